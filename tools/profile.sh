#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of one bench
# command, on the gpurun box. Outputs under gpurun_out/prof_<tag>/.
#   tools/profile.sh <tag> <bench args...>
set -u
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
  -- python3 "$R/bench.py" "$@" > "$out/trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$c" -o run \
    -- python3 "$R/bench.py" "$@" > "$out/pmc_$c.log" 2>&1 || { echo "pmc $c rc=$?"; exit 1; }
done
echo done
