#!/bin/bash
# rocprofv3 kernel-trace + stats only (no PMC) of one bench command.  tools/profile_trace.sh <tag> <bench args...>
set -u
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
  -- python3 "$R/bench.py" "$@" > "$out/trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
echo done
