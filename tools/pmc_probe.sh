#!/bin/bash
# rocprofv3 kernel trace + one PMC pass per counter set of any python tool, on the gpurun box.
#   tools/pmc_probe.sh <tag> "<counters pass 1>" ["<counters pass 2>" ...] -- <script.py> [args...]
# Outputs under gpurun_out/pmc_<tag>/{trace,pass1,pass2,...}. Each pass is its own run (never
# combined with tracing domains), each under its own time limit.
set -u
tag=$1; shift
sets=()
while [ "$#" -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
script=$1; shift
case $script in /*) ;; *) script=$R/$script;; esac
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
  -- python3 "$script" "$@" > "$out/trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
i=0
for s in "${sets[@]}"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $s --output-format csv -d "$out/pass$i" -o run \
    -- python3 "$script" "$@" > "$out/pass$i.log" 2>&1 || { echo "pmc pass $i ($s) rc=$?"; exit 1; }
done
echo done
