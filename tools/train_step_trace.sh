#!/bin/bash
# Memory-copy trace of tools/train_step_trace.py at two step counts (kernel + memory-copy
# domains only, no PMC). Outputs under gpurun_out/memcpy_<N>/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
for N in 10 40; do
  out=$R/gpurun_out/memcpy_$N
  mkdir -p "$out"
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d "$out" -o run -- python3 "$R/tools/train_step_trace.py" --steps $N > "$out/log.txt" 2>&1 \
    || { echo "trace N=$N rc=$?"; exit 1; }
done
echo done
