#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit, logging to
# gpurun_out/<name>.log. Ordinary failures (test failures, Python exceptions: rc 1/2/5) go on to
# the next step; a fault, abort, segfault or time limit (any other rc) ends the script at once.
#   tools/gpu_steps.sh "name:timeout_s:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name (limit ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 8 "gpurun_out/$name.log"
  case $rc in 0|1|2|5) ;; *) echo "=== fatal rc=$rc: stopping"; exit "$rc";; esac
  # a GPU fault caught as a Python exception still ends the call
  if grep -q -E "illegal memory access|hipErrorIllegalAddress|Memory access fault|HSA_STATUS_ERROR|page fault" "gpurun_out/$name.log"; then
    echo "=== GPU fault signature in $name.log: stopping"; exit 99
  fi
done
