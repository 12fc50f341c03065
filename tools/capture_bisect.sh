#!/bin/bash
# Bisect the two-lane HIP-graph capture crash: each case in its own process (a host segfault in
# hipStreamEndCapture ends only that process). Usage: tools/capture_bisect.sh [K...]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for K in ${@:-1 2 3}; do
  for bf in 1 0; do
    for aux in 3 4 5 7; do
      LGCN_CAPTURE_AUX=$aux LGCN_BLOCKS_FIRST=$bf timeout -k 5 120 python -u tools/capture_probe.py $aux $K > gpurun_out/cap.txt 2>&1
      rc=$?
      echo "K=$K blocks_first=$bf aux=$aux rc=$rc :: $(tail -2 gpurun_out/cap.txt | tr '\n' ' ')"
    done
  done
done
