# round 6: the row-sparse backward on lane 0's streams shared by both lanes (LGCN_SCHED_LANE1_SHARED)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sides.py tests/test_gpu_training.py tests/test_gpu_exact.py tests/test_gpu_capture.py \
  > gpurun_out/r06_t8.log 2>&1 || { tail -40 gpurun_out/r06_t8.log; exit 1; }
tail -2 gpurun_out/r06_t8.log
rm -f gpurun_out/ab.log
export DENSE=1
bash tools/gpu_ab.sh product || exit 1
grep -E "^==|median" gpurun_out/ab.log
bash tools/trace_fwd.sh r06b || exit 1
