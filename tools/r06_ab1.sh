# round 6 A/B 1: layer-K items kernel at normal priority, NT stage stores, dense backward mask skip
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sides.py tests/test_gpu_training.py > gpurun_out/r06_t1.log 2>&1 || { tail -30 gpurun_out/r06_t1.log; exit 1; }
tail -2 gpurun_out/r06_t1.log
export DENSE=1
bash tools/gpu_ab.sh product 'product@LGCN_LK_NORMAL=1' stnt 'product@LGCN_DENSE_SKIP_MASK=0' || exit 1
cat gpurun_out/ab.log
bash tools/trace_fwd.sh lkn LGCN_LK_NORMAL=1 || exit 1
