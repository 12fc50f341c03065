# Final-tree check: GPU suite + smoke (outputs under gpurun_out/final2/)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/final2/gpu_tests.log 2>&1 || { tail -40 gpurun_out/final2/gpu_tests.log; exit 1; }
tail -2 gpurun_out/final2/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/final2/gpu_tests.log 2>&1 || exit 1
tail -1 gpurun_out/final2/gpu_tests.log
