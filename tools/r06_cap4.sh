# round 6: GPU suite on the current tree, then the torch-capture discrimination (prealloc: the
# library call alone under torch.cuda.graph; relaxed: CapturedForward-like, relaxed capture mode)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r06_gpu_tests.log
export LGCN_LIB=gcn_recommendation_amd/_variants/liblgcn_capaux.so
timeout -k 10 300 python -u tools/capture_torch.py prealloc > gpurun_out/cap_torch_prealloc.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/cap_torch_prealloc.log | tail -8; echo "prealloc rc=$rc"; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u tools/capture_torch.py relaxed > gpurun_out/cap_torch_relaxed.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/cap_torch_relaxed.log | tail -8; echo "relaxed rc=$rc"
exit $rc
