# round 6: the capture fix — C host (7.2 runtime: full schedule captured), the same binary on the
# torch wheel's 7.0 runtime (restricted schedule), the torch probe, and the sided / capture GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/capture_host 3 both > gpurun_out/cap6_host72.log 2>&1 \
  || { cat gpurun_out/cap6_host72.log; exit 1; }
cat gpurun_out/cap6_host72.log
TL=$(python -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/hip70 && ln -sf $TL/libamdhip64.so /tmp/hip70/libamdhip64.so.7
LD_LIBRARY_PATH=/tmp/hip70:$TL timeout -k 10 120 ./tools/capture_host 3 both > gpurun_out/cap6_host70.log 2>&1 \
  || { cat gpurun_out/cap6_host70.log; exit 1; }
cat gpurun_out/cap6_host70.log
timeout -k 10 300 python -u tools/capture_torch.py engine > gpurun_out/cap6_torch.log 2>&1 \
  || { grep -v amdgpu.ids gpurun_out/cap6_torch.log | tail; exit 1; }
grep -v amdgpu.ids gpurun_out/cap6_torch.log | tail -4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sides.py tests/test_gpu_capture.py tests/test_gpu_training.py > gpurun_out/r06_t6.log 2>&1 \
  || { tail -40 gpurun_out/r06_t6.log; exit 1; }
tail -2 gpurun_out/r06_t6.log
