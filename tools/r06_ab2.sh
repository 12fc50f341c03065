# round 6 A/B 2: dedicated hardware queues for the backward's lane 1; C-host capture of the
# library's sided forward (product library, then the LGCN_CAPTURE_AUX_EXP build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_sides.py tests/test_gpu_training.py tests/test_gpu_exact.py > gpurun_out/r06_t2.log 2>&1 \
  || { tail -40 gpurun_out/r06_t2.log; exit 1; }
tail -2 gpurun_out/r06_t2.log
rm -f gpurun_out/ab.log
export DENSE=1
bash tools/gpu_ab.sh product 'product@LGCN_DEDICATED_Q=1' || exit 1
cat gpurun_out/ab.log
timeout -k 10 120 ./tools/capture_host_engine 3 both > gpurun_out/cap_engine.log 2>&1
rc=$?; cat gpurun_out/cap_engine.log; echo "capture_host_engine rc=$rc"; [ $rc = 0 ] || exit 1
timeout -k 10 120 ./tools/capture_host_capaux 3 forward > gpurun_out/cap_aux_fwd.log 2>&1
rc=$?; cat gpurun_out/cap_aux_fwd.log; echo "capture_host_capaux forward rc=$rc"
exit $rc
