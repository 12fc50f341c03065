# round 6: forward timeline of the current product, then the C host capture of the library on the
# HIP runtime bundled with the torch wheel (ROCm 7.0) instead of /opt/rocm's (7.2) — last: may crash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/trace_fwd.sh r06 || exit 1
for rep in 1 2; do for L in "" gcn_recommendation_amd/_variants/liblgcn_evthr.so; do
  LGCN_LIB=$L timeout -k 10 180 python -u tools/eval_probe.py --reps 5 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/eval_ab.log || exit 1
done; done
TL=$(python -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/hip70 && ln -sf $TL/libamdhip64.so /tmp/hip70/libamdhip64.so.7
echo "torch HIP runtime: $TL/libamdhip64.so"
LD_LIBRARY_PATH=/tmp/hip70:$TL timeout -k 10 120 ./tools/capture_host_engine 3 both > gpurun_out/cap_engine_hip70.log 2>&1
rc=$?; cat gpurun_out/cap_engine_hip70.log; echo "capture_host_engine on torch's runtime rc=$rc"; [ $rc = 0 ] || exit 1
LD_LIBRARY_PATH=/tmp/hip70:$TL timeout -k 10 120 ./tools/capture_host_capaux 3 forward > gpurun_out/cap_aux_hip70.log 2>&1
rc=$?; cat gpurun_out/cap_aux_hip70.log; echo "capture_host_capaux on torch's runtime rc=$rc"
exit $rc
