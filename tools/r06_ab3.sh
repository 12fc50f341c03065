# round 6 A/B 3: the walk at issue priority 3 (s_setprio) vs product; C-host capture with brand
# hubs (LGCN_CAPTURE_AUX_EXP library); torch capture of the same library (last: may crash)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
bash tools/gpu_ab.sh product wprio || exit 1
cat gpurun_out/ab.log
timeout -k 10 120 ./tools/capture_host_capaux 3 both > gpurun_out/cap_aux_both.log 2>&1
rc=$?; cat gpurun_out/cap_aux_both.log; echo "capture_host_capaux both rc=$rc"; [ $rc = 0 ] || exit 1
LGCN_LIB=gcn_recommendation_amd/_variants/liblgcn_capaux.so timeout -k 10 300 python -u tools/capture_torch.py > gpurun_out/cap_torch.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/cap_torch.log | tail -30; echo "capture_torch rc=$rc"
exit $rc
