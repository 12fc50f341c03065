# round 6 A/B 10: the walk's prediction margin (LGCN_TUNE_EMU_MARGIN = base << 4 | shift;
# default 128 << 4 | 4): wider margins fetch more blocks ahead, fewer on-demand fetches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
bash tools/gpu_ab.sh product 'product@TUNE=6:8194' 'product@TUNE=6:32769' 'product@TUNE=6:2051' || exit 1
grep -E "^==|median" gpurun_out/ab.log
LGCN_LIB=gcn_recommendation_amd/_variants/liblgcn_emustats.so timeout -k 10 300 python -u tools/walk_phase_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/walk_phases.log
