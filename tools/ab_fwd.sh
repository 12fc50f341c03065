# A/B of C3 forward / BPR backward timing over library variants and environments, interleaved
# twice (product = the in-tree build; lib@VAR=v;VAR2=w adds environment settings):
#   bash tools/ab_fwd.sh product s32 'product@LGCN_MEAN_EARLY=0;LGCN_EMU_SLOTS=20,4'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    lib=${spec%%@*}; envs=""
    [ "$spec" != "$lib" ] && envs=$(echo "${spec#*@}" | tr ';' ' ')
    if [ $lib = product ]; then L=""; else L=gcn_recommendation_amd/_variants/liblgcn_$lib.so; fi
    echo "== $spec" >> gpurun_out/ab.log
    env $envs LGCN_LIB=$L FWD_ONLY=1 REPS=15 timeout -k 10 180 python -u tools/fwd_trace.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab.log || exit 1
  done
done
