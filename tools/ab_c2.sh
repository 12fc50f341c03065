# C2 forward A/B over environments (same spec syntax as tools/ab_fwd.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    lib=${spec%%@*}; envs=""
    [ "$spec" != "$lib" ] && envs=$(echo "${spec#*@}" | tr ';' ' ')
    if [ $lib = product ]; then L=""; else L=gcn_recommendation_amd/_variants/liblgcn_$lib.so; fi
    echo "== $spec" >> gpurun_out/abc2.log
    env $envs CFG=c2 LGCN_LIB=$L FWD_ONLY=1 REPS=30 timeout -k 10 180 python -u tools/fwd_trace.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/abc2.log || exit 1
  done
done
