# A/B of the C3 forward / BPR backward (tools/fwd_trace.py medians), interleaved twice:
#   bash tools/gpu_ab.sh product 'product@LGCN_CLASSES=0' r04
# product = this tree; r04 = the round-4 tree in _r04/ (git worktree, its own library); any
# other name = this tree with gcn_recommendation_amd/_variants/liblgcn_<name>.so (LGCN_LIB);
# spec@VAR=v;VAR2=w adds environment settings.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    tree=${spec%%@*}; envs=""
    [ "$spec" != "$tree" ] && envs=$(echo "${spec#*@}" | tr ';' ' ')
    dir=.; [ $tree = r04 ] && dir=_r04
    L=""; [ $tree != product ] && [ $tree != r04 ] && L=gcn_recommendation_amd/_variants/liblgcn_$tree.so
    echo "== $spec" >> gpurun_out/ab.log
    (cd $dir && env $envs LGCN_LIB=$L FWD_ONLY=1 REPS=15 timeout -k 10 240 python -u tools/fwd_trace.py 2>&1 | grep -v amdgpu.ids) >> gpurun_out/ab.log || exit 1
  done
done
