# eval kernel A/B: tools/eval_probe.py per variant library, interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    L=gcn_recommendation_amd/_variants/liblgcn_$v.so; [ $v = product ] && L=""
    LGCN_LIB=$L timeout -k 10 120 python -u tools/eval_probe.py --reps 3 2>&1 | grep -v amdgpu.ids >> gpurun_out/eval_ab.log || exit 1
  done
done
cat gpurun_out/eval_ab.log
