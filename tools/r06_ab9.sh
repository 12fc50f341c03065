# round 6 A/B 9: the row-sparse backward's lane 1 on lane 0's streams (shared) vs round 5's four
# pooled torch streams (HIP pairs them with lane 0's queues)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
bash tools/gpu_ab.sh product 'product@LGCN_BWD_R05=1' || exit 1
grep -E "^==|median" gpurun_out/ab.log
