# A/B of C3 forward / BPR backward timing over library variants (product = the in-tree build):
#   bash tools/ab_fwd.sh product s32 s64   (each twice, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    if [ $lib = product ]; then L=""; else L=gcn_recommendation_amd/_variants/liblgcn_$lib.so; fi
    LGCN_LIB=$L FWD_ONLY=1 REPS=15 timeout -k 10 180 python -u tools/fwd_trace.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab.log || exit 1
  done
done
