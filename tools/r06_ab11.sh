# round 6 A/B 11: the walk's vmcnt waits on a finer ladder (refills no longer wait for the ~6
# refills issued after their own), vs product; the hint-ring test on the current engine
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sides.py \
  -k "hint_ring or shared or bitwise" > gpurun_out/r06_t11.log 2>&1 || { tail -30 gpurun_out/r06_t11.log; exit 1; }
tail -1 gpurun_out/r06_t11.log
rm -f gpurun_out/ab.log
export DENSE=1
bash tools/gpu_ab.sh product vmfine || exit 1
grep -E "^==|median" gpurun_out/ab.log
