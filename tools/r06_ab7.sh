# round 6 A/B 7: the chain kernel's grid resident at once (LGCN_TUNE_CHAIN_PER_CU 1, 2) vs one
# workgroup per (row, slice) item; plus the chain-grid bitwise test
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_exact.py -k "chain_grid or widths or giant" > gpurun_out/r06_t7.log 2>&1 \
  || { tail -40 gpurun_out/r06_t7.log; exit 1; }
tail -2 gpurun_out/r06_t7.log
rm -f gpurun_out/ab.log
bash tools/gpu_ab.sh product 'product@TUNE_CHAIN=1' 'product@TUNE_CHAIN=2' 'product@LGCN_TORCH_STREAMS=1' || exit 1
cat gpurun_out/ab.log
