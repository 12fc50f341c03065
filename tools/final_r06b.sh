# Round-6 remaining evidence: GPU suite + smoke, C2 / C5 bench lines, featsplit per-rank sweeps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/final/gpu_tests.log 2>&1 || { tail -40 gpurun_out/final/gpu_tests.log; exit 1; }
tail -2 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/final/gpu_tests.log 2>&1 || exit 1
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 600 python -u bench.py --config c2 > gpurun_out/final/bench_c2.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/final/bench_c5.log 2>&1 || exit 1
LGCN_SIDES_FEATSPLIT=1 timeout -k 10 900 python -u tools/featsplit_sweep.py --config c4 --dims 256,128,64,32 --steps 3 > gpurun_out/final/featsplit_c4.log 2>&1 || exit 1
LGCN_SIDES_FEATSPLIT=1 timeout -k 10 600 python -u tools/featsplit_sweep.py --config c3 --steps 5 > gpurun_out/final/featsplit_c3.log 2>&1 || exit 1
grep ms_per_step gpurun_out/final/featsplit_c4.log gpurun_out/final/featsplit_c3.log | cut -c1-200
