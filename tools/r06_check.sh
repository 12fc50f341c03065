# Re-entry check of the restored tree: eval probe (new kernel), GPU suite + smoke, default C3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/chk
timeout -k 10 300 python -u tools/eval_probe.py --reps 3 > gpurun_out/chk/eval.log 2>&1 || { tail -20 gpurun_out/chk/eval.log; exit 1; }
cat gpurun_out/chk/eval.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/chk/gpu_tests.log 2>&1 || { tail -40 gpurun_out/chk/gpu_tests.log; exit 1; }
tail -2 gpurun_out/chk/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/chk/gpu_tests.log 2>&1 || exit 1
tail -1 gpurun_out/chk/gpu_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/chk/bench_c3.log 2>&1 || exit 1
tail -1 gpurun_out/chk/bench_c3.log | cut -c1-600
