# Round-6 C3 evidence in one call (outputs under gpurun_out/final/, copied into profiles/ after):
# rocprofv3 kernel trace + separate PMC passes of the bench command, the stamped traffic file,
# then the default bench line that reads it, and the GPU suite + smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
bash tools/profile.sh c3 --steps 10 --no-cpu-baseline --train-steps 0 --recall-epochs 0 --no-c4 || exit 1
python tools/summarize_profile.py gpurun_out/prof_c3 c3_powerlaw r06 6828419628 > gpurun_out/final/summary.txt 2>&1 || exit 1
cp profiles/traffic_c3_powerlaw.json profiles/r06_c3_powerlaw_kernel_stats.csv gpurun_out/final/
timeout -k 10 900 python -u bench.py > gpurun_out/final/bench_c3.log 2>&1 || exit 1
tail -1 gpurun_out/final/bench_c3.log | cut -c1-400
