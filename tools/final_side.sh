# Round-end side evidence in one call: smoke(), the C2 and C5 bench lines, the N>1 bench path at
# world size 1 over RCCL. Outputs under gpurun_out/final2/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final2/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --config c2 > gpurun_out/final2/bench_c2.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --config c5 > gpurun_out/final2/bench_c5.log 2>&1 || exit 1
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --force-dist --steps 10 --warmup 2 > gpurun_out/final2/bench_dist_world1.log 2>&1 || exit 1
