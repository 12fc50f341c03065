set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_training.py > gpurun_out/t_train.log 2>&1 || exit 1
for rep in 1 2; do
  for dir in . _ab; do
    echo "== $dir" >> gpurun_out/ab_train.log
    (cd $dir && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --recall-epochs 0 --no-c4 --train-steps 10 2>&1 | grep -E "train|^\{" ) >> gpurun_out/ab_train.log || exit 1
  done
done
