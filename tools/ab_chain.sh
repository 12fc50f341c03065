# GPU suite, then the C3 forward / BPR-backward A/B of this tree vs a variant library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || exit 1
bash tools/gpu_ab.sh product "$@"
