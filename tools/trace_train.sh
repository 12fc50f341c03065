# rocprofv3 kernel trace of one C3 training step (tools/train_trace_c3.py) + its per-kernel sum:
#   bash tools/trace_train.sh <tag> [VAR=value ...]
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/trace_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp || exit 1
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/raw" -o run \
  -- python3 "$R/tools/train_trace_c3.py" > "$out/run.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
python3 "$R/tools/timeline.py" "$out/raw" --bursts -1 --sum > "$out/sum.txt" 2>&1
echo done $tag
