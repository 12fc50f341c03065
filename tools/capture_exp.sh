# One capture-crash experiment (LGCN_CAPTURE_EXP bits, lgcn_engine.hip cap_exp; capdbg variant
# build): the sided C3-like forward captured with 7 aux streams. A host segfault ends the call:
# run it as the LAST step of a GPU command.  Usage: tools/capture_exp.sh EXP [K]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
LGCN_LIB=gcn_recommendation_amd/_variants/liblgcn_capdbg.so LGCN_CAPTURE_EXP=$1 \
  timeout -k 5 120 python -u tools/capture_probe.py 7 ${2:-3} > gpurun_out/capexp_$1.txt 2>&1
rc=$?
echo "EXP=$1 rc=$rc :: $(tail -2 gpurun_out/capexp_$1.txt | tr '\n' ' ')" | tee -a gpurun_out/capexp.log
exit $rc
