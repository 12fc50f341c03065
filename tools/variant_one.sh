# A/B variant library: the product objects with ONE source rebuilt under extra defines
#   bash tools/variant_one.sh name lgcn_exact.hip "-DX=1 -DY=2"   -> _variants/liblgcn_name.so
set -e
cd "$(dirname "$0")/.."
O=gcn_recommendation_amd/_obj
n=$1; src=$2; defs=$3
mkdir -p gcn_recommendation_amd/_variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -I include \
  -I gcn_recommendation_amd/csrc $defs -c gcn_recommendation_amd/csrc/$src -o /tmp/var_$n.o
objs=$(ls $O/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/var_$n.o \
  -o gcn_recommendation_amd/_variants/liblgcn_$n.so
echo built $n
