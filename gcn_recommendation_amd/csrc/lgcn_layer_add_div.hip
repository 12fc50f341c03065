// lgcn_layer_add_div.hip — k_layer instantiations for the ADD epilogue, X = G / (K+1) on load: the backward's first layer.
// One translation unit per epilogue variant so hipcc compiles them in parallel (lgcn_kernels.h).
#include "lgcn_kernels.h"

namespace lgcn_detail {
int layer_add_div(const LayerArgs& a, int xd) {
    return xd == 2 ? layer_mode<LGCN_EPI_ADD, 2>(a) : layer_mode<LGCN_EPI_ADD, 1>(a);
}
}  // namespace lgcn_detail
