// lgcn_layer_add.hip — k_layer instantiations for the ADD epilogue, X gathered as is: the backward's layers 2..K.
// One translation unit per epilogue variant so hipcc compiles them in parallel (lgcn_kernels.h).
#include "lgcn_kernels.h"

namespace lgcn_detail {
int layer_add(const LayerArgs& a, int) { return layer_mode<LGCN_EPI_ADD, 0>(a); }
}  // namespace lgcn_detail
