// lgcn_layer_store.hip — k_layer instantiations for the STORE epilogue (Y = Â·X): the forward's layers 1..K-1.
// One translation unit per epilogue variant so hipcc compiles them in parallel (lgcn_kernels.h).
#include "lgcn_kernels.h"

namespace lgcn_detail {
int layer_store(const LayerArgs& a) { return layer_mode<LGCN_EPI_STORE>(a); }
}  // namespace lgcn_detail
