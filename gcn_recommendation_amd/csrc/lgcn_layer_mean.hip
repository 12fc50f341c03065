// lgcn_layer_mean.hip — k_layer instantiations for the MEAN epilogue: the forward's last layer with the fused K+1-layer mean.
// One translation unit per epilogue variant so hipcc compiles them in parallel (lgcn_kernels.h).
#include "lgcn_kernels.h"

namespace lgcn_detail {
int layer_mean(const LayerArgs& a) { return layer_mode<LGCN_EPI_MEAN>(a); }
}  // namespace lgcn_detail
