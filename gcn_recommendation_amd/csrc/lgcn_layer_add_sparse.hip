// lgcn_layer_add_sparse.hip — k_layer instantiations for the ADD epilogue over a row-sparse G (zero rows skipped): the backward's first layer of a BPR batch.
// One translation unit per epilogue variant so hipcc compiles them in parallel (lgcn_kernels.h).
#include "lgcn_kernels.h"

namespace lgcn_detail {
int layer_add_sparse(const LayerArgs& a, int xd) {
    switch (xd) {
        case 4: return layer_mode<LGCN_EPI_ADD, 4>(a);
        case 5: return layer_mode<LGCN_EPI_ADD, 5>(a);
        default: return layer_mode<LGCN_EPI_ADD, 6>(a);
    }
}
}  // namespace lgcn_detail
