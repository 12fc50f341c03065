// lgcn_engine.hip — MI355X (gfx950, CDNA4) kernels + C ABI for LightGCN propagation.
//
// Replaces, for a HIP device, the reference hot path (models/lightgcn.py:37-59 and
// models/lightgcn_fusion.py:52-59): E_{k+1} = Â·E_k for K layers (torch.sparse.mm, lightgcn.py:45),
// the layer mean (lightgcn.py:54), and the autograd backward of both. Declarations and the
// numerics contract: include/lgcn.h. Design and byte model: DESIGN.md.
//
// Kernel shape (HBM-bound sparse gather-reduce, no MFMA):
//  * a row of Â is owned by a group of G lanes (G = d/4 rounded to a power of two, <= 64), each
//    lane holding NV float4 columns of the output row: a gathered 256-B row of X at d=64 is ONE
//    coalesced 16-lane dwordx4 access; a wave64 works on 64/G rows at once.
//  * each group walks its row's 8-byte {col,val} edge records in stored order, issues U gathers
//    before consuming any (memory-level parallelism), then folds them with v_fma_f32 in order —
//    the same sequential fmaf chain ATen's CPU addmm_sparse_dense loop runs, so results are bitwise
//    identical to the reference CPU path for every row the chain covers.
//  * rows longer than hub_threshold are cut into chunks (host plan) that run in the SAME launch
//    (blocks [0, hub_blocks)), writing partial sums; k_hub_combine finishes them in fixed order.
//  * the epilogue is fused: store, the K+1-layer mean (reads E0..E_{K-1} rows, sums in order,
//    divides), or the backward's Horner add. E0 is read as three segments (no torch.cat copy).
#include "lgcn_kernels.h"

#include <string.h>
#include <algorithm>
#include <functional>
#include <new>
#include <vector>

namespace lgcn_detail {
int g_rows_per_group = 0;
int g_unroll = 0;
int g_mean_prefetch = 0;
int g_min_groups = 0;
int g_emu_margin = (128 << 4) | 4;  // LGCN_TUNE_EMU_MARGIN (the walk's prediction margin)
}  // namespace lgcn_detail

namespace {
// ---------------------------------------------------------------------------------------------
// COO -> CSR preparation kernels
// ---------------------------------------------------------------------------------------------
__global__ void k_coo_inspect(const int64_t* __restrict__ rows, const int64_t* __restrict__ cols,
                              int64_t nnz, int32_t n_rows, int32_t n_cols, int32_t* flags) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    const int64_t r = rows[j], c = cols[j];
    int f = 0;
    if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) f |= LGCN_COO_OUT_OF_RANGE;
    if (j > 0) {
        const int64_t rp = rows[j - 1];
        if (r < rp) f |= LGCN_COO_ROWS_UNSORTED;
        else if (r == rp && c <= cols[j - 1]) f |= LGCN_COO_COLS_UNSORTED;
    }
    if (f) atomicOr(flags, f);
}

__global__ void k_csr_edges(const int64_t* __restrict__ other, const float* __restrict__ vals,
                            int64_t nnz, const int32_t* __restrict__ perm,
                            lgcn_edge_t* __restrict__ edges) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    const int64_t src = perm ? perm[j] : j;
    const uint32_t c = (uint32_t)other[src];
    const uint32_t v = __float_as_uint(vals[src]);
    edges[j] = (lgcn_edge_t)(((uint64_t)v << 32) | c);
}

// rowptr[r] = first j with key(j) >= r (binary search; keys sorted): no atomics, deterministic.
__global__ void k_csr_rowptr(const int64_t* __restrict__ keys64, const int32_t* __restrict__ keys32,
                             int64_t nnz, int32_t n_rows, int32_t* __restrict__ rowptr) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > n_rows) return;
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int64_t k = keys32 ? (int64_t)keys32[mid] : keys64[mid];
        if (k < r) lo = mid + 1; else hi = mid;
    }
    rowptr[r] = (int32_t)lo;
}

__global__ void k_keys_iota(const int64_t* __restrict__ keys, int64_t nnz, int32_t* __restrict__ k32,
                            int32_t* __restrict__ perm) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    k32[j] = (int32_t)keys[j];
    perm[j] = (int32_t)j;
}

__global__ void k_csr_symmetric(const int32_t* __restrict__ rowptr,
                                const lgcn_edge_t* __restrict__ edges, int32_t n_rows,
                                int64_t nnz, int32_t* asym) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    // row of edge j: last r with rowptr[r] <= j
    int32_t lo = 0, hi = n_rows - 1;
    while (lo < hi) {
        const int32_t mid = (lo + hi + 1) >> 1;
        if (rowptr[mid] <= j) lo = mid; else hi = mid - 1;
    }
    const int32_t r = lo;
    const int2 e = load_edge(edges + j);
    const int32_t c = e.x;
    int32_t a = rowptr[c], b = rowptr[c + 1];
    while (a < b) {
        const int32_t mid = (a + b) >> 1;
        if (load_edge(edges + mid).x < r) a = mid + 1; else b = mid;
    }
    if (a >= rowptr[c + 1] || load_edge(edges + a).x != r || load_edge(edges + a).y != e.y)
        atomicOr(asym, 1);
}

// Processing order: slots sorted by degree (descending, stable). The lane groups of a wave then
// stream rows of equal length (no group idles while a longer neighbour finishes) and hub rows
// come first. Each row keeps its own edge order, so every output row is the same fp32 chain.
// side_bit: set on the rows outside [lo, hi) (sorted descending, they take the first slots)
__device__ __forceinline__ int32_t side_flag(int64_t r, int32_t lo, int32_t hi, int32_t side_bit) {
    return (r >= lo && r < hi) ? 0 : side_bit;
}

__global__ void k_csr_degrees(const int32_t* __restrict__ rowptr, int32_t n, int32_t lo,
                              int32_t hi, int32_t side_bit, int32_t* __restrict__ deg,
                              int32_t* __restrict__ iota) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    deg[r] = (rowptr[r + 1] - rowptr[r]) | side_flag(r, lo, hi, side_bit);
    iota[r] = (int32_t)r;
}

__global__ void k_csr_mask_degrees(int32_t* __restrict__ deg, int32_t n, int32_t mask) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) deg[s] &= mask;
}

// bad |= some edge joins two rows on the same side of [lo, hi) (row of edge j by binary search)
__global__ void k_csr_bipartite(const int32_t* __restrict__ rowptr,
                                const lgcn_edge_t* __restrict__ edges,
                                const int32_t* __restrict__ row_ids, int32_t n_rows, int64_t nnz,
                                int32_t lo, int32_t hi, int32_t* bad) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    int32_t a = 0, b = n_rows - 1;
    while (a < b) {
        const int32_t mid = (a + b + 1) >> 1;
        if (rowptr[mid] <= j) a = mid; else b = mid - 1;
    }
    const int32_t r = row_ids ? row_ids[a] : a;
    const int32_t c = load_edge(edges + j).x;
    if ((r >= lo && r < hi) == (c >= lo && c < hi)) atomicOr(bad, 1);
}

// rank[row_ids[s]] = s: position of every row in the degree-descending order
__global__ void k_csr_rank(const int32_t* __restrict__ row_ids, int32_t n, int32_t* __restrict__ rank) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    rank[row_ids[s]] = (int32_t)s;
}

// Tie-break key of the slot order: among rows of equal degree, rows whose least popular
// neighbour (highest degree rank) is the same sit next to each other, so a neighbour's row
// gathers them from consecutive slots (several rows of a narrow shard per 128-B line).
// comp = deg << 32 | ~(key + 1), sorted descending: degree descending, then key ascending;
// rows above kKeyMaxDeg (hubs: their degrees rarely tie) and empty rows get key 0.
constexpr int32_t kKeyMaxDeg = 256;
__global__ void k_csr_degree_key(const int32_t* __restrict__ rowptr,
                                 const lgcn_edge_t* __restrict__ edges, int32_t n,
                                 const int32_t* __restrict__ rank, int32_t lo, int32_t hi,
                                 int32_t side_bit, uint64_t* __restrict__ comp,
                                 int32_t* __restrict__ iota) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int32_t b = rowptr[r], e = rowptr[r + 1];
    uint32_t key = 0;
    if (e - b <= kKeyMaxDeg)
        for (int32_t j = b; j < e; ++j) {
            const uint32_t k = (uint32_t)rank[(int32_t)edges[j]] + 1u;
            key = k > key ? k : key;
        }
    comp[r] = ((uint64_t)(uint32_t)((e - b) | side_flag(r, lo, hi, side_bit)) << 32) |
              (uint64_t)(0xFFFFFFFFu - key);
    iota[r] = (int32_t)r;
}

__global__ void k_csr_slot_degrees(const int32_t* __restrict__ row_ids,
                                   const int32_t* __restrict__ deg, int32_t n, int32_t mask,
                                   int32_t* __restrict__ deg_sorted) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    deg_sorted[s] = deg[row_ids[s]] & mask;
}

// edges_out[j] = the edge record of slot s (binary search: rowptr_out[s] <= j < rowptr_out[s+1])
__global__ void k_csr_gather_rows(const int32_t* __restrict__ rowptr_out,
                                  const int32_t* __restrict__ row_ids,
                                  const int32_t* __restrict__ rowptr,
                                  const lgcn_edge_t* __restrict__ edges, int32_t n, int64_t nnz,
                                  lgcn_edge_t* __restrict__ edges_out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    int32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const int32_t mid = (lo + hi + 1) >> 1;
        if (rowptr_out[mid] <= j) lo = mid; else hi = mid - 1;
    }
    edges_out[j] = edges[rowptr[row_ids[lo]] + (j - rowptr_out[lo])];
}

// edges_out[j] = edges[j] with its column id c replaced by new_id[c] (value bits kept)
__global__ void k_csr_relabel_cols(const lgcn_edge_t* __restrict__ edges, int64_t nnz,
                                   const int32_t* __restrict__ new_id,
                                   lgcn_edge_t* __restrict__ edges_out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    const int2 e = load_edge(edges + j);
    edges_out[j] = (lgcn_edge_t)(((uint64_t)(uint32_t)e.y << 32) | (uint32_t)new_id[e.x]);
}

// ---------------------------------------------------------------------------------------------
// side-0 classes of a bipartite slot order (lgcn_csr_side_classes): a side-0 row (user / brand)
// is class 0 when it is linked to a side-1 row of part 0 (the longest, walked item rows), class 1
// when linked to a part-1 row only, class 2 otherwise. Stored class-major (each class keeps its
// degree order), the half-layers of side 0 run one class at a time, and a walked part of the
// next side-1 half-layer waits only for the classes it reads (lgcn_propagate_*_sides).
// ---------------------------------------------------------------------------------------------
__global__ void k_fill_i32(int32_t* __restrict__ p, int64_t n, int32_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// mark[col] = min(mark[col], part) for every edge of side-1 slot s_lo + blockIdx.x (part 0 below
// s_mid, 1 above); gridDim.y blocks stride over the slot's edges
__global__ void k_class_mark(const int32_t* __restrict__ rowptr,
                             const lgcn_edge_t* __restrict__ edges, int32_t s_lo, int32_t s_mid,
                             int32_t* __restrict__ mark) {
    const int32_t slot = s_lo + (int32_t)blockIdx.x;
    const int32_t part = slot < s_mid ? 0 : 1;
    const int64_t end = rowptr[slot + 1];
    for (int64_t j = rowptr[slot] + (int64_t)blockIdx.y * blockDim.x + threadIdx.x; j < end;
         j += (int64_t)gridDim.y * blockDim.x)
        atomicMin(mark + load_edge(edges + j).x, part);
}

// partof[row_ids[s_lo + i]] = part of side-1 slot s_lo + i (0 below s_mid, 1 above)
__global__ void k_class_partof(const int32_t* __restrict__ row_ids, int32_t s_lo, int32_t s_mid,
                               int32_t s_hi, int32_t* __restrict__ partof) {
    const int64_t s = s_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= s_hi) return;
    partof[row_ids[s]] = s < s_mid ? 0 : 1;
}

// the other direction (Â need not be structurally symmetric): side-0 slot s reads a walked
// side-1 row -> mark[row_ids[s]] = min(mark, that row's part); one thread per side-0 slot
__global__ void k_class_mark_rev(const int32_t* __restrict__ rowptr,
                                 const lgcn_edge_t* __restrict__ edges,
                                 const int32_t* __restrict__ row_ids, int32_t n0,
                                 const int32_t* __restrict__ partof, int32_t* __restrict__ mark) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n0) return;
    int m = 2;
    for (int64_t j = rowptr[s], end = rowptr[s + 1]; j < end && m > 0; ++j)
        m = min(m, partof[load_edge(edges + j).x]);
    if (m < 2) atomicMin(mark + row_ids[s], m);
}

__global__ void k_class_keys(const int32_t* __restrict__ row_ids, const int32_t* __restrict__ mark,
                             int32_t n0, int32_t* __restrict__ key, int32_t* __restrict__ iota) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n0) return;
    key[s] = mark[row_ids[s]];
    iota[s] = (int32_t)s;
}

// the new slot s takes old slot src = perm0[s] (side 0, class-sorted) or s (side 1)
__global__ void k_class_apply(const int32_t* __restrict__ perm0, const int32_t* __restrict__ rowptr,
                              const int32_t* __restrict__ row_ids, int32_t split, int32_t n,
                              int32_t* __restrict__ perm, int32_t* __restrict__ deg,
                              int32_t* __restrict__ row_ids_out) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const int32_t src = s < split ? perm0[s] : (int32_t)s;
    perm[s] = src;
    deg[s] = rowptr[src + 1] - rowptr[src];
    row_ids_out[s] = row_ids[src];
}

// class_end[c] = first side-0 slot of a class above c (keys sorted ascending); one thread
__global__ void k_class_bounds(const int32_t* __restrict__ key_sorted, int32_t n0,
                               int32_t* __restrict__ class_end) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int c = 0; c < 2; ++c) {
        int32_t a = 0, b = n0;
        while (a < b) {
            const int32_t mid = (a + b) >> 1;
            if (key_sorted[mid] <= c) a = mid + 1; else b = mid;
        }
        class_end[c] = a;
    }
}

// ---------------------------------------------------------------------------------------------
// adjacency builder (main.py:313-336 on the device): degree histogram, duplicate merge by a
// 64-bit radix sort of row*n+col keys + run-length encode, values fp32((d_r * m) * d_c)
// ---------------------------------------------------------------------------------------------
// deg[r] = (first sorted key >= (r+1)*n) - (first sorted key >= r*n): raw edges of row r,
// duplicates included; binary search, no atomics (a 2.77M-degree hub made atomics serialise)
__global__ void k_adj_degree(const uint64_t* __restrict__ keys, int64_t n_edges, int64_t n,
                             int32_t* __restrict__ deg) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    int64_t b[2];
    for (int t = 0; t < 2; ++t) {
        const uint64_t target = (uint64_t)(r + t) * (uint64_t)n;
        int64_t lo = 0, hi = n_edges;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < target) lo = mid + 1; else hi = mid;
        }
        b[t] = lo;
    }
    deg[r] = (int32_t)(b[1] - b[0]);
}

__global__ void k_adj_keys(const int64_t* __restrict__ rows, const int64_t* __restrict__ cols,
                           int64_t n_edges, int64_t n, uint64_t* __restrict__ keys) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n_edges) keys[j] = (uint64_t)rows[j] * (uint64_t)n + (uint64_t)cols[j];
}

__global__ void k_adj_finish(const uint64_t* __restrict__ uniq, const int32_t* __restrict__ counts,
                             int64_t nnz, int64_t n, const float* __restrict__ dinv,
                             int64_t* __restrict__ coo_rows, int64_t* __restrict__ coo_cols,
                             float* __restrict__ vals, lgcn_edge_t* __restrict__ edges) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    const uint64_t k = uniq[j];
    const int64_t r = (int64_t)(k / (uint64_t)n);
    const int64_t c = (int64_t)(k - (uint64_t)r * (uint64_t)n);
    // scipy: D.dot(A) -> d_r * m ; .dot(D) -> (d_r * m) * d_c   (fp32, each product rounded)
    const float v = __fmul_rn(__fmul_rn(dinv[r], (float)counts[j]), dinv[c]);
    coo_rows[j] = r;
    coo_cols[j] = c;
    vals[j] = v;
    edges[j] = (lgcn_edge_t)(((uint64_t)__float_as_uint(v) << 32) | (uint32_t)c);
}

int check_epi(const lgcn_epilogue_t* ep) {
    if (!ep) return LGCN_EINVAL;
    if (ep->mode < LGCN_EPI_STORE || ep->mode > LGCN_EPI_ADD) return LGCN_EINVAL;
    if (ep->mode == LGCN_EPI_MEAN) {
        if (ep->n_prev < 1) return LGCN_EINVAL;
        if (ep->n_prev - 1 > LGCN_MAX_LAYERS) return LGCN_ETOOMANY;
        if (!(ep->div > 0.f)) return LGCN_EINVAL;
    }
    if (ep->mode == LGCN_EPI_ADD && (!ep->addend.p0 || !(ep->div > 0.f))) return LGCN_EINVAL;
    return 0;
}

struct CombineF {
    const lgcn_hub_row_t* rows; int32_t n; const float* partials; float* y; int64_t ldy;
    int32_t d, dW; const lgcn_epilogue_t* ep; hipStream_t s;
    template <typename V, int G, int NV> int operator()() const {
        return launch_combine_t<V, G, NV>(rows, n, partials, y, ldy, d, dW, *ep, s);
    }
};

struct ScaleF {
    const lgcn_rows_t* x; int32_t n; int32_t dW; float div; float* y; int64_t ldy; hipStream_t s;
    template <typename V, int G, int NV> int operator()() const {
        return launch_scale_t<V, G, NV>(*x, n, dW, div, y, ldy, s);
    }
};

struct NonzeroF {
    const lgcn_rows_t* x; int32_t n; int32_t dW; uint32_t* mask; int32_t* count; hipStream_t s;
    template <typename V, int G, int NV> int operator()() const {
        const int64_t grid = ((int64_t)n + 255) / 256;
        if (grid == 0) return 0;
        hipLaunchKernelGGL((k_rows_nonzero<V, G, NV>), dim3((uint32_t)grid), dim3(kBlock), 0, s,
                           *x, n, dW, mask, count);
        return last_err();
    }
};

lgcn_epilogue_t with_pow2(const lgcn_epilogue_t& ep) {
    lgcn_epilogue_t e = ep;
    // internal: divisions by a power-of-two div become multiplies by its exact reciprocal
    if (is_pow2f(ep.div)) {
        const float inv = 1.0f / ep.div;
        memcpy(&e.pad, &inv, sizeof(inv));
    } else {
        e.pad = 0;
    }
    return e;
}

int spmm_layer(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
               int32_t n_rows, int32_t thr,
               const lgcn_hub_item_t* items, int32_t n_items, float* partials, lgcn_rows_t x,
               float* y, int64_t ldy, int32_t d, const lgcn_epilogue_t& ep_in, float xdiv,
               const uint32_t* x_nz, hipStream_t s) {
    const lgcn_epilogue_t ep = with_pow2(ep_in);
    const bool vec_ok = rows_aligned(x) && al16(y) && (ldy % 4 == 0) && epi_aligned(ep) &&
                        (n_items == 0 || al16(partials));
    const Geo g = pick_geo(d, vec_ok);
    const lgcn_detail::LayerArgs a{rowptr, edges, row_ids, n_rows, thr, items, n_items, partials,
                                   x, y, ldy, d, g.dW, ep, xdiv, x_nz, s, g.vec, g.G, g.NV};
    if (ep.mode != LGCN_EPI_ADD && (xdiv != 1.f || x_nz)) return LGCN_EINVAL;  // backward only
    switch (ep.mode) {
        case LGCN_EPI_STORE: return lgcn_detail::layer_store(a);
        case LGCN_EPI_MEAN: return lgcn_detail::layer_mean(a);
        case LGCN_EPI_ADD: {
            const int xd = (xdiv == 1.f ? 0 : is_pow2f(xdiv) ? 2 : 1) | (x_nz ? 4 : 0);
            if (xd & 4) return lgcn_detail::layer_add_sparse(a, xd);
            return xd ? lgcn_detail::layer_add_div(a, xd) : lgcn_detail::layer_add(a, xd);
        }
        default: return LGCN_EINVAL;
    }
}

int hub_combine(const lgcn_hub_row_t* rows, int32_t n, int32_t n_pre, float* partials, float* y,
                int64_t ldy, int32_t d, const lgcn_epilogue_t& ep_in, hipStream_t s) {
    if (n <= 0) return 0;
    if (n_pre > 0) {  // level 1: runs of partial slots summed into partial slots (plain store)
        lgcn_epilogue_t st;
        memset(&st, 0, sizeof(st));
        st.mode = LGCN_EPI_STORE;
        st.div = 1.f;
        const Geo g1 = pick_geo(d, al16(partials) && (d % 4 == 0));
        CombineF f1{rows, n_pre, partials, partials, d, d, g1.dW, &st, s};
        if (int e = dispatch_geo(g1, f1)) return e;
        rows += n_pre;
        n -= n_pre;
    }
    const lgcn_epilogue_t ep = with_pow2(ep_in);
    const bool vec_ok = al16(partials) && al16(y) && (ldy % 4 == 0) && epi_aligned(ep);
    const Geo g = pick_geo(d, vec_ok);
    CombineF f{rows, n, partials, y, ldy, d, g.dW, &ep, s};
    return dispatch_geo(g, f);
}

int scale_rows(const lgcn_rows_t& x, int32_t n_rows, int32_t d, float div, float* y, int64_t ldy,
               hipStream_t s) {
    const bool vec_ok = rows_aligned(x) && al16(y) && (ldy % 4 == 0);
    const Geo g = pick_geo(d, vec_ok);
    ScaleF f{&x, n_rows, g.dW, div, y, ldy, s};
    return dispatch_geo(g, f);
}

lgcn_rows_t dense_rows(const float* p, int32_t n, int64_t ld) {
    lgcn_rows_t r;
    r.p0 = r.p1 = r.p2 = p;
    r.end0 = r.end1 = n;
    r.ld = ld;
    return r;
}

int valid_geom(int32_t n_rows, int32_t d) {
    if (n_rows < 0 || d < 1 || d > 2048) return LGCN_EINVAL;
    return 0;
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
// dst += src where src != 0, elementwise (lgcn_add_nonzero): src is a row-sparse gradient (the
// rows main.py gathers), dst a dense one that is never -0 (every engine output row is a chain from
// +0 or a sum with one: DESIGN §4d), so dst + (+-0) == dst and skipping the zeros gives the dense
// add's bits while reading dst only where src holds a value. NaN != 0: added.
template <typename V>
__global__ __launch_bounds__(256) void k_add_nonzero(const V* __restrict__ src, V* __restrict__ dst,
                                                     int64_t m) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m;
         i += (int64_t)gridDim.x * 256) {
        const V v = src[i];
        if constexpr (sizeof(V) == 16) {
            if (v.x != 0.f || v.y != 0.f || v.z != 0.f || v.w != 0.f) {
                V a = dst[i];
                a.x = a.x + v.x;
                a.y = a.y + v.y;
                a.z = a.z + v.z;
                a.w = a.w + v.w;
                dst[i] = a;
            }
        } else if (v != 0.f) {
            dst[i] = dst[i] + v;
        }
    }
}

extern "C" {

int lgcn_abi_version(void) { return LGCN_ABI_VERSION; }

int lgcn_tune(int knob, int value) {
    switch (knob) {
        case LGCN_TUNE_ROWS_PER_GROUP: {
            const int old = lgcn_detail::g_rows_per_group;
            if (value >= 0) lgcn_detail::g_rows_per_group = value;
            return old;
        }
        case LGCN_TUNE_UNROLL: {
            const int old = lgcn_detail::g_unroll;
            if (value >= 0) lgcn_detail::g_unroll = value;
            return old;
        }
        case LGCN_TUNE_MEAN_PREFETCH: {
            const int old = lgcn_detail::g_mean_prefetch;
            if (value >= 0) lgcn_detail::g_mean_prefetch = value;
            return old;
        }
        case LGCN_TUNE_MIN_GROUPS: {
            const int old = lgcn_detail::g_min_groups;
            if (value >= 0) lgcn_detail::g_min_groups = value;
            return old;
        }
        case LGCN_TUNE_EMU_MARGIN: {
            const int old = lgcn_detail::g_emu_margin;
            if (value >= 0) lgcn_detail::g_emu_margin = value;
            return old;
        }
        default:
            return LGCN_EINVAL;
    }
}

const char* lgcn_error_string(int code) {
    switch (code) {
        case 0: return "success";
        case LGCN_EINVAL: return "lgcn: invalid argument";
        case LGCN_EALIGN: return "lgcn: misaligned operand";
        case LGCN_ETOOMANY: return "lgcn: too many layers for the fused mean epilogue";
        default: break;
    }
    if (code > 0) return hipGetErrorString((hipError_t)code);
    return "lgcn: unknown error";
}

int32_t lgcn_chain_max_default(int64_t nnz) {
    // the forward's cut: a chain row must stay short against a whole layer; on a small graph the
    // floor: a walk's fixed costs (block pass + walk ~0.4 ms per layer at C2) outweigh a 8k-edge
    // chain (C2: 2048 -> 8192: forward 1.10 -> 0.94 ms). C3 (56M nonzeros): 55k / 110k / 220k /
    // 330k edges: 13.4 / 13.06 / 12.65 / 12.8 ms (round 5, A/B on one box: 220k)
    return (int32_t)std::min<int64_t>(std::max<int64_t>(nnz / 256, 8192), 262144);
}

int32_t lgcn_chain_max_backward_default(int64_t nnz) {
    // the backward's (Âᵀ) cut: its row-sparse first layer turns chain rows into live-edge chains
    // and the longer rows into walks or live chains by their live edges; C3 BPR-batch backward
    // 110k / 220k / 330k edges: 9.06 / 10.47 / 12.05 ms (round 5; 55k: 9.7 ms, round 4)
    return (int32_t)std::min<int64_t>(std::max<int64_t>(nnz / 512, 8192), 131072);
}

int lgcn_plan_exact(const int32_t* rowptr_host, const int32_t* row_ids_host, int32_t n_rows,
                    int32_t emu_min_degree, int32_t chain_max, int32_t part0_blocks,
                    lgcn_emu_row_t* rows_host, lgcn_emu_block_t* blocks_host,
                    lgcn_hub_plan_t* plan) {
    if (!plan || n_rows < 0 || (n_rows > 0 && !rowptr_host) || emu_min_degree < 0)
        return LGCN_EINVAL;
    if ((rows_host == nullptr) != (blocks_host == nullptr)) return LGCN_EINVAL;
    constexpr int64_t B = LGCN_EMU_BLOCK;
    if (n_rows > 0 && (rowptr_host[0] < 0 || rowptr_host[n_rows] < rowptr_host[0]))
        return LGCN_EINVAL;
    if (chain_max <= 0)
        chain_max = lgcn_chain_max_default(n_rows > 0 ? rowptr_host[n_rows] - rowptr_host[0] : 0);
    if (part0_blocks <= 0) part0_blocks = 8192;
    // the emulated rows, longest first; equal degrees keep their slot order
    std::vector<int32_t> em;
    for (int32_t s = 0; s < n_rows; ++s) {
        const int64_t deg = (int64_t)rowptr_host[s + 1] - rowptr_host[s];
        if (deg < 0) return LGCN_EINVAL;
        if (deg > emu_min_degree) em.push_back(s);
    }
    std::stable_sort(em.begin(), em.end(), [&](int32_t a, int32_t b) {
        return rowptr_host[a + 1] - rowptr_host[a] > rowptr_host[b + 1] - rowptr_host[b];
    });
    const int64_t b1 = (chain_max + B - 1) / B;                  // chain rows: <= b1 blocks
    const int64_t b0 = std::max<int64_t>(part0_blocks, b1);      // part 0: > b0 blocks
    int64_t nb_total = 0;
    int32_t pr[2] = {0, 0}, pb[2] = {0, 0}, pm[2] = {0, 0};
    for (size_t i = 0; i < em.size(); ++i) {
        const int32_t s = em[i];
        const int64_t beg = rowptr_host[s], deg = (int64_t)rowptr_host[s + 1] - beg;
        const int64_t nb = (deg + B - 1) / B;
        if (nb_total + nb > INT32_MAX) return LGCN_EINVAL;
        if (nb > b0) pr[0] = (int32_t)(i + 1), pb[0] = (int32_t)(nb_total + nb);
        if (nb > b1) pr[1] = (int32_t)(i + 1), pb[1] = (int32_t)(nb_total + nb);
        // the first (longest) row of each part
        if (nb > b0 && !pm[0]) pm[0] = (int32_t)nb;
        if (nb <= b0 && nb > b1 && !pm[1]) pm[1] = (int32_t)nb;
        if (rows_host) {
            rows_host[i].row = row_ids_host ? row_ids_host[s] : s;
            rows_host[i].first_block = (int32_t)nb_total;
            rows_host[i].n_blocks = (int32_t)nb;
            rows_host[i].pad = 0;
            for (int64_t k = 0; k < nb; ++k) {
                lgcn_emu_block_t& bl = blocks_host[nb_total + k];
                bl.row = (int32_t)i;
                bl.beg = (int32_t)(beg + k * B);
                bl.end = (int32_t)std::min(beg + (k + 1) * B, beg + deg);
                bl.first = k == 0;
            }
        }
        nb_total += nb;
    }
    plan->n_emu_rows = (int32_t)em.size();
    plan->n_emu_blocks = (int32_t)nb_total;
    plan->emu_part_rows[0] = pr[0];
    plan->emu_part_rows[1] = pr[1];
    plan->emu_part_blocks[0] = pb[0];
    plan->emu_part_blocks[1] = pb[1];
    plan->emu_scratch_blocks = pb[1];
    plan->emu_part_max_blocks[0] = pm[0];
    plan->emu_part_max_blocks[1] = pm[1];
    return 0;
}

int32_t lgcn_emu_min_default(int64_t nnz) {
    // rows up to this degree run as whole-row items of the layer kernel (dispatched first in its
    // grid); at 2^23+ nonzeros that beats a chain kernel launched beside it (C3: 14.0-14.4 ->
    // 12.6-13.0 ms, round 4); on a small graph a 1024-edge item is the layer's tail (C2: 0.81 ->
    // 1.14 ms), so none
    return nnz >= (int64_t)1 << 23 ? 1024 : 0;
}

int lgcn_plan_items(const int32_t* rowptr_host, const int32_t* row_ids_host, int32_t n_rows,
                    int32_t threshold, int32_t emu_min_degree, lgcn_hub_item_t* items_host,
                    int32_t* n_items_host) {
    if (!n_items_host || n_rows < 0 || (n_rows > 0 && !rowptr_host) || threshold < 0)
        return LGCN_EINVAL;
    int32_t m = 0;
    for (int32_t s = 0; s < n_rows; ++s) {
        const int64_t deg = (int64_t)rowptr_host[s + 1] - rowptr_host[s];
        if (deg < 0) return LGCN_EINVAL;
        if (deg > threshold && deg <= emu_min_degree) {
            if (items_host)
                items_host[m] = lgcn_hub_item_t{row_ids_host ? row_ids_host[s] : s,
                                                rowptr_host[s], rowptr_host[s + 1], -1};
            ++m;
        }
    }
    *n_items_host = m;
    return 0;
}

int lgcn_plan_scratch_bytes(const lgcn_hub_plan_t* plan, int32_t d, int32_t walk_all,
                            size_t* bytes_host) {
    if (!plan || !bytes_host || d < 1 || d > 2048) return LGCN_EINVAL;
    const int64_t nb = walk_all ? plan->n_emu_blocks : plan->emu_part_blocks[1];
    bytes_host[0] = (size_t)nb * d * LGCN_EMU_CANDS * 4;
    bytes_host[1] = (size_t)nb * d * LGCN_EMU_META_BYTES;
    bytes_host[2] = (size_t)nb * (d + 1) * LGCN_EMU_BLOCK * 4;
    return 0;
}

int lgcn_device_info(int device, int32_t* n_cu_host, int32_t* arch_major_host) {
    hipDeviceProp_t p;
    const hipError_t e = hipGetDeviceProperties(&p, device);
    if (e != hipSuccess) return (int)e;
    if (n_cu_host) *n_cu_host = p.multiProcessorCount;
    if (arch_major_host) *arch_major_host = p.major;
    return 0;
}

int lgcn_stream_create(int32_t high, void** stream) {
    if (!stream) return LGCN_EINVAL;
    int least = 0, greatest = 0;
    if (hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest)) return (int)e;
    hipStream_t s = nullptr;
    if (hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking,
                                                   high ? greatest : least))
        return (int)e;
    *stream = s;
    return 0;
}

int lgcn_stream_destroy(void* stream) {
    return stream ? herr(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream))) : 0;
}

int lgcn_coo_inspect(const int64_t* rows, const int64_t* cols, int64_t nnz, int32_t n_rows,
                     int32_t n_cols, int32_t* flags, void* stream) {
    if (nnz < 0 || !flags) return LGCN_EINVAL;
    if (nnz == 0) return 0;
    if (!rows || !cols) return LGCN_EINVAL;
    const int64_t grid = (nnz + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_coo_inspect, dim3((uint32_t)grid), dim3(kBlock), 0, S(stream), rows, cols,
                       nnz, n_rows, n_cols, flags);
    return last_err();
}

int lgcn_coo_to_csr(const int64_t* rows, const int64_t* cols, const float* vals, int64_t nnz,
                    int32_t n_rows, const int32_t* perm, const int32_t* keys_sorted,
                    int32_t* rowptr, lgcn_edge_t* edges, void* stream) {
    if (nnz < 0 || nnz > 0x7fffffffLL || n_rows < 0 || !rowptr) return LGCN_EINVAL;
    if (nnz > 0 && (!cols || !vals || !edges || (!rows && !keys_sorted))) return LGCN_EINVAL;
    if ((perm == nullptr) != (keys_sorted == nullptr)) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (nnz > 0) {
        hipLaunchKernelGGL(k_csr_edges, dim3((uint32_t)((nnz + kBlock - 1) / kBlock)), dim3(kBlock),
                           0, s, cols, vals, nnz, perm, edges);
        if (int e = last_err()) return e;
    }
    const int64_t nr = (int64_t)n_rows + 1;
    hipLaunchKernelGGL(k_csr_rowptr, dim3((uint32_t)((nr + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, keys_sorted ? nullptr : rows, keys_sorted, nnz, n_rows, rowptr);
    return last_err();
}

int lgcn_coo_sort_perm(const int64_t* keys, int64_t nnz, int32_t n_keys, int32_t* keys_tmp,
                       int32_t* keys_sorted, int32_t* perm_tmp, int32_t* perm, void* temp,
                       size_t* temp_bytes_host, void* stream) {
    if (nnz < 0 || nnz > 0x7fffffffLL || !temp_bytes_host || n_keys < 0) return LGCN_EINVAL;
    int end_bit = 1;
    while (end_bit < 31 && (1LL << end_bit) < (int64_t)n_keys) ++end_bit;
    hipStream_t s = S(stream);
    if (temp == nullptr) {
        size_t bytes = 0;
        const hipError_t e = hipcub::DeviceRadixSort::SortPairs(
            nullptr, bytes, keys_tmp, keys_sorted, perm_tmp, perm, (int)nnz, 0, end_bit, s);
        *temp_bytes_host = bytes;
        return herr(e);
    }
    if (nnz == 0) return 0;
    if (!keys || !keys_tmp || !keys_sorted || !perm_tmp || !perm) return LGCN_EINVAL;
    hipLaunchKernelGGL(k_keys_iota, dim3((uint32_t)((nnz + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, keys, nnz, keys_tmp, perm_tmp);
    if (int e = last_err()) return e;
    size_t bytes = *temp_bytes_host;
    // LSD radix sort: stable, so equal keys keep their stored order (torch's summation order).
    return herr(hipcub::DeviceRadixSort::SortPairs(temp, bytes, keys_tmp, keys_sorted, perm_tmp,
                                                   perm, (int)nnz, 0, end_bit, s));
}

int lgcn_csr_check_symmetric(const int32_t* rowptr, const lgcn_edge_t* edges, int32_t n_rows,
                             int64_t nnz, int32_t* asym, void* stream) {
    if (!rowptr || !asym || n_rows < 0 || nnz < 0) return LGCN_EINVAL;
    if (nnz == 0 || n_rows == 0) return 0;
    hipLaunchKernelGGL(k_csr_symmetric, dim3((uint32_t)((nnz + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, S(stream), rowptr, edges, n_rows, nnz, asym);
    return last_err();
}

int lgcn_csr_order_by_degree(const int32_t* rowptr, const lgcn_edge_t* edges, int32_t n_rows,
                             int64_t nnz, int32_t side_lo, int32_t side_hi, int32_t* deg_tmp,
                             int32_t* deg_sorted, int32_t* iota_tmp,
                             int32_t* row_ids, int32_t* rowptr_out, lgcn_edge_t* edges_out,
                             uint64_t* key_tmp, uint64_t* key_sorted,
                             void* temp, size_t* temp_bytes_host, void* stream) {
    if (n_rows < 0 || nnz < 0 || nnz > 0x7fffffffLL || !temp_bytes_host) return LGCN_EINVAL;
    if ((key_tmp == nullptr) != (key_sorted == nullptr)) return LGCN_EINVAL;
    if (side_lo < 0 || side_lo > side_hi || side_hi > n_rows) return LGCN_EINVAL;
    int end_bit = 1;  // degrees are <= nnz
    while (end_bit < 31 && (1LL << end_bit) <= nnz) ++end_bit;
    // sides: one more key bit above the degree, set on the rows outside [side_lo, side_hi)
    const bool sided = side_lo < side_hi;
    if (sided && end_bit > 30) return LGCN_EINVAL;  // (2^30 nonzeros)
    const int32_t side_bit = sided ? (int32_t)(1u << end_bit) : 0;
    const int32_t deg_mask = sided ? side_bit - 1 : -1;
    const int sort_bits = end_bit + (sided ? 1 : 0);
    hipStream_t s = S(stream);
    const int n = n_rows;
    const bool keyed = key_tmp != nullptr;
    if (temp == nullptr) {
        size_t b1 = 0, b2 = 0, b3 = 0;
        hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(
            nullptr, b1, deg_tmp, deg_sorted, iota_tmp, row_ids, n, 0, sort_bits, s);
        if (e != hipSuccess) return (int)e;
        e = hipcub::DeviceScan::InclusiveSum(nullptr, b2, deg_sorted, rowptr_out, n, s);
        if (e != hipSuccess) return (int)e;
        if (keyed) {
            e = hipcub::DeviceRadixSort::SortPairsDescending(
                nullptr, b3, key_tmp, key_sorted, iota_tmp, row_ids, n, 0, 32 + sort_bits, s);
            if (e != hipSuccess) return (int)e;
        }
        size_t b = b1 > b2 ? b1 : b2;
        *temp_bytes_host = b > b3 ? b : b3;
        return 0;
    }
    if (!rowptr || !rowptr_out || (n > 0 && (!deg_tmp || !deg_sorted || !iota_tmp || !row_ids)))
        return LGCN_EINVAL;
    if (nnz > 0 && (!edges || !edges_out)) return LGCN_EINVAL;
    if (int e = herr(hipMemsetAsync(rowptr_out, 0, sizeof(int32_t), s))) return e;
    if (n == 0) return 0;
    const dim3 gn((uint32_t)((n + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(k_csr_degrees, gn, dim3(kBlock), 0, s, rowptr, n, side_lo, side_hi,
                       side_bit, deg_tmp, iota_tmp);
    if (int e = last_err()) return e;
    size_t bytes = *temp_bytes_host;
    // LSD radix sort: stable, so rows of equal degree keep their id order
    if (int e = herr(hipcub::DeviceRadixSort::SortPairsDescending(
            temp, bytes, deg_tmp, deg_sorted, iota_tmp, row_ids, n, 0, sort_bits, s)))
        return e;
    if (keyed) {  // second, stable sort by (side, degree, neighbour key); the permutation only
        // reorders work and slots, every row keeps its edges (bitwise-neutral)
        hipLaunchKernelGGL(k_csr_rank, gn, dim3(kBlock), 0, s, row_ids, n, deg_sorted);
        if (int e = last_err()) return e;
        hipLaunchKernelGGL(k_csr_degree_key, gn, dim3(kBlock), 0, s, rowptr, edges, n, deg_sorted,
                           side_lo, side_hi, side_bit, key_tmp, iota_tmp);
        if (int e = last_err()) return e;
        bytes = *temp_bytes_host;
        if (int e = herr(hipcub::DeviceRadixSort::SortPairsDescending(
                temp, bytes, key_tmp, key_sorted, iota_tmp, row_ids, n, 0, 32 + sort_bits, s)))
            return e;
        hipLaunchKernelGGL(k_csr_slot_degrees, gn, dim3(kBlock), 0, s, row_ids, deg_tmp, n,
                           deg_mask, deg_sorted);
        if (int e = last_err()) return e;
    } else if (sided) {
        hipLaunchKernelGGL(k_csr_mask_degrees, gn, dim3(kBlock), 0, s, deg_sorted, n, deg_mask);
        if (int e = last_err()) return e;
    }
    bytes = *temp_bytes_host;
    if (int e = herr(hipcub::DeviceScan::InclusiveSum(temp, bytes, deg_sorted, rowptr_out + 1, n, s)))
        return e;
    if (nnz == 0) return 0;
    hipLaunchKernelGGL(k_csr_gather_rows, dim3((uint32_t)((nnz + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, s, rowptr_out, row_ids, rowptr, edges, n, nnz, edges_out);
    return last_err();
}

int lgcn_csr_check_bipartite(const int32_t* rowptr, const lgcn_edge_t* edges,
                             const int32_t* row_ids, int32_t n_rows, int64_t nnz,
                             int32_t side_lo, int32_t side_hi, int32_t* bad, void* stream) {
    if (n_rows < 0 || nnz < 0 || !bad || side_lo < 0 || side_lo > side_hi || side_hi > n_rows)
        return LGCN_EINVAL;
    if (nnz == 0) return 0;
    if (!rowptr || !edges || n_rows == 0) return LGCN_EINVAL;
    hipLaunchKernelGGL(k_csr_bipartite, dim3((uint32_t)((nnz + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, S(stream), rowptr, edges, row_ids, n_rows, nnz, side_lo,
                       side_hi, bad);
    return last_err();
}

int lgcn_csr_side_classes(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
                          int32_t n_rows, int64_t nnz, int32_t split, int32_t part_rows0,
                          int32_t part_rows1, int32_t* work, int32_t* row_ids_out,
                          int32_t* rowptr_out, lgcn_edge_t* edges_out, int32_t* class_end,
                          void* temp, size_t* temp_bytes_host, void* stream) {
    if (n_rows < 0 || nnz < 0 || nnz > 0x7fffffffLL || !temp_bytes_host) return LGCN_EINVAL;
    if (split < 0 || split > n_rows || part_rows0 < 0 || part_rows0 > part_rows1 ||
        part_rows1 > n_rows - split)
        return LGCN_EINVAL;
    hipStream_t s = S(stream);
    const int32_t n = n_rows, n0 = split;
    int32_t* mark = work;
    int32_t* key = work + n;
    int32_t* key_sorted = work + 2 * (int64_t)n;
    int32_t* iota = work + 3 * (int64_t)n;
    int32_t* perm0 = work + 4 * (int64_t)n;
    if (temp == nullptr) {
        size_t b1 = 0, b2 = 0;
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b1, key, key_sorted, iota,
                                                          perm0, n0, 0, 2, s);
        if (e != hipSuccess) return (int)e;
        e = hipcub::DeviceScan::InclusiveSum(nullptr, b2, key, rowptr_out, n, s);
        if (e != hipSuccess) return (int)e;
        *temp_bytes_host = std::max(b1, b2);
        return 0;
    }
    if (!rowptr || !rowptr_out || !row_ids_out || !class_end || !work ||
        (n > 0 && !row_ids) || (nnz > 0 && (!edges || !edges_out)))
        return LGCN_EINVAL;
    if (int e = herr(hipMemsetAsync(rowptr_out, 0, sizeof(int32_t), s))) return e;
    if (int e = herr(hipMemsetAsync(class_end, 0, 2 * sizeof(int32_t), s))) return e;
    if (n == 0) return 0;
    auto grid = [](int64_t m) { return dim3((uint32_t)((m + kBlock - 1) / kBlock)); };
    hipLaunchKernelGGL(k_fill_i32, grid(n), dim3(kBlock), 0, s, mark, (int64_t)n, 2);
    if (int e = last_err()) return e;
    if (part_rows1 > 0) {
        hipLaunchKernelGGL(k_class_mark, dim3((uint32_t)part_rows1, 256), dim3(kBlock), 0, s, rowptr,
                           edges, split, split + part_rows0, mark);
        if (int e = last_err()) return e;
        if (n0 > 0) {
            // the side-0 rows that read a walked row (not implied without structural
            // symmetry); key_sorted holds partof[row id] until the sort below rewrites it
            int32_t* partof = key_sorted;
            hipLaunchKernelGGL(k_fill_i32, grid(n), dim3(kBlock), 0, s, partof, (int64_t)n, 2);
            if (int e = last_err()) return e;
            hipLaunchKernelGGL(k_class_partof, grid(part_rows1), dim3(kBlock), 0, s, row_ids,
                               split, split + part_rows0, split + part_rows1, partof);
            if (int e = last_err()) return e;
            hipLaunchKernelGGL(k_class_mark_rev, grid(n0), dim3(kBlock), 0, s, rowptr, edges,
                               row_ids, n0, partof, mark);
            if (int e = last_err()) return e;
        }
    }
    if (n0 > 0) {
        hipLaunchKernelGGL(k_class_keys, grid(n0), dim3(kBlock), 0, s, row_ids, mark, n0, key, iota);
        if (int e = last_err()) return e;
        size_t bytes = *temp_bytes_host;
        // LSD radix sort: stable, so every class keeps the degree order of its rows
        if (int e = herr(hipcub::DeviceRadixSort::SortPairs(temp, bytes, key, key_sorted, iota,
                                                            perm0, n0, 0, 2, s)))
            return e;
        hipLaunchKernelGGL(k_class_bounds, dim3(1), dim3(64), 0, s, key_sorted, n0, class_end);
        if (int e = last_err()) return e;
    }
    // full permutation (key: new slot -> old slot) and the degrees in the new order
    int32_t* perm = key;
    int32_t* deg = iota;
    hipLaunchKernelGGL(k_class_apply, grid(n), dim3(kBlock), 0, s, perm0, rowptr, row_ids, n0, n,
                       perm, deg, row_ids_out);
    if (int e = last_err()) return e;
    size_t bytes = *temp_bytes_host;
    if (int e = herr(hipcub::DeviceScan::InclusiveSum(temp, bytes, deg, rowptr_out + 1, n, s)))
        return e;
    if (nnz == 0) return 0;
    hipLaunchKernelGGL(k_csr_gather_rows, grid(nnz), dim3(kBlock), 0, s, rowptr_out, perm, rowptr,
                       edges, n, nnz, edges_out);
    return last_err();
}

int lgcn_csr_relabel_cols(const lgcn_edge_t* edges, int64_t nnz, const int32_t* new_id,
                          lgcn_edge_t* edges_out, void* stream) {
    if (nnz < 0 || (nnz > 0 && (!edges || !new_id || !edges_out))) return LGCN_EINVAL;
    if (nnz == 0) return 0;
    hipLaunchKernelGGL(k_csr_relabel_cols, dim3((uint32_t)((nnz + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, S(stream), edges, nnz, new_id, edges_out);
    return last_err();
}

int lgcn_adj_degree(const uint64_t* keys_sorted, int64_t n_edges, int32_t n, int32_t* deg,
                    void* stream) {
    if (n_edges < 0 || n < 0 || (n_edges > 0 && !keys_sorted) || (n > 0 && !deg))
        return LGCN_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_adj_degree, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       S(stream), keys_sorted, n_edges, (int64_t)n, deg);
    return last_err();
}

int lgcn_adj_sort_unique(const int64_t* rows, const int64_t* cols, int64_t n_edges, int32_t n,
                         uint64_t* keys_a, uint64_t* keys_b, uint64_t* uniq, int32_t* counts,
                         int32_t* n_unique, void* temp, size_t* temp_bytes_host, void* stream) {
    if (n_edges < 0 || n_edges > 0x7fffffffLL || n < 0 || !temp_bytes_host) return LGCN_EINVAL;
    const uint64_t nn = (uint64_t)n * (uint64_t)n;
    int end_bit = 1;
    while (end_bit < 64 && (1ULL << end_bit) < nn) ++end_bit;
    hipStream_t s = S(stream);
    const int ne = (int)n_edges;
    if (temp == nullptr) {
        size_t b1 = 0, b2 = 0;
        hipError_t e = hipcub::DeviceRadixSort::SortKeys(nullptr, b1, keys_a, keys_b, ne, 0,
                                                         end_bit, s);
        if (e != hipSuccess) return (int)e;
        e = hipcub::DeviceRunLengthEncode::Encode(nullptr, b2, keys_b, uniq, counts, n_unique, ne, s);
        *temp_bytes_host = b1 > b2 ? b1 : b2;
        return herr(e);
    }
    if (!rows || !cols || !keys_a || !keys_b || !uniq || !counts || !n_unique) return LGCN_EINVAL;
    if (n_edges == 0) return herr(hipMemsetAsync(n_unique, 0, sizeof(int32_t), s));
    hipLaunchKernelGGL(k_adj_keys, dim3((uint32_t)((n_edges + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, s, rows, cols, n_edges, (int64_t)n, keys_a);
    if (int e = last_err()) return e;
    size_t bytes = *temp_bytes_host;
    if (int e = herr(hipcub::DeviceRadixSort::SortKeys(temp, bytes, keys_a, keys_b, ne, 0,
                                                       end_bit, s)))
        return e;
    bytes = *temp_bytes_host;
    return herr(hipcub::DeviceRunLengthEncode::Encode(temp, bytes, keys_b, uniq, counts, n_unique,
                                                      ne, s));
}

int lgcn_adj_finish(const uint64_t* uniq, const int32_t* counts, int64_t nnz, int32_t n,
                    const float* dinv, int64_t* coo_rows, int64_t* coo_cols, float* vals,
                    int32_t* rowptr, lgcn_edge_t* edges, void* stream) {
    if (nnz < 0 || nnz > 0x7fffffffLL || n < 0 || !rowptr) return LGCN_EINVAL;
    if (nnz > 0 && (!uniq || !counts || !dinv || !coo_rows || !coo_cols || !vals || !edges))
        return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (nnz > 0) {
        hipLaunchKernelGGL(k_adj_finish, dim3((uint32_t)((nnz + kBlock - 1) / kBlock)), dim3(kBlock),
                           0, s, uniq, counts, nnz, (int64_t)n, dinv, coo_rows, coo_cols, vals,
                           edges);
        if (int e = last_err()) return e;
    }
    const int64_t nr = (int64_t)n + 1;
    hipLaunchKernelGGL(k_csr_rowptr, dim3((uint32_t)((nr + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, coo_rows, nullptr, nnz, n, rowptr);
    return last_err();
}

int lgcn_spmm_layer(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
                    int32_t n_rows, int32_t hub_threshold, const lgcn_hub_item_t* hub_items, int32_t n_hub_items,
                    float* partials, lgcn_rows_t x, float x_div, const uint32_t* x_nz, float* y,
                    int64_t ldy, int32_t d, const lgcn_epilogue_t* epi_host, void* stream) {
    if (int e = valid_geom(n_rows, d)) return e;
    if (int e = check_epi(epi_host)) return e;
    if (n_rows > 0 && (!rowptr || !y || ldy < d)) return LGCN_EINVAL;
    if (n_hub_items < 0 || (n_hub_items > 0 && (!hub_items || !partials))) return LGCN_EINVAL;
    if (!(x_div > 0.f)) return LGCN_EINVAL;
    return spmm_layer(rowptr, edges, row_ids, n_rows, hub_threshold, hub_items, n_hub_items,
                      partials, x, y, ldy, d, *epi_host, x_div, x_nz, S(stream));
}

int lgcn_rows_nonzero(lgcn_rows_t x, int32_t n_rows, int32_t d, uint32_t* mask, int32_t* count,
                      void* stream) {
    if (int e = valid_geom(n_rows, d)) return e;
    if (!count || (n_rows > 0 && !mask)) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (int e = herr(hipMemsetAsync(count, 0, sizeof(int32_t), s))) return e;
    const Geo g = pick_geo(d, rows_aligned(x));
    NonzeroF f{&x, n_rows, g.dW, mask, count, s};
    return dispatch_geo(g, f);
}

int lgcn_add_nonzero(const float* src, float* dst, int64_t n, void* stream) {
    if (n < 0) return LGCN_EINVAL;
    if (n == 0) return 0;
    if (!src || !dst) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    const bool vec = n % 4 == 0 && !(reinterpret_cast<uintptr_t>(src) & 15) &&
                     !(reinterpret_cast<uintptr_t>(dst) & 15);
    const int64_t m = vec ? n / 4 : n;
    const int64_t grid = std::min<int64_t>((m + 255) / 256, 1 << 20);
    if (vec)
        hipLaunchKernelGGL((k_add_nonzero<float4>), dim3((uint32_t)grid), dim3(256), 0, s,
                           reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), m);
    else
        hipLaunchKernelGGL((k_add_nonzero<float>), dim3((uint32_t)grid), dim3(256), 0, s, src,
                           dst, m);
    return herr(hipGetLastError());
}

int lgcn_hub_combine(const lgcn_hub_row_t* hub_rows, int32_t n_hub_rows, int32_t n_pre_rows,
                     float* partials, float* y, int64_t ldy, int32_t d,
                     const lgcn_epilogue_t* epi_host, void* stream) {
    if (d < 1 || d > 2048 || n_hub_rows < 0) return LGCN_EINVAL;
    if (n_pre_rows < 0 || n_pre_rows > n_hub_rows) return LGCN_EINVAL;
    if (int e = check_epi(epi_host)) return e;
    if (n_hub_rows > 0 && (!hub_rows || !partials || !y || ldy < d)) return LGCN_EINVAL;
    return hub_combine(hub_rows, n_hub_rows, n_pre_rows, partials, y, ldy, d, *epi_host,
                       S(stream));
}

int lgcn_scale_rows(lgcn_rows_t x, int32_t n_rows, int32_t d, float div, float* y, int64_t ldy,
                    void* stream) {
    if (int e = valid_geom(n_rows, d)) return e;
    if (n_rows > 0 && (!y || ldy < d)) return LGCN_EINVAL;
    return scale_rows(x, n_rows, d, div, y, ldy, S(stream));
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// The concurrent schedule of the exact layers (lgcn_sched_create): auxiliary streams the
// emulated and chain rows run on beside the layer kernel, the bipartite lanes, and the events
// that fork and join them (graph-capture safe: a captured fork/join is a graph dependency).
// ---------------------------------------------------------------------------------------------
namespace {
// Every event record of one call takes a fresh event from this pool, so no event is recorded
// twice inside one call (a captured graph's edges follow the records one to one); the next call
// starts over. Created by lgcn_sched_create — nothing is created while a stream is captured. A
// call that would need more fails with LGCN_ETOOMANY instead of reusing an event (a reused event
// could bind a cross-layer wait to a later record; ~30 records per layer, K <= 17, use < 600).
constexpr int kPoolEvents = 1024;
struct EventPool {
    hipEvent_t ev[kPoolEvents];
    int n = 0;
    int next = 0;
    int32_t state[5] = {0, 0, 0, 0, 0};  // the latest call's schedule (lgcn_sched_state)
};
}  // namespace

struct lgcn_sched {
    hipStream_t aux[3];
    int n_aux;
    EventPool* pool;        // owned by the root schedule; lane 1's view shares it
    int32_t slots[2];       // walk LDS slots of part 0 / part 1 (0 = default)
    int chain;              // 0: chain rows are walked too (tests / A-B)
    hipEvent_t t0, t1;      // optional: recorded on the caller's stream around the layer kernel
    hipEvent_t* trace;      // optional [8]: phase events (LGCN_SCHED_TRACE)
    // bipartite lanes (lgcn_propagate_*_sides; created with >= 4 aux streams): the second lane's
    // main stream and its own view (aux streams)
    hipStream_t lane1_main;
    lgcn_sched* lane1;
    hipEvent_t* trace_sides;   // optional [32 K] (LGCN_SCHED_TRACE_SIDES)
    hipEvent_t* timing_sides;  // optional [8 K] (LGCN_SCHED_TIMING_SIDES)
    int classes;               // LGCN_SCHED_CLASSES (default 1)
    int lk_normal;             // LGCN_SCHED_LK_NORMAL (default 1)
    // LGCN_SCHED_LANE1_SHARED: lane 1 on the caller's stream and lane 0's aux streams in reverse
    // order (lane1s: that view), so each of lane 1's streams is one of lane 0's
    int lane1_shared;
    lgcn_sched* lane1s;
};

namespace {
struct EmuPart {
    int32_t r0, r1, b0, b1;
};

int ev_next(const lgcn_sched* sc, hipEvent_t* e) {
    EventPool* p = sc->pool;
    if (p->n <= 0) return LGCN_EINVAL;
    if (p->next >= p->n) return LGCN_ETOOMANY;
    *e = p->ev[p->next++];
    return 0;
}

// an event recorded on `from` that `to` waits for
int link(const lgcn_sched* sc, hipStream_t from, hipStream_t to) {
    hipEvent_t e;
    if (int r = ev_next(sc, &e)) return r;
    if (int r = herr(hipEventRecord(e, from))) return r;
    return herr(hipStreamWaitEvent(to, e, 0));
}

int record(const lgcn_sched* sc, hipStream_t st, hipEvent_t* out) {
    if (int r = ev_next(sc, out)) return r;
    return herr(hipEventRecord(*out, st));
}

int wait_ev(hipStream_t st, hipEvent_t e) { return e ? herr(hipStreamWaitEvent(st, e, 0)) : 0; }

// Cross-stream dependencies of one layer under a schedule (all optional):
//  - late: the epilogue's operands (a MEAN's earlier layers, made on the other lane) — every
//    kernel that writes Y waits for them; the block passes (they read X only) do not;
//  - part_wait[i]: walked part i (0, 1) reads only the X rows this event covers, so its block pass
//    starts after it instead of after everything before the layer on `s`;
//  - defer: parts 0 and 1 are not joined back into `s`; part_done[i] (written here) fires when
//    part i's rows are written, and whoever reads them waits for it.
// part_wait / defer take effect when parts 0, 1 and the chain rows have a stream each; otherwise
// the parts fork and join with the rest and part_done fires with the joined layer.
struct Deps {
    hipEvent_t late[3] = {nullptr, nullptr, nullptr};
    // late_emu: operands only the emulated rows' epilogue reads (their own rows of the earlier
    // layers, made by the other lane's walked parts): with a deferred epilogue only it waits for
    // them, otherwise they count as `late`
    hipEvent_t late_emu[2] = {nullptr, nullptr};
    hipEvent_t part_wait[2] = {nullptr, nullptr};
    bool defer = false;
    hipEvent_t part_done[2] = {nullptr, nullptr};
    // lk: the layer kernel (and its chunk combine) runs on this stream, forked from and joined
    // back into `s` (a normal-priority stream for a high-priority lane's last layer kernel)
    hipStream_t lk = nullptr;
};

int wait_late(hipStream_t st, const Deps* dp, bool emu = true) {
    if (!dp) return 0;
    for (hipEvent_t e : dp->late)
        if (int r = wait_ev(st, e)) return r;
    if (emu)
        for (hipEvent_t e : dp->late_emu)
            if (int r = wait_ev(st, e)) return r;
    return 0;
}

// rows [r0, r1) of the emulated-row list: block pass (blocks [b0, b1)) into the scratch at the
// part's block offset
// live: NULL, or lgcn_live_rows' per-row flags over the whole emulated-row list (rows the
// live-edge chains ran are skipped)
int part_blocks(const lgcn_edge_t* edges, const lgcn_hub_plan_t& p, const EmuPart& q,
                const lgcn_rows_t& x, float xdiv, const uint32_t* x_nz, int32_t d,
                const lgcn_emu_row_t* live, hipStream_t s) {
    if (q.b1 <= q.b0) return 0;
    const int64_t b0 = q.b0;
    return lgcn_emu_blocks(edges, p.emu_blocks + b0, q.b1 - q.b0, x, xdiv, x_nz, d,
                           p.emu_rel + b0 * d * LGCN_EMU_CANDS,
                           static_cast<char*>(p.emu_meta) + b0 * d * LGCN_EMU_META_BYTES,
                           p.emu_stage ? p.emu_stage + b0 * (d + 1) * LGCN_EMU_BLOCK : nullptr,
                           live, s);
}

int part_walk(const lgcn_edge_t* edges, const lgcn_hub_plan_t& p, const EmuPart& q,
              const lgcn_rows_t& x, float xdiv, const uint32_t* x_nz, float* y, int64_t ldy,
              int32_t d, const lgcn_epilogue_t& ep, int slots, const lgcn_emu_row_t* live,
              hipStream_t s) {
    if (q.r1 <= q.r0) return 0;
    return lgcn_emu_walk(edges, p.emu_blocks, p.emu_rows + q.r0, q.r1 - q.r0, p.emu_rel,
                         p.emu_meta, p.emu_stage, x, xdiv, x_nz, y, ldy, d, &ep, slots,
                         live ? live + q.r0 : nullptr, s);
}

bool chain_ok(const lgcn_rows_t& x, int32_t d) {
    return lgcn_chain_supported(d) && x.ld % 4 == 0 && al16(x.p0) && al16(x.p1) && al16(x.p2);
}

// One layer under a hub plan (every row of Y written once):
//  - bundles, hub chunks and whole long rows: the layer kernel (spmm_layer) + chunk combine;
//  - emulated rows, longest first, in three parts (lgcn_hub_plan_t emu_part_*): parts 0 and 1
//    block pass + walk, part 2 the sequential chain kernel (or walked, when the chain kernel
//    cannot take d / the alignment, or the schedule turns it off).
// Without a schedule everything runs in that order on `s`. With one, the emulated parts run on
// the auxiliary streams beside the layer kernel: part 0 (the longest rows, whose walk is the
// layer's critical path) on aux[0], part 1 on aux[1], the chain rows on aux[2] (with fewer aux
// streams the later parts share the last one); the block passes are enqueued first and the
// layer kernel waits for part 0's, so the longest walk starts before the layer kernel fills the
// chip (C3 forward 18.58 -> 18.06 ms, round 3).
int plan_layer(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
               int32_t n, const lgcn_hub_plan_t& p, const lgcn_rows_t& x, float xdiv,
               const uint32_t* x_nz, float* y, int64_t ldy, int32_t d, const lgcn_epilogue_t& ep,
               const lgcn_sched* sc, hipStream_t s, Deps* dp = nullptr) {
    const int32_t ne = p.n_emu_rows;
    // row-sparse X (the backward's first layer on a BPR batch): every emulated row is a chain
    // over its live edges (lgcn_live_rows) — no block pass, no walk
    const bool live = x_nz && p.emu_live && ne > 0 && chain_ok(x, d) && (!sc || sc->chain);
    const bool chains = !live && ne > p.emu_part_rows[1] && chain_ok(x, d) && (!sc || sc->chain);
    // walked rows read the block-pass scratch, which must cover their blocks
    if ((chains || live ? p.emu_part_blocks[1] : p.n_emu_blocks) > p.emu_scratch_blocks)
        return LGCN_EINVAL;
    hipEvent_t* tr = sc ? sc->trace : nullptr;
    auto mark = [&](int k, hipStream_t st) -> int {
        return tr && tr[k] ? herr(hipEventRecord(tr[k], st)) : 0;
    };
    const EmuPart parts[3] = {{0, p.emu_part_rows[0], 0, p.emu_part_blocks[0]},
                              {p.emu_part_rows[0], p.emu_part_rows[1], p.emu_part_blocks[0],
                               p.emu_part_blocks[1]},
                              {p.emu_part_rows[1], ne, p.emu_part_blocks[1], p.n_emu_blocks}};
    const int slots[3] = {sc ? sc->slots[0] : 0, sc ? sc->slots[1] : 0, sc ? sc->slots[1] : 0};
    auto layer_kernel = [&](hipStream_t st) -> int {
        if (sc && sc->t0)
            if (int e = herr(hipEventRecord(sc->t0, st))) return e;
        if (int e = spmm_layer(rowptr, edges, row_ids, n, p.threshold, p.items, p.n_items,
                               p.partials, x, y, ldy, d, ep, xdiv, x_nz, st))
            return e;
        if (sc && sc->t1)
            if (int e = herr(hipEventRecord(sc->t1, st))) return e;
        return hub_combine(p.rows, p.n_rows, p.n_pre, p.partials, y, ldy, d, ep, st);
    };
    // a MEAN whose operands arrive late (the other lane's layer K-1) with an emu_out scratch: the
    // walks and chains write their rows' sums there (LGCN_EPI_ROWS) without waiting for them, and
    // the mean of those rows follows on `s` once they are ready (lgcn_emu_epilogue)
    const bool has_late = dp && (dp->late[0] || dp->late[1] || dp->late[2] ||
                                 dp->late_emu[0] || dp->late_emu[1]);
    const bool defer_epi = sc && has_late && ep.mode == LGCN_EPI_MEAN && p.emu_out && ne > 0 &&
                           !live;
    lgcn_epilogue_t ep_rows;
    memset(&ep_rows, 0, sizeof(ep_rows));
    ep_rows.mode = LGCN_EPI_ROWS;
    // where the emulated rows of part i go: Y, or emu_out rows [r0, r1) when deferred
    auto emu_y = [&](int i) { return defer_epi ? p.emu_out + (int64_t)parts[i].r0 * d : y; };
    const int64_t emu_ld = defer_epi ? d : ldy;
    const lgcn_epilogue_t& emu_ep = defer_epi ? ep_rows : ep;
    auto chain_rows = [&](hipStream_t st) -> int {
        const EmuPart& q = parts[2];
        if (q.r1 <= q.r0) return 0;
        return lgcn_chain_rows(edges, p.emu_blocks, p.emu_rows + q.r0, q.r1 - q.r0, x, xdiv,
                               emu_y(2), emu_ld, d, &emu_ep, st);
    };
    // live path: the live-edge chains take every chain row (part 2) and every walked row with at
    // most LGCN_LIVE_MAX live edges; block pass + walk run the rest (their waves of the live
    // rows exit at once). Dense X: every walked row stays walked, the chains cover part 2.
    const lgcn_emu_row_t* lflags =
        live ? lgcn_live_flags(p.emu_live, ne, p.n_emu_blocks) : nullptr;
    auto live_rows = [&](hipStream_t st) -> int {
        return lgcn_live_rows(edges, p.emu_blocks, p.n_emu_blocks, p.emu_rows, ne, x, xdiv, x_nz,
                              y, ldy, d, &ep, p.emu_part_rows[1], LGCN_LIVE_MAX, p.emu_live, st);
    };
    auto walked = [&](int i, hipStream_t st) -> int {
        if (int e = part_blocks(edges, p, parts[i], x, xdiv, x_nz, d, lflags, st)) return e;
        return part_walk(edges, p, parts[i], x, xdiv, x_nz, y, ldy, d, ep, slots[i], lflags, st);
    };
    // everything joined into `s`: the deferred parts are done with it
    auto done_on_s = [&]() -> int {
        if (dp && dp->defer && sc)
            for (int i = 0; i < 2; ++i)
                if (int e = record(sc, s, &dp->part_done[i])) return e;
        return 0;
    };
    if (!sc || ne == 0 || live) {
        if (int e = wait_late(s, dp)) return e;
    }
    if (live && sc) {
        // aux[0]: the live-edge flags (they gate the walks), then part 0's block pass + walk;
        // aux[1] (after the flags): part 1; aux[2] (after the flags): the live-edge chains —
        // beside the walks rather than before them (a dense G keeps every walked row walked and
        // makes every chain row a chain over all its edges: round 5, the dense backward's first
        // layer no longer waits for its chains before its walks start)
        const int na = sc->n_aux;
        hipStream_t a0 = sc->aux[0], a1 = sc->aux[na > 1 ? 1 : 0], a2 = sc->aux[na > 2 ? 2 : 0];
        if (int e = mark(0, s)) return e;
        if (int e = link(sc, s, a0)) return e;
        if (int e = lgcn_detail::live_prepare(edges, p.emu_blocks, p.n_emu_blocks, p.emu_rows, ne,
                                              x_nz, d, xdiv, &ep, y, ldy, x.p0,
                                              p.emu_part_rows[1], LGCN_LIVE_MAX, p.emu_live, a0))
            return e;
        if (a2 != a0)
            if (int e = link(sc, a0, a2)) return e;
        if (int e = lgcn_detail::live_chains(p.n_emu_blocks, ne, x, xdiv, y, ldy, d, &ep,
                                             p.emu_live, a2))
            return e;
        if (int e = mark(4, a2)) return e;
        if (a1 != a0 && a1 != a2)
            if (int e = link(sc, a0, a1)) return e;
        if (int e = walked(0, a0)) return e;
        if (int e = mark(5, a0)) return e;
        if (int e = walked(1, a1)) return e;
        if (int e = mark(6, a1)) return e;
        if (int e = layer_kernel(s)) return e;
        if (int e = mark(3, s)) return e;
        if (int e = link(sc, a0, s)) return e;
        if (a1 != a0)
            if (int e = link(sc, a1, s)) return e;
        if (a2 != a0 && a2 != a1)
            if (int e = link(sc, a2, s)) return e;
        if (int e = mark(7, s)) return e;
        return done_on_s();
    }
    if (live) {
        if (int e = live_rows(s)) return e;
        for (int i = 0; i < 2; ++i)
            if (int e = walked(i, s)) return e;
        if (int e = layer_kernel(s)) return e;
        return done_on_s();
    }
    if (!sc || ne == 0) {
        for (int i = 0; i < 3; ++i)
            if (i < 2 || !chains)
                if (int e = part_blocks(edges, p, parts[i], x, xdiv, x_nz, d, nullptr, s)) return e;
        if (int e = layer_kernel(s)) return e;
        for (int i = 0; i < 3; ++i)
            if (i < 2 || !chains)
                if (int e = part_walk(edges, p, parts[i], x, xdiv, x_nz, y, ldy, d, ep, slots[i],
                                      nullptr, s))
                    return e;
        if (chains)
            if (int e = chain_rows(s)) return e;
        return done_on_s();
    }
    // fork: X is ready on `s` (parts 0 / 1 with a stream of their own: once their part_wait fires)
    const int na = sc->n_aux;
    const bool own = dp && na >= 3;
    auto aux_of = [&](int part) { return sc->aux[part < na ? part : na - 1]; };
    if (int e = mark(0, s)) return e;
    hipEvent_t fork;
    if (int e = record(sc, s, &fork)) return e;
    for (int i = 0; i < na; ++i) {
        const hipEvent_t w = own && i < 2 && dp->part_wait[i] ? dp->part_wait[i] : fork;
        if (int e = wait_ev(sc->aux[i], w)) return e;
    }
    // block passes first (the walk of part 0 starts as soon as its own is done), then the layer
    // kernel, then the walks and the chains
    for (int i = 0; i < 3; ++i)
        if (i < 2 || !chains) {
            if (int e = part_blocks(edges, p, parts[i], x, xdiv, x_nz, d, nullptr, aux_of(i)))
                return e;
            if (i < 2)
                if (int e = mark(1 + i, aux_of(i))) return e;
        }
    // the block passes read X only; every kernel after them writes Y, whose epilogue operands
    // are ready once `late` fires (the walks and chains write emu_out instead when deferred, and
    // only their epilogue waits for late_emu)
    if (int e = wait_late(s, dp, !defer_epi)) return e;
    if (!defer_epi)
        for (int i = 0; i < na; ++i)
            if (int e = wait_late(sc->aux[i], dp)) return e;
    // the layer kernel waits for part 0's block pass (round 5: the mean half-layers without this
    // wait measured the same, 12.40 / 12.68 vs 12.38 / 12.64 ms)
    if (parts[0].b1 > parts[0].b0)
        if (int e = link(sc, aux_of(0), s)) return e;
    if (dp && dp->lk && dp->lk != s) {
        if (int e = link(sc, s, dp->lk)) return e;
        if (int e = layer_kernel(dp->lk)) return e;
        if (int e = link(sc, dp->lk, s)) return e;
    } else if (int e = layer_kernel(s)) {
        return e;
    }
    if (int e = mark(3, s)) return e;
    if (chains) {
        if (int e = chain_rows(aux_of(2))) return e;
        if (int e = mark(4, aux_of(2))) return e;
    }
    for (int i = 0; i < 3; ++i)
        if (i < 2 || !chains) {
            if (int e = part_walk(edges, p, parts[i], x, xdiv, x_nz, emu_y(i), emu_ld, d, emu_ep,
                                  slots[i], nullptr, aux_of(i)))
                return e;
            if (i < 2)
                if (int e = mark(5 + i, aux_of(i))) return e;
        }
    // join: every row of Y written before `s` goes on — except deferred parts 0 and 1
    for (int i = 0; i < na; ++i) {
        if (own && dp->defer && i < 2) {
            if (int e = record(sc, sc->aux[i], &dp->part_done[i])) return e;
        } else if (int e = link(sc, sc->aux[i], s)) {
            return e;
        }
    }
    if (defer_epi) {
        for (hipEvent_t e : dp->late_emu)
            if (int r = wait_ev(s, e)) return r;
        if (int e = lgcn_emu_epilogue(p.emu_rows, ne, p.emu_out, d, y, ldy, d, &ep, s)) return e;
    }
    if (int e = mark(7, s)) return e;
    return own ? 0 : done_on_s();
}

// The bipartite schedule (lgcn_propagate_*_sides): a lane = the stream its half-layers' layer
// kernels run on + the schedule view whose aux streams take their emulated / chain rows.
struct Lane {
    hipStream_t main;
    const lgcn_sched* view;
};

bool capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}

// The two lanes: lane 1 on its own streams when the schedule has them, else both lanes share
// the caller's stream (half-layers then run in layer order, each still overlapped inside).
// Captures: HIP runtimes before 7.2 segfault in hipStreamEndCapture on the full schedule — lane
// 1's aux streams forked from its main stream and joined back, deferred parts, cross-lane waits
// on aux streams (round 6, DESIGN §4e: the same C host binary captures, instantiates and replays
// it bitwise on /opt/rocm's 7.2 runtime and crashes on the 7.0 runtime that the torch 2.10.0
// +rocm7.0 wheel bundles, which is the one a torch process loads). Under a capture on such a
// runtime lane 1 runs its half-layers on its main stream alone and the parts are joined every
// half-layer; from 7.2 on a capture records the eager schedule itself.
bool runtime_captures_full() {
    static const bool ok = [] {
        int v = 0;
        return hipRuntimeGetVersion(&v) == hipSuccess && v >= 70200000;
    }();
    return ok;
}

// the capture restrictions above apply to this call: `s` is being captured on an older runtime
bool capture_restricted(hipStream_t s) { return capturing(s) && !runtime_captures_full(); }

bool make_lanes(const lgcn_sched* sc, hipStream_t s, Lane lanes[2], bool& l1_aux) {
    lanes[0] = Lane{s, sc};
    const bool shared = sc && sc->lane1_shared && sc->lane1s;
    const bool two = sc && (sc->lane1 || shared);
    const lgcn_sched* l1v = shared ? sc->lane1s : (sc ? sc->lane1 : nullptr);
    const bool cap = capturing(s);
    l1_aux = two && l1v->n_aux > 0 && !(cap && !runtime_captures_full());
    lanes[1] = two ? Lane{shared ? s : sc->lane1_main, l1_aux ? l1v : nullptr} : lanes[0];
    if (sc) {
        sc->pool->state[0] = two ? 2 : 1;
        sc->pool->state[1] = l1_aux ? l1v->n_aux : 0;
        sc->pool->state[2] = cap ? 1 : 0;
        sc->pool->state[4] = cap && runtime_captures_full() ? 1 : 0;
    }
    return two;
}

// Lane 1 forked from the caller's stream: its main stream and its aux streams wait on `s`.
int fork_lanes(const lgcn_sched* sc, bool two, const Lane& l1, hipStream_t s) {
    if (!two) return 0;
    hipEvent_t f;
    if (int e = record(sc, s, &f)) return e;
    if (int e = wait_ev(l1.main, f)) return e;
    for (int i = 0; i < (l1.view ? l1.view->n_aux : 0); ++i)
        if (int e = wait_ev(l1.view->aux[i], f)) return e;
    return 0;
}

// Lane 1 back into the caller's stream: its main stream and its aux streams, each joined into
// `s` directly.
int join_lanes(const lgcn_sched* sc, bool two, const Lane& l1, hipStream_t s) {
    if (!two) return 0;
    if (int e = link(sc, l1.main, s)) return e;
    for (int i = 0; i < (l1.view ? l1.view->n_aux : 0); ++i)
        if (int e = link(sc, l1.view->aux[i], s)) return e;
    return 0;
}

int check_plan(const lgcn_hub_plan_t* p) {
    if (!p) return LGCN_EINVAL;
    if (p->n_items < 0 || (p->n_items > 0 && !p->items)) return LGCN_EINVAL;
    if (p->n_rows < 0 || p->n_pre < 0 || p->n_pre > p->n_rows) return LGCN_EINVAL;
    if (p->n_rows > 0 && (!p->rows || !p->partials)) return LGCN_EINVAL;
    if (p->n_emu_rows < 0 || p->n_emu_blocks < 0) return LGCN_EINVAL;
    if (p->n_emu_rows > 0 && (!p->emu_rows || !p->emu_blocks)) return LGCN_EINVAL;
    const int32_t* pr = p->emu_part_rows;
    const int32_t* pb = p->emu_part_blocks;
    if (pr[0] < 0 || pr[0] > pr[1] || pr[1] > p->n_emu_rows || pb[0] < 0 || pb[0] > pb[1] ||
        pb[1] > p->n_emu_blocks)
        return LGCN_EINVAL;
    // walked rows need the block-pass scratch
    if (p->emu_scratch_blocks < 0 || p->emu_scratch_blocks > p->n_emu_blocks) return LGCN_EINVAL;
    if (p->emu_scratch_blocks > 0 && (!p->emu_rel || !p->emu_meta)) return LGCN_EINVAL;
    return 0;
}

// segments of a sided propagation: 0..2 = the side-0 classes, 3 = side 1
constexpr int kSegs = 4;

int check_sides(const int32_t* rowptr, const int32_t* row_ids, int32_t n, const lgcn_sides_t* sd,
                const lgcn_hub_plan_t* plans) {
    if (!plans || !rowptr || !sd || (n > 0 && !row_ids)) return LGCN_EINVAL;
    const int32_t c0 = sd->class_end[0], c1 = sd->class_end[1], sp = sd->split;
    if (c0 < 0 || c0 > c1 || c1 > sp || sp > n) return LGCN_EINVAL;
    if (sd->part_rows[0] < 0 || sd->part_rows[0] > sd->part_rows[1] ||
        sd->part_rows[1] > n - sp)
        return LGCN_EINVAL;
    for (int i = 0; i < 2 * kSegs; ++i)
        if (int e = check_plan(plans + i)) return e;
    return 0;
}

// The classes hold when side 1's walked parts are covered by the rows they were built from:
// plan part 0 = side-1 slots [split, split + emu_part_rows[0]) (a plan over a degree-ordered
// slot range lists its emulated rows in slot order), part 1 up to emu_part_rows[1].
bool classes_hold(const lgcn_sides_t& sd, const lgcn_hub_plan_t* plans) {
    for (int j = 0; j < 2; ++j) {
        const lgcn_hub_plan_t& p = plans[2 * 3 + j];
        if (p.emu_part_rows[0] > sd.part_rows[0] || p.emu_part_rows[1] > sd.part_rows[1])
            return false;
    }
    return true;
}

// What layer k of a sided propagation reads and writes.
struct LayerIO {
    lgcn_rows_t x;
    float xdiv;
    const uint32_t* x_nz;
    float* y;
    lgcn_epilogue_t ep;
};

// Segment g of layer k: slots [lo, hi) under plans[2 * g + (k & 1)] on lane L.
int seg_layer(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
              int32_t lo, int32_t hi, const lgcn_hub_plan_t* plans, int k, int g,
              const LayerIO& io, int32_t d, const lgcn_sched* sc, const Lane& L, Deps* dp) {
    if (hi <= lo) {  // nothing to run: the deferred parts are "done" here
        if (dp && dp->defer && sc)
            for (int i = 0; i < 2; ++i)
                if (int e = record(sc, L.main, &dp->part_done[i])) return e;
        return 0;
    }
    const int h = (k - 1) * kSegs + g;
    lgcn_sched v;
    const lgcn_sched* vp = nullptr;
    if (L.view) {
        v = *L.view;
        v.t0 = sc->timing_sides ? sc->timing_sides[2 * h] : nullptr;
        v.t1 = sc->timing_sides ? sc->timing_sides[2 * h + 1] : nullptr;
        v.trace = sc->trace_sides ? sc->trace_sides + h * 8 : nullptr;
        vp = &v;
    }
    Deps local;
    Deps* dq = dp;
    if (!vp && dp && dp->defer && sc) {
        // (no view: everything runs on L.main; plan_layer records nothing without a schedule)
        local = *dp;
        local.defer = false;
        dq = &local;
    }
    if (int e = plan_layer(rowptr + lo, edges, row_ids + lo, hi - lo, plans[2 * g + (k & 1)],
                           io.x, io.xdiv, io.x_nz, io.y, d, d, io.ep, vp, L.main, dq))
        return e;
    if (dq == &local)
        for (int i = 0; i < 2; ++i)
            if (int e = record(sc, L.main, &dp->part_done[i])) return e;
    return 0;
}

// The sided propagation (forward and backward): layer k of one side reads layer k-1 of the
// other. Half-layer (k, side) runs on lane (k + side + K) % 2, so each lane is a chain of
// half-layers that alternate sides, and layer k of one side follows layer k-1 of the other on
// its own lane. Side 0 runs as its classes (class A = rows linked to side 1's walked part 0, B =
// to part 1 only, C = the rest; lgcn_csr_side_classes), and the walked parts of side 1 wait
// only for the classes they read:
//  - layer 1 of side 0 runs A, B, C: layer 2's part 0 (the longest walk) starts once A is done;
//  - side 1's parts 0 and 1 are not joined into their lane: layer k+1 of side 0 runs C (reads
//    side 1's other rows), then B after part 1, then A after part 0, so the classes that do not
//    read the longest walks run while it is still going;
//  - a mean (forward, k = K) waits, per class / per part, only for the rows of layer K-1 it reads.
// Backward buffers alternate (layer k overwrites layer k-2's rows): a part of side 1 overwrites
// rows that only the classes it waited for read, and a class of side 0 overwrites rows that only
// the parts it waited for read.
int run_sides(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
              const lgcn_sides_t& sd, const lgcn_hub_plan_t* plans, int32_t d, int32_t K,
              const std::function<LayerIO(int)>& layer, const lgcn_sched* sched, hipStream_t s) {
    Lane lanes[2];
    bool l1_aux = false;
    if (sched) sched->pool->next = 0;
    const bool two = make_lanes(sched, s, lanes, l1_aux);
    // Under a HIP-graph capture on a runtime before 7.2 the parts are joined into their lane at
    // the end of every half-layer (no deferred parts, no early starts, no cross-lane waits on an
    // aux stream: runtime_captures_full); the captured graph keeps the per-class launches and
    // the two lanes.
    const bool cap = capture_restricted(s);
    const bool classes = sched && sched->classes && classes_hold(sd, plans) && !cap;
    if (sched) sched->pool->state[3] = classes ? 1 : 0;
    const int32_t lo[kSegs] = {0, sd.class_end[0], sd.class_end[1], sd.split};
    const int32_t hi[kSegs] = {sd.class_end[0], sd.class_end[1], sd.split, 0};
    auto seg_hi = [&](int g, int32_t n) { return g == 3 ? n : hi[g]; };
    const int32_t n = sd.n;
    if (int e = fork_lanes(sched, two, lanes[1], s)) return e;  // lane 1 starts where `s` is
    constexpr int KM = LGCN_MAX_LAYERS + 2;
    hipEvent_t cls[KM][3] = {}, ab[KM] = {}, rest[KM] = {}, part[KM][2] = {};
    for (int k = 1; k <= K; ++k) {
        const LayerIO io = layer(k);
        const bool mean = io.ep.mode == LGCN_EPI_MEAN;
        {  // side 1
            const Lane& L = lanes[(k + 1 + K) & 1];
            Deps dp;
            if (classes && k >= 2) {
                dp.part_wait[0] = cls[k - 1][0];
                dp.part_wait[1] = ab[k - 1];
            }
            dp.defer = k < K && sched && !cap;
            // the final mean's side-1 layer kernel (lane 1's last) on lane 0's chain stream at
            // normal priority: on lane 1's high-priority stream its grid held the dispatcher, and
            // side 0's mean layer (lane 0, the critical path) started ~1.3 ms after the walk it
            // waits for; sharing the queues they overlap (round 6: C3 forward -0.25..0.35 ms)
            if (k == K && mean && sched && sched->lk_normal && two && l1_aux && !cap &&
                sched->n_aux >= 3)
                dp.lk = sched->aux[2];
            if (mean && k >= 2) {  // the layer kernel's rows read layer K-1's layer-kernel rows
                dp.late[0] = rest[k - 1];
                dp.late_emu[0] = part[k - 1][0];
                dp.late_emu[1] = part[k - 1][1];
            }
            if (int e = seg_layer(rowptr, edges, row_ids, sd.split, n, plans, k, 3, io, d, sched,
                                  L, &dp))
                return e;
            if (k < K && sched) {
                if (int e = record(sched, L.main, &rest[k])) return e;
                part[k][0] = dp.part_done[0];
                part[k][1] = dp.part_done[1];
            }
        }
        {  // side 0, one class at a time
            const Lane& L = lanes[(k + K) & 1];
            static const int up[3] = {0, 1, 2}, down[3] = {2, 1, 0};
            const int* order = k == 1 ? up : down;
            for (int t = 0; t < 3; ++t) {
                const int c = order[t];
                // (without classes every class reads everything: all wait for both parts)
                if (k >= 2 && (c <= 1 || !classes))
                    if (int e = wait_ev(L.main, part[k - 1][1])) return e;
                if (k >= 2 && (c == 0 || !classes))
                    if (int e = wait_ev(L.main, part[k - 1][0])) return e;
                Deps dp;
                if (mean && k >= 2) dp.late[0] = cls[k - 1][c];
                if (int e = seg_layer(rowptr, edges, row_ids, lo[c], seg_hi(c, n), plans, k, c,
                                      io, d, sched, L, &dp))
                    return e;
                if (sched)
                    if (int e = record(sched, L.main, &cls[k][c])) return e;
            }
            ab[k] = k == 1 ? cls[k][1] : cls[k][0];
        }
    }
    return join_lanes(sched, two, lanes[1], s);
}
}  // namespace

extern "C" {

int lgcn_sched_create(void* const* aux_streams, int32_t n_aux, lgcn_sched_t** out) {
    if (!out || n_aux < 1 || n_aux > 7 || !aux_streams) return LGCN_EINVAL;
    for (int i = 0; i < n_aux; ++i)
        if (!aux_streams[i]) return LGCN_EINVAL;
    lgcn_sched* sc = new (std::nothrow) lgcn_sched();
    EventPool* pool = new (std::nothrow) EventPool();
    if (!sc || !pool) {
        delete sc;
        delete pool;
        return LGCN_EINVAL;
    }
    memset(sc, 0, sizeof(*sc));
    sc->pool = pool;
    const int n0 = n_aux < 3 ? n_aux : 3;
    sc->n_aux = n0;
    sc->chain = 1;
    sc->classes = 1;
    sc->lk_normal = 1;
    for (int i = 0; i < n0; ++i) sc->aux[i] = reinterpret_cast<hipStream_t>(aux_streams[i]);
    int e = 0;
    for (; pool->n < kPoolEvents && !e; ++pool->n)
        e = herr(hipEventCreateWithFlags(&pool->ev[pool->n], hipEventDisableTiming));
    if (e) --pool->n;  // (the failed slot holds no event)
    if (!e) {
        sc->lane1s = new (std::nothrow) lgcn_sched();
        if (!sc->lane1s) e = LGCN_EINVAL;
        if (!e) {
            lgcn_sched* l1 = sc->lane1s;
            memset(l1, 0, sizeof(*l1));
            l1->pool = pool;
            l1->n_aux = n0;
            l1->chain = 1;
            l1->classes = 1;
            for (int i = 0; i < n0; ++i) l1->aux[i] = sc->aux[n0 - 1 - i];
        }
    }
    if (!e && n_aux >= 4) {
        sc->lane1_main = reinterpret_cast<hipStream_t>(aux_streams[3]);
        sc->lane1 = new (std::nothrow) lgcn_sched();
        if (!sc->lane1) e = LGCN_EINVAL;
        if (!e) {
            lgcn_sched* l1 = sc->lane1;
            memset(l1, 0, sizeof(*l1));
            l1->pool = pool;
            l1->n_aux = n_aux - 4;
            l1->chain = 1;
            l1->classes = 1;
            for (int i = 0; i < l1->n_aux; ++i)
                l1->aux[i] = reinterpret_cast<hipStream_t>(aux_streams[4 + i]);
        }
    }
    if (e) {
        lgcn_sched_destroy(sc);
        return e;
    }
    *out = sc;
    return 0;
}

int lgcn_sched_destroy(lgcn_sched_t* sc) {
    if (!sc) return 0;
    if (sc->pool) {
        for (int i = 0; i < sc->pool->n; ++i) (void)hipEventDestroy(sc->pool->ev[i]);
        delete sc->pool;
    }
    delete sc->lane1;  // (views: share the root's pool)
    delete sc->lane1s;
    delete sc;
    return 0;
}

int lgcn_sched_set(lgcn_sched_t* sc, int32_t knob, int64_t value) {
    if (!sc) return LGCN_EINVAL;
    switch (knob) {
        case LGCN_SCHED_SLOTS0:
        case LGCN_SCHED_SLOTS1:
            if (value < 0 || value > LGCN_EMU_MAX_WALK_SLOTS) return LGCN_EINVAL;
            sc->slots[knob - LGCN_SCHED_SLOTS0] = (int32_t)value;
            if (sc->lane1) sc->lane1->slots[knob - LGCN_SCHED_SLOTS0] = (int32_t)value;
            if (sc->lane1s) sc->lane1s->slots[knob - LGCN_SCHED_SLOTS0] = (int32_t)value;
            return 0;
        case LGCN_SCHED_CHAIN:
            sc->chain = value != 0;
            if (sc->lane1) sc->lane1->chain = value != 0;
            if (sc->lane1s) sc->lane1s->chain = value != 0;
            return 0;
        case LGCN_SCHED_LANE1_SHARED:
            sc->lane1_shared = value != 0;
            return 0;
        case LGCN_SCHED_TIMING_START:
            sc->t0 = reinterpret_cast<hipEvent_t>(value);
            return 0;
        case LGCN_SCHED_TIMING_END:
            sc->t1 = reinterpret_cast<hipEvent_t>(value);
            return 0;
        case LGCN_SCHED_TRACE:
            sc->trace = reinterpret_cast<hipEvent_t*>(value);
            return 0;
        case LGCN_SCHED_TRACE_SIDES:
            sc->trace_sides = reinterpret_cast<hipEvent_t*>(value);
            return 0;
        case LGCN_SCHED_TIMING_SIDES:
            sc->timing_sides = reinterpret_cast<hipEvent_t*>(value);
            return 0;
        case LGCN_SCHED_CLASSES:
            sc->classes = value != 0;
            return 0;
        case LGCN_SCHED_LK_NORMAL:
            sc->lk_normal = value != 0;
            return 0;
        default:
            return LGCN_EINVAL;
    }
}

int lgcn_capture_full_schedule(void) { return runtime_captures_full() ? 1 : 0; }

int64_t lgcn_sched_state(const lgcn_sched_t* sc, int32_t what) {
    if (!sc || what < LGCN_SCHED_STATE_LANES || what > LGCN_SCHED_STATE_CAPTURE_FULL)
        return LGCN_EINVAL;
    return sc->pool->state[what - LGCN_SCHED_STATE_LANES];
}

int lgcn_layer(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
               int32_t n_rows, const lgcn_hub_plan_t* plan, lgcn_rows_t x, float x_div,
               const uint32_t* x_nz, float* y, int64_t ldy, int32_t d,
               const lgcn_epilogue_t* epi_host, const lgcn_sched_t* sched, void* stream) {
    if (int e = valid_geom(n_rows, d)) return e;
    if (int e = check_epi(epi_host)) return e;
    if (int e = check_plan(plan)) return e;
    if (n_rows > 0 && (!rowptr || !y || ldy < d)) return LGCN_EINVAL;
    if (!(x_div > 0.f)) return LGCN_EINVAL;
    if (epi_host->mode != LGCN_EPI_ADD && (x_div != 1.f || x_nz)) return LGCN_EINVAL;
    if (sched) sched->pool->next = 0;
    return plan_layer(rowptr, edges, row_ids, n_rows, *plan, x, x_div, x_nz, y, ldy, d,
                      *epi_host, sched, S(stream));
}

int lgcn_propagate_forward(const int32_t* rowptr, const lgcn_edge_t* edges,
                           const int32_t* row_ids, int32_t n, const lgcn_hub_plan_t* plan,
                           lgcn_rows_t emb, int32_t d,
                           int32_t K, float* const* layer_bufs_host, float* out,
                           void* const* ev_host, const lgcn_sched_t* sched, void* stream) {
    if (int e = valid_geom(n, d)) return e;
    if (K < 0 || K - 1 > LGCN_MAX_LAYERS || !out) return K < 0 || !out ? LGCN_EINVAL : LGCN_ETOOMANY;
    if (K > 1 && !layer_bufs_host) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (K == 0) return scale_rows(emb, n, d, 1.0f, out, d, s);
    if (int e = check_plan(plan)) return e;
    if (sched) sched->pool->next = 0;
    for (int k = 1; k <= K; ++k) {
        const lgcn_rows_t x = (k == 1) ? emb : dense_rows(layer_bufs_host[k - 2], n, d);
        lgcn_epilogue_t ep;
        memset(&ep, 0, sizeof(ep));
        float* y;
        if (k < K) {
            ep.mode = LGCN_EPI_STORE;
            y = layer_bufs_host[k - 1];
        } else {
            ep.mode = LGCN_EPI_MEAN;
            ep.n_prev = K;
            ep.div = (float)(K + 1);
            ep.prev0 = emb;
            for (int i = 0; i + 1 < K; ++i) ep.prev_dense[i] = layer_bufs_host[i];
            ep.ld_prev = d;
            y = out;
        }
        if (ev_host) {
            if (int e = herr(hipEventRecord((hipEvent_t)ev_host[2 * (k - 1)], s))) return e;
        }
        if (int e = plan_layer(rowptr, edges, row_ids, n, *plan, x, 1.f, nullptr, y, d, d, ep,
                               sched, s))
            return e;
        if (ev_host) {
            if (int e = herr(hipEventRecord((hipEvent_t)ev_host[2 * (k - 1) + 1], s))) return e;
        }
    }
    return 0;
}

int lgcn_propagate_forward_sides(const int32_t* rowptr, const lgcn_edge_t* edges,
                                 const int32_t* row_ids, const lgcn_sides_t* sides,
                                 const lgcn_hub_plan_t* plans, lgcn_rows_t emb, int32_t d,
                                 int32_t K, float* const* layer_bufs_host, float* out,
                                 const lgcn_sched_t* sched, void* stream) {
    const int32_t n = sides ? sides->n : -1;
    if (int e = valid_geom(n, d)) return e;
    if (K < 0 || K - 1 > LGCN_MAX_LAYERS || !out) return K < 0 || !out ? LGCN_EINVAL : LGCN_ETOOMANY;
    if (K > 1 && !layer_bufs_host) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (K == 0) return scale_rows(emb, n, d, 1.0f, out, d, s);
    if (int e = check_sides(rowptr, row_ids, n, sides, plans)) return e;
    auto layer = [&](int k) {
        LayerIO io;
        memset(&io, 0, sizeof(io));
        io.x = (k == 1) ? emb : dense_rows(layer_bufs_host[k - 2], n, d);
        io.xdiv = 1.f;
        if (k < K) {
            io.ep.mode = LGCN_EPI_STORE;
            io.y = layer_bufs_host[k - 1];
        } else {
            io.ep.mode = LGCN_EPI_MEAN;
            io.ep.n_prev = K;
            io.ep.div = (float)(K + 1);
            io.ep.prev0 = emb;
            for (int i = 0; i + 1 < K; ++i) io.ep.prev_dense[i] = layer_bufs_host[i];
            io.ep.ld_prev = d;
            io.y = out;
        }
        return io;
    };
    return run_sides(rowptr, edges, row_ids, *sides, plans, d, K, layer, sched, s);
}

int lgcn_propagate_backward_sides(const int32_t* rowptr, const lgcn_edge_t* edges,
                                  const int32_t* row_ids, const lgcn_sides_t* sides,
                                  const lgcn_hub_plan_t* plans, lgcn_rows_t grad_out,
                                  const uint32_t* grad_nz, int32_t d, int32_t K, float* work_h,
                                  float* grad_e0, const lgcn_sched_t* sched, void* stream) {
    const int32_t n = sides ? sides->n : -1;
    if (int e = valid_geom(n, d)) return e;
    if (K < 0 || !grad_out.p0 || !grad_e0) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (K == 0) return scale_rows(grad_out, n, d, 1.0f, grad_e0, d, s);
    if (K > 1 && !work_h) return LGCN_EINVAL;
    if (int e = check_sides(rowptr, row_ids, n, sides, plans)) return e;
    // as lgcn_propagate_backward: h = G/(K+1) + Âᵀ h, layer k into grad_e0 or work_h alternately
    auto out_of = [&](int k) { return ((K - k) % 2 == 0) ? grad_e0 : work_h; };
    auto layer = [&](int k) {
        LayerIO io;
        memset(&io, 0, sizeof(io));
        io.x = k == 1 ? grad_out : dense_rows(out_of(k - 1), n, d);
        io.xdiv = k == 1 ? (float)(K + 1) : 1.f;
        io.x_nz = k == 1 ? grad_nz : nullptr;
        io.y = out_of(k);
        io.ep.mode = LGCN_EPI_ADD;
        io.ep.addend = grad_out;
        io.ep.addend_nz = grad_nz;
        io.ep.div = (float)(K + 1);
        return io;
    };
    // (round 5: the backward with its lanes flipped, the high-priority lane carrying the chain
    // of half-layers that starts with side 0, measured 9.74 / 9.76 vs 9.65 / 9.64 ms: not kept)
    return run_sides(rowptr, edges, row_ids, *sides, plans, d, K, layer, sched, s);
}

int lgcn_propagate_backward(const int32_t* rowptr, const lgcn_edge_t* edges,
                            const int32_t* row_ids, int32_t n, const lgcn_hub_plan_t* plan,
                            lgcn_rows_t grad_out,
                            const uint32_t* grad_nz, int32_t d, int32_t K, float* work_h,
                            float* grad_e0, const lgcn_sched_t* sched, void* stream) {
    if (int e = valid_geom(n, d)) return e;
    if (K < 0 || !grad_out.p0 || !grad_e0) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (K == 0) return scale_rows(grad_out, n, d, 1.0f, grad_e0, d, s);
    if (K > 1 && !work_h) return LGCN_EINVAL;
    if (int e = check_plan(plan)) return e;
    if (sched) sched->pool->next = 0;
    // MeanBackward hands every layer c = G / (K+1); it is never materialised: layer 1 gathers
    // G / (K+1) on load and every epilogue adds G[row] / (K+1) (same rounding as c).
    const float div = (float)(K + 1);
    lgcn_epilogue_t ep;
    memset(&ep, 0, sizeof(ep));
    ep.mode = LGCN_EPI_ADD;
    ep.addend = grad_out;
    ep.addend_nz = grad_nz;
    ep.div = div;
    lgcn_rows_t h = grad_out;
    float xdiv = div;
    const uint32_t* x_nz = grad_nz;
    for (int k = 1; k <= K; ++k) {
        float* y = ((K - k) % 2 == 0) ? grad_e0 : work_h;
        if (int e = plan_layer(rowptr, edges, row_ids, n, *plan, h, xdiv, x_nz, y, d, d, ep, sched,
                               s))
            return e;
        h = dense_rows(y, n, d);
        xdiv = 1.f;
        x_nz = nullptr;
    }
    return 0;
}

}  // extern "C"
