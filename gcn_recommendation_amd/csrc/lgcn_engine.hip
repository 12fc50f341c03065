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
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>
#include <string.h>

#include "lgcn.h"

namespace {

constexpr int kBlock = 256;

// ---------------------------------------------------------------------------------------------
// small vector helpers: V = float4 (vector path) or float (scalar path)
// ---------------------------------------------------------------------------------------------
template <typename V> struct VT;
template <> struct VT<float4> {
    static constexpr int W = 4;
    __device__ static float4 zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
    __device__ static float4 load(const float* p) { return *reinterpret_cast<const float4*>(p); }
    __device__ static void store(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
    __device__ static float4 fma(float a, float4 x, float4 y) {
        return make_float4(__builtin_fmaf(a, x.x, y.x), __builtin_fmaf(a, x.y, y.y),
                           __builtin_fmaf(a, x.z, y.z), __builtin_fmaf(a, x.w, y.w));
    }
    __device__ static float4 add(float4 a, float4 b) {
        return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
    __device__ static float4 div(float4 a, float b) {
        return make_float4(a.x / b, a.y / b, a.z / b, a.w / b);
    }
};
template <> struct VT<float> {
    static constexpr int W = 1;
    __device__ static float zero() { return 0.f; }
    __device__ static float load(const float* p) { return *p; }
    __device__ static void store(float* p, float v) { *p = v; }
    __device__ static float fma(float a, float x, float y) { return __builtin_fmaf(a, x, y); }
    __device__ static float add(float a, float b) { return a + b; }
    __device__ static float div(float a, float b) { return a / b; }
};

__device__ __forceinline__ const float* seg_row(const lgcn_rows_t& s, int32_t r) {
    if (r < s.end0) return s.p0 + (int64_t)r * s.ld;
    if (r < s.end1) return s.p1 + (int64_t)(r - s.end0) * s.ld;
    return s.p2 + (int64_t)(r - s.end1) * s.ld;
}

__device__ __forceinline__ int2 load_edge(const lgcn_edge_t* e) {
    return *reinterpret_cast<const int2*>(e);
}

// Sequential fmaf chain over edge records [beg, end) — the ATen CPU order (one row's nonzeros in
// stored order, y = fma(val, x, y) starting from +0). U gathers are in flight before the folds.
// x / div, correctly rounded. When div is a power of two, x * (1/div) is the same real number,
// so it rounds identically and costs one multiply instead of the IEEE division sequence.
template <typename V>
__device__ __forceinline__ V mul_s(V v, float s) {
    if constexpr (VT<V>::W == 4) return make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
    else return v * s;
}

// inv_bits: 0, or the bits of 1/div when div is a power of two (precomputed on the host)
template <typename V>
__device__ __forceinline__ V div_exact(V v, float div, int32_t inv_bits) {
    if (inv_bits != 0) return mul_s<V>(v, __int_as_float(inv_bits));
    return VT<V>::div(v, div);
}

__host__ __device__ __forceinline__ bool is_pow2f(float x) {
    int e;
    return x > 0.f && frexpf(x, &e) == 0.5f;
}

// XD & 3: 0 = gather X as is, 1 = X / xdiv (IEEE division), 2 = X * xdiv where the host
// already replaced a power-of-two divisor by its (exact) reciprocal.
// XD & 4: X is row-sparse; x_nz is a bitmask of its rows that hold a nonzero. Edges into an
// all-zero row are skipped: fma(v, ±0, acc) == acc for every acc a chain can hold (a chain
// starts at +0 and never reaches -0), so the result is bitwise that of the dense chain.
template <typename V, int XD>
__device__ __forceinline__ V load_x(const float* p, float xdiv) {
    const V v = VT<V>::load(p);
    if constexpr ((XD & 3) == 1) return VT<V>::div(v, xdiv);  // X / xdiv, rounded once
    else if constexpr ((XD & 3) == 2) return mul_s<V>(v, xdiv);  // host passes 1/xdiv (exact)
    else return v;
}

__device__ __forceinline__ bool row_live(const uint32_t* __restrict__ nz, int32_t r) {
    return (nz[r >> 5] >> (r & 31)) & 1u;
}

template <typename V, int G, int NV, int U, int XD = 0>
__device__ __forceinline__ void accumulate(const lgcn_edge_t* __restrict__ edges, int32_t beg,
                                           int32_t end, const lgcn_rows_t& x, int lane, int dW,
                                           V (&acc)[NV], float xdiv = 1.f,
                                           const uint32_t* __restrict__ x_nz = nullptr) {
    using T = VT<V>;
    for (int32_t j = beg; j < end; j += U) {
        const int n = min(U, end - j);
        int2 e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = (u < n) ? load_edge(edges + j + u) : make_int2(0, 0);
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (XD & 4) live[u] = u < n && row_live(x_nz, e[u].x);
            else live[u] = u < n;
        }
        V xv[U][NV];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float* rp = seg_row(x, e[u].x);
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int c = lane + q * G;
                xv[u][q] = (live[u] && c < dW) ? load_x<V, XD>(rp + c * T::W, xdiv) : T::zero();
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (live[u]) {
                const float v = __int_as_float(e[u].y);
#pragma unroll
                for (int q = 0; q < NV; ++q) acc[q] = T::fma(v, xv[u][q], acc[q]);
            }
        }
    }
}

// Fused epilogue for one output row (lanes of the row's group).
template <typename V, int G, int NV, int MODE>
__device__ __forceinline__ void epilogue_store(const lgcn_epilogue_t& ep, int32_t row, int lane,
                                               int dW, V (&acc)[NV], float* __restrict__ y,
                                               int64_t ldy) {
    using T = VT<V>;
    float* yr = y + (int64_t)row * ldy;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const int c = lane + q * G;
        if (c >= dW) continue;
        V out = acc[q];
        if constexpr (MODE == LGCN_EPI_MEAN) {
            // ((E0 + E1) + ... + E_{K-1}) + E_K, then / (K+1): torch.mean(torch.stack(.), 0)
            V s = T::load(seg_row(ep.prev0, row) + c * T::W);
            for (int i = 0; i + 1 < ep.n_prev; ++i)
                s = T::add(s, T::load(ep.prev_dense[i] + (int64_t)row * ep.ld_prev + c * T::W));
            s = T::add(s, out);
            out = div_exact<V>(s, ep.div, ep.pad);
        } else if constexpr (MODE == LGCN_EPI_ADD) {
            // Horner step: (Z / div) + Â·X, Z read in place (segments), Z / div rounded once.
            // A row outside addend_nz is all ±0: ±0/div + out == out (out is never -0).
            if (!ep.addend_nz || row_live(ep.addend_nz, row))
                out = T::add(div_exact<V>(T::load(seg_row(ep.addend, row) + c * T::W), ep.div,
                                          ep.pad), out);
        }
        T::store(yr + c * T::W, out);
    }
}

// Rows of one group, RPG at a time: the group walks the bundle's edges as ONE stream (hub rows
// skipped) and folds them in stored order, flushing a row's accumulator (fused epilogue) when the
// stream passes its end. Each row is still one sequential fmaf chain, so results are identical to
// one row per group; what changes is the latency structure:
//  * edge records arrive in windows of G records (one coalesced load per window, lane l holding
//    record wb+l) with the next window prefetched, and reach every lane by shuffles — the only
//    memory latency left on the critical path is the gather itself;
//  * U gathers are in flight per group across row boundaries.
template <typename V, int G, int NV, int MODE, int RPG, int U, int XD>
__device__ __forceinline__ void rows_bundle(const int32_t* __restrict__ rowptr,
                                            const lgcn_edge_t* __restrict__ edges,
                                            const int32_t* __restrict__ row_ids, int32_t n_rows,
                                            int32_t hub_thr, int32_t r0, const lgcn_rows_t& x,
                                            float* __restrict__ y, int64_t ldy, int lane, int dW,
                                            const lgcn_epilogue_t& ep, float xdiv,
                                            const uint32_t* __restrict__ x_nz) {
    using T = VT<V>;
    static_assert(RPG < G, "row boundaries are held one per lane");
    const int nrows = min(RPG, n_rows - r0);
    // lane l (l <= nrows) holds rowptr[r0 + l]; boundaries are read back by shuffles
    const int32_t rpl = (lane <= nrows) ? rowptr[r0 + lane] : 0;
    auto bnd = [&](int i) { return __shfl(rpl, i, G); };
    // lane l (l < nrows) holds the output row of slot r0 + l (the CSR may be stored in a
    // processing order: slot s holds the edges of row row_ids[s])
    const int32_t orl = (lane < nrows) ? (row_ids ? row_ids[r0 + lane] : r0 + lane) : 0;
    const int32_t eend = bnd(nrows);
    auto load_win = [&](int32_t b) {
        return (b + lane < eend) ? load_edge(edges + b + lane) : make_int2(0, 0);
    };
    V acc[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) acc[q] = T::zero();
    int fr = 0;                              // next row to flush (bundle-relative)
    int lr = 0;                              // row the load cursor is in
    int32_t lend = bnd(1);
    int32_t j = bnd(0);
    if (lend - j > hub_thr) j = lend;        // hub rows: edges owned by the chunk path
    int32_t wb = j;                          // window base
    int2 win = load_win(wb);
    int2 nxt = load_win(wb + G);
    auto flush = [&](int i) {
        const int32_t deg = bnd(i + 1) - bnd(i);
        const int32_t orow = __shfl(orl, i, G);
        if (deg <= hub_thr) epilogue_store<V, G, NV, MODE>(ep, orow, lane, dW, acc, y, ldy);
#pragma unroll
        for (int q = 0; q < NV; ++q) acc[q] = T::zero();
    };
    while (true) {
        int col[U];
        float val[U];
        int rid[U];
        int cnt = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            while (j >= lend && lr < nrows) {
                ++lr;
                if (lr < nrows) {
                    const int32_t b = bnd(lr);
                    lend = bnd(lr + 1);
                    j = (lend - b > hub_thr) ? lend : b;
                }
            }
            rid[u] = lr;
            col[u] = 0;
            val[u] = 0.f;
            if (lr < nrows) {
                if (j >= wb + G) {
                    if (j < wb + 2 * G) {
                        win = nxt;
                        wb += G;
                    } else {  // jumped over a hub row
                        wb = j;
                        win = load_win(wb);
                    }
                    nxt = load_win(wb + G);
                }
                const int idx = j - wb;
                col[u] = __shfl(win.x, idx, G);
                val[u] = __int_as_float(__shfl(win.y, idx, G));
                ++j;
                ++cnt;
            }
        }
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (XD & 4) live[u] = u < cnt && row_live(x_nz, col[u]);
            else live[u] = u < cnt;
        }
        V xv[U][NV];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float* rp = seg_row(x, col[u]);
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int c = lane + q * G;
                xv[u][q] = (live[u] && c < dW) ? load_x<V, XD>(rp + c * T::W, xdiv) : T::zero();
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u < cnt) {
                while (fr < rid[u]) flush(fr++);
                if (live[u]) {
#pragma unroll
                    for (int q = 0; q < NV; ++q) acc[q] = T::fma(val[u], xv[u][q], acc[q]);
                }
            }
        }
        if (cnt < U) break;
    }
    while (fr < nrows) flush(fr++);
}

// MEAN epilogue with its NP previous-layer rows loaded before the gathers (they do not depend on
// them) and pre-summed in the reference order ((E0 + E1) + ...) + E_K.
template <typename V, int G, int NV, int NP>
__device__ __forceinline__ void mean_prefetch(const lgcn_epilogue_t& ep, int32_t row, int lane,
                                              int dW, V (&pre)[NP][NV]) {
    using T = VT<V>;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const float* src = p == 0 ? seg_row(ep.prev0, row)
                                  : ep.prev_dense[p - 1] + (int64_t)row * ep.ld_prev;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int c = lane + q * G;
            pre[p][q] = c < dW ? T::load(src + c * T::W) : T::zero();
        }
    }
}

template <typename V, int G, int NV, int MODE, int RPG, int U, int NP = 0, int XD = 0>
__global__ __launch_bounds__(kBlock) void k_layer(
    const int32_t* __restrict__ rowptr, const lgcn_edge_t* __restrict__ edges,
    const int32_t* __restrict__ row_ids, int32_t n_rows,
    int32_t hub_thr, const lgcn_hub_item_t* __restrict__ items, int32_t n_items,
    int32_t hub_blocks, float* __restrict__ partials, lgcn_rows_t x, float* __restrict__ y,
    int64_t ldy, int32_t d, int32_t dW, lgcn_epilogue_t ep, float xdiv,
    const uint32_t* __restrict__ x_nz) {
    using T = VT<V>;
    constexpr int RPB = kBlock / G;
    const int lane = threadIdx.x & (G - 1);
    const int grp = threadIdx.x / G;

    if ((int32_t)blockIdx.x < hub_blocks) {  // hub chunks first: the longest work starts earliest
        const int32_t it = blockIdx.x * RPB + grp;
        if (it >= n_items) return;
        const lgcn_hub_item_t w = items[it];
        V acc[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) acc[q] = T::zero();
        constexpr int UH = NV >= 8 ? 1 : 8 / NV;  // hub chunks are long: deep unroll
        accumulate<V, G, NV, UH, XD>(edges, w.beg, w.end, x, lane, dW, acc, xdiv, x_nz);
        float* pr = partials + (int64_t)w.slot * d;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int c = lane + q * G;
            if (c < dW) T::store(pr + c * T::W, acc[q]);
        }
        return;
    }
    const int64_t gidx = (int64_t)(blockIdx.x - hub_blocks) * RPB + grp;
    if constexpr (RPG == 1) {
        if (gidx >= n_rows) return;
        const int32_t slot = (int32_t)gidx;
        const int32_t beg = rowptr[slot];
        const int32_t end = rowptr[slot + 1];
        if (end - beg > hub_thr) return;  // owned by the hub chunks + k_hub_combine
        const int32_t row = row_ids ? row_ids[slot] : slot;  // output row of this slot
        V acc[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) acc[q] = T::zero();
        if constexpr (MODE == LGCN_EPI_MEAN && NP > 0) {
            V pre[NP][NV];
            mean_prefetch<V, G, NV, NP>(ep, row, lane, dW, pre);
            accumulate<V, G, NV, U, XD>(edges, beg, end, x, lane, dW, acc, xdiv, x_nz);
            float* yr = y + (int64_t)row * ldy;
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int c = lane + q * G;
                if (c >= dW) continue;
                V s = pre[0][q];
#pragma unroll
                for (int p = 1; p < NP; ++p) s = T::add(s, pre[p][q]);
                T::store(yr + c * T::W, div_exact<V>(T::add(s, acc[q]), ep.div, ep.pad));
            }
        } else {
            accumulate<V, G, NV, U, XD>(edges, beg, end, x, lane, dW, acc, xdiv, x_nz);
            epilogue_store<V, G, NV, MODE>(ep, row, lane, dW, acc, y, ldy);
        }
    } else {
        const int64_t r0 = gidx * RPG;
        if (r0 >= n_rows) return;
        rows_bundle<V, G, NV, MODE, RPG, U, XD>(rowptr, edges, row_ids, n_rows, hub_thr,
                                                (int32_t)r0, x, y, ldy, lane, dW, ep, xdiv,
                                                x_nz);
    }
}

// One block per hub row: group g sums slots g, g+NG, ... in order; groups are then added in
// group order. Deterministic (fixed order), not the CPU's single chain.
template <typename V, int G, int NV, int MODE>
__global__ __launch_bounds__(kBlock) void k_hub_combine(const lgcn_hub_row_t* __restrict__ rows,
                                                        const float* __restrict__ partials,
                                                        float* __restrict__ y, int64_t ldy,
                                                        int32_t d, int32_t dW, lgcn_epilogue_t ep) {
    using T = VT<V>;
    constexpr int NG = kBlock / G;
    __shared__ V red[NG][G * NV];
    const int lane = threadIdx.x & (G - 1);
    const int grp = threadIdx.x / G;
    const lgcn_hub_row_t hr = rows[blockIdx.x];
    V acc[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) acc[q] = T::zero();
    constexpr int UC = 8;  // slot loads in flight per group; added in slot order
    for (int s0 = grp; s0 < hr.n_slots; s0 += NG * UC) {
        V pv[UC][NV];
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const int s = s0 + u * NG;
            const float* pr = partials + (int64_t)(hr.first_slot + s) * d;
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int c = lane + q * G;
                pv[u][q] = (s < hr.n_slots && c < dW) ? T::load(pr + c * T::W) : T::zero();
            }
        }
#pragma unroll
        for (int u = 0; u < UC; ++u)
            if (s0 + u * NG < hr.n_slots)
#pragma unroll
                for (int q = 0; q < NV; ++q) acc[q] = T::add(acc[q], pv[u][q]);
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) red[grp][lane + q * G] = acc[q];
    __syncthreads();
    if (grp != 0) return;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        V t = red[0][lane + q * G];
        for (int g = 1; g < NG; ++g) t = T::add(t, red[g][lane + q * G]);
        acc[q] = t;
    }
    epilogue_store<V, G, NV, MODE>(ep, hr.row, lane, dW, acc, y, ldy);
}

template <typename V, int G, int NV>
__global__ __launch_bounds__(kBlock) void k_scale_rows(lgcn_rows_t x, int32_t n_rows, int32_t dW,
                                                       float div, float* __restrict__ y,
                                                       int64_t ldy) {
    using T = VT<V>;
    constexpr int RPB = kBlock / G;
    const int lane = threadIdx.x & (G - 1);
    const int32_t row = blockIdx.x * RPB + threadIdx.x / G;
    if (row >= n_rows) return;
    const float* xr = seg_row(x, row);
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const int c = lane + q * G;
        if (c < dW) T::store(y + (int64_t)row * ldy + c * T::W, T::div(T::load(xr + c * T::W), div));
    }
}

// Row-sparsity mask of a block: bit r of mask = row r holds a value != 0 (NaN counts). A block
// owns 256 rows = 8 mask words (plain stores, no global atomics); one atomicAdd per block
// accumulates the live-row count.
template <typename V, int G, int NV>
__global__ __launch_bounds__(kBlock) void k_rows_nonzero(lgcn_rows_t x, int32_t n_rows, int32_t dW,
                                                         uint32_t* __restrict__ mask,
                                                         int32_t* __restrict__ count) {
    using T = VT<V>;
    constexpr int RPB = kBlock / G;          // rows per pass
    constexpr int ROWS = 256;                // rows per block
    __shared__ uint32_t words[ROWS / 32];
    const int lane = threadIdx.x & (G - 1);
    const int grp = threadIdx.x / G;
    if (threadIdx.x < ROWS / 32) words[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * ROWS;
    for (int i = grp; i < ROWS; i += RPB) {
        const int64_t r = base + i;
        bool nz = false;
        if (r < n_rows) {
            const float* xr = seg_row(x, (int32_t)r);
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int c = lane + q * G;
                if (c < dW) {
                    const V v = T::load(xr + c * T::W);
                    if constexpr (T::W == 4) nz |= !(v.x == 0.f && v.y == 0.f && v.z == 0.f && v.w == 0.f);
                    else nz |= !(v == 0.f);
                }
            }
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) nz |= __shfl_xor((int)nz, o, G) != 0;
        if (lane == 0 && nz) atomicOr(&words[i >> 5], 1u << (i & 31));
    }
    __syncthreads();
    if (threadIdx.x < ROWS / 32) {
        const int64_t w = (int64_t)blockIdx.x * (ROWS / 32) + threadIdx.x;
        if (w * 32 < n_rows) mask[w] = words[threadIdx.x];
        const int c = __popc(words[threadIdx.x]);
        int t = c;
#pragma unroll
        for (int o = 4; o > 0; o >>= 1) t += __shfl_xor(t, o, 8);
        if (threadIdx.x == 0 && t) atomicAdd(count, t);
    }
}

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
__global__ void k_csr_degrees(const int32_t* __restrict__ rowptr, int32_t n,
                              int32_t* __restrict__ deg, int32_t* __restrict__ iota) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    deg[r] = rowptr[r + 1] - rowptr[r];
    iota[r] = (int32_t)r;
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

// ---------------------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------------------
inline int herr(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }
inline int last_err() { return herr(hipGetLastError()); }
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Launch geometry from d: (vector?) G lanes per row, NV elements-of-V per lane.
struct Geo {
    bool vec;
    int G;
    int NV;
    int dW;
};

inline int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

inline Geo pick_geo(int d, bool vec_ok) {
    Geo g;
    g.vec = vec_ok && (d % 4 == 0);
    g.dW = g.vec ? d / 4 : d;
    g.G = next_pow2(g.dW);
    if (g.G < 4) g.G = 4;
    if (g.G > 64) g.G = 64;
    int nv = (g.dW + g.G - 1) / g.G;
    g.NV = next_pow2(nv);
    return g;
}

bool rows_aligned(const lgcn_rows_t& r) {
    return al16(r.p0) && al16(r.p1) && al16(r.p2) && (r.ld % 4 == 0);
}

bool epi_aligned(const lgcn_epilogue_t& ep) {
    if (ep.mode == LGCN_EPI_MEAN) {
        if (!rows_aligned(ep.prev0) || ep.ld_prev % 4) return false;
        for (int i = 0; i + 1 < ep.n_prev; ++i)
            if (!al16(ep.prev_dense[i])) return false;
    }
    if (ep.mode == LGCN_EPI_ADD && !rows_aligned(ep.addend)) return false;
    return true;
}

// tuning knobs (lgcn_tune): 0 = automatic choice; explicit (rows per group, gathers in flight)
// pairs select a fixed d = 64 variant for A/B timing
int g_rows_per_group = 0;
int g_unroll = 0;

template <typename V, int G, int NV, int RPG, int U, int NP = 0>
int launch_layer_rpg(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
                     int32_t n_rows, int32_t thr,
                     const lgcn_hub_item_t* items, int32_t n_items, float* partials,
                     const lgcn_rows_t& x, float* y, int64_t ldy, int32_t d, int32_t dW,
                     const lgcn_epilogue_t& ep, float xdiv, const uint32_t* x_nz, hipStream_t s) {
    constexpr int RPB = kBlock / G;
    const int32_t hub_blocks = (n_items + RPB - 1) / RPB;
    const int64_t row_groups = ((int64_t)n_rows + RPG - 1) / RPG;
    const int64_t row_blocks = (row_groups + RPB - 1) / RPB;
    const int64_t grid = hub_blocks + row_blocks;
    if (grid == 0) return 0;
    if (grid > 0x7fffffffLL) return LGCN_EINVAL;
    // gather scaling and row-sparse X exist for the backward (ADD) only
    if (ep.mode != LGCN_EPI_ADD && (xdiv != 1.f || x_nz)) return LGCN_EINVAL;
#define LGCN_LAUNCH(MODE_, NP_, XD_, XDIV_)                                                      \
    hipLaunchKernelGGL((k_layer<V, G, NV, MODE_, RPG, U, NP_, XD_>), dim3((uint32_t)grid),       \
                       dim3(kBlock), 0, s, rowptr, edges, row_ids, n_rows, thr, items, n_items,  \
                       hub_blocks, partials, x, y, ldy, d, dW, ep, XDIV_, x_nz)
    switch (ep.mode) {
        case LGCN_EPI_STORE:
            LGCN_LAUNCH(LGCN_EPI_STORE, 0, 0, 1.f);
            break;
        case LGCN_EPI_MEAN:
            LGCN_LAUNCH(LGCN_EPI_MEAN, NP, 0, 1.f);
            break;
        case LGCN_EPI_ADD: {
            const int xd = (xdiv == 1.f ? 0 : is_pow2f(xdiv) ? 2 : 1) | (x_nz ? 4 : 0);
            const float xa = (xd & 3) == 2 ? 1.0f / xdiv : xdiv;
            switch (xd) {
                case 0: LGCN_LAUNCH(LGCN_EPI_ADD, 0, 0, xa); break;
                case 1: LGCN_LAUNCH(LGCN_EPI_ADD, 0, 1, xa); break;
                case 2: LGCN_LAUNCH(LGCN_EPI_ADD, 0, 2, xa); break;
                case 4: LGCN_LAUNCH(LGCN_EPI_ADD, 0, 4, xa); break;
                case 5: LGCN_LAUNCH(LGCN_EPI_ADD, 0, 5, xa); break;
                default: LGCN_LAUNCH(LGCN_EPI_ADD, 0, 6, xa); break;
            }
            break;
        }
        default:
            return LGCN_EINVAL;
    }
#undef LGCN_LAUNCH
    return last_err();
}

template <typename V, int G, int NV>
int launch_layer_t(const int32_t* rowptr, const lgcn_edge_t* edges, const int32_t* row_ids,
                   int32_t n_rows, int32_t thr,
                   const lgcn_hub_item_t* items, int32_t n_items, float* partials,
                   const lgcn_rows_t& x, float* y, int64_t ldy, int32_t d, int32_t dW,
                   const lgcn_epilogue_t& ep, float xdiv, const uint32_t* x_nz,
                   hipStream_t s) {
    // one row per group (deep unroll) on small graphs, row bundles (shallow unroll) otherwise
    constexpr int U1 = NV >= 8 ? 1 : 8 / NV;
    constexpr int UB = NV >= 4 ? 1 : 4 / NV;
    constexpr int RB = G >= 16 ? 15 : G - 1;
#define LGCN_ARGS rowptr, edges, row_ids, n_rows, thr, items, n_items, partials, x, y, ldy, d, dW, ep, xdiv, x_nz, s
    if constexpr (VT<V>::W == 4 && G == 16 && NV == 1) {  // d = 64: explicit variants (lgcn_tune)
#define LGCN_V(R_, U_) \
        if (g_rows_per_group == R_ && g_unroll == U_) return launch_layer_rpg<V, G, NV, R_, U_>(LGCN_ARGS);
        LGCN_V(1, 8) LGCN_V(8, 4) LGCN_V(15, 4) LGCN_V(8, 6) LGCN_V(15, 6) LGCN_V(8, 8)
        LGCN_V(15, 8)
#undef LGCN_V
    }
    // keep >= ~64k lane groups in the grid: small graphs (the reference's real datasets) run
    // one row per group, Books-scale graphs 15-row bundles (with degree-ordered slots the rows
    // of a bundle have equal length, which also pays for the MEAN epilogue's row reads)
    const int64_t per = (int64_t)n_rows / 65536;
    if (RB <= 1 || g_rows_per_group == 1 || per < 2) {
        if (ep.mode == LGCN_EPI_MEAN && NV <= 2) {  // early-issued E0..E_{K-1} row loads
            if (ep.n_prev == 2) return launch_layer_rpg<V, G, NV, 1, U1, 2>(LGCN_ARGS);
            if (ep.n_prev == 3) return launch_layer_rpg<V, G, NV, 1, U1, 3>(LGCN_ARGS);
            if (ep.n_prev == 4) return launch_layer_rpg<V, G, NV, 1, U1, 4>(LGCN_ARGS);
        }
        return launch_layer_rpg<V, G, NV, 1, U1>(LGCN_ARGS);
    }
    if (per >= RB) return launch_layer_rpg<V, G, NV, RB, UB>(LGCN_ARGS);
    if constexpr (RB >= 8) {
        if (per >= 8) return launch_layer_rpg<V, G, NV, 8, UB>(LGCN_ARGS);
    }
    if constexpr (RB >= 4) {
        if (per >= 4) return launch_layer_rpg<V, G, NV, 4, UB>(LGCN_ARGS);
    }
    if constexpr (RB >= 2) {
        if (per >= 2) return launch_layer_rpg<V, G, NV, 2, UB>(LGCN_ARGS);
    }
    return launch_layer_rpg<V, G, NV, 1, U1>(LGCN_ARGS);
#undef LGCN_ARGS
}

template <typename V, int G, int NV>
int launch_combine_t(const lgcn_hub_row_t* rows, int32_t n, const float* partials, float* y,
                     int64_t ldy, int32_t d, int32_t dW, const lgcn_epilogue_t& ep, hipStream_t s) {
    if (n <= 0) return 0;
    switch (ep.mode) {
        case LGCN_EPI_STORE:
            hipLaunchKernelGGL((k_hub_combine<V, G, NV, LGCN_EPI_STORE>), dim3(n), dim3(kBlock), 0, s,
                               rows, partials, y, ldy, d, dW, ep);
            break;
        case LGCN_EPI_MEAN:
            hipLaunchKernelGGL((k_hub_combine<V, G, NV, LGCN_EPI_MEAN>), dim3(n), dim3(kBlock), 0, s,
                               rows, partials, y, ldy, d, dW, ep);
            break;
        case LGCN_EPI_ADD:
            hipLaunchKernelGGL((k_hub_combine<V, G, NV, LGCN_EPI_ADD>), dim3(n), dim3(kBlock), 0, s,
                               rows, partials, y, ldy, d, dW, ep);
            break;
        default:
            return LGCN_EINVAL;
    }
    return last_err();
}

template <typename V, int G, int NV>
int launch_scale_t(const lgcn_rows_t& x, int32_t n_rows, int32_t dW, float div, float* y,
                   int64_t ldy, hipStream_t s) {
    constexpr int RPB = kBlock / G;
    const int64_t grid = ((int64_t)n_rows + RPB - 1) / RPB;
    if (grid == 0) return 0;
    hipLaunchKernelGGL((k_scale_rows<V, G, NV>), dim3((uint32_t)grid), dim3(kBlock), 0, s, x, n_rows,
                       dW, div, y, ldy);
    return last_err();
}

// Geometry dispatch: F is a generic lambda taking (V tag, G, NV) as template parameters via
// a functor with a templated call operator.
template <typename F>
int dispatch_geo(const Geo& g, const F& f) {
#define LGCN_CASE(VT_, G_, NV_) \
    if (g.G == G_ && g.NV == NV_) return f.template operator()<VT_, G_, NV_>();
    if (g.vec) {
        LGCN_CASE(float4, 4, 1)
        LGCN_CASE(float4, 8, 1)
        LGCN_CASE(float4, 16, 1)
        LGCN_CASE(float4, 32, 1)
        LGCN_CASE(float4, 64, 1)
        LGCN_CASE(float4, 64, 2)
        LGCN_CASE(float4, 64, 4)
        LGCN_CASE(float4, 64, 8)
    } else {
        LGCN_CASE(float, 4, 1)
        LGCN_CASE(float, 8, 1)
        LGCN_CASE(float, 16, 1)
        LGCN_CASE(float, 32, 1)
        LGCN_CASE(float, 64, 1)
        LGCN_CASE(float, 64, 2)
        LGCN_CASE(float, 64, 4)
        LGCN_CASE(float, 64, 8)
        LGCN_CASE(float, 64, 16)
        LGCN_CASE(float, 64, 32)
    }
#undef LGCN_CASE
    return LGCN_EINVAL;
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

struct LayerF {
    const int32_t* rowptr; const lgcn_edge_t* edges; const int32_t* row_ids; int32_t n_rows, thr;
    const lgcn_hub_item_t* items; int32_t n_items; float* partials; const lgcn_rows_t* x;
    float* y; int64_t ldy; int32_t d, dW; const lgcn_epilogue_t* ep; float xdiv;
    const uint32_t* x_nz; hipStream_t s;
    template <typename V, int G, int NV> int operator()() const {
        return launch_layer_t<V, G, NV>(rowptr, edges, row_ids, n_rows, thr, items, n_items,
                                        partials, *x, y, ldy, d, dW, *ep, xdiv, x_nz, s);
    }
};

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
    LayerF f{rowptr, edges, row_ids, n_rows, thr, items, n_items, partials, &x, y, ldy, d, g.dW,
             &ep, xdiv, x_nz, s};
    return dispatch_geo(g, f);
}

int hub_combine(const lgcn_hub_row_t* rows, int32_t n, const float* partials, float* y,
                int64_t ldy, int32_t d, const lgcn_epilogue_t& ep_in, hipStream_t s) {
    if (n <= 0) return 0;
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
extern "C" {

int lgcn_abi_version(void) { return LGCN_ABI_VERSION; }

int lgcn_tune(int knob, int value) {
    switch (knob) {
        case LGCN_TUNE_ROWS_PER_GROUP: {
            const int old = g_rows_per_group;
            if (value >= 0) g_rows_per_group = value;
            return old;
        }
        case LGCN_TUNE_UNROLL: {
            const int old = g_unroll;
            if (value >= 0) g_unroll = value;
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

int lgcn_device_info(int device, int32_t* n_cu_host, int32_t* arch_major_host) {
    hipDeviceProp_t p;
    const hipError_t e = hipGetDeviceProperties(&p, device);
    if (e != hipSuccess) return (int)e;
    if (n_cu_host) *n_cu_host = p.multiProcessorCount;
    if (arch_major_host) *arch_major_host = p.major;
    return 0;
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
                             int64_t nnz, int32_t* deg_tmp, int32_t* deg_sorted, int32_t* iota_tmp,
                             int32_t* row_ids, int32_t* rowptr_out, lgcn_edge_t* edges_out,
                             void* temp, size_t* temp_bytes_host, void* stream) {
    if (n_rows < 0 || nnz < 0 || nnz > 0x7fffffffLL || !temp_bytes_host) return LGCN_EINVAL;
    int end_bit = 1;  // degrees are <= nnz
    while (end_bit < 31 && (1LL << end_bit) <= nnz) ++end_bit;
    hipStream_t s = S(stream);
    const int n = n_rows;
    if (temp == nullptr) {
        size_t b1 = 0, b2 = 0;
        hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(
            nullptr, b1, deg_tmp, deg_sorted, iota_tmp, row_ids, n, 0, end_bit, s);
        if (e != hipSuccess) return (int)e;
        e = hipcub::DeviceScan::InclusiveSum(nullptr, b2, deg_sorted, rowptr_out, n, s);
        *temp_bytes_host = b1 > b2 ? b1 : b2;
        return herr(e);
    }
    if (!rowptr || !rowptr_out || (n > 0 && (!deg_tmp || !deg_sorted || !iota_tmp || !row_ids)))
        return LGCN_EINVAL;
    if (nnz > 0 && (!edges || !edges_out)) return LGCN_EINVAL;
    if (int e = herr(hipMemsetAsync(rowptr_out, 0, sizeof(int32_t), s))) return e;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_csr_degrees, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, rowptr, n, deg_tmp, iota_tmp);
    if (int e = last_err()) return e;
    size_t bytes = *temp_bytes_host;
    // LSD radix sort: stable, so rows of equal degree keep their id order
    if (int e = herr(hipcub::DeviceRadixSort::SortPairsDescending(
            temp, bytes, deg_tmp, deg_sorted, iota_tmp, row_ids, n, 0, end_bit, s)))
        return e;
    bytes = *temp_bytes_host;
    if (int e = herr(hipcub::DeviceScan::InclusiveSum(temp, bytes, deg_sorted, rowptr_out + 1, n, s)))
        return e;
    if (nnz == 0) return 0;
    hipLaunchKernelGGL(k_csr_gather_rows, dim3((uint32_t)((nnz + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, s, rowptr_out, row_ids, rowptr, edges, n, nnz, edges_out);
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

int lgcn_hub_combine(const lgcn_hub_row_t* hub_rows, int32_t n_hub_rows, const float* partials,
                     float* y, int64_t ldy, int32_t d, const lgcn_epilogue_t* epi_host,
                     void* stream) {
    if (d < 1 || d > 2048 || n_hub_rows < 0) return LGCN_EINVAL;
    if (int e = check_epi(epi_host)) return e;
    if (n_hub_rows > 0 && (!hub_rows || !partials || !y || ldy < d)) return LGCN_EINVAL;
    return hub_combine(hub_rows, n_hub_rows, partials, y, ldy, d, *epi_host, S(stream));
}

int lgcn_scale_rows(lgcn_rows_t x, int32_t n_rows, int32_t d, float div, float* y, int64_t ldy,
                    void* stream) {
    if (int e = valid_geom(n_rows, d)) return e;
    if (n_rows > 0 && (!y || ldy < d)) return LGCN_EINVAL;
    return scale_rows(x, n_rows, d, div, y, ldy, S(stream));
}

int lgcn_propagate_forward(const int32_t* rowptr, const lgcn_edge_t* edges,
                           const int32_t* row_ids, int32_t n,
                           int32_t hub_threshold, const lgcn_hub_item_t* hub_items,
                           int32_t n_hub_items, const lgcn_hub_row_t* hub_rows,
                           int32_t n_hub_rows, float* partials, lgcn_rows_t emb, int32_t d,
                           int32_t K, float* const* layer_bufs_host, float* out,
                           void* const* ev_host, void* stream) {
    if (int e = valid_geom(n, d)) return e;
    if (K < 0 || K - 1 > LGCN_MAX_LAYERS || !out) return K < 0 || !out ? LGCN_EINVAL : LGCN_ETOOMANY;
    if (K > 1 && !layer_bufs_host) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (K == 0) return scale_rows(emb, n, d, 1.0f, out, d, s);
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
        if (int e = spmm_layer(rowptr, edges, row_ids, n, hub_threshold, hub_items, n_hub_items,
                               partials, x, y, d, d, ep, 1.f, nullptr, s))
            return e;
        if (ev_host) {
            if (int e = herr(hipEventRecord((hipEvent_t)ev_host[2 * (k - 1) + 1], s))) return e;
        }
        if (int e = hub_combine(hub_rows, n_hub_rows, partials, y, d, d, ep, s)) return e;
    }
    return 0;
}

int lgcn_propagate_backward(const int32_t* rowptr, const lgcn_edge_t* edges,
                            const int32_t* row_ids, int32_t n,
                            int32_t hub_threshold, const lgcn_hub_item_t* hub_items,
                            int32_t n_hub_items, const lgcn_hub_row_t* hub_rows,
                            int32_t n_hub_rows, float* partials, lgcn_rows_t grad_out,
                            const uint32_t* grad_nz, int32_t d, int32_t K, float* work_h,
                            float* grad_e0, void* stream) {
    if (int e = valid_geom(n, d)) return e;
    if (K < 0 || !grad_out.p0 || !grad_e0) return LGCN_EINVAL;
    hipStream_t s = S(stream);
    if (K == 0) return scale_rows(grad_out, n, d, 1.0f, grad_e0, d, s);
    if (K > 1 && !work_h) return LGCN_EINVAL;
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
        if (int e = spmm_layer(rowptr, edges, row_ids, n, hub_threshold, hub_items, n_hub_items,
                               partials, h, y, d, d, ep, xdiv, x_nz, s))
            return e;
        if (int e = hub_combine(hub_rows, n_hub_rows, partials, y, d, d, ep, s)) return e;
        h = dense_rows(y, n, d);
        xdiv = 1.f;
        x_nz = nullptr;
    }
    return 0;
}

}  // extern "C"
