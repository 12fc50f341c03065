// lgcn_kernels.h — internal to liblgcn_engine.so: the propagation kernel templates
// (k_layer and its helpers, k_hub_combine, k_scale_rows, k_rows_nonzero) and their host-side
// dispatch. Included by lgcn_engine.hip (graph preparation + C ABI) and by one translation unit
// per epilogue mode (lgcn_layer_{store,mean,add}.hip), so the many k_layer instantiations
// compile in parallel. Not part of the C ABI (include/lgcn.h is). Design: DESIGN.md §4.
#pragma once
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>
#include <string.h>

#include "lgcn.h"


namespace lgcn_detail {
// tuning knobs (lgcn_tune): 0 = automatic choice; explicit (rows per group, gathers in flight)
// pairs select a fixed d = 64 variant for A/B timing
extern int g_rows_per_group;
extern int g_unroll;
extern int g_mean_prefetch;  // LGCN_TUNE_MEAN_PREFETCH: 2 = off
extern int g_min_groups;     // LGCN_TUNE_MIN_GROUPS: 0 = 65536

// one lgcn_spmm_layer launch, geometry already chosen (dW = d / lanes' element width)
struct LayerArgs {
    const int32_t* rowptr;
    const lgcn_edge_t* edges;
    const int32_t* row_ids;
    int32_t n_rows, thr;
    const lgcn_hub_item_t* items;
    int32_t n_items;
    float* partials;
    lgcn_rows_t x;
    float* y;
    int64_t ldy;
    int32_t d, dW;
    lgcn_epilogue_t ep;
    float xdiv;
    const uint32_t* x_nz;
    hipStream_t s;
    bool vec;
    int G, NV;
};
int layer_store(const LayerArgs& a);       // lgcn_layer_store.hip
int layer_mean(const LayerArgs& a);        // lgcn_layer_mean.hip
// ADD: by the gather variant XD (see load_x): 0 | 1, 2 (G / (K+1) on load) | 4, 5, 6 (row-sparse)
int layer_add(const LayerArgs& a, int xd);         // lgcn_layer_add.hip
int layer_add_div(const LayerArgs& a, int xd);     // lgcn_layer_add_div.hip
int layer_add_sparse(const LayerArgs& a, int xd);  // lgcn_layer_add_sparse.hip
// lgcn_live_rows in two steps (lgcn_exact.hip): the live-edge flags and compaction, then the
// chains over the compacted live edges — so a schedule can run the chains on a stream of their
// own once the flags (which gate the walks) are done
int live_prepare(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks, int32_t n_blocks,
                 const lgcn_emu_row_t* rows, int32_t n_rows, const uint32_t* x_nz, int32_t d,
                 float x_div, const lgcn_epilogue_t* epi_host, float* y, int64_t ldy,
                 const void* x_p0, int32_t live_min, int32_t max_live, void* scratch,
                 hipStream_t s);
int live_chains(int32_t n_blocks, int32_t n_rows, lgcn_rows_t x, float x_div, float* y,
                int64_t ldy, int32_t d, const lgcn_epilogue_t* epi_host, void* scratch,
                hipStream_t s);
}  // namespace lgcn_detail

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

// Streams touched once per layer (edge records, output rows, the mean epilogue's row reads) can
// be marked non-temporal so they do not displace the gathered rows in L2 (LGCN_NT build flag).
#ifndef LGCN_NT
#define LGCN_NT 0
#endif
typedef float f4_t __attribute__((ext_vector_type(4)));

// MEAN bundle prefetch: widest lane group it is used for (8: d <= 32; 16 adds d = 64 with
// bundles of LGCN_MEAN_PF_RPG16 rows) — build-time A/B knobs
#ifndef LGCN_MEAN_PF_MAX_G
#define LGCN_MEAN_PF_MAX_G 8
#endif
#ifndef LGCN_MEAN_PF_RPG16
#define LGCN_MEAN_PF_RPG16 4
#endif

__device__ __forceinline__ int2 load_edge(const lgcn_edge_t* e) {
    if constexpr (LGCN_NT & 1) {
        const long long v = __builtin_nontemporal_load(reinterpret_cast<const long long*>(e));
        return make_int2((int)(v & 0xffffffffLL), (int)(v >> 32));
    } else {
        return *reinterpret_cast<const int2*>(e);
    }
}

template <typename V>
__device__ __forceinline__ void store_out(float* p, V v) {
    if constexpr ((LGCN_NT & 2) && VT<V>::W == 4) {
        f4_t t = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(t, reinterpret_cast<f4_t*>(p));
    } else if constexpr (LGCN_NT & 2) {
        __builtin_nontemporal_store(v, p);
    } else {
        VT<V>::store(p, v);
    }
}

template <typename V>
__device__ __forceinline__ V load_stream(const float* p) {
    if constexpr ((LGCN_NT & 4) && VT<V>::W == 4) {
        const f4_t t = __builtin_nontemporal_load(reinterpret_cast<const f4_t*>(p));
        return make_float4(t.x, t.y, t.z, t.w);
    } else if constexpr (LGCN_NT & 4) {
        return __builtin_nontemporal_load(p);
    } else {
        return VT<V>::load(p);
    }
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
    if constexpr (XD & 4) {
        // row-sparse X: windows of G records, one per lane; every lane looks up its record's
        // mask bit (in parallel, the next window already in flight), the group's live edges come
        // out of the ballot in stored order and are folded in that order
        const int base = (int)(threadIdx.x & 63) - lane;  // the group's first lane in the wave
        int2 rec = (beg + lane < end) ? load_edge(edges + beg + lane) : make_int2(0, 0);
        for (int32_t wb = beg; wb < end; wb += G) {
            const int2 nrec = (wb + G + lane < end) ? load_edge(edges + wb + G + lane)
                                                    : make_int2(0, 0);
            const bool lvb = wb + lane < end && row_live(x_nz, rec.x);
            unsigned long long m = __ballot(lvb) >> base;
            if constexpr (G < 64) m &= (1ull << G) - 1;
            while (m) {
                const int i = __builtin_ctzll(m);
                m &= m - 1;
                const int c = __shfl(rec.x, i, G);
                const float v = __int_as_float(__shfl(rec.y, i, G));
                const float* rp = seg_row(x, c);
#pragma unroll
                for (int q = 0; q < NV; ++q) {
                    const int cc = lane + q * G;
                    if (cc < dW) acc[q] = T::fma(v, load_x<V, XD>(rp + cc * T::W, xdiv), acc[q]);
                }
            }
            rec = nrec;
        }
        return;
    }
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
                                               int64_t ldy, int alive = -1) {
    using T = VT<V>;
    float* yr = y + (int64_t)row * ldy;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const int c = lane + q * G;
        if (c >= dW) continue;
        V out = acc[q];
        if constexpr (MODE == LGCN_EPI_MEAN) {
            // ((E0 + E1) + ... + E_{K-1}) + E_K, then / (K+1): torch.mean(torch.stack(.), 0)
            V s = load_stream<V>(seg_row(ep.prev0, row) + c * T::W);
            for (int i = 0; i + 1 < ep.n_prev; ++i)
                s = T::add(s, load_stream<V>(ep.prev_dense[i] + (int64_t)row * ep.ld_prev + c * T::W));
            s = T::add(s, out);
            out = div_exact<V>(s, ep.div, ep.pad);
        } else if constexpr (MODE == LGCN_EPI_ADD) {
            // Horner step: (Z / div) + Â·X, Z read in place (segments), Z / div rounded once.
            // A row outside addend_nz is all ±0: ±0/div + out == out (out is never -0).
            // alive: the row's addend_nz bit when the caller looked it up ahead, else -1
            if (alive >= 0 ? alive != 0 : (!ep.addend_nz || row_live(ep.addend_nz, row)))
                out = T::add(div_exact<V>(T::load(seg_row(ep.addend, row) + c * T::W), ep.div,
                                          ep.pad), out);
        }
        store_out<V>(yr + c * T::W, out);
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
// NP > 0 (MEAN epilogue; NV == 1 and dW a power of two, so dW divides G): the bundle's
// E0..E_{K-1} rows are loaded before its edge stream starts — they do not depend on the gathers,
// so their latency leaves the flush. Element e of the bundle's row-major [nrows x dW] block sits
// in lane e % G, register slot e / G; all dW elements of a row share one slot, and a flush
// fetches them with one shuffle per layer.
template <typename V>
__device__ __forceinline__ V shfl_v(V v, int src, int width) {
    if constexpr (VT<V>::W == 4)
        return make_float4(__shfl(v.x, src, width), __shfl(v.y, src, width),
                           __shfl(v.z, src, width), __shfl(v.w, src, width));
    else return __shfl(v, src, width);
}

template <typename V, int G, int NV, int MODE, int RPG, int U, int XD, int NP = 0>
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
    // ADD: the addend_nz bits of the bundle's rows, looked up once in parallel (lane l: row l)
    // rather than one dependent lookup per flush
    int alv = 1;
    if constexpr (MODE == LGCN_EPI_ADD)
        alv = (ep.addend_nz && lane < nrows) ? (int)row_live(ep.addend_nz, orl) : 1;
    constexpr bool PRE = MODE == LGCN_EPI_MEAN && NP > 0;
    static_assert(!PRE || NV == 1, "bundle prefetch: one element per lane and slot");
    V pre[PRE ? NP : 1][PRE ? RPG : 1];
    if constexpr (PRE) {
#pragma unroll
        for (int s = 0; s < RPG; ++s) {
            const int e = s * G + lane;
            const int i = e / dW;
            const int c = e - i * dW;
            const int32_t orow = __shfl(orl, min(i, G - 1), G);
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const float* src = p == 0 ? seg_row(ep.prev0, orow)
                                          : ep.prev_dense[p - 1] + (int64_t)orow * ep.ld_prev;
                pre[p][s] = i < nrows ? load_stream<V>(src + c * T::W) : T::zero();
            }
        }
    }
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
    // XD & 4 (row-sparse X): each lane looks up the mask bit of ITS record once per window (one
    // round trip per G edges, in parallel) instead of every lane per edge; edges read it by shuffle
    auto win_live = [&](const int2& w, int32_t b) -> int {
        if constexpr (XD & 4) return (b + lane < eend && row_live(x_nz, w.x)) ? 1 : 0;
        else return 1;
    };
    int2 win = load_win(wb);
    int2 nxt = load_win(wb + G);
    int wlv = win_live(win, wb);
    auto flush = [&](int i) {
        const int32_t deg = bnd(i + 1) - bnd(i);
        const int32_t orow = __shfl(orl, i, G);
        if constexpr (PRE) {
            // ((E0 + E1) + ... + E_{K-1}) + E_K, then / (K+1) — epilogue_store's order
            const int s = (i * dW) / G;                 // the row's slot, uniform in the group
            const int src = (i * dW + lane) & (G - 1);  // lane holding column `lane` of row i
            V sum = T::zero();
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                V v = pre[p][0];
#pragma unroll
                for (int q = 1; q < RPG; ++q)
                    if (q == s) v = pre[p][q];
                v = shfl_v<V>(v, src, G);
                sum = p == 0 ? v : T::add(sum, v);
            }
            if (deg <= hub_thr && lane < dW)
                store_out<V>(y + (int64_t)orow * ldy + lane * T::W,
                             div_exact<V>(T::add(sum, acc[0]), ep.div, ep.pad));
        } else {
            const int al = MODE == LGCN_EPI_ADD ? __shfl(alv, i, G) : -1;
            if (deg <= hub_thr)
                epilogue_store<V, G, NV, MODE>(ep, orow, lane, dW, acc, y, ldy, al);
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) acc[q] = T::zero();
    };
    while (true) {
        int col[U];
        float val[U];
        int rid[U];
        int lv[U];
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
            lv[u] = 0;
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
                    wlv = win_live(win, wb);
                }
                const int idx = j - wb;
                col[u] = __shfl(win.x, idx, G);
                val[u] = __int_as_float(__shfl(win.y, idx, G));
                if constexpr (XD & 4) lv[u] = __shfl(wlv, idx, G);
                ++j;
                ++cnt;
            }
        }
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (XD & 4) live[u] = u < cnt && lv[u];
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
            pre[p][q] = c < dW ? load_stream<V>(src + c * T::W) : T::zero();
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
        if (w.slot < 0) {  // a whole long row: one exact chain, epilogue in place
            epilogue_store<V, G, NV, MODE>(ep, w.row, lane, dW, acc, y, ldy);
            return;
        }
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
                store_out<V>(yr + c * T::W, div_exact<V>(T::add(s, acc[q]), ep.div, ep.pad));
            }
        } else {
            accumulate<V, G, NV, U, XD>(edges, beg, end, x, lane, dW, acc, xdiv, x_nz);
            epilogue_store<V, G, NV, MODE>(ep, row, lane, dW, acc, y, ldy);
        }
    } else {
        const int64_t r0 = gidx * RPG;
        if (r0 >= n_rows) return;
        rows_bundle<V, G, NV, MODE, RPG, U, XD, NP>(rowptr, edges, row_ids, n_rows, hub_thr,
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

inline bool rows_aligned(const lgcn_rows_t& r) {
    return al16(r.p0) && al16(r.p1) && al16(r.p2) && (r.ld % 4 == 0);
}

inline bool epi_aligned(const lgcn_epilogue_t& ep) {
    if (ep.mode == LGCN_EPI_MEAN) {
        if (!rows_aligned(ep.prev0) || ep.ld_prev % 4) return false;
        for (int i = 0; i + 1 < ep.n_prev; ++i)
            if (!al16(ep.prev_dense[i])) return false;
    }
    if (ep.mode == LGCN_EPI_ADD && !rows_aligned(ep.addend)) return false;
    return true;
}

template <typename V, int G, int NV, int MODE, int XD, int RPG, int U, int NP = 0>
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
#define LGCN_LAUNCH(NP_, XD_, XDIV_)                                                             \
    hipLaunchKernelGGL((k_layer<V, G, NV, MODE, RPG, U, NP_, XD_>), dim3((uint32_t)grid),         \
                       dim3(kBlock), 0, s, rowptr, edges, row_ids, n_rows, thr, items, n_items,  \
                       hub_blocks, partials, x, y, ldy, d, dW, ep, XDIV_, x_nz)
    if constexpr (MODE == LGCN_EPI_ADD) {
        const float xa = (XD & 3) == 2 ? 1.0f / xdiv : xdiv;  // power of two: exact reciprocal
        LGCN_LAUNCH(0, XD, xa);
    } else {
        // gather scaling and row-sparse X exist for the backward (ADD) only
        if (xdiv != 1.f || x_nz) return LGCN_EINVAL;
        LGCN_LAUNCH(NP, 0, 1.f);
    }
#undef LGCN_LAUNCH
    return last_err();
}

template <typename V, int G, int NV, int MODE, int XD>
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
        if (lgcn_detail::g_rows_per_group == R_ && lgcn_detail::g_unroll == U_) return launch_layer_rpg<V, G, NV, MODE, XD, R_, U_>(LGCN_ARGS);
        LGCN_V(1, 8) LGCN_V(8, 4) LGCN_V(15, 4) LGCN_V(8, 6) LGCN_V(15, 6) LGCN_V(8, 8)
        LGCN_V(15, 8)
#undef LGCN_V
    }
    // keep >= ~64k lane groups in the grid: small graphs (the reference's real datasets) run
    // one row per group, Books-scale graphs 15-row bundles (with degree-ordered slots the rows
    // of a bundle have equal length, which also pays for the MEAN epilogue's row reads)
    const int64_t per = (int64_t)n_rows /
                        (lgcn_detail::g_min_groups > 0 ? lgcn_detail::g_min_groups : 65536);
    if (RB <= 1 || lgcn_detail::g_rows_per_group == 1 || per < 2) {
        if (MODE == LGCN_EPI_MEAN && NV <= 2) {  // early-issued E0..E_{K-1} row loads
            if (ep.n_prev == 2) return launch_layer_rpg<V, G, NV, MODE, XD, 1, U1, 2>(LGCN_ARGS);
            if (ep.n_prev == 3) return launch_layer_rpg<V, G, NV, MODE, XD, 1, U1, 3>(LGCN_ARGS);
            if (ep.n_prev == 4) return launch_layer_rpg<V, G, NV, MODE, XD, 1, U1, 4>(LGCN_ARGS);
        }
        return launch_layer_rpg<V, G, NV, MODE, XD, 1, U1>(LGCN_ARGS);
    }
    if constexpr (MODE == LGCN_EPI_MEAN && NV == 1 && G >= 4 && G <= LGCN_MEAN_PF_MAX_G) {
        // small d (featsplit shards): the flush's E0..E_{K-1} row reads are latency on the
        // critical path; bundles of RM rows prefetch them (RM register slots per layer)
        constexpr int RM = G >= 16 ? LGCN_MEAN_PF_RPG16 : G >= 8 ? 4 : RB;
        if (lgcn_detail::g_mean_prefetch != 2 && per >= RM && (dW & (dW - 1)) == 0) {
            if (ep.n_prev == 2) return launch_layer_rpg<V, G, NV, MODE, XD, RM, UB, 2>(LGCN_ARGS);
            if (ep.n_prev == 3) return launch_layer_rpg<V, G, NV, MODE, XD, RM, UB, 3>(LGCN_ARGS);
            if (ep.n_prev == 4) return launch_layer_rpg<V, G, NV, MODE, XD, RM, UB, 4>(LGCN_ARGS);
        }
    }
    if (per >= RB) return launch_layer_rpg<V, G, NV, MODE, XD, RB, UB>(LGCN_ARGS);
    if constexpr (RB >= 8) {
        if (per >= 8) return launch_layer_rpg<V, G, NV, MODE, XD, 8, UB>(LGCN_ARGS);
    }
    if constexpr (RB >= 4) {
        if (per >= 4) return launch_layer_rpg<V, G, NV, MODE, XD, 4, UB>(LGCN_ARGS);
    }
    if constexpr (RB >= 2) {
        if (per >= 2) return launch_layer_rpg<V, G, NV, MODE, XD, 2, UB>(LGCN_ARGS);
    }
    return launch_layer_rpg<V, G, NV, MODE, XD, 1, U1>(LGCN_ARGS);
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

template <int MODE, int XD>
struct LayerF {
    const lgcn_detail::LayerArgs* a;
    template <typename V, int G, int NV> int operator()() const {
        return launch_layer_t<V, G, NV, MODE, XD>(a->rowptr, a->edges, a->row_ids, a->n_rows, a->thr,
                                              a->items, a->n_items, a->partials, a->x, a->y,
                                              a->ldy, a->d, a->dW, a->ep, a->xdiv, a->x_nz, a->s);
    }
};

template <int MODE, int XD = 0>
int layer_mode(const lgcn_detail::LayerArgs& a) {
    const Geo g{a.vec, a.G, a.NV, a.dW};
    LayerF<MODE, XD> f{&a};
    return dispatch_geo(g, f);
}

}  // namespace
