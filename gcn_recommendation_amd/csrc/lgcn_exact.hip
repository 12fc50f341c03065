// lgcn_exact.hip — hub rows summed with the reference's exact arithmetic at any degree.
//
// The reference (models/lightgcn.py:45, torch.sparse.mm -> ATen addmm_sparse_dense_cpu) folds
// every row of Â·X as ONE sequential chain acc = fma(val_j, X[col_j, c], acc) per column c, in
// stored edge order, from +0. On a power-law graph one item row holds millions of edges; a chain
// that long is millions of dependent FMAs (~4.6 ms per layer for the 2.77M-edge row of the
// Books-scale graph even at one FMA per 4 cycles). This file reproduces that chain bit for bit
// without running it step by step.
//
// Translation invariance. Let e be a binade (|a| in [2^e, 2^(e+1))) and u = 2^(e-23) its ulp.
// If a chain value a is a multiple of u and a + p stays inside binade e, then
// fma-rounding gives RN(a + p) = a + RN_u(p) (RN_u: nearest multiple of u; the tie case depends
// on a's parity). So two chains over the same steps, started from a and a' in binade e, stay
// exactly a - a' apart as long as both trajectories stay inside the binade (and no step is an
// exact tie). Hence:
//   * k_emu_blocks cuts a hub row into blocks of <= 256 edges. For each (block, column) it runs
//     32 CANDIDATE chains from a' = +-1.5 * 2^e, e in a 16-binade window chosen from the block's
//     own first products, and records rel = chain_end - a' (exact), bounds lo/hi on the exact
//     running sum of its products (from the block's own chain from +0, widened by its rounding
//     error; every trajectory of the block stays within 128 ulps of that sum), and the largest
//     lowest-set-bit exponent of its products (a product can be an exact tie only if that
//     exponent reaches e - 24). Block 0 of a row keeps its chain from +0: the true value.
//   * k_emu_walk (one wave per (row, column)) walks the blocks in order with the true value a:
//     if a's binade has a candidate, both trajectories provably stay inside it and no tie is
//     possible, a += rel (exact); otherwise the block is re-run as the sequential fma chain.
// Every step is therefore either the reference's own fma or a proven-identical translation:
// the result is bitwise the reference's, whatever the data (ties, zero crossings, subnormals,
// inf/NaN all take the sequential path). oracle/lgcn_oracle.c holds the sequential chain the
// tests compare against; DESIGN.md §3 has the argument and the measured slow-block fractions.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "lgcn.h"

namespace {

constexpr int kW = LGCN_EMU_CANDS / 2;  // binades per sign
constexpr int kEOff = 2;                // window starts 2 binades above the first 64 steps' reach
constexpr int16_t kIdentity = -32768;   // maxlsb sentinel: no nonzero product in the block
constexpr int16_t kNoFast = 32000;      // maxlsb sentinel: never take the fast path
constexpr int kSlack = 132;             // ulps: 128 for <= 256 steps of <= 1/2 ulp + margin

struct EmuMeta {
    int32_t lo;      // floor(L * 2^(23 - ebase)), L a lower bound of the block's exact running sum
    int32_t hi;      // ceil(H * 2^(23 - ebase)), H an upper bound
    int16_t ebase;   // binade of candidate pair 0
    int16_t maxlsb;  // max over nonzero products of the exponent of their lowest set bit
                     // (kIdentity: no nonzero product; kNoFast: bounds too wide for int32)
    float r0;        // block 0 of a row: the exact chain from +0
};
static_assert(sizeof(EmuMeta) == LGCN_EMU_META_BYTES, "meta record size");

__device__ __forceinline__ const float* seg_row_x(const lgcn_rows_t& s, int32_t r) {
    if (r < s.end0) return s.p0 + (int64_t)r * s.ld;
    if (r < s.end1) return s.p1 + (int64_t)(r - s.end0) * s.ld;
    return s.p2 + (int64_t)(r - s.end1) * s.ld;
}

__device__ __forceinline__ bool row_live_x(const uint32_t* __restrict__ nz, int32_t r) {
    return (nz[r >> 5] >> (r & 31)) & 1u;
}

// X element as the layer kernels read it (lgcn_kernels.h load_x): XD & 3 = 1: / xdiv (IEEE),
// 2: * xdiv (host passes the exact reciprocal of a power-of-two divisor); XD & 4: row-sparse X
// (dead rows are all zero: fma(v, +-0, acc) == acc for every value a chain holds).
// Branch-free: the segment is chosen by selects and every load is issued unconditionally at a
// valid address (`ok` masks the value), so a batch of these loads is all in flight at once.
__device__ __forceinline__ const float* seg_row_sel(const lgcn_rows_t& s, int32_t r) {
    // p0 + an integer offset: a per-lane select between the three base POINTERS is turned by
    // the compiler into a per-lane load from the kernel-argument segment (a dependent round
    // trip before the element load); selecting between integer deltas keeps it in registers
    const char* b = reinterpret_cast<const char*>(s.p0);
    const int64_t row_b = s.ld * 4;
    const int64_t d1 = (reinterpret_cast<const char*>(s.p1) - b) - (int64_t)s.end0 * row_b;
    const int64_t d2 = (reinterpret_cast<const char*>(s.p2) - b) - (int64_t)s.end1 * row_b;
    const int64_t off = (int64_t)r * row_b + (r < s.end0 ? 0 : (r < s.end1 ? d1 : d2));
    return reinterpret_cast<const float*>(b + off);
}

template <int XD>
__device__ __forceinline__ float load_elem(const lgcn_rows_t& x, const uint32_t* x_nz, int32_t col,
                                           int c, float xdiv, bool ok = true) {
    // uniform row base + a 32-bit lane offset (global_load ... saddr form)
    float v = *reinterpret_cast<const float*>(
        reinterpret_cast<const char*>(seg_row_sel(x, col)) + (uint32_t)c * 4u);
    if constexpr ((XD & 4) != 0) ok = ok && row_live_x(x_nz, col);
    v = ok ? v : 0.f;
    if constexpr ((XD & 3) == 1) return v / xdiv;
    else if constexpr ((XD & 3) == 2) return v * xdiv;
    else return v;
}

// exponent of the lowest set bit of a finite nonzero float (subnormals included)
__device__ __forceinline__ int lsb_exp(float f) {
    const uint32_t b = __float_as_uint(f);
    const int E = (int)((b >> 23) & 255u);
    const uint32_t M = b & 0x7fffffu;
    if (E == 0) return -149 + __builtin_ctz(M);
    return E - 150 + __builtin_ctz(M | 0x800000u);
}

// ---------------------------------------------------------------------------------------------
// block pass: one wave per (block, 64-column slice); lane = column
// ---------------------------------------------------------------------------------------------
template <int XD>
__global__ __launch_bounds__(64) void k_emu_blocks(const lgcn_edge_t* __restrict__ edges,
                                                   const lgcn_emu_block_t* __restrict__ blocks,
                                                   lgcn_rows_t x, float xdiv,
                                                   const uint32_t* __restrict__ x_nz, int32_t d,
                                                   int32_t* __restrict__ rel,
                                                   EmuMeta* __restrict__ meta,
                                                   float* __restrict__ stage) {
    constexpr int SW = 16;  // steps gathered per sub-window (all in flight at once)
    const int lane = threadIdx.x;
    const int c = blockIdx.y * 64 + lane;
    const bool act = c < d;
    const lgcn_emu_block_t blk = blocks[blockIdx.x];
    // T: the sequential fma chain of the block from +0. It is the true chain for block 0; for
    // every block it tracks the exact running sum S of the products to within 1/2 ulp(|T|) per
    // step, which bounds every trajectory of the block (EmuMeta lo/hi)
    float T = 0.f, tlo = 0.f, thi = 0.f;
    int maxlsb = -100000;
    float cand[LGCN_EMU_CANDS];
    bool init = false;
    int ebase = 0;
    const int cc = act ? c : d - 1;  // lanes past d load a valid element and mask it
    // lane l holds edge record j0 + l of the current 64-edge window ((0, 0) past the block)
    auto load_rec = [&](int32_t j0) {
        const int32_t j = min(j0 + lane, blk.end - 1);
        const int2 r = *reinterpret_cast<const int2*>(edges + j);
        return j0 + lane < blk.end ? r : make_int2(0, 0);
    };
    auto load_sub = [&](const int2& rec, int s0, int n, float (&xv)[SW], float (&vv)[SW]) {
#pragma unroll
        for (int t = 0; t < SW; ++t) {
            const int32_t col = __builtin_amdgcn_readlane(rec.x, s0 + t);
            vv[t] = __int_as_float(__builtin_amdgcn_readlane(rec.y, s0 + t));
            xv[t] = load_elem<XD>(x, x_nz, col, cc, xdiv, act && s0 + t < n);
        }
    };
    // one sub-window: steps past the block end read as (0, 0), and fma(0, 0, c) == c for every
    // chain value (a chain is never -0), so the unrolled steps need no guard
    // this (block, column)'s elements, in step order (the walk re-runs a block from here)
    // stage layout [block][d + 1][BLOCK]: column c's X elements, then (column d) the edge values
    float* st = stage ? stage + ((int64_t)blockIdx.x * (d + 1) + cc) * LGCN_EMU_BLOCK : nullptr;
    float* sv = stage && blockIdx.y == 0
                    ? stage + ((int64_t)blockIdx.x * (d + 1) + d) * LGCN_EMU_BLOCK : nullptr;
    auto stage_sub = [&](const float (&xv)[SW], int step0) {
        if (!st || !act) return;
#pragma unroll
        for (int q = 0; q < SW / 4; ++q)
            *reinterpret_cast<float4*>(st + step0 + 4 * q) =
                make_float4(xv[4 * q], xv[4 * q + 1], xv[4 * q + 2], xv[4 * q + 3]);
    };
    auto run_sub = [&](const float (&xv)[SW], const float (&vv)[SW]) {
        if (!init) {
            // candidates start at the first sub-window holding a nonzero product (before it the
            // block is the identity for every start value); their binade window starts kEOff
            // above this sub-window's reach
            float s = T, m = 0.f;
#pragma unroll
            for (int t = 0; t < SW; ++t) {
                s = __builtin_fmaf(vv[t], xv[t], s);
                m = fmaxf(m, fabsf(s));
            }
            if (m > 0.f && m <= 3.0e38f) {
                init = true;
                int e;
                frexpf(m, &e);
                ebase = max(-200, min(e - 1 + kEOff + 1, 200));  // 16 steps reach ~1/2 of 64
#pragma unroll
                for (int k = 0; k < LGCN_EMU_CANDS; ++k) {
                    const int eb = ebase + (k >> 1);
                    const float a0 = (eb >= -126 && eb <= 127) ? ldexpf(1.5f, eb) : 1.5f;
                    cand[k] = (k & 1) ? -a0 : a0;
                }
            }
        }
#pragma unroll
        for (int t = 0; t < SW; ++t) {
            T = __builtin_fmaf(vv[t], xv[t], T);
            tlo = fminf(tlo, T);
            thi = fmaxf(thi, T);
            const int le = lsb_exp(vv[t]) + lsb_exp(xv[t]);
            maxlsb = (vv[t] != 0.f && xv[t] != 0.f) ? max(maxlsb, le) : maxlsb;
        }
        if (init) {
#pragma unroll
            for (int t = 0; t < SW; ++t) {
#pragma unroll
                for (int k = 0; k < LGCN_EMU_CANDS; ++k)
                    cand[k] = __builtin_fmaf(vv[t], xv[t], cand[k]);
            }
        }
    };
    int2 rec = load_rec(blk.beg);
    for (int32_t j0 = blk.beg; j0 < blk.end; j0 += 64) {
        const int n = min(64, blk.end - j0);
        const int2 nrec = load_rec(j0 + 64);  // next window's records, in flight meanwhile
        if (sv) sv[j0 - blk.beg + lane] = __int_as_float(rec.y);  // (0 past the block end)
        float xa[SW], va[SW], xb[SW], vb[SW];
        // the loads of sub-window k + 1 are issued before sub-window k is computed
        const int w0 = j0 - blk.beg;
        load_sub(rec, 0, n, xa, va);
        load_sub(rec, 16, n, xb, vb);
        run_sub(xa, va);
        stage_sub(xa, w0);
        load_sub(rec, 32, n, xa, va);
        run_sub(xb, vb);
        stage_sub(xb, w0 + 16);
        load_sub(rec, 48, n, xb, vb);
        run_sub(xa, va);
        stage_sub(xa, w0 + 32);
        run_sub(xb, vb);
        stage_sub(xb, w0 + 48);
        rec = nrec;
    }
    if (!act) return;
    const int64_t rc = (int64_t)blockIdx.x * d + c;
    // candidate k's translation in units of its ulp u_k = 2^(ebase + k/2 - 23): exact integer
    // when the candidate's chain stayed in its binade (the walker checks exactly that)
    int4* rp = reinterpret_cast<int4*>(rel + rc * LGCN_EMU_CANDS);
#pragma unroll
    for (int q = 0; q < LGCN_EMU_CANDS / 4; ++q) {
        int r4[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int k = 4 * q + t;
            const int eb = ebase + (k >> 1);
            const float a0 = (eb >= -126 && eb <= 127) ? ldexpf(1.5f, eb) : 1.5f;
            const float dlt = cand[k] - ((k & 1) ? -a0 : a0);
            const float ku = ldexpf(dlt, 23 - eb);
            r4[t] = (init && fabsf(ku) < 16777216.f) ? (int)ku : 0;
        }
        rp[q] = make_int4(r4[0], r4[1], r4[2], r4[3]);
    }
    // |T_j - S_j| <= j * ulp(max|T|) / 2 <= 128 * ulp(max|T|) for a block of <= 256 steps
    const float M = fmaxf(-tlo, thi);
    double err = 0.0;
    if (M > 0.f) {
        int e;
        frexpf(M, &e);  // M in [2^(e-1), 2^e): ulp(M) <= 2^(e-24) (subnormal ulp: 2^-149)
        err = (LGCN_EMU_BLOCK / 2) * ldexp(1.0, max(e - 24, -149));
    }
    const double lo_u = floor(ldexp((double)tlo - err, 23 - ebase));
    const double hi_u = ceil(ldexp((double)thi + err, 23 - ebase));
    const bool fits = lo_u >= -1073741824.0 && hi_u <= 1073741824.0;
    EmuMeta m;
    m.lo = fits ? (int32_t)lo_u : 0;
    m.hi = fits ? (int32_t)hi_u : 0;
    m.ebase = (int16_t)ebase;
    m.maxlsb = (maxlsb == -100000) ? kIdentity
               : !fits ? kNoFast : (int16_t)max(-32000, min(maxlsb, 31999));
    m.r0 = T;
    meta[rc] = m;
}

// ---------------------------------------------------------------------------------------------
// walker: one wave per (hub row, column). The chain value is wave-uniform.
// ---------------------------------------------------------------------------------------------
// A block the walk re-runs as the reference does: a = fma(val_j, x_j, a) in stored order.
// SlowData holds one lane's share of a block's (val, x) pairs, fetched with every load in
// flight at once: x from the staged copy (contiguous) or gathered from X (a second round trip).
struct SlowData {
    int2 rec[LGCN_EMU_BLOCK / 64];   // edge records of steps t * 64 + lane
    float xg[LGCN_EMU_BLOCK / 64];   // gathered x of the same steps (no stage)
    float4 xs;                       // staged x of steps 4 * lane .. 4 * lane + 3
};

template <int XD>
__device__ __forceinline__ void slow_load(SlowData& sd, const lgcn_edge_t* __restrict__ edges,
                                          int32_t beg, int32_t end, const lgcn_rows_t& x,
                                          float xdiv, const uint32_t* __restrict__ x_nz,
                                          const float* __restrict__ st, int c) {
    constexpr int Q = LGCN_EMU_BLOCK / 64;
    const int lane = threadIdx.x;
    const int n = end - beg;
#pragma unroll
    for (int t = 0; t < Q; ++t)  // clamped addresses, masked values: all loads in flight
        sd.rec[t] = *reinterpret_cast<const int2*>(edges + beg + min(t * 64 + lane, n - 1));
    if (st) {
        sd.xs = *reinterpret_cast<const float4*>(st + 4 * lane);
    } else {
#pragma unroll
        for (int t = 0; t < Q; ++t)
            sd.xg[t] = load_elem<XD>(x, x_nz, sd.rec[t].x, c, xdiv, t * 64 + lane < n);
    }
}

// LDS ordering point for the walker (a one-wave workgroup: a wave's LDS operations complete in
// order, so only the compiler must not move LDS accesses across this point). __syncthreads()
// would also make the compiler drain every global load in flight (vmcnt(0)) — the prefetched
// re-run blocks and the next chunk's records — exposing their latency at every re-run block.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// A re-run block's (val, x) pairs from a SlowData slot to LDS (sq[step] = (val, x)).
__device__ __forceinline__ void slow_stage(const SlowData& sd, int n, bool staged, float2* sq) {
    constexpr int Q = LGCN_EMU_BLOCK / 64;
    const int lane = threadIdx.x;
    wave_lds_sync();  // the previous chain's reads of sq are done
#pragma unroll
    for (int t = 0; t < Q; ++t) {
        const bool in = t * 64 + lane < n;
        sq[t * 64 + lane] = make_float2(in ? __int_as_float(sd.rec[t].y) : 0.f,
                                        staged ? 0.f : sd.xg[t]);
    }
    if (staged) {
        wave_lds_sync();
        const float xv[4] = {sd.xs.x, sd.xs.y, sd.xs.z, sd.xs.w};
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (4 * lane + t < n) sq[4 * lane + t].y = xv[t];
    }
    wave_lds_sync();
}

// The sequential chain over a staged block: a = fma(val_j, x_j, a), j = 0 .. n-1.
__device__ __forceinline__ float slow_chain(int n, float a, const float2* sq) {
    int i = 0;
    if (n == LGCN_EMU_BLOCK) {
        // full block: the LDS reads run PF groups of 8 steps ahead of the FMAs, so only the
        // dependent FMA chain is on the critical path
        constexpr int NG = LGCN_EMU_BLOCK / 8, PF = 4;
        float4 w[PF][4];
#pragma unroll
        for (int g = 0; g < PF; ++g)
#pragma unroll
            for (int k = 0; k < 4; ++k) w[g][k] = reinterpret_cast<const float4*>(sq + 8 * g)[k];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            float4 cur[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) cur[k] = w[g % PF][k];
            if (g + PF < NG) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    w[g % PF][k] = reinterpret_cast<const float4*>(sq + 8 * (g + PF))[k];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a = __builtin_fmaf(cur[k].x, cur[k].y, a);
                a = __builtin_fmaf(cur[k].z, cur[k].w, a);
            }
        }
        return a;
    }
    for (; i + 8 <= n; i += 8) {
        float2 w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = sq[i + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) a = __builtin_fmaf(w[k].x, w[k].y, a);
    }
    for (; i < n; ++i) a = __builtin_fmaf(sq[i].x, sq[i].y, a);
    return a;
}

// LGCN_EMU_STATS builds (diagnostics only, tools/exact_probe.py): walker decision counters
// [fast, slow, identity, slow: zero/subnormal, slow: window, slow: tie, slow: bounds, slow steps]
#ifdef LGCN_EMU_STATS
__device__ unsigned long long g_emu_stats[8];
// per emulated row (first 256 rows): fast blocks, slow blocks, cycles in slow blocks, max cycles
__device__ unsigned long long g_emu_row_stats[256][4];
#endif
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
// timing experiments only: 1 = re-run blocks skip their chain, 2 = every block translates
__device__ int g_emu_mode;
#define LGCN_EMU_FORCE(f) do { if (g_emu_mode == 2) (f) = true; } while (0)
#else
#define LGCN_EMU_FORCE(f) ((void)0)
#endif
#ifdef LGCN_EMU_STATS
// phase timer of the walker wave (row 0, column 0): s_memtime deltas per phase, then counts
// [stage, predict, fetch+wait, scans, chains, on-demand fetch, -, -, chunks, predicted, re-run,
//  not predicted]
__device__ unsigned long long g_emu_phase[16];
#define PH_MARK(k) do { const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
                        ph[k] += now_ - ph_last; ph_last = now_; } while (0)
#define PH_COUNT(k, v) (ph[k] += (v))
#else
#define PH_MARK(k) ((void)0)
#define PH_COUNT(k, v) ((void)0)
#endif
#ifdef LGCN_EMU_STATS
#define EMU_STAT(k, v) \
    do { if (threadIdx.x == 0) atomicAdd(&g_emu_stats[k], (unsigned long long)(v)); } while (0)
#else
#define EMU_STAT(k, v) ((void)0)
#endif

// Fast-path test (k_emu_walk): with e = binade(a), u = 2^(e-23), M = the integer mantissa
// (a = +-M u, 2^23 <= M < 2^24) and [lo, hi] the block's bounds in units of u, every trajectory
// value a + (c_j - a) stays in [2^e + u, 2^(e+1) - u] iff its mantissa stays in
// [2^23 + 1, 2^24 - 1]; kSlack covers the per-step rounding drift. For a < 0 the magnitude moves
// by -[lo, hi]. The candidate's own chain (from +-1.5 * 2^e) must pass the same test.

// The walk over one row for one column, 64 blocks at a time. Records are staged per chunk of 64
// blocks: while a chunk is walked, the next one's raw records are loaded into registers; at the
// chunk boundary they go to LDS together with, for every (block, candidate), the range of start
// mantissas the candidate's translation is valid for (the bounds test above, precomputed by all
// 64 lanes). Within a chunk the walk is a SPECULATIVE SCAN: with the chain value's binade, sign
// and mantissa (E, s, M) fixed, lane i takes block i's translation for (E, s), an exclusive
// prefix sum over the lanes gives the mantissa block i starts from if every block before it
// translates, and each lane tests its own block at that start. Up to the first failing block f
// every block translates, so the prefix at f is exactly what a block-by-block walk computes; f
// is re-run as the sequential chain and the scan resumes after it. A chunk of fast blocks costs
// one scan instead of 64 dependent steps.
// Re-run blocks need their (val, x) pairs, a global-memory round trip each. They are PREDICTED
// per chunk before the walk: the same scan run with approximate continuation (after a failing
// block f the value is taken as a + T_f, block f's chain from +0 — the true value to within its
// rounding) names the blocks likely to fail; their staged edge values and X elements go straight
// to LDS slots by LDS-DMA (global_load_lds_dwordx4) in one batch, so a chunk waits for memory
// once.
// A block that fails without having been predicted is fetched on demand into a spare slot.
#define LGCN_EMU_CH 64
#define LGCN_EMU_SLOTS 15   // default predicted re-run blocks per chunk with LDS slots (+1 spare)

struct EmuChunk {  // one lane's share of a chunk's raw records
    int32_t lo, hi, pk;                 // meta of block `lane`
    float t;                            // its chain from +0 (EmuMeta::r0)
    int32_t k[LGCN_EMU_CH / 2];         // translation (lane & 31) of block 2 j + (lane >> 5)
};

// Inclusive prefix sum over the 64 lanes of a wave by DPP row shifts and row broadcasts (no LDS
// round trips: the walker's scan is on its critical path).
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// A block's staged edge values and X elements -> an LDS slot by LDS-DMA
// (global_load_lds_dwordx4: the LDS destination is base + lane * 16 B; both sources are 1 KB,
// 1 KB-aligned rows of the stage).
__device__ __forceinline__ void fetch_block_lds(const float* __restrict__ sv,
                                                const float* __restrict__ sx, float* v, float* xs) {
    const int lane = threadIdx.x;
    __builtin_amdgcn_global_load_lds(sv + 4 * lane, v, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(sx + 4 * lane, xs, 16, 0, 0);
}

// The sequential chain over a block held in an LDS slot: a = fma(v_j, x_j, a), j < n.
__device__ __forceinline__ float slot_chain(int n, float a, const float* __restrict__ v,
                                            const float* __restrict__ xs) {
    if (n == LGCN_EMU_BLOCK) {
        // full block: the LDS reads run PF groups of 8 steps ahead of the FMAs, so only the
        // dependent FMA chain is on the critical path
        constexpr int NG = LGCN_EMU_BLOCK / 8, PF = 4;
        float4 wv[PF][2], wx[PF][2];
#pragma unroll
        for (int g = 0; g < PF; ++g) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                wv[g][k] = reinterpret_cast<const float4*>(v + 8 * g)[k];
                wx[g][k] = reinterpret_cast<const float4*>(xs + 8 * g)[k];
            }
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const float4 cv = wv[g % PF][k], cx = wx[g % PF][k];
                a = __builtin_fmaf(cv.x, cx.x, a);
                a = __builtin_fmaf(cv.y, cx.y, a);
                a = __builtin_fmaf(cv.z, cx.z, a);
                a = __builtin_fmaf(cv.w, cx.w, a);
            }
            if (g + PF < NG) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    wv[g % PF][k] = reinterpret_cast<const float4*>(v + 8 * (g + PF))[k];
                    wx[g % PF][k] = reinterpret_cast<const float4*>(xs + 8 * (g + PF))[k];
                }
            }
            // keep the reads PF groups ahead (the scheduler would otherwise sink them next to
            // their use and wait for each group's LDS round trip)
            __builtin_amdgcn_sched_barrier(0);
        }
        return a;
    }
    for (int i = 0; i < n; ++i) a = __builtin_fmaf(v[i], xs[i], a);
    return a;
}

template <int MODE, int XD>
__global__ __launch_bounds__(64) void k_emu_walk(const lgcn_edge_t* __restrict__ edges,
                                                 const lgcn_emu_block_t* __restrict__ blocks,
                                                 const lgcn_emu_row_t* __restrict__ rows,
                                                 const int32_t* __restrict__ rel,
                                                 const EmuMeta* __restrict__ meta,
                                                 const float* __restrict__ stage, lgcn_rows_t x,
                                                 float xdiv, const uint32_t* __restrict__ x_nz,
                                                 int32_t d, float* __restrict__ y, int64_t ldy,
                                                 lgcn_epilogue_t ep, int NS) {
    constexpr int CH = LGCN_EMU_CH;
    constexpr int NC = LGCN_EMU_CANDS;
    static_assert(CH == 64, "one lane per block of a chunk");
    __shared__ int32_t s_k[CH * NC], s_min[CH * NC], s_max[CH * NC];
    __shared__ float2 sq[LGCN_EMU_BLOCK];            // no-stage mode: gathered (val, x)
    // NS + 1 slots (dynamic LDS, sized at launch): re-run blocks' edge values, then their X
    // elements. Fewer slots = less LDS per wave = more walk waves per CU (short-row parts).
    extern __shared__ __attribute__((aligned(16))) float s_dyn[];
    auto s_v = [&](int sl) { return s_dyn + sl * LGCN_EMU_BLOCK; };
    auto s_xs = [&](int sl) { return s_dyn + (NS + 1 + sl) * LGCN_EMU_BLOCK; };
    const int lane = threadIdx.x;
    const int c = blockIdx.y;
    const lgcn_emu_row_t er = rows[blockIdx.x];
    // the chain value, as its bits (wave-uniform)
    uint32_t ab = __float_as_uint(meta[(int64_t)er.first_block * d + c].r0);
    auto stage_of = [&](int64_t bi) -> const float* {
        return stage ? stage + (bi * (d + 1) + c) * LGCN_EMU_BLOCK : nullptr;
    };
    auto load_chunk = [&](int32_t b0, EmuChunk& ck) {
        const int nb = min(CH, er.n_blocks - b0);
        const int64_t bl = er.first_block + b0 + min(lane, max(nb - 1, 0));
        const int4 mv = *reinterpret_cast<const int4*>(meta + bl * d + c);
        ck.lo = mv.x;
        ck.hi = mv.y;
        ck.pk = lane < nb ? mv.z : (int)0x80000000;  // past the row: identity
        ck.t = __int_as_float(mv.w);
        const int64_t base = (int64_t)(er.first_block + b0) * d + c;
#pragma unroll
        for (int j = 0; j < CH / 2; ++j) {
            const int bb = min(2 * j + (lane >> 5), max(nb - 1, 0));
            ck.k[j] = rel[(base + (int64_t)bb * d) * NC + (lane & 31)];
        }
    };
    // chunk -> LDS: translations and, per (block, candidate k = 2 w + sign), the valid range of
    // the start mantissa M (empty when the candidate's own chain may have left its binade)
    auto stage_chunk = [&](const EmuChunk& ck) {
        constexpr int LB = (1 << 23) + kSlack, HB = (1 << 24) - kSlack, C = 3 << 22;
        const int k = lane & 31;
        const int w = k >> 1;
        const bool neg = k & 1;
#pragma unroll
        for (int j = 0; j < CH / 2; ++j) {
            const int b = 2 * j + (lane >> 5);
            const int32_t lo0 = __shfl(ck.lo, b);
            const int32_t hi0 = __shfl(ck.hi, b);
            const int lo = lo0 >> w, hi = -((-hi0) >> w);
            const int mlo = neg ? -hi : lo, mhi = neg ? -lo : hi;  // magnitude offsets
            const bool valid = C + mlo >= LB && C + mhi <= HB;
            s_k[b * NC + k] = ck.k[j];
            s_min[b * NC + k] = valid ? LB - mlo : 1 << 24;
            s_max[b * NC + k] = valid ? HB - mhi : 0;
        }
    };
    // block k of the row holds edges [row_beg + k * BLOCK, min(.. + BLOCK, row_end)) (plan_emulation)
    const int32_t row_beg = blocks[er.first_block].beg;
    const int32_t row_end = blocks[er.first_block + er.n_blocks - 1].end;
    auto fetch_slot = [&](int32_t kb, int s) {
        const int64_t bi = er.first_block + kb;
        fetch_block_lds(stage + (bi * (d + 1) + d) * LGCN_EMU_BLOCK, stage_of(bi), s_v(s),
                        s_xs(s));
    };
#ifdef LGCN_EMU_STATS
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    unsigned long long n_fast = 0, n_slow = 0, t_slow = 0;
    unsigned long long ph[16] = {0};
    unsigned long long ph_last = t_start;
#endif
    EmuChunk nxt;
    if (er.n_blocks > 1) load_chunk(1, nxt);
    for (int32_t b0 = 1; b0 < er.n_blocks; b0 += CH) {
        const int nb = min(CH, er.n_blocks - b0);
        wave_lds_sync();  // the previous chunk's LDS rows and slots are no longer read
        stage_chunk(nxt);
        const int my_eb = (int)(int16_t)(nxt.pk & 0xffff);   // lane i: block i's ebase,
        const int my_ml = (int)(int16_t)(nxt.pk >> 16);      // maxlsb,
        const float my_t = nxt.t;                            // and chain from +0
        const bool my_id = my_ml == kIdentity;  // every product zero: translation by 0
        wave_lds_sync();
        PH_MARK(0);
        PH_COUNT(8, 1);
        // The speculative test from block `from` with chain value bits `a`: lane i's start
        // mantissa if every block in [from, i) translates (exclusive prefix of the mantissa
        // changes), and the mask of blocks that cannot translate from there. `incl` returns the
        // inclusive prefix, `dm` the lane's own change.
        auto test = [&](uint32_t a, int from, int& incl, int& dm) -> unsigned long long {
            const int E = (int)((a >> 23) & 255u);
            const int neg = (int)(a >> 31);
            const int M = (int)((a & 0x7fffffu) | 0x800000u);
            const int w = E - 127 - my_eb;
            const int idx = lane * NC + 2 * min(max(w, 0), kW - 1) + neg;
            const int32_t K = s_k[idx], mn = s_min[idx], mx = s_max[idx];
            const bool act = lane < nb && lane >= from;
            dm = act && !my_id ? (neg ? -K : K) : 0;  // |K| < 2^24: the sums fit in int32
            incl = wave_incl_scan(dm);
            const int start = M + incl - dm;
            bool ok = my_id || (((unsigned)(E - 1) < 254u) & ((unsigned)w < (unsigned)kW) &
                                (my_ml < E - 127 - 24) & (start >= mn) & (start <= mx));
            LGCN_EMU_FORCE(ok);
            return __ballot(act && !ok);
        };
        // predicted re-run blocks of this chunk (stage mode: their data goes to LDS slots)
        unsigned long long pred = 0;
        if (stage) {
            uint32_t pa = ab;
            int from = 0;
            for (int it = 0; it < NS && from < nb; ++it) {
                int incl, dm;
                const unsigned long long bad = test(pa, from, incl, dm);
                if (!bad) break;
                const int f = (int)__builtin_ctzll(bad);
                pred |= 1ull << f;
                pa += (uint32_t)__builtin_amdgcn_readlane(incl - dm, f);
                pa = __float_as_uint(__uint_as_float(pa) + __int_as_float(
                         __builtin_amdgcn_readlane(__float_as_int(my_t), f)));
                from = f + 1;
            }
        }
        PH_MARK(1);
        PH_COUNT(9, __builtin_popcountll(pred));
        if (b0 + CH < er.n_blocks) load_chunk(b0 + CH, nxt);  // in flight during this chunk
        if (pred) {
            int s = 0;
            for (unsigned long long m = pred; m; m &= m - 1, ++s)
                fetch_slot(b0 + (int)__builtin_ctzll(m), s);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slots (and the next chunk) landed
        }
        PH_MARK(2);
        // lane i: the slot holding block i's data, or -1
        const int my_slot = ((pred >> lane) & 1ull)
            ? (int)__builtin_popcountll(pred & ((1ull << lane) - 1ull)) : -1;
        int from = 0;
        while (true) {
            int incl, dm;
            const unsigned long long bad = test(ab, from, incl, dm);
            const int f = bad ? (int)__builtin_ctzll(bad) : nb;
            // blocks [from, f) translate: their mantissa changes add to the bits (same binade)
            ab += (uint32_t)(f < nb ? __builtin_amdgcn_readlane(incl - dm, f)
                                    : __builtin_amdgcn_readlane(incl, 63));
            PH_MARK(3);
            EMU_STAT(0, f - from);
#ifdef LGCN_EMU_STATS
            n_fast += f - from;
#endif
            if (f >= nb) break;
            // re-run block f as the reference does
            const int32_t kb = b0 + f;
            const int32_t f_beg = row_beg + kb * LGCN_EMU_BLOCK;
            const int32_t n = min(f_beg + LGCN_EMU_BLOCK, row_end) - f_beg;
            EMU_STAT(1, 1);
            EMU_STAT(7, n);
#ifdef LGCN_EMU_STATS
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            EMU_STAT(2, __builtin_amdgcn_readlane(my_slot, f) < 0);  // not predicted
#endif
            float a;
            if (stage) {
                int sl = __builtin_amdgcn_readlane(my_slot, f);
                if (sl < 0) {  // not predicted: fetch now into the spare slot
                    sl = NS;
                    wave_lds_sync();
                    fetch_slot(kb, sl);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    PH_MARK(5);
                    PH_COUNT(11, 1);
                }
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
                a = g_emu_mode == 1 ? __uint_as_float(ab)
                                    : slot_chain(n, __uint_as_float(ab), s_v(sl), s_xs(sl));
#else
                a = slot_chain(n, __uint_as_float(ab), s_v(sl), s_xs(sl));
#endif
            } else {
                SlowData sd;
                slow_load<XD>(sd, edges, f_beg, f_beg + n, x, xdiv, x_nz, nullptr, c);
                slow_stage(sd, n, false, sq);
                a = slow_chain(n, __uint_as_float(ab), sq);
            }
            ab = (uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(a));
            PH_MARK(4);
            PH_COUNT(10, 1);
#ifdef LGCN_EMU_STATS
            ++n_slow;
            t_slow += __builtin_amdgcn_s_memtime() - t0;
#endif
            from = f + 1;
            if (from >= nb) break;
        }
    }
#ifdef LGCN_EMU_STATS
    if (lane == 0 && blockIdx.x == 0 && blockIdx.y == 0)
        for (int k = 0; k < 16; ++k) g_emu_phase[k] += ph[k];
    if (lane == 0 && blockIdx.x < 256) {
        atomicAdd(&g_emu_row_stats[blockIdx.x][0], n_fast);
        atomicAdd(&g_emu_row_stats[blockIdx.x][1], n_slow);
        atomicAdd(&g_emu_row_stats[blockIdx.x][2], t_slow);
        atomicMax(&g_emu_row_stats[blockIdx.x][3], __builtin_amdgcn_s_memtime() - t_start);
    }
#endif
    if (lane != 0) return;
    const int32_t row = er.row;
    float out = __uint_as_float(ab);
    if constexpr (MODE == LGCN_EPI_MEAN) {
        // ((E0 + E1) + ... + E_{K-1}) + E_K, then / (K+1)  (lightgcn.py:54)
        float s = seg_row_x(ep.prev0, row)[c];
        for (int i = 0; i + 1 < ep.n_prev; ++i) s = s + ep.prev_dense[i][(int64_t)row * ep.ld_prev + c];
        s = s + out;
        out = ep.pad ? s * __int_as_float(ep.pad) : s / ep.div;
    } else if constexpr (MODE == LGCN_EPI_ADD) {
        if (!ep.addend_nz || row_live_x(ep.addend_nz, row)) {
            const float z = seg_row_x(ep.addend, row)[c];
            out = (ep.pad ? z * __int_as_float(ep.pad) : z / ep.div) + out;
        }
    }
    y[(int64_t)row * ldy + c] = out;
}

inline int herr_x(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

bool is_pow2(float x) {
    int e;
    return x > 0.f && frexpf(x, &e) == 0.5f;
}

template <int XD>
int launch_blocks(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks, int32_t n_blocks,
                  const lgcn_rows_t& x, float xdiv, const uint32_t* x_nz, int32_t d, int32_t* rel,
                  EmuMeta* meta, float* stage, hipStream_t s) {
    const dim3 grid((uint32_t)n_blocks, (uint32_t)((d + 63) / 64));
    hipLaunchKernelGGL((k_emu_blocks<XD>), grid, dim3(64), 0, s, edges, blocks, x, xdiv, x_nz, d,
                       rel, meta, stage);
    return herr_x(hipGetLastError());
}

template <int MODE, int XD>
int launch_walk(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks,
                const lgcn_emu_row_t* rows, int32_t n_rows, const int32_t* rel, const EmuMeta* meta,
                const float* stage, const lgcn_rows_t& x, float xdiv, const uint32_t* x_nz, float* y,
                int64_t ldy, int32_t d, const lgcn_epilogue_t& ep, int slots, hipStream_t s) {
    const dim3 grid((uint32_t)n_rows, (uint32_t)d);
    const size_t lds = (size_t)2 * (slots + 1) * LGCN_EMU_BLOCK * sizeof(float);
    hipLaunchKernelGGL((k_emu_walk<MODE, XD>), grid, dim3(64), lds, s, edges, blocks, rows, rel,
                       meta, stage, x, xdiv, x_nz, d, y, ldy, ep, slots);
    return herr_x(hipGetLastError());
}

int xd_of(float xdiv, const uint32_t* x_nz) {
    return (xdiv == 1.f ? 0 : is_pow2(xdiv) ? 2 : 1) | (x_nz ? 4 : 0);
}

template <int MODE>
int walk_mode(int xd, const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks,
              const lgcn_emu_row_t* rows, int32_t n_rows, const int32_t* rel, const EmuMeta* meta,
              const float* stage, const lgcn_rows_t& x, float xdiv, const uint32_t* x_nz, float* y,
              int64_t ldy, int32_t d, const lgcn_epilogue_t& ep, int slots, hipStream_t s) {
#define LGCN_W(XD_) \
    case XD_: return launch_walk<MODE, XD_>(edges, blocks, rows, n_rows, rel, meta, stage, x, xdiv, x_nz, y, ldy, d, ep, slots, s);
    switch (xd) {
        LGCN_W(0) LGCN_W(1) LGCN_W(2) LGCN_W(4) LGCN_W(5) LGCN_W(6)
        default: return LGCN_EINVAL;
    }
#undef LGCN_W
}


// ---------------------------------------------------------------------------------------------
// mid-size hub rows: the reference's sequential chain itself, latency-hidden
// ---------------------------------------------------------------------------------------------
// For a row of a few thousand to ~10^5 edges the chain itself is cheap (deg dependent FMAs); what
// makes it slow in the layer kernel is the gathers. One wave per (row, W-column slice): the
// wave keeps two 64-edge windows of gathered X rows in flight by LDS-DMA (global_load_lds
// dwordx4: no registers held, up to 2 * W/4 + 1 loads outstanding) while it folds the window
// before them, lane c = column c, acc = fma(val_j, x_j, acc) in stored order from +0 — the
// reference's arithmetic, no emulation, no block pass. Edge records come in by LDS-DMA one
// window further ahead, so the gather addresses are read from LDS, never waited on alone.
// Ring: X windows w (folding), w+1 (in flight), w+2 (being issued); records w .. w+3.
template <int W>
struct ChainCfg {
    static constexpr int LPR = W / 4;       // lanes per gathered row slice (16 B each)
    static constexpr int RPI = 64 / LPR;    // rows per 1-KB LDS-DMA instruction
    static constexpr int NI = 64 / RPI;     // instructions per 64-edge window
    static constexpr int XWIN = 64 * W;     // floats per X window
    // X windows in flight while one is folded: as many as vmcnt (<= 63 outstanding) allows
    // with NI + 2 loads per window (W=64: 3 x 18, W=32: 6 x 10, W=16: 8 x 6)
    static constexpr int AHEAD = W == 64 ? 3 : W == 32 ? 6 : 8;
    static constexpr int NX = AHEAD + 1;    // X windows in the ring
    static constexpr int NR = 2 * AHEAD + 1;  // record windows in the ring
};

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)reinterpret_cast<uintptr_t>(p);
}

// 16 LDS reads at a + OFF + t * STRIDE, completed before the values are used. Inline asm on
// purpose: LDS written by LDS-DMA makes the compiler wait for EVERY outstanding global load
// before any compiler-visible LDS read (it cannot tell the ring slots apart), which would drain
// the gathers in flight; here the waits are explicit (vmcnt before, lgkmcnt inside).
template <int OFF, int STRIDE>
__device__ __forceinline__ void lds_read16(uint32_t a, float (&v)[16]) {
    asm volatile(
        "ds_read_b32 %0, %16 offset:%17\n\tds_read_b32 %1, %16 offset:%18\n\t"
        "ds_read_b32 %2, %16 offset:%19\n\tds_read_b32 %3, %16 offset:%20\n\t"
        "ds_read_b32 %4, %16 offset:%21\n\tds_read_b32 %5, %16 offset:%22\n\t"
        "ds_read_b32 %6, %16 offset:%23\n\tds_read_b32 %7, %16 offset:%24\n\t"
        "ds_read_b32 %8, %16 offset:%25\n\tds_read_b32 %9, %16 offset:%26\n\t"
        "ds_read_b32 %10, %16 offset:%27\n\tds_read_b32 %11, %16 offset:%28\n\t"
        "ds_read_b32 %12, %16 offset:%29\n\tds_read_b32 %13, %16 offset:%30\n\t"
        "ds_read_b32 %14, %16 offset:%31\n\tds_read_b32 %15, %16 offset:%32\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]),
          "=&v"(v[6]), "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]),
          "=&v"(v[12]), "=&v"(v[13]), "=&v"(v[14]), "=&v"(v[15])
        : "v"(a), "n"(OFF), "n"(OFF + STRIDE), "n"(OFF + 2 * STRIDE), "n"(OFF + 3 * STRIDE),
          "n"(OFF + 4 * STRIDE), "n"(OFF + 5 * STRIDE), "n"(OFF + 6 * STRIDE),
          "n"(OFF + 7 * STRIDE), "n"(OFF + 8 * STRIDE), "n"(OFF + 9 * STRIDE),
          "n"(OFF + 10 * STRIDE), "n"(OFF + 11 * STRIDE), "n"(OFF + 12 * STRIDE),
          "n"(OFF + 13 * STRIDE), "n"(OFF + 14 * STRIDE), "n"(OFF + 15 * STRIDE)
        : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MODE, int XD, int W>
__global__ __launch_bounds__(64) void k_chain_rows(const lgcn_edge_t* __restrict__ edges,
                                                   const lgcn_emu_block_t* __restrict__ blocks,
                                                   const lgcn_emu_row_t* __restrict__ rows,
                                                   lgcn_rows_t x, float xdiv, int32_t d,
                                                   float* __restrict__ y, int64_t ldy,
                                                   lgcn_epilogue_t ep) {
    using C = ChainCfg<W>;
    constexpr int NX = C::NX, NR = C::NR, AHEAD = C::AHEAD;
    static_assert(AHEAD * (C::NI + 2) <= 63, "vmcnt holds at most 63 outstanding loads");
    __shared__ __attribute__((aligned(16))) float s_x[NX][C::XWIN];
    __shared__ __attribute__((aligned(16))) int2 s_rec[NR][64];
    const int lane = threadIdx.x;
    const int c0 = blockIdx.y * W;
    const lgcn_emu_row_t er = rows[blockIdx.x];
    const int32_t beg = blocks[er.first_block].beg;
    const int32_t end = blocks[er.first_block + er.n_blocks - 1].end;
    const int32_t nwin = (end - beg + 63) >> 6;
    // records of window w -> s_rec[w % NR]: 128 dwords in two dword LDS-DMA loads. Dwords past
    // the row repeat its last record (col and val kept apart by parity), so windows past the
    // end load valid records and gather valid rows: every iteration issues the same number of
    // loads, which keeps the vmcnt arithmetic below exact. They are never folded.
    const int32_t* ew = reinterpret_cast<const int32_t*>(edges);
    const int64_t dl = 2 * (int64_t)end - 1, dlast = 2 * (int64_t)end - 2 + (lane & 1);
    auto rec_dma = [&](int32_t w) {
        const int64_t d0 = 2 * ((int64_t)beg + 64 * w) + lane;
        int32_t* dst = reinterpret_cast<int32_t*>(&s_rec[w % NR][0]);
        __builtin_amdgcn_global_load_lds(ew + (d0 <= dl ? d0 : dlast), dst, 4, 0, 0);
        __builtin_amdgcn_global_load_lds(ew + (d0 + 64 <= dl ? d0 + 64 : dlast), dst + 64, 4, 0, 0);
    };
    // gathered X of window w -> s_x[w % NX]: instruction k moves rows k*RPI .. k*RPI + RPI - 1
    // (lane -> row sub = lane / LPR, 16-B piece q = lane % LPR); the columns come from LDS
    const int sub = lane / C::LPR, q = lane % C::LPR;
    auto x_dma = [&](int32_t w) {
        float cols[16];
        lds_read16<0, C::RPI * 8>(lds_addr(&s_rec[w % NR][sub]), cols);
        float* dst = s_x[w % NX];
#pragma unroll
        for (int k = 0; k < C::NI; ++k) {
            const float* src = seg_row_sel(x, __float_as_int(cols[k])) + c0 + 4 * q;
            __builtin_amdgcn_global_load_lds(src, dst + k * 256, 16, 0, 0);
        }
    };
    // Pipeline (A = AHEAD): iteration v issues x(v + A) then rec(v + 2A); the prologue runs
    // v = -A .. -1 after rec(0 .. A-1) have landed. At iteration w, x(w) and rec(w + A) (both
    // issued by iteration w - A) must have landed: A - 1 later iterations of NI + 2 loads each
    // may still be in flight. Ring slots: x(w + A) reuses window w - 1's slot (NX = A + 1),
    // rec(w + 2A) record window w - 1's (NR = 2A + 1).
    static_assert(NX == AHEAD + 1 && NR == 2 * AHEAD + 1, "ring sizes");
    for (int w = 0; w < AHEAD; ++w) rec_dma(w);
    wait_vm<0>();
    for (int v = -AHEAD; v < 0; ++v) {
        x_dma(v + AHEAD);
        rec_dma(v + 2 * AHEAD);
    }
    float acc = 0.f;
    const int cc = lane < W ? lane : 0;
    for (int32_t w = 0; w < nwin; ++w) {
        wait_vm<(AHEAD - 1) * (C::NI + 2)>();
        x_dma(w + AHEAD);
        rec_dma(w + 2 * AHEAD);
        const int n = min(64, end - beg - 64 * w);
        const uint32_t xa = lds_addr(&s_x[w % NX][cc]);
        const uint32_t va = lds_addr(&s_rec[w % NR][0].y);  // same address in every lane
        // 16 steps at a time: X elements and (broadcast) edge values from LDS, then the chain;
        // only the row's last window is partial (steps past n leave acc alone)
#define LGCN_CHAIN_FOLD(G, FULL)                                                              \
        {                                                                                     \
            float xv[16], vv[16];                                                             \
            lds_read16<(G) * W * 4, W * 4>(xa, xv);                                           \
            lds_read16<(G) * 8, 8>(va, vv);                                                   \
            _Pragma("unroll") for (int t = 0; t < 16; ++t) {                                  \
                float xe = xv[t];                                                             \
                if constexpr ((XD & 3) == 1) xe = xe / xdiv;                                  \
                else if constexpr ((XD & 3) == 2) xe = xe * xdiv;                             \
                if (FULL) acc = __builtin_fmaf(vv[t], xe, acc);                               \
                else acc = (G) + t < n ? __builtin_fmaf(vv[t], xe, acc) : acc;                \
            }                                                                                 \
        }
        if (n == 64) {
            LGCN_CHAIN_FOLD(0, true)
            LGCN_CHAIN_FOLD(16, true)
            LGCN_CHAIN_FOLD(32, true)
            LGCN_CHAIN_FOLD(48, true)
        } else {
            LGCN_CHAIN_FOLD(0, false)
            LGCN_CHAIN_FOLD(16, false)
            LGCN_CHAIN_FOLD(32, false)
            LGCN_CHAIN_FOLD(48, false)
        }
#undef LGCN_CHAIN_FOLD
    }
    wait_vm<0>();  // no LDS-DMA may land after the wave (and its LDS) is gone
    if (lane >= W || c0 + lane >= d) return;
    const int c = c0 + lane;
    const int32_t row = er.row;
    float out = acc;
    if constexpr (MODE == LGCN_EPI_MEAN) {
        float s = seg_row_x(ep.prev0, row)[c];
        for (int i = 0; i + 1 < ep.n_prev; ++i) s = s + ep.prev_dense[i][(int64_t)row * ep.ld_prev + c];
        s = s + out;
        out = ep.pad ? s * __int_as_float(ep.pad) : s / ep.div;
    } else if constexpr (MODE == LGCN_EPI_ADD) {
        if (!ep.addend_nz || row_live_x(ep.addend_nz, row)) {
            const float z = seg_row_x(ep.addend, row)[c];
            out = (ep.pad ? z * __int_as_float(ep.pad) : z / ep.div) + out;
        }
    }
    y[(int64_t)row * ldy + c] = out;
}

template <int MODE, int XD>
int launch_chain(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks,
                 const lgcn_emu_row_t* rows, int32_t n_rows, const lgcn_rows_t& x, float xdiv,
                 float* y, int64_t ldy, int32_t d, const lgcn_epilogue_t& ep, hipStream_t s) {
    // 128-B slices (one line per gathered row piece) for every d that is a multiple of 32: two
    // or more waves per row, each with twice the windows in flight of a 64-column wave
    const int w = d % 32 == 0 ? 32 : 16;  // 16, 32 or a multiple of 64 (checked by the caller)
    const dim3 grid((uint32_t)n_rows, (uint32_t)((d + w - 1) / w));
    if (w == 32)
        hipLaunchKernelGGL((k_chain_rows<MODE, XD, 32>), grid, dim3(64), 0, s, edges, blocks, rows,
                           x, xdiv, d, y, ldy, ep);
    else
        hipLaunchKernelGGL((k_chain_rows<MODE, XD, 16>), grid, dim3(64), 0, s, edges, blocks, rows,
                           x, xdiv, d, y, ldy, ep);
    return herr_x(hipGetLastError());
}

template <int MODE>
int chain_mode(int xd, const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks,
               const lgcn_emu_row_t* rows, int32_t n_rows, const lgcn_rows_t& x, float xdiv,
               float* y, int64_t ldy, int32_t d, const lgcn_epilogue_t& ep, hipStream_t s) {
    // the row mask of X (XD & 4) only saves gathers; the chain reads the (all-zero) dead rows
    switch (xd & 3) {
        case 0: return launch_chain<MODE, 0>(edges, blocks, rows, n_rows, x, xdiv, y, ldy, d, ep, s);
        case 1: return launch_chain<MODE, 1>(edges, blocks, rows, n_rows, x, xdiv, y, ldy, d, ep, s);
        case 2: return launch_chain<MODE, 2>(edges, blocks, rows, n_rows, x, xdiv, y, ldy, d, ep, s);
        default: return LGCN_EINVAL;
    }
}
}  // namespace

extern "C" {

#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
int lgcn_emu_set_mode(int mode) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_emu_mode), &mode, sizeof(int)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef LGCN_EMU_STATS
// diagnostics builds only (not in lgcn.h): read and reset the walker counters
int lgcn_emu_stats(unsigned long long* out_host) {
    if (hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_emu_stats), sizeof(g_emu_stats)) != hipSuccess)
        return -1;
    unsigned long long z[8] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_emu_stats), z, sizeof(z)) == hipSuccess ? 0 : -1;
}


int lgcn_emu_phase(unsigned long long* out_host) {  // [16], then reset
    if (hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_emu_phase), sizeof(g_emu_phase)) != hipSuccess)
        return -1;
    unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_emu_phase), z, sizeof(z)) == hipSuccess ? 0 : -1;
}

int lgcn_emu_row_stats(unsigned long long* out_host) {  // [256][4], then reset
    if (hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_emu_row_stats), sizeof(g_emu_row_stats)) !=
        hipSuccess)
        return -1;
    static unsigned long long z[256][4];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_emu_row_stats), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

int lgcn_emu_blocks(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks, int32_t n_blocks,
                    lgcn_rows_t x, float x_div, const uint32_t* x_nz, int32_t d, float* rel,
                    void* meta, float* stage, void* stream) {
    if (n_blocks < 0 || d < 1 || d > 2048 || !(x_div > 0.f)) return LGCN_EINVAL;
    if (n_blocks == 0) return 0;
    if (!edges || !blocks || !rel || !meta || !x.p0) return LGCN_EINVAL;
    const int xd = xd_of(x_div, x_nz);
    const float xa = (xd & 3) == 2 ? 1.0f / x_div : x_div;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    EmuMeta* mp = static_cast<EmuMeta*>(meta);
    int32_t* rp = reinterpret_cast<int32_t*>(rel);
#define LGCN_B(XD_) \
    case XD_: return launch_blocks<XD_>(edges, blocks, n_blocks, x, xa, x_nz, d, rp, mp, stage, s);
    switch (xd) {
        LGCN_B(0) LGCN_B(1) LGCN_B(2) LGCN_B(4) LGCN_B(5) LGCN_B(6)
        default: return LGCN_EINVAL;
    }
#undef LGCN_B
}

int lgcn_emu_walk(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks,
                  const lgcn_emu_row_t* rows, int32_t n_rows, const float* rel, const void* meta,
                  const float* stage, lgcn_rows_t x, float x_div, const uint32_t* x_nz, float* y,
                  int64_t ldy, int32_t d, const lgcn_epilogue_t* epi_host, int32_t slots,
                  void* stream) {
    if (slots == 0) slots = LGCN_EMU_SLOTS;
    if (n_rows < 0 || d < 1 || d > 2048 || !(x_div > 0.f) || !epi_host || slots < 1 ||
        slots > 63)
        return LGCN_EINVAL;
    if (n_rows == 0) return 0;
    if (!edges || !blocks || !rows || !rel || !meta || !y || ldy < d || !x.p0) return LGCN_EINVAL;
    lgcn_epilogue_t ep = *epi_host;
    if (ep.mode == LGCN_EPI_MEAN && (ep.n_prev < 1 || ep.n_prev - 1 > LGCN_MAX_LAYERS))
        return LGCN_EINVAL;
    if (ep.mode == LGCN_EPI_ADD && !ep.addend.p0) return LGCN_EINVAL;
    if (ep.mode != LGCN_EPI_STORE && !(ep.div > 0.f)) return LGCN_EINVAL;
    // a power-of-two divisor becomes a multiply by its exact reciprocal (same rounding)
    if (ep.mode != LGCN_EPI_STORE && is_pow2(ep.div)) {
        const float inv = 1.0f / ep.div;
        memcpy(&ep.pad, &inv, sizeof(inv));
    } else {
        ep.pad = 0;
    }
    const int xd = xd_of(x_div, x_nz);
    const float xa = (xd & 3) == 2 ? 1.0f / x_div : x_div;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const EmuMeta* mp = static_cast<const EmuMeta*>(meta);
    const int32_t* rl = reinterpret_cast<const int32_t*>(rel);
    switch (ep.mode) {
        case LGCN_EPI_STORE:
            return walk_mode<LGCN_EPI_STORE>(xd, edges, blocks, rows, n_rows, rl, mp, stage, x, xa, x_nz, y, ldy, d, ep, slots, s);
        case LGCN_EPI_MEAN:
            return walk_mode<LGCN_EPI_MEAN>(xd, edges, blocks, rows, n_rows, rl, mp, stage, x, xa, x_nz, y, ldy, d, ep, slots, s);
        case LGCN_EPI_ADD:
            return walk_mode<LGCN_EPI_ADD>(xd, edges, blocks, rows, n_rows, rl, mp, stage, x, xa, x_nz, y, ldy, d, ep, slots, s);
        default:
            return LGCN_EINVAL;
    }
}


int lgcn_chain_supported(int32_t d) { return d == 16 || d == 32 || (d > 0 && d % 64 == 0); }

int lgcn_chain_rows(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks,
                    const lgcn_emu_row_t* rows, int32_t n_rows, lgcn_rows_t x, float x_div,
                    float* y, int64_t ldy, int32_t d, const lgcn_epilogue_t* epi_host,
                    void* stream) {
    if (n_rows < 0 || !lgcn_chain_supported(d) || d > 2048 || !(x_div > 0.f) || !epi_host)
        return LGCN_EINVAL;
    if (n_rows == 0) return 0;
    if (!edges || !blocks || !rows || !y || ldy < d || !x.p0) return LGCN_EINVAL;
    // 16-B row slices: every X segment and the row stride 16-B aligned
    if (x.ld % 4 || (reinterpret_cast<uintptr_t>(x.p0) & 15) ||
        (reinterpret_cast<uintptr_t>(x.p1) & 15) || (reinterpret_cast<uintptr_t>(x.p2) & 15))
        return LGCN_EALIGN;
    lgcn_epilogue_t ep = *epi_host;
    if (ep.mode == LGCN_EPI_MEAN && (ep.n_prev < 1 || ep.n_prev - 1 > LGCN_MAX_LAYERS))
        return LGCN_EINVAL;
    if (ep.mode == LGCN_EPI_ADD && !ep.addend.p0) return LGCN_EINVAL;
    if (ep.mode != LGCN_EPI_STORE && !(ep.div > 0.f)) return LGCN_EINVAL;
    if (ep.mode != LGCN_EPI_STORE && is_pow2(ep.div)) {
        const float inv = 1.0f / ep.div;
        memcpy(&ep.pad, &inv, sizeof(inv));
    } else {
        ep.pad = 0;
    }
    const int xd = xd_of(x_div, nullptr);
    const float xa = (xd & 3) == 2 ? 1.0f / x_div : x_div;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (ep.mode) {
        case LGCN_EPI_STORE: return chain_mode<LGCN_EPI_STORE>(xd, edges, blocks, rows, n_rows, x, xa, y, ldy, d, ep, s);
        case LGCN_EPI_MEAN: return chain_mode<LGCN_EPI_MEAN>(xd, edges, blocks, rows, n_rows, x, xa, y, ldy, d, ep, s);
        case LGCN_EPI_ADD: return chain_mode<LGCN_EPI_ADD>(xd, edges, blocks, rows, n_rows, x, xa, y, ldy, d, ep, s);
        default: return LGCN_EINVAL;
    }
}

}  // extern "C"
