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
// If a chain value a is a multiple of u and the exact a + p lies inside binade e, fma-rounding
// gives RN(a + p) = a + RN_u(p) (RN_u: nearest multiple of u; only an exact tie would depend on
// a's parity). RN_u(p) does not depend on a — nor on a's SIGN. So along a stretch of steps whose
// results all stay inside binade e, the chain is an integer prefix sum: in units of u its
// magnitude mantissa M moves by +-q_j, q_j = RN_u(p_j) / u. Hence:
//   * k_emu_blocks cuts a hub row into blocks of <= 256 edges. For each (block, column) it runs
//     16 CANDIDATE chains from +1.5 * 2^e, e in a 16-binade window chosen from the block's own
//     first products; candidate e's end minus its start is K_e = sum_j q_j (exact, when the
//     candidate stayed in its binade). It records K_e, bounds on the block's exact running sum
//     (from its own chain from +0, widened by that chain's rounding: every trajectory of the
//     block stays within 128 ulps of it) and a per-binade validity mask (candidate inside its
//     binade, bounds representable, and no product able to be an exact tie at ulp u_e: the
//     lowest set bit of every product lies below u_e / 2). Block 0 of a row keeps its chain from
//     +0: the true value. It also stages the block's X elements per column (and the edge
//     values), so a block the walk must resolve is one contiguous 2-KB fetch.
//   * k_emu_walk (one wave per (row, column)) walks the blocks in order with the true value a,
//     64 blocks per scan (lane = block): a DPP prefix sum of the translations gives every lane
//     its start mantissa if all earlier blocks translate, and each lane tests that its whole
//     trajectory stays inside the binade. The first block that fails is RESOLVED IN PARALLEL:
//     lane l holds steps 4l..4l+3, computes q_j = (fma(v_j, x_j, C) - C) / u with C = 1.5 * 2^e
//     (exact, C's binade is e), a wave prefix sum gives the magnitude after every step, and the
//     first step whose result could leave the binade (or whose product could be a tie) is done
//     as the reference's own fma; the scan restarts after it in the new binade. A block costs
//     one scan per binade change instead of 256 dependent FMAs.
// Every step is therefore either the reference's own fma or a proven-identical integer step:
// the result is bitwise the reference's, whatever the data (zero, subnormal, inf and NaN values
// take the sequential fma). oracle/lgcn_oracle.c holds the sequential chain the tests compare
// against; DESIGN.md §3 has the argument and the measured decision mix.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>

#include "lgcn.h"

namespace lgcn_detail {
extern int g_emu_margin;   // LGCN_TUNE_EMU_MARGIN (lgcn_engine.hip)
// (declared for lgcn_engine.hip in lgcn_kernels.h; defined at the end of this file)
int live_prepare(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks, int32_t n_blocks,
                 const lgcn_emu_row_t* rows, int32_t n_rows, const uint32_t* x_nz, int32_t d,
                 float x_div, const lgcn_epilogue_t* epi_host, float* y, int64_t ldy,
                 const void* x_p0, int32_t live_min, int32_t max_live, void* scratch,
                 hipStream_t s);
int live_chains(int32_t n_blocks, int32_t n_rows, lgcn_rows_t x, float x_div, float* y,
                int64_t ldy, int32_t d, const lgcn_epilogue_t* epi_host, void* scratch,
                hipStream_t s);
}

namespace {

constexpr int kNB = LGCN_EMU_CANDS;           // binades per (block, column) table
constexpr int kEOff = 2;                      // window starts 2 binades above the first 64 steps' reach
constexpr int kSlack = 132;                   // ulps: 128 for <= 256 steps of <= 1/2 ulp + margin
constexpr int kLB = (1 << 23) + kSlack;       // a trajectory's mantissa must stay in [kLB, kHB]
constexpr int kHB = (1 << 24) - kSlack;
constexpr int kC = 3 << 22;                   // a candidate's start mantissa (1.5 * 2^23)
constexpr int kIdentEb = -32768;              // meta ebase of a block without a nonzero product
static_assert(kNB == 16, "tables hold 16 binades (4 x int4 per (block, column))");

// The walk's and the chain kernel's grids: (column or slice, row) — LGCN_ROWMAJOR=0 builds round
// 5's (row, column) order for A/B
#ifndef LGCN_ROWMAJOR
#define LGCN_ROWMAJOR 1
#endif
#if LGCN_ROWMAJOR  // one dimension (a y extent is limited to 65535 rows): row * cols + column
#define LGCN_GRID_COL(nc) (blockIdx.x % (uint32_t)(nc))
#define LGCN_GRID_ROW(nc) (blockIdx.x / (uint32_t)(nc))
#define LGCN_GRID_DIM(cols, rows) dim3((cols) * (rows))
#else
#define LGCN_GRID_COL(nc) blockIdx.y
#define LGCN_GRID_ROW(nc) blockIdx.x
#define LGCN_GRID_DIM(cols, rows) dim3((rows), (cols))
#endif
static_assert(LGCN_EMU_META_BYTES == 16, "meta record is one int4");

// Records written by k_emu_blocks per (block, column) rc = block * d + column:
//   meta[rc] = int4 {lo0, hi0, pk, r0}: lo0 / hi0 = floor / ceil of bounds on the block's exact
//     running sum in units of u_ebase; pk = ebase (low 16 bits, signed; kIdentEb: every product
//     is zero) | valid mask << 16 (bit w: binade ebase + w may translate); r0 = bits of the
//     block's chain from +0 (the true chain for block 0 of a row);
//   ktab[4 rc .. 4 rc + 3] = int4 x 4: K[w], the translation of binade ebase + w in its ulps.

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

// exponent of the lowest set bit of a finite nonzero float (subnormals included), branch-free:
// the lowest set bit of the mantissa with the implicit bit 23 set (the exponent bits above it do
// not matter; a subnormal's bits lie below it). A zero gives -126, below any nonzero float's.
__device__ __forceinline__ int lsb_exp(float f) {
    const uint32_t b = __float_as_uint(f);
    const int E = (int)((b >> 23) & 255u);
    return __builtin_ctz(b | 0x800000u) + max(E, 1) - 150;
}

// lsb_exp, and -100000 for +-0: the sum of two of them is < -50000 iff the product is zero
__device__ __forceinline__ int lsb_exp_z(float f) {
    return (__float_as_uint(f) << 1) ? lsb_exp(f) : -100000;
}


// ---------------------------------------------------------------------------------------------
// block pass: one wave per (block, 64-column slice); lane = column
// ---------------------------------------------------------------------------------------------
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
// timing experiments only (tools/exact_layer_probe.py --blk-modes): bit 1 = no stage writes,
// 2 = no candidate chains, 4 = no lowest-set-bit tracking (the tables are then wrong)
__device__ int g_blk_mode;
#define LGCN_BLK_OFF(b) ((blk_mode & (b)) != 0)
#else
#define LGCN_BLK_OFF(b) false
#endif
template <int XD>
__global__ __launch_bounds__(64) void k_emu_blocks(const lgcn_edge_t* __restrict__ edges,
                                                   const lgcn_emu_block_t* __restrict__ blocks,
                                                   lgcn_rows_t x, float xdiv,
                                                   const uint32_t* __restrict__ x_nz, int32_t d,
                                                   int4* __restrict__ ktab,
                                                   int4* __restrict__ meta,
                                                   float* __restrict__ stage,
                                                   const lgcn_emu_row_t* __restrict__ live) {
    // steps gathered per sub-window (all in flight at once), two sub-windows in flight
#ifndef LGCN_BLK_SW
#define LGCN_BLK_SW 16
#endif
    constexpr int SW = LGCN_BLK_SW;
    static_assert(SW == 8 || SW == 16, "sub-window");
    const int lane = threadIdx.x;
    const int c = blockIdx.y * 64 + lane;
    const bool act = c < d;
    const int64_t bi = blockIdx.x;
    const lgcn_emu_block_t blk = blocks[bi];
    // a row the live-edge chains run (lgcn_live_rows flags it) needs no block pass
    if (live && live[blk.row].n_blocks) return;
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
    const int blk_mode = __builtin_amdgcn_readfirstlane(g_blk_mode);
#endif
    // T: the sequential fma chain of the block from +0. It is the true chain for block 0; for
    // every block it tracks the exact running sum S of the products to within 1/2 ulp(|T|) per
    // step, which bounds every trajectory of the block (meta lo0/hi0)
    float T = 0.f, tlo = 0.f, thi = 0.f;
    int maxlsb = -100000;
    float cand[kNB];
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
    // this (block, column)'s elements, in step order (the walk resolves a block from here)
    // stage layout [block][d + 1][BLOCK]: column c's X elements, then (column d) the edge values.
    // Written through an LDS tile of 32 steps x 64 columns: each flush stores 8 whole 128-B
    // column runs per instruction. (A lane storing its own column's 16-B pieces at a 1-KB
    // stride scattered 64 half-written lines over L2 per instruction: ~60% of the pass's time.)
    constexpr int TP = 36;  // tile pitch in floats: 32 steps + 4 (ds_write_b128 conflict-free)
    __shared__ __attribute__((aligned(16))) float s_tile[64 * TP];
    float* const st0 = stage ? stage + bi * (d + 1) * LGCN_EMU_BLOCK : nullptr;
    float* sv = stage && blockIdx.y == 0 ? stage + (bi * (d + 1) + d) * LGCN_EMU_BLOCK : nullptr;
    const bool staging = st0 && !LGCN_BLK_OFF(1);
    auto stage_sub = [&](const float (&xv)[SW], int part) {  // SW steps into the tile
        if (!staging) return;
        float* tp = s_tile + lane * TP + SW * part;
#pragma unroll
        for (int q = 0; q < SW / 4; ++q)
            *reinterpret_cast<float4*>(tp + 4 * q) =
                make_float4(xv[4 * q], xv[4 * q + 1], xv[4 * q + 2], xv[4 * q + 3]);
    };
    // the tile is written by each lane for its own column and read across lanes: a wave barrier
    // with wavefront-scope release/acquire orders the LDS writes before the reads (and the reads
    // before the next sub-window rewrites the tile) under the memory model, not only by issue order
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto stage_flush = [&](int step0) {  // the tile's 32 steps -> stage, 8 columns a store
        if (!staging) return;
        wave_sync();
        const int sub = lane >> 3, q = lane & 7;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int col = 8 * i + sub;
            const float4 v = *reinterpret_cast<const float4*>(s_tile + col * TP + 4 * q);
            const int cg = blockIdx.y * 64 + col;
            // non-temporal: the walk re-reads ~10% of the stage, much later; streaming stores
            // keep the layer kernels' gathered rows in L2 / MALL (round 6: forward -0.15..0.4 ms,
            // BPR backward -0.1 ms, A/B on one box)
            if (cg < d) {
                typedef float f4v __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(
                    f4v{v.x, v.y, v.z, v.w},
                    reinterpret_cast<f4v*>(st0 + (int64_t)cg * LGCN_EMU_BLOCK + step0 + 4 * q));
            }
        }
        wave_sync();
    };
    // one sub-window: steps past the block end read as (0, 0), and fma(0, 0, c) == c for every
    // chain value (a chain is never -0), so the unrolled steps need no guard
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
                for (int k = 0; k < kNB; ++k) {
                    const int eb = ebase + k;
                    cand[k] = (eb >= -126 && eb <= 127) ? ldexpf(1.5f, eb) : 1.5f;
                }
            }
        }
#pragma unroll
        for (int t = 0; t < SW; ++t) {
            T = __builtin_fmaf(vv[t], xv[t], T);
            tlo = fminf(tlo, T);
            thi = fmaxf(thi, T);
            // a product's lowest set bit: lsb(v) (scalar) + lsb(x); -100000 when v or x is a zero
            if (!LGCN_BLK_OFF(4)) maxlsb = max(maxlsb, lsb_exp_z(vv[t]) + lsb_exp_z(xv[t]));
        }
        if (init && !LGCN_BLK_OFF(2)) {
#pragma unroll
            for (int t = 0; t < SW; ++t) {
#pragma unroll
                for (int k = 0; k < kNB; ++k) cand[k] = __builtin_fmaf(vv[t], xv[t], cand[k]);
            }
        }
    };
    int2 rec = load_rec(blk.beg);
    float xa[SW], va[SW], xb[SW], vb[SW];
    // the loads of sub-window k + 1 are issued before sub-window k is computed — across the
    // 64-edge windows too: the last sub-window of a window is computed while the next window's
    // first sub-window is in flight (its records were loaded at the window's start)
    load_sub(rec, 0, min(64, blk.end - blk.beg), xa, va);
    for (int32_t j0 = blk.beg; j0 < blk.end; j0 += 64) {
        const int n = min(64, blk.end - j0);
        const bool more = j0 + 64 < blk.end;
        const int2 nrec = load_rec(j0 + 64);  // next window's records, in flight meanwhile
        if (sv) sv[j0 - blk.beg + lane] = __int_as_float(rec.y);  // (0 past the block end)
        const int w0 = j0 - blk.beg;
#pragma unroll
        for (int k = 0; k < 64 / SW; k += 2) {
            load_sub(rec, (k + 1) * SW, n, xb, vb);
            run_sub(xa, va);
            stage_sub(xa, k % (32 / SW));
            if (k + 2 < 64 / SW)
                load_sub(rec, (k + 2) * SW, n, xa, va);
            else if (more)  // (round 5: 12.98 / 13.07 vs 13.04 / 13.29 ms forward, A/B)
                load_sub(nrec, 0, min(64, blk.end - j0 - 64), xa, va);
            run_sub(xb, vb);
            stage_sub(xb, (k + 1) % (32 / SW));
            if ((k + 2) % (32 / SW) == 0) stage_flush(w0 + (k + 2 - 32 / SW) * SW);
        }
        rec = nrec;
    }
    if (!act) return;
    const int64_t rc = bi * d + c;
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
    const int32_t lo0 = fits ? (int32_t)lo_u : 0, hi0 = fits ? (int32_t)hi_u : 0;
    // candidate k: translation in units of its ulp u_k = 2^(ebase + k - 23) — an exact integer
    // when the candidate's chain stayed in its binade, which the validity bit certifies
    uint32_t vm = 0;
    int K[kNB];
#pragma unroll
    for (int k = 0; k < kNB; ++k) {
        const int eb = ebase + k;
        const bool normal = eb >= -126 && eb <= 127;
        const float a0 = normal ? ldexpf(1.5f, eb) : 1.5f;
        const float ku = ldexpf(cand[k] - a0, 23 - eb);
        const bool kfit = fabsf(ku) < 16777216.f;
        K[k] = (init && kfit) ? (int)ku : 0;
        const int lo = lo0 >> k, hi = -((-hi0) >> k);
        const bool ok = init && fits && normal && kfit && kC + lo >= kLB && kC + hi <= kHB &&
                        maxlsb < eb - 24;
        vm |= ok ? (1u << k) : 0u;
    }
    const bool ident = maxlsb < -50000;
    const int pk = ident ? (kIdentEb & 0xffff) : (int)(((uint32_t)ebase & 0xffffu) | (vm << 16));
    meta[rc] = make_int4(lo0, hi0, pk, __float_as_int(T));
    int4* kp = ktab + rc * 4;
#pragma unroll
    for (int q = 0; q < kNB / 4; ++q)
        kp[q] = make_int4(K[4 * q], K[4 * q + 1], K[4 * q + 2], K[4 * q + 3]);
}

// ---------------------------------------------------------------------------------------------
// walker: one wave per (hub row, column). The chain value is wave-uniform.
// ---------------------------------------------------------------------------------------------
// LGCN_EMU_STATS builds (diagnostics only, tools/exact_probe.py): walker counters
// [translated blocks, resolved blocks, identity blocks, not predicted, resolve iterations,
//  sequential steps, -, -]
#ifdef LGCN_EMU_STATS
__device__ unsigned long long g_emu_stats[8];
// per emulated row (first 256 rows): translated, resolved, cycles resolving, max wave cycles
__device__ unsigned long long g_emu_row_stats[256][4];
#endif
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
__device__ int g_emu_mode;
// timing experiments only: 1 = failing blocks are not resolved (value kept), 2 = every block
// translates, 3 = every block is resolved, 4 = every block fails and is not resolved, 5 = as 4
// with no slot fetched
#define LGCN_EMU_FORCE(f) do { if (g_emu_mode == 2) (f) = true; \
                               if (g_emu_mode >= 3) (f) = false; } while (0)
#else
#define LGCN_EMU_FORCE(f) ((void)0)
#endif
#ifdef LGCN_EMU_STATS
// phase timer of the walker wave (row 0, column 0): s_memtime deltas per phase, then counts
// [tables, predict, slot wait, scans, resolve, on-demand fetch, -, -, chunks, predicted,
//  resolved, not predicted, resolve iterations]
__device__ unsigned long long g_emu_phase[16];
#define PH_MARK(k) do { const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
                        ph[k] += now_ - ph_last; ph_last = now_; } while (0)
#define PH_COUNT(k, v) (ph[k] += (v))
// counted per wave in registers, flushed once at the end: an atomic per event would count in
// vmcnt and make the walker's explicit waits wait for it
#define EMU_STAT(k, v) (est[k] += (unsigned long long)(v))
#else
#define PH_MARK(k) ((void)0)
#define PH_COUNT(k, v) ((void)0)
#define EMU_STAT(k, v) ((void)0)
#endif

#define LGCN_EMU_CH 64
#define LGCN_EMU_SLOTS 12   // default LDS slots per chunk for predicted resolve blocks
// static LDS of k_emu_walk (two 16 x 64 translation tables, 8 KB) + (2 * slots + 1) 2-KB slots
// within a CU's 160 KB; and a chunk's slot fetches (2 per slot) + the 5 table loads after them
// within the 63 outstanding loads a vmcnt wait can count
#define LGCN_EMU_MAX_SLOTS 28

// Inclusive prefix sum over the 64 lanes of a wave by DPP row shifts and row broadcasts (no LDS
// round trips: the walker's scans are on its critical path).
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// inclusive prefix sum of floats over the 64 lanes (DPP, as wave_incl_scan); the order of the
// additions is the scan's, not sequential: for approximations only
__device__ __forceinline__ float wave_incl_scan_f(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x112, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x114, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x118, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xa, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x143, 0xc, 0xf, false));
    return x;
}


__device__ __forceinline__ uint32_t lds_byte(const void* p) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)reinterpret_cast<uintptr_t>(p));
}

// 1 KB by LDS-DMA: lane l's 16 bytes at gsrc -> LDS byte address dst + 16 l (dst wave-uniform).
// Inline asm on purpose: a compiler-visible LDS-DMA makes the compiler drain every global load
// in flight (vmcnt(0)) before any later LDS access of the kernel, which would serialise the
// walker's prefetches; hidden from it, the DMA is waited for by this file's explicit vmcnt.
// dma16x2: two of them to consecutive KB of LDS (dst, dst + 1024) under one m0 save/restore.
__device__ __forceinline__ void dma16x2(const void* g0, const void* g1, uint32_t dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g0), "v"(g1),
                   "s"(__builtin_amdgcn_readfirstlane((int)dst)) : "memory", "scc");
}

// N (4 or 8) 1-KB LDS-DMAs to consecutive KB of LDS (dst + 1024 k): a chain window's gathers
// under one m0 save/restore (k_chain_rows; 3 scalar instructions per load saved).
#define LGCN_DMA16_NEXT(i) \
    "global_load_lds_dwordx4 %" #i ", off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
template <int N>
__device__ __forceinline__ void dma16_run(const char* const (&g)[N], uint32_t dst) {
    static_assert(N == 2 || N == 4 || N == 8, "window sizes of k_chain_rows");
    uint32_t keep;
    if constexpr (N == 2) {
        dma16x2(g[0], g[1], dst);
    } else if constexpr (N == 4) {
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 0\n\t"
                     LGCN_DMA16_NEXT(1) LGCN_DMA16_NEXT(2) LGCN_DMA16_NEXT(3)
                     "global_load_lds_dwordx4 %4, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "s"(dst)
                     : "memory", "scc");
    } else {
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %9\n\ts_nop 0\n\t"
                     LGCN_DMA16_NEXT(1) LGCN_DMA16_NEXT(2) LGCN_DMA16_NEXT(3)
                     LGCN_DMA16_NEXT(4) LGCN_DMA16_NEXT(5) LGCN_DMA16_NEXT(6)
                     LGCN_DMA16_NEXT(7)
                     "global_load_lds_dwordx4 %8, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "v"(g[4]),
                       "v"(g[5]), "v"(g[6]), "v"(g[7]), "s"(dst)
                     : "memory", "scc");
    }
}
#undef LGCN_DMA16_NEXT

// s_waitcnt vmcnt(m) for the largest m in {32, 16, 8, 4, 2, 1, 0} not above a wave-uniform n:
// at most n younger operations may stay outstanding, a few of them may be waited for too. The
// walk's common cases (a refill NS blocks old, n ~ 2 NS) take one or two compares instead of a
// branch tree over every count.
__device__ __forceinline__ void wait_vm_coarse(int n) {
    if (n >= 63) return;
    if (n >= 32) {
        asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    } else if (n >= 16) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else if (n >= 8) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (n >= 4) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else if (n >= 2) {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else if (n == 1) {
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// The reference's chain itself over steps [j0, j1) of a block whose (val, x) pairs lane l holds
// for steps 4l..4l+3 (vv, xv): the value travels down the lanes — lane l applies its steps,
// then hands the value to lane l + 1 (DPP wave_shr:1). Every lane computes with its own pairs;
// only the lane holding the value matters, the others' results are overwritten by the shift.
// No memory access on the chain. Returns the bits of the value after step j1 - 1.
__device__ __forceinline__ float dpp_wave_shr1(float v) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x138, 0xf, 0xf, false));
}

__device__ __forceinline__ uint32_t seq_reg(const float (&vv)[4], const float (&xv)[4], int j0,
                                            int j1, uint32_t a) {
    const int lane = threadIdx.x;
    float acc = __uint_as_float(a);
    const int L0 = j0 >> 2, L1 = (j1 - 1) >> 2;
    if (j0 == 0 && j1 == LGCN_EMU_BLOCK) {  // a whole block: no step masks
        for (int L = 0; L < 64; ++L) {
            if (L > 0) acc = dpp_wave_shr1(acc);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc = __builtin_fmaf(vv[k], xv[k], acc);
        }
    } else {
        for (int L = L0; L <= L1; ++L) {
            if (L > L0) acc = dpp_wave_shr1(acc);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 4 * lane + k;
                const float f = __builtin_fmaf(vv[k], xv[k], acc);
                acc = (j >= j0 && j < j1) ? f : acc;
            }
        }
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(acc), L1);
}

// A whole block's chain (256 steps) over its (val, x) pairs in an LDS slot, S steps per lane:
// lane l < 256/S holds steps S*l .. S*l+S-1 in registers and the value travels down those lanes
// by DPP wave_shr:1 — 256/S - 1 lane transitions instead of seq_reg's 63 (a transition costs the
// wait states around the DPP move on the dependent chain). The other lanes mirror the first
// lanes' pairs and compute values nobody reads. Returns the bits of the value after step 255.
#ifndef LGCN_SEQ_STEPS
#define LGCN_SEQ_STEPS 16
#endif
template <int S>
__device__ __forceinline__ uint32_t seq_block(const float* __restrict__ sv,
                                              const float* __restrict__ sx, uint32_t a) {
    constexpr int NL = LGCN_EMU_BLOCK / S;
    static_assert(S % 4 == 0 && NL >= 1 && NL <= 64, "steps per lane");
    const int l = threadIdx.x & (NL - 1);
    const float4* v4 = reinterpret_cast<const float4*>(sv + S * l);
    const float4* x4 = reinterpret_cast<const float4*>(sx + S * l);
    float vv[S], xv[S];
#pragma unroll
    for (int q = 0; q < S / 4; ++q) {
        const float4 v = v4[q], x = x4[q];
        vv[4 * q] = v.x, vv[4 * q + 1] = v.y, vv[4 * q + 2] = v.z, vv[4 * q + 3] = v.w;
        xv[4 * q] = x.x, xv[4 * q + 1] = x.y, xv[4 * q + 2] = x.z, xv[4 * q + 3] = x.w;
    }
    float acc = __uint_as_float(a);
#pragma unroll
    for (int L = 0; L < NL; ++L) {
        if (L > 0) acc = dpp_wave_shr1(acc);
#pragma unroll
        for (int k = 0; k < S; ++k) acc = __builtin_fmaf(vv[k], xv[k], acc);
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(acc), NL - 1);
}

// The resolution of one block: the sequential chain a = fma(v_j, x_j, a), j < n, over the
// block's (val, x) pairs in an LDS slot (sv, sx): a whole block LGCN_SEQ_STEPS steps per lane
// (seq_block), a shorter last block 4 steps per lane (seq_reg). (Round 3 measured parallel
// runs of exact integer steps before the chain: a chain value next to a binade boundary crosses
// it ~19 times per resolved block on the Books-scale graph, so they did not pay and are gone.)
// Returns the bits of the value after the block.
__device__ __forceinline__ uint32_t resolve_block(const float* __restrict__ sv,
                                                  const float* __restrict__ sx, int n, uint32_t a) {
    const int lane = threadIdx.x;
    if (n == LGCN_EMU_BLOCK) return seq_block<LGCN_SEQ_STEPS>(sv, sx, a);
    const float4 v4 = *reinterpret_cast<const float4*>(sv + 4 * lane);
    const float4 x4 = *reinterpret_cast<const float4*>(sx + 4 * lane);
    const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
    const float xv[4] = {x4.x, x4.y, x4.z, x4.w};
    return seq_reg(vv, xv, 0, n, a);
}

template <int MODE, int XD>
__global__ __launch_bounds__(64) void k_emu_walk(const lgcn_edge_t* __restrict__ edges,
                                                 const lgcn_emu_block_t* __restrict__ blocks,
                                                 const lgcn_emu_row_t* __restrict__ rows,
                                                 const int4* __restrict__ ktab,
                                                 const int4* __restrict__ meta,
                                                 const float* __restrict__ stage, lgcn_rows_t x,
                                                 float xdiv, const uint32_t* __restrict__ x_nz,
                                                 int32_t d, float* __restrict__ y, int64_t ldy,
                                                 lgcn_epilogue_t ep, int NS, int pmargin,
                                                 const lgcn_emu_row_t* __restrict__ live) {
    constexpr int CH = LGCN_EMU_CH;
    constexpr int B = LGCN_EMU_BLOCK;
    static_assert(CH == 64, "one lane per block of a chunk");
    // translation tables of two chunks, [binade][block]: lane reads are conflict-free
    __shared__ int32_t sK[2][kNB][CH];
    // 2 sets x NS slots (chunk c uses set c & 1) + one spare: a block's edge values, then its
    // X elements (dynamic LDS, sized at launch)
    extern __shared__ __attribute__((aligned(16))) float s_dyn[];
    const int lane = threadIdx.x;
    // grid (column, row): a row's column waves are dispatched together, longest row first (the
    // rows are in descending length), so a long row's last columns do not queue behind every
    // shorter row's first ones
    const int c = (int)LGCN_GRID_COL(d);
    const uint32_t rix = LGCN_GRID_ROW(d);
#ifdef LGCN_WALK_PRIO
    // issue priority over the co-resident waves of other kernels on this SIMD (build flag A/B)
    __builtin_amdgcn_s_setprio(LGCN_WALK_PRIO);
#endif
    // a row the live-edge chains run (lgcn_live_rows flags it, aligned with `rows`) is theirs
    if (live && live[rix].n_blocks) return;
    const lgcn_emu_row_t er = rows[rix];
    const int64_t fb = er.first_block;
    const int nb_all = er.n_blocks;
    // block k of the row holds edges [row_beg + k * B, min(.. + B, row_end)) (plan_emulation)
    const int32_t row_beg = blocks[fb].beg;
    const int32_t row_end = blocks[fb + nb_all - 1].end;
    // chunks of blocks 1, 2, ... (64 blocks each)
    const int nch = (nb_all - 1 + CH - 1) / CH;
    constexpr int ch_lo = 0;
    // the chain value as its bits (wave-uniform): block 0's chain from +0 is the true chain
    uint32_t ab = (uint32_t)__builtin_amdgcn_readfirstlane(meta[fb * d + c].w);
    const bool staged = stage != nullptr;
    const int spare = 2 * NS;
#ifdef LGCN_EMU_STATS
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    unsigned long long n_fast = 0, n_slow = 0, t_slow = 0;
    unsigned long long ph[16] = {0};
    unsigned long long est[8] = {0};
    unsigned long long ph_last = t_start;
#endif
    struct Tab {
        int4 m;
        int4 k[4];
    };
    auto chunk_nb = [&](int ch) { return min(CH, nb_all - 1 - ch * CH); };
    auto load_tab = [&](int ch, Tab& t) {  // 5 loads per lane (lane = block)
        const int nb = chunk_nb(ch);
        const int64_t rc = (fb + 1 + (int64_t)ch * CH + min(lane, nb - 1)) * d + c;
        t.m = meta[rc];
        const int4* kp = ktab + rc * 4;
        t.k[0] = kp[0];
        t.k[1] = kp[1];
        t.k[2] = kp[2];
        t.k[3] = kp[3];
    };
    auto stage_tab = [&](const Tab& t, int buf) {
        const int kk[kNB] = {t.k[0].x, t.k[0].y, t.k[0].z, t.k[0].w, t.k[1].x, t.k[1].y,
                             t.k[1].z, t.k[1].w, t.k[2].x, t.k[2].y, t.k[2].z, t.k[2].w,
                             t.k[3].x, t.k[3].y, t.k[3].z, t.k[3].w};
#pragma unroll
        for (int w = 0; w < kNB; ++w) sK[buf][w][lane] = kk[w];
    };
    // The speculative test of chunk blocks [from, nb) from chain value bits a, with table `buf`
    // and the lane's block meta m: lane i's start mantissa if every block in [from, i)
    // translates (exclusive prefix of the magnitude changes), and the ballot of the blocks that
    // cannot translate from there. `incl` returns the inclusive prefix, `dm` the lane's change.
    // margin: the prediction widens the bounds (its start value is approximate).
    auto test = [&](uint32_t a, int from, int nb, int buf, const int4& m, bool margin, int& incl,
                    int& dm) -> unsigned long long {
        const int E = (int)((a >> 23) & 255u);
        const int neg = (int)(a >> 31);
        const int M = (int)((a & 0x7fffffu) | 0x800000u);
        const int eb = (int)(int16_t)(m.z & 0xffff);
        const uint32_t vm = (uint32_t)m.z >> 16;
        const bool ident = eb == kIdentEb;
        const int w = E - 127 - eb;
        const bool inw = ((unsigned)(E - 1) < 254u) && ((unsigned)w < (unsigned)kNB) &&
                         ((vm >> (w & (kNB - 1))) & 1u);
        const int wc = inw ? w : 0;
        const int K = sK[buf][wc][lane];
        const int lo = m.x >> wc, hi = -((-m.y) >> wc);
        const bool act = lane >= from && lane < nb;
        dm = (act && inw && !ident) ? (neg ? -K : K) : 0;  // |K| < 2^24: the sums fit in int32
        incl = wave_incl_scan(dm);
        const int start = M + incl - dm;
        const int alo = neg ? -hi : lo, ahi = neg ? -lo : hi;
        const int mg = margin ? ((hi - lo) >> 4) + 64 : 0;
        bool ok = ident || (inw && start + alo >= kLB + mg && start + ahi <= kHB - mg);
        LGCN_EMU_FORCE(ok);
        return __ballot(act && !ok);
    };
    // Chunk ch's blocks predicted to need a resolve, from the approximate start bits pa, in ONE
    // pass: block i's start is taken as pa + the chains from +0 (meta r0) of the blocks before
    // it — the true contributions to within their rounding — and every lane tests its own block
    // from its own start with widened bounds. All predicted blocks are recorded (the first NS
    // are fetched ahead of the chunk, the rest refill slots as the walk passes them).
    // Returns the approximate end value.
    auto predict = [&](int ch, int buf, const int4& m, uint32_t pa,
                       unsigned long long& pred) -> uint32_t {
        const int nb = chunk_nb(ch);
        const bool act = lane < nb;
        const float r0 = act ? __int_as_float(m.w) : 0.f;
        const float incl = wave_incl_scan_f(r0);
        const uint32_t a = __float_as_uint(__uint_as_float(pa) + (incl - r0));
        const int E = (int)((a >> 23) & 255u);
        const int neg = (int)(a >> 31);
        const int M = (int)((a & 0x7fffffu) | 0x800000u);
        const int eb = (int)(int16_t)(m.z & 0xffff);
        const uint32_t vm = (uint32_t)m.z >> 16;
        const bool ident = eb == kIdentEb;
        const int w = E - 127 - eb;
        const bool inw = ((unsigned)(E - 1) < 254u) && ((unsigned)w < (unsigned)kNB) &&
                         ((vm >> (w & (kNB - 1))) & 1u);
        const int wc = inw ? w : 0;
        const int lo = m.x >> wc, hi = -((-m.y) >> wc);
        const int alo = neg ? -hi : lo, ahi = neg ? -lo : hi;
        // widened bounds: (hi - lo) >> shift + base (pmargin = base << 4 | shift; default 4, 128)
        const int mg = ((hi - lo) >> (pmargin & 15)) + (pmargin >> 4);
        bool ok = ident || (inw && M + alo >= kLB + mg && M + ahi <= kHB - mg);
        LGCN_EMU_FORCE(ok);
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
        if (g_emu_mode == 5) ok = true;  // nothing predicted (and nothing fetched: mode 5)
#endif
        pred = __ballot(act && !ok);
#ifdef LGCN_WALK_NO_REFILL  // build-time A/B: the first NS only, the rest fetched on demand
        {
            unsigned long long keep = 0, m = pred;
            for (int i = 0; i < NS && m; ++i, m &= m - 1) keep |= m & (~m + 1ull);
            pred = keep;
        }
#endif
        const float tot = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
        return (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)__float_as_uint(__uint_as_float(pa) + tot));
    };
    // Slots by LDS float offset from s_dyn: slot i at 2 B i (values, then X). The ring: lane k
    // holds the offset of slot k % NS of set 0 — predicted block #k of a chunk lives there —
    // read back by readlane, no division on the walk's per-block path.
    const uint32_t lds0 = lds_byte(s_dyn);
    const int ring = (lane % NS) * 2 * B;
    const int set_off = NS * 2 * B;
    // block kb of the row: its staged values at st_v + kb * (d + 1) B, column c at st_x + ...
    const float* st_v = stage + ((fb * (d + 1)) + d) * B + 4 * lane;
    const float* st_x = stage + ((fb * (d + 1)) + c) * B + 4 * lane;
    const int64_t blk_stride = (int64_t)(d + 1) * B;
    auto fetch = [&](int kb, int off) {  // block kb's staged values -> LDS at float offset off
        const int64_t o = (int64_t)kb * blk_stride;
        dma16x2(st_v + o, st_x + o, lds0 + 4u * (uint32_t)off);
    };
    // the first NS predicted blocks of chunk ch into slot set `set`; returns the predicted
    // blocks left for refills (nvm: this wave's vector-memory operations issued so far)
    auto issue_slots = [&](int ch, unsigned long long pred, int set,
                           int& nvm) -> unsigned long long {
        unsigned long long m = pred;
        for (int s = 0; s < NS && m; ++s, m &= m - 1) {
            fetch(1 + ch * CH + __builtin_ctzll(m), (set * NS + s) * 2 * B);
            nvm += 2;
        }
        return m;
    };
    if (nch > ch_lo) {
        Tab tn;
        int4 mc, mn = make_int4(0, 0, 0, 0);
        // vmcnt bookkeeping: nvm counts this wave's vector-memory operations (5 per table load,
        // 2 per block fetch); an operation stamped s has landed once at most nvm - s younger
        // ones are outstanding (they complete in issue order)
        int nvm = 0;
        load_tab(ch_lo, tn);
        nvm += 5;
        stage_tab(tn, 0);
        mc = tn.m;
        unsigned long long pred_c = 0, pred_n = 0;
        uint32_t start_c = ab;                     // assumed start of chunk ch's prediction
        uint32_t end_c = predict(ch_lo, 0, mc, ab, pred_c);  // and its predicted end
        if (!staged) pred_c = 0;
        // predicted blocks of chunk ch not fetched yet, how many are issued, and the stamp of
        // its first NS fetches; lane k of `stamp`: nvm after the fetch of predicted block #k
        unsigned long long rem_c = issue_slots(ch_lo, pred_c, 0, nvm), rem_n = 0;
        int iss_c = min(__builtin_popcountll(pred_c), NS), iss_n = 0;
        int stamp_c = nvm, stamp_n = 0;
        int stamp = 0;
        if (nch > ch_lo + 1) {
            load_tab(ch_lo + 1, tn);
            nvm += 5;
            stage_tab(tn, 1);
            mn = tn.m;
        }
        if (nch > ch_lo + 2) {  // in flight during the first chunk
            load_tab(ch_lo + 2, tn);
            nvm += 5;
        }
        PH_MARK(0);
        for (int ch = ch_lo; ch < nch; ++ch) {
            const int buf = (ch - ch_lo) & 1;
            const int nb = chunk_nb(ch);
            const int buf_off = buf ? set_off : 0;
            // prediction of chunk ch + 1 (its start: chunk ch's predicted end, moved by the
            // error of chunk ch's assumed start) and its first slot fetches, in flight during ch
            uint32_t start_n = 0, end_n = 0;
            if (ch + 1 < nch) {
                start_n = __float_as_uint(__uint_as_float(end_c) +
                                          (__uint_as_float(ab) - __uint_as_float(start_c)));
                start_n = (uint32_t)__builtin_amdgcn_readfirstlane((int)start_n);
                end_n = predict(ch + 1, buf ^ 1, mn, start_n, pred_n);
                if (!staged) pred_n = 0;
                rem_n = issue_slots(ch + 1, pred_n, buf ^ 1, nvm);
                iss_n = min(__builtin_popcountll(pred_n), NS);
                stamp_n = nvm;
            }
            PH_MARK(1);
            PH_COUNT(8, 1);
            PH_COUNT(9, __builtin_popcountll(pred_c));
            wait_vm_coarse(nvm - stamp_c);  // chunk ch's first slots have landed
            PH_MARK(2);
            int from = 0;
            bool direct = false;  // block `from` is re-run without a test (a predicted run)
            while (true) {
                int f = from;
                if (!direct) {
                    int incl, dm;
                    const unsigned long long bad = test(ab, from, nb, buf, mc, false, incl, dm);
                    f = bad ? (int)__builtin_ctzll(bad) : nb;
                    // blocks [from, f) translate: their mantissa changes add to the bits
                    const int tv = f < nb ? incl - dm : incl;
                    ab += (uint32_t)__builtin_amdgcn_readlane(tv, f < nb ? f : 63);
                    PH_MARK(3);
                    EMU_STAT(0, f - from);
#ifdef LGCN_EMU_STATS
                    n_fast += f - from;
#endif
                    if (f >= nb) break;
                }
                // refills: the predicted blocks before f are done, their slots take the next
                // predicted ones (at most NS ahead of f, so f's own slot is kept)
                const int done = __builtin_popcountll(pred_c & ((1ull << f) - 1ull));
                while (rem_c && iss_c < done + NS) {
                    fetch(1 + ch * CH + __builtin_ctzll(rem_c),
                          buf_off + __builtin_amdgcn_readlane(ring, iss_c));
                    nvm += 2;
                    stamp = lane == iss_c ? nvm : stamp;
                    rem_c &= rem_c - 1;
                    ++iss_c;
                }
                const int kb = 1 + ch * CH + f;  // block index in the row
                const int32_t bbeg = row_beg + kb * B;
                const int n = min(bbeg + B, row_end) - bbeg;
                EMU_STAT(1, 1);
#ifdef LGCN_EMU_STATS
                const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
                int sl;  // the block's slot: float offset from s_dyn
                if ((pred_c >> f) & 1ull) {
                    sl = buf_off + __builtin_amdgcn_readlane(ring, done);
                    if (done >= NS) {  // a refill: wait for its own fetch only
                        wait_vm_coarse(nvm - __builtin_amdgcn_readlane(stamp, done));
                        PH_MARK(5);
                    }
                } else {  // not predicted: fetched now into the spare slot
                    sl = spare * 2 * B;
                    EMU_STAT(3, 1);
                    PH_COUNT(11, 1);
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
                    if (g_emu_mode == 5) {
                    } else
#endif
                    if (staged) {
                        fetch(kb, sl);
                        nvm += 2;
                        // the youngest operation: everything older lands before it anyway
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    } else {
                        // no stage: the block's edge records and X elements, gathered
                        float vq[4], xq[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const int j = 4 * lane + k;
                            const int2 r = *reinterpret_cast<const int2*>(
                                edges + bbeg + min(j, n - 1));
                            vq[k] = j < n ? __int_as_float(r.y) : 0.f;
                            xq[k] = load_elem<XD>(x, x_nz, r.x, c, xdiv, j < n);
                        }
                        *reinterpret_cast<float4*>(s_dyn + sl + 4 * lane) =
                            make_float4(vq[0], vq[1], vq[2], vq[3]);
                        *reinterpret_cast<float4*>(s_dyn + sl + B + 4 * lane) =
                            make_float4(xq[0], xq[1], xq[2], xq[3]);
                    }
                    PH_MARK(5);
                }
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
                if (g_emu_mode != 1 && g_emu_mode < 4)
#endif
                    ab = resolve_block(s_dyn + sl, s_dyn + sl + B, n, ab);
                PH_MARK(4);
                PH_COUNT(10, 1);
#ifdef LGCN_EMU_STATS
                ++n_slow;
                t_slow += __builtin_amdgcn_s_memtime() - t0;
#endif
                from = f + 1;
                if (from >= nb) break;
                // the next block predicted to fail too (runs of them: the chain value wanders
                // near zero or along a binade boundary): re-run it without a test — a re-run
                // is the reference's chain, exact whether or not the block would translate, and
                // it costs about what the test does (~0.6 us either way)
                direct = (pred_c >> from) & 1ull;
#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
                if (g_emu_mode == 2) direct = false;
#endif
            }
            // rotate: chunk ch + 2's table into chunk ch's buffer, chunk ch + 3's loads
            if (ch + 2 < nch) {
                stage_tab(tn, buf);
                mc = mn;
                mn = tn.m;
            } else {
                mc = mn;
            }
            if (ch + 3 < nch) {
                load_tab(ch + 3, tn);
                nvm += 5;
            }
            PH_MARK(0);
            pred_c = pred_n;
            rem_c = rem_n;
            iss_c = iss_n;
            stamp_c = stamp_n;
            start_c = start_n;
            end_c = end_n;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA lands after the wave is gone
#ifdef LGCN_EMU_STATS
    if (lane == 0 && rix == 0 && c == 0)
        for (int k = 0; k < 16; ++k) g_emu_phase[k] += ph[k];
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&g_emu_stats[k], est[k]);
    if (lane == 0 && rix < 256) {
        atomicAdd(&g_emu_row_stats[rix][0], n_fast);
        atomicAdd(&g_emu_row_stats[rix][1], n_slow);
        atomicAdd(&g_emu_row_stats[rix][2], t_slow);
        atomicMax(&g_emu_row_stats[rix][3], __builtin_amdgcn_s_memtime() - t_start);
    }
#endif
    if (lane != 0) return;
    const int32_t row = er.row;
    float out = __uint_as_float(ab);
    if constexpr (MODE == LGCN_EPI_ROWS) {  // the chain value itself, to row i of the list
        y[(int64_t)rix * ldy + c] = out;
        return;
    }
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

// n_blocks blocks from `blocks`
template <int XD>
int launch_blocks(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks, int32_t n_blocks,
                  const lgcn_rows_t& x, float xdiv, const uint32_t* x_nz, int32_t d, int4* ktab,
                  int4* meta, float* stage, const lgcn_emu_row_t* live, hipStream_t s) {
    const dim3 grid((uint32_t)n_blocks, (uint32_t)((d + 63) / 64));
    hipLaunchKernelGGL((k_emu_blocks<XD>), grid, dim3(64), 0, s, edges, blocks, x, xdiv, x_nz, d,
                       ktab, meta, stage, live);
    return herr_x(hipGetLastError());
}

template <int MODE, int XD>
int launch_walk(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks,
                const lgcn_emu_row_t* rows, int32_t n_rows, const int4* ktab, const int4* meta,
                const float* stage, const lgcn_rows_t& x, float xdiv, const uint32_t* x_nz, float* y,
                int64_t ldy, int32_t d, const lgcn_epilogue_t& ep, int slots,
                const lgcn_emu_row_t* live, hipStream_t s) {
    const dim3 grid = LGCN_GRID_DIM((uint32_t)d, (uint32_t)n_rows);
    const size_t lds = (size_t)(2 * slots + 1) * 2 * LGCN_EMU_BLOCK * sizeof(float);
    if (lds > 56 * 1024) {
        // beyond the default dynamic-LDS limit: raise it once per kernel and DEVICE (the
        // attribute applies to the device current at the call)
        static std::atomic<uint64_t> raised{0};
        int dev = 0;
        if (hipError_t e = hipGetDevice(&dev)) return (int)e;
        const uint64_t bit = dev < 64 ? (1ull << dev) : 0;
        if (!bit || !(raised.load(std::memory_order_relaxed) & bit)) {
            const hipError_t e = hipFuncSetAttribute(
                reinterpret_cast<const void*>(&k_emu_walk<MODE, XD>),
                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 8 * 1024);
            if (e != hipSuccess) return (int)e;
            raised.fetch_or(bit, std::memory_order_relaxed);
        }
    }
    hipLaunchKernelGGL((k_emu_walk<MODE, XD>), grid, dim3(64), lds, s, edges, blocks, rows, ktab,
                       meta, stage, x, xdiv, x_nz, d, y, ldy, ep, slots,
                       lgcn_detail::g_emu_margin, live);
    return herr_x(hipGetLastError());
}

int xd_of(float xdiv, const uint32_t* x_nz) {
    return (xdiv == 1.f ? 0 : is_pow2(xdiv) ? 2 : 1) | (x_nz ? 4 : 0);
}

template <int MODE>
int walk_mode(int xd, const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks,
              const lgcn_emu_row_t* rows, int32_t n_rows, const int4* ktab, const int4* meta,
              const float* stage, const lgcn_rows_t& x, float xdiv, const uint32_t* x_nz, float* y,
              int64_t ldy, int32_t d, const lgcn_epilogue_t& ep, int slots,
              const lgcn_emu_row_t* live, hipStream_t s) {
#define LGCN_W(XD_) \
    case XD_: return launch_walk<MODE, XD_>(edges, blocks, rows, n_rows, ktab, meta, stage, x, xdiv, x_nz, y, ldy, d, ep, slots, live, s);
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
#ifndef LGCN_CHAIN_AHEAD32
#define LGCN_CHAIN_AHEAD32 6  // X windows in flight per 32-column chain wave (build-time A/B)
#endif
template <int W>
struct ChainCfg {
    static constexpr int LPR = W / 4;       // lanes per gathered row slice (16 B each)
    static constexpr int RPI = 64 / LPR;    // rows per 1-KB LDS-DMA instruction
    static constexpr int NI = 64 / RPI;     // instructions per 64-edge window
    static constexpr int XWIN = 64 * W;     // floats per X window
    // X windows in flight while one is folded: as many as vmcnt (<= 63 outstanding) allows
    // with NI + 2 loads per window (W=64: 3 x 18, W=32: 6 x 10, W=16: 8 x 6)
    static constexpr int AHEAD = W == 64 ? 3 : W == 32 ? LGCN_CHAIN_AHEAD32 : 8;
    // rings: X windows (>= AHEAD + 1), record windows (>= 2 AHEAD + 1); at W = 32 powers of two
    // (8 and 16: the ring index is a mask, not a division; 72 KB of LDS, still 2 waves per CU)
    static constexpr int NX = W == 32 && AHEAD <= 7 ? 8 : AHEAD + 1;
    static constexpr int NR = W == 32 && AHEAD <= 7 ? 16 : 2 * AHEAD + 1;
};

// the two dword LDS-DMAs of a window's edge records (column -> dst0, value -> dst1; lane l's
// dword to dst + 4 l), one m0 save/restore; hidden from the compiler like dma16x2
__device__ __forceinline__ void dma4x2(const void* g0, uint32_t dst0, const void* g1,
                                       uint32_t dst1) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                 "global_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g0), "v"(g1), "s"(dst0), "s"(dst1) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MODE, int XD, int W, bool SEG1>
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
    __shared__ __attribute__((aligned(16))) int32_t s_col[NR][64];
    __shared__ __attribute__((aligned(16))) float s_val[NR][64];
    const int lane = threadIdx.x;
    // grid (slice, row): a row's slices are dispatched together, longest row first
    const int c0 = (int)LGCN_GRID_COL((d + W - 1) / W) * W;
    const uint32_t rix = LGCN_GRID_ROW((d + W - 1) / W);
    const lgcn_emu_row_t er = rows[rix];
    if (er.n_blocks <= 0) return;  // (a live-edge row left to the walk: lgcn_live_rows)
    const int32_t beg = blocks[er.first_block].beg;
    const int32_t end = blocks[er.first_block + er.n_blocks - 1].end;
    const int32_t nwin = (end - beg + 63) >> 6;
    // records of window w: lane l's column -> s_col[w % NR][l], its value -> s_val[w % NR][l]
    // (two dword LDS-DMA loads). Windows past the row repeat its last record, so they load
    // valid records and gather valid rows: every iteration issues the same number of loads,
    // which keeps the vmcnt arithmetic below exact. They are never folded.
    const int32_t* ew = reinterpret_cast<const int32_t*>(edges);
    auto rec_dma = [&](int32_t w) {
        const int64_t j = min((int64_t)beg + 64 * w + lane, (int64_t)end - 1);
        dma4x2(ew + 2 * j, lds_byte(&s_col[w % NR][0]), ew + 2 * j + 1,
               lds_byte(&s_val[w % NR][0]));
    };
    // gathered X of window w -> s_x[w % NX]: instruction k moves rows k*RPI .. k*RPI + RPI - 1
    // (lane -> row sub = lane / LPR, 16-B piece q = lane % LPR); the columns come from LDS
    const int sub = lane / C::LPR, q = lane % C::LPR;
    const char* xb = reinterpret_cast<const char*>(x.p0) + (c0 + 4 * q) * 4;
    const uint32_t row_b = (uint32_t)(x.ld * 4);  // d <= 2048: a row is at most 8 KB
    auto x_dma = [&](int32_t w) {
        int32_t cols[C::NI];
#pragma unroll
        for (int k = 0; k < C::NI; ++k) cols[k] = s_col[w % NR][k * C::RPI + sub];
        const uint32_t dst = lds_byte(s_x[w % NX]);
        const char* g[C::NI];
#pragma unroll
        for (int k = 0; k < C::NI; ++k) {
            if constexpr (SEG1)  // one buffer: a row is base + col * ld
                g[k] = xb + (uint64_t)(uint32_t)cols[k] * row_b;
            else
                g[k] = reinterpret_cast<const char*>(seg_row_sel(x, cols[k]) + c0 + 4 * q);
        }
        dma16_run<C::NI>(g, dst);  // instruction k -> dst + 1024 k
    };
    // Pipeline (A = AHEAD): iteration v issues x(v + A) then rec(v + 2A); the prologue runs
    // v = -A .. -1 after rec(0 .. A-1) have landed. At iteration w, x(w) and rec(w + A) (both
    // issued by iteration w - A) must have landed: A - 1 later iterations of NI + 2 loads each
    // may still be in flight. Ring slots: x(w + A) takes a slot no window in [w, w + A) holds
    // (NX >= A + 1), rec(w + 2A) one no record window in [w, w + 2A) holds (NR >= 2A + 1); with
    // the minimum sizes that is window w - 1's. The LDS-DMA is hidden from the compiler
    // (dma4 / dma16): its LDS reads are then ordinary, scheduled and counted by it, and the
    // explicit vmcnt waits (asm, "memory") keep them behind the data they read.
    static_assert(NX >= AHEAD + 1 && NR >= 2 * AHEAD + 1, "ring sizes");
    float acc = 0.f;
    if (nwin > 0) {  // (an empty row — live-edge rows may have none — reads no record)
    for (int w = 0; w < AHEAD; ++w) rec_dma(w);
    wait_vm<0>();
    for (int v = -AHEAD; v < 0; ++v) {
        x_dma(v + AHEAD);
        rec_dma(v + 2 * AHEAD);
    }
    const int cc = lane < W ? lane : 0;
    for (int32_t w = 0; w < nwin; ++w) {
        wait_vm<(AHEAD - 1) * (C::NI + 2)>();
        x_dma(w + AHEAD);
        rec_dma(w + 2 * AHEAD);
        const int n = min(64, end - beg - 64 * w);
        const float* xs = &s_x[w % NX][cc];  // step j's element of column cc: xs[j * W]
        const float4* vs = reinterpret_cast<const float4*>(s_val[w % NR]);  // broadcast reads
        // groups of 8 steps, two groups' LDS reads (2 x 16-B edge values + 8 X elements, the
        // latter paired by ds_read2) issued ahead of the group being folded; the sched_barriers
        // keep the compiler from sinking them next to their use
        float xg[3][8];
        float4 vg[3][2];
        auto load8 = [&](int slot, int g) {
#pragma unroll
            for (int t = 0; t < 8; ++t) xg[slot][t] = xs[(8 * g + t) * W];
            vg[slot][0] = vs[2 * g];
            vg[slot][1] = vs[2 * g + 1];
        };
        auto fold8 = [&](int slot, int g, bool full) {
            const float vv[8] = {vg[slot][0].x, vg[slot][0].y, vg[slot][0].z, vg[slot][0].w,
                                 vg[slot][1].x, vg[slot][1].y, vg[slot][1].z, vg[slot][1].w};
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                float xe = xg[slot][t];
                if constexpr ((XD & 3) == 1) xe = xe / xdiv;
                else if constexpr ((XD & 3) == 2) xe = xe * xdiv;
                const float f = __builtin_fmaf(vv[t], xe, acc);
                acc = (full || 8 * g + t < n) ? f : acc;
            }
        };
        load8(0, 0);
        load8(1, 1);
        if (n == 64) {
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                if (g + 2 < 8) load8((g + 2) % 3, g + 2);
                __builtin_amdgcn_sched_barrier(0);
                fold8(g % 3, g, true);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {  // the row's last window: steps past n leave acc alone
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                if (g + 2 < 8) load8((g + 2) % 3, g + 2);
                __builtin_amdgcn_sched_barrier(0);
                fold8(g % 3, g, false);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    wait_vm<0>();  // no LDS-DMA may land after the wave (and its LDS) is gone
    }
    if (lane >= W || c0 + lane >= d) return;
    const int c = c0 + lane;
    const int32_t row = er.row;
    float out = acc;
    if constexpr (MODE == LGCN_EPI_ROWS) {  // the chain value itself, to row i of the list
        y[(int64_t)rix * ldy + c] = out;
        return;
    }
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
    // (16- and 8-column slices: the d/P columns of a featsplit shard — d=64 at P=4, P=8)
    const int w = d % 32 == 0 ? 32 : d % 16 == 0 ? 16 : 8;  // d % 8 == 0 (checked by the caller)
    const dim3 grid = LGCN_GRID_DIM((uint32_t)((d + w - 1) / w), (uint32_t)n_rows);
    const bool seg1 = x.p0 == x.p1 && x.p1 == x.p2;
#define LGCN_CH(W_, S_) \
    hipLaunchKernelGGL((k_chain_rows<MODE, XD, W_, S_>), grid, dim3(64), 0, s, edges, blocks, \
                       rows, x, xdiv, d, y, ldy, ep)
    if (w == 32) {
        if (seg1) LGCN_CH(32, true);
        else LGCN_CH(32, false);
    } else if (w == 16) {
        if (seg1) LGCN_CH(16, true);
        else LGCN_CH(16, false);
    } else {
        if (seg1) LGCN_CH(8, true);
        else LGCN_CH(8, false);
    }
#undef LGCN_CH
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
// The epilogue of emulated rows a walk / chain wrote with LGCN_EPI_ROWS (their chain values, row
// i of the list in tmp row i), applied once the epilogue's operands are ready: the same
// arithmetic, in the same order, as the kernels' own epilogue.
template <int MODE>
__global__ __launch_bounds__(256) void k_emu_epilogue(const lgcn_emu_row_t* __restrict__ rows,
                                                      const float* __restrict__ tmp, int64_t ldt,
                                                      float* __restrict__ y, int64_t ldy,
                                                      int32_t d, lgcn_epilogue_t ep) {
    const int32_t row = rows[blockIdx.x].row;
    for (int c = threadIdx.x; c < d; c += blockDim.x) {
        float out = tmp[(int64_t)blockIdx.x * ldt + c];
        if constexpr (MODE == LGCN_EPI_MEAN) {
            float s = seg_row_x(ep.prev0, row)[c];
            for (int i = 0; i + 1 < ep.n_prev; ++i)
                s = s + ep.prev_dense[i][(int64_t)row * ep.ld_prev + c];
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
}

// ---------------------------------------------------------------------------------------------
// row-sparse X (the backward's first layer on a BPR batch's gradient): emulated rows as chains
// over their LIVE edges only
// ---------------------------------------------------------------------------------------------
// An edge into an all-zero row of X adds fma(v, +-0, acc) == acc to the chain (v finite: the
// chain value is unchanged, +0 stays +0), so the reference's chain over a row equals the chain
// over its live edges in stored order. A BPR batch leaves a few thousand live rows of millions,
// so a 2.77M-edge row keeps a few hundred live edges: compacted (three launches over the rows'
// blocks, no host sync) they run as ordinary chain rows (k_chain_rows) — no block pass, no walk.
// Edges with a non-finite value are kept (inf * 0 is NaN in the reference's chain too).
//
// Scratch layout (lgcn_live_scratch_bytes): int32 off[n_blocks] | lgcn_emu_row_t lrows[n_rows] |
// lgcn_emu_block_t lblocks[n_rows] | lgcn_edge_t ledges[n_blocks * LGCN_EMU_BLOCK]; emulated row
// i's live edges go to ledges[first_block_i * LGCN_EMU_BLOCK ...] (its blocks' own span).
struct LiveScratch {
    int32_t* off;
    lgcn_emu_row_t* lrows;
    lgcn_emu_block_t* lblocks;
    lgcn_edge_t* ledges;
};

__host__ __device__ inline size_t live_align(size_t b) { return (b + 255) & ~(size_t)255; }

__host__ __device__ inline LiveScratch live_layout(void* base, int32_t n_rows, int32_t n_blocks) {
    char* p = static_cast<char*>(base);
    LiveScratch s;
    s.off = reinterpret_cast<int32_t*>(p);
    p += live_align((size_t)n_blocks * 4);
    s.lrows = reinterpret_cast<lgcn_emu_row_t*>(p);
    p += live_align((size_t)n_rows * sizeof(lgcn_emu_row_t));
    s.lblocks = reinterpret_cast<lgcn_emu_block_t*>(p);
    p += live_align((size_t)n_rows * sizeof(lgcn_emu_block_t));
    s.ledges = reinterpret_cast<lgcn_edge_t*>(p);
    return s;
}

inline size_t live_bytes(int32_t n_rows, int32_t n_blocks) {
    return live_align((size_t)n_blocks * 4) + live_align((size_t)n_rows * sizeof(lgcn_emu_row_t)) +
           live_align((size_t)n_rows * sizeof(lgcn_emu_block_t)) +
           (size_t)n_blocks * LGCN_EMU_BLOCK * sizeof(lgcn_edge_t);
}

// lane l's 4 edges of block b (steps 4l .. 4l+3): live flags (bit k) and the records
__device__ __forceinline__ int live_flags(const lgcn_edge_t* __restrict__ edges,
                                          const lgcn_emu_block_t& blk,
                                          const uint32_t* __restrict__ x_nz, int2 (&rec)[4]) {
    const int lane = threadIdx.x;
    int f = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int32_t j = blk.beg + 4 * lane + k;
        const bool in = j < blk.end;
        rec[k] = *reinterpret_cast<const int2*>(edges + (in ? j : blk.beg));
        const float v = __int_as_float(rec[k].y);
        const bool live = in && (row_live_x(x_nz, rec[k].x) || !__builtin_isfinite(v));
        f |= live ? (1 << k) : 0;
    }
    return f;
}

// per block: its live-edge count -> off[b]
__global__ __launch_bounds__(64) void k_live_count(const lgcn_edge_t* __restrict__ edges,
                                                   const lgcn_emu_block_t* __restrict__ blocks,
                                                   const uint32_t* __restrict__ x_nz,
                                                   int32_t* __restrict__ off) {
    int2 rec[4];
    const int f = live_flags(edges, blocks[blockIdx.x], x_nz, rec);
    const int tot = wave_incl_scan(__builtin_popcount((unsigned)f));
    if (threadIdx.x == 63) off[blockIdx.x] = tot;
}

// per emulated row (256 threads): exclusive scan of its blocks' counts in place, and the row's
// descriptors of the compacted edges (one block per row, lgcn_chain_rows reads its span)
__global__ __launch_bounds__(256) void k_live_scan(const lgcn_emu_row_t* __restrict__ rows,
                                                   int32_t* __restrict__ off,
                                                   lgcn_emu_row_t* __restrict__ lrows,
                                                   lgcn_emu_block_t* __restrict__ lblocks,
                                                   int32_t live_min, int32_t max_live) {
    __shared__ int32_t s_wave[4];
    __shared__ int32_t s_carry;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const lgcn_emu_row_t er = rows[blockIdx.x];
    if (t == 0) s_carry = 0;
    __syncthreads();
    for (int32_t b0 = 0; b0 < er.n_blocks; b0 += 256) {
        const int32_t b = b0 + t;
        const int32_t c = b < er.n_blocks ? off[er.first_block + b] : 0;
        const int incl = wave_incl_scan(c);
        if (lane == 63) s_wave[w] = incl;
        __syncthreads();
        int base = s_carry;
        for (int i = 0; i < w; ++i) base += s_wave[i];
        const int tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
        if (b < er.n_blocks) off[er.first_block + b] = base + incl - c;
        __syncthreads();
        if (t == 0) s_carry += tot;
        __syncthreads();
    }
    if (t == 0) {
        const int32_t beg = er.first_block * LGCN_EMU_BLOCK;
        // n_blocks = 1: the live-edge chain runs the row; 0: left to the caller (block pass +
        // walk skip the rows flagged 1)
        // (a walk costs ~0.45 us per block, a chain ~1.2 us per 64 edges: 16 live edges per
        // block is where the chain stops paying)
        const bool mine = (int32_t)blockIdx.x >= live_min ||
                          (int64_t)s_carry <= min((int64_t)max_live, (int64_t)er.n_blocks * 16);
        lrows[blockIdx.x] = lgcn_emu_row_t{er.row, (int32_t)blockIdx.x, mine ? 1 : 0, 0};
        lblocks[blockIdx.x] = lgcn_emu_block_t{(int32_t)blockIdx.x, beg, beg + s_carry, 1};
    }
}

// per block: its live edges, in stored order, to the row's compacted span
__global__ __launch_bounds__(64) void k_live_scatter(const lgcn_edge_t* __restrict__ edges,
                                                     const lgcn_emu_block_t* __restrict__ blocks,
                                                     const lgcn_emu_row_t* __restrict__ rows,
                                                     const uint32_t* __restrict__ x_nz,
                                                     const int32_t* __restrict__ off,
                                                     const lgcn_emu_row_t* __restrict__ lrows,
                                                     lgcn_edge_t* __restrict__ ledges) {
    const lgcn_emu_block_t blk = blocks[blockIdx.x];
    if (!lrows[blk.row].n_blocks) return;  // the walk's row
    int2 rec[4];
    const int f = live_flags(edges, blk, x_nz, rec);
    const int cnt = __builtin_popcount((unsigned)f);
    int pos = wave_incl_scan(cnt) - cnt;
    const int64_t base = (int64_t)rows[blk.row].first_block * LGCN_EMU_BLOCK + off[blockIdx.x];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if ((f >> k) & 1) {
            *reinterpret_cast<int2*>(ledges + base + pos) = rec[k];
            ++pos;
        }
    }
}

}  // namespace

extern "C" {

#if defined(LGCN_EMU_STATS) || defined(LGCN_EMU_MODES)
int lgcn_emu_set_mode(int mode) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_emu_mode), &mode, sizeof(int)) == hipSuccess ? 0 : -1;
}
int lgcn_emu_set_blk_mode(int mode) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_blk_mode), &mode, sizeof(int)) == hipSuccess ? 0 : -1;
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
                    void* meta, float* stage, const lgcn_emu_row_t* live, void* stream) {
    if (n_blocks < 0 || d < 1 || d > 2048 || !(x_div > 0.f)) return LGCN_EINVAL;
    if (n_blocks == 0) return 0;
    if (!edges || !blocks || !rel || !meta || !x.p0) return LGCN_EINVAL;
    if ((reinterpret_cast<uintptr_t>(rel) & 15) || (reinterpret_cast<uintptr_t>(meta) & 15) ||
        (reinterpret_cast<uintptr_t>(stage) & 15))
        return LGCN_EALIGN;
    const int xd = xd_of(x_div, x_nz);
    const float xa = (xd & 3) == 2 ? 1.0f / x_div : x_div;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int4* mp = static_cast<int4*>(meta);
    int4* kp = reinterpret_cast<int4*>(rel);
#ifdef LGCN_EXP_NOSTAGE  // timing experiment only (wrong results): no stage writes after N calls
    static int calls = 0;
    if (++calls > LGCN_EXP_NOSTAGE) stage = nullptr;
#endif
#define LGCN_B(XD_) \
    case XD_: return launch_blocks<XD_>(edges, blocks, n_blocks, x, xa, x_nz, d, kp, mp, stage, live, s);
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
                  const lgcn_emu_row_t* live, void* stream) {
    if (slots == 0) slots = LGCN_EMU_SLOTS;
    // static LDS (two translation tables, 8 KB) + (2 slots + 1) x 2 KB within 64 KB
    if (n_rows < 0 || d < 1 || d > 2048 || !(x_div > 0.f) || !epi_host || slots < 1 ||
        slots > LGCN_EMU_MAX_SLOTS)
        return LGCN_EINVAL;
    if (n_rows == 0) return 0;
    if (!edges || !blocks || !rows || !rel || !meta || !y || ldy < d || !x.p0) return LGCN_EINVAL;
    if ((reinterpret_cast<uintptr_t>(rel) & 15) || (reinterpret_cast<uintptr_t>(meta) & 15) ||
        (reinterpret_cast<uintptr_t>(stage) & 15))
        return LGCN_EALIGN;
    lgcn_epilogue_t ep = *epi_host;
    if (ep.mode == LGCN_EPI_MEAN && (ep.n_prev < 1 || ep.n_prev - 1 > LGCN_MAX_LAYERS))
        return LGCN_EINVAL;
    if (ep.mode == LGCN_EPI_ADD && !ep.addend.p0) return LGCN_EINVAL;
    if ((ep.mode == LGCN_EPI_MEAN || ep.mode == LGCN_EPI_ADD) && !(ep.div > 0.f)) return LGCN_EINVAL;
    if (ep.mode < LGCN_EPI_STORE || ep.mode > LGCN_EPI_ROWS) return LGCN_EINVAL;
    // a power-of-two divisor becomes a multiply by its exact reciprocal (same rounding)
    if ((ep.mode == LGCN_EPI_MEAN || ep.mode == LGCN_EPI_ADD) && is_pow2(ep.div)) {
        const float inv = 1.0f / ep.div;
        memcpy(&ep.pad, &inv, sizeof(inv));
    } else {
        ep.pad = 0;
    }
    const int xd = xd_of(x_div, x_nz);
    const float xa = (xd & 3) == 2 ? 1.0f / x_div : x_div;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int4* mp = static_cast<const int4*>(meta);
    const int4* kp = reinterpret_cast<const int4*>(rel);
    switch (ep.mode) {
        case LGCN_EPI_STORE:
            return walk_mode<LGCN_EPI_STORE>(xd, edges, blocks, rows, n_rows, kp, mp, stage, x, xa, x_nz, y, ldy, d, ep, slots, live, s);
        case LGCN_EPI_MEAN:
            return walk_mode<LGCN_EPI_MEAN>(xd, edges, blocks, rows, n_rows, kp, mp, stage, x, xa, x_nz, y, ldy, d, ep, slots, live, s);
        case LGCN_EPI_ADD:
            return walk_mode<LGCN_EPI_ADD>(xd, edges, blocks, rows, n_rows, kp, mp, stage, x, xa, x_nz, y, ldy, d, ep, slots, live, s);
        case LGCN_EPI_ROWS:  // (a forward's deferred mean: X read as is)
            return xd == 0 ? launch_walk<LGCN_EPI_ROWS, 0>(edges, blocks, rows, n_rows, kp, mp, stage, x, xa, x_nz, y, ldy, d, ep, slots, live, s) : LGCN_EINVAL;
        default:
            return LGCN_EINVAL;
    }
}

int lgcn_emu_epilogue(const lgcn_emu_row_t* rows, int32_t n_rows, const float* tmp, int64_t ld_tmp,
                      float* y, int64_t ldy, int32_t d, const lgcn_epilogue_t* epi_host,
                      void* stream) {
    if (n_rows < 0 || d < 1 || d > 2048 || !epi_host) return LGCN_EINVAL;
    if (n_rows == 0) return 0;
    if (!rows || !tmp || !y || ld_tmp < d || ldy < d) return LGCN_EINVAL;
    lgcn_epilogue_t ep = *epi_host;
    if (ep.mode < LGCN_EPI_STORE || ep.mode > LGCN_EPI_ADD) return LGCN_EINVAL;
    if (ep.mode == LGCN_EPI_MEAN && (ep.n_prev < 1 || ep.n_prev - 1 > LGCN_MAX_LAYERS))
        return LGCN_EINVAL;
    if (ep.mode == LGCN_EPI_ADD && !ep.addend.p0) return LGCN_EINVAL;
    if ((ep.mode == LGCN_EPI_MEAN || ep.mode == LGCN_EPI_ADD) && !(ep.div > 0.f)) return LGCN_EINVAL;
    if ((ep.mode == LGCN_EPI_MEAN || ep.mode == LGCN_EPI_ADD) && is_pow2(ep.div)) {
        const float inv = 1.0f / ep.div;
        memcpy(&ep.pad, &inv, sizeof(inv));
    } else {
        ep.pad = 0;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((uint32_t)n_rows), block((uint32_t)std::min(d, 256));
    switch (ep.mode) {
        case LGCN_EPI_STORE:
            hipLaunchKernelGGL(k_emu_epilogue<LGCN_EPI_STORE>, grid, block, 0, s, rows, tmp, ld_tmp, y, ldy, d, ep);
            break;
        case LGCN_EPI_MEAN:
            hipLaunchKernelGGL(k_emu_epilogue<LGCN_EPI_MEAN>, grid, block, 0, s, rows, tmp, ld_tmp, y, ldy, d, ep);
            break;
        default:
            hipLaunchKernelGGL(k_emu_epilogue<LGCN_EPI_ADD>, grid, block, 0, s, rows, tmp, ld_tmp, y, ldy, d, ep);
            break;
    }
    return herr_x(hipGetLastError());
}

int lgcn_chain_supported(int32_t d) { return d > 0 && d <= 2048 && d % 8 == 0; }

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
    if ((ep.mode == LGCN_EPI_MEAN || ep.mode == LGCN_EPI_ADD) && !(ep.div > 0.f)) return LGCN_EINVAL;
    if (ep.mode < LGCN_EPI_STORE || ep.mode > LGCN_EPI_ROWS) return LGCN_EINVAL;
    if ((ep.mode == LGCN_EPI_MEAN || ep.mode == LGCN_EPI_ADD) && is_pow2(ep.div)) {
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
        case LGCN_EPI_ROWS:
            return xd == 0 ? launch_chain<LGCN_EPI_ROWS, 0>(edges, blocks, rows, n_rows, x, xa, y, ldy, d, ep, s) : LGCN_EINVAL;
        default: return LGCN_EINVAL;
    }
}

}  // extern "C"

extern "C" {

size_t lgcn_live_scratch_bytes(int32_t n_rows, int32_t n_blocks) {
    if (n_rows < 0 || n_blocks < 0) return 0;
    return live_bytes(n_rows, n_blocks);
}

const lgcn_emu_row_t* lgcn_live_flags(const void* scratch, int32_t n_rows, int32_t n_blocks) {
    if (!scratch || n_rows < 0 || n_blocks < 0) return nullptr;
    return live_layout(const_cast<void*>(scratch), n_rows, n_blocks).lrows;
}

int lgcn_live_rows(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks, int32_t n_blocks,
                   const lgcn_emu_row_t* rows, int32_t n_rows, lgcn_rows_t x, float x_div,
                   const uint32_t* x_nz, float* y, int64_t ldy, int32_t d,
                   const lgcn_epilogue_t* epi_host, int32_t live_min, int32_t max_live,
                   void* scratch, void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (int e = lgcn_detail::live_prepare(edges, blocks, n_blocks, rows, n_rows, x_nz, d, x_div,
                                          epi_host, y, ldy, x.p0, live_min, max_live, scratch, s))
        return e;
    return lgcn_detail::live_chains(n_blocks, n_rows, x, x_div, y, ldy, d, epi_host, scratch, s);
}

}  // extern "C"

namespace lgcn_detail {

int live_prepare(const lgcn_edge_t* edges, const lgcn_emu_block_t* blocks, int32_t n_blocks,
                 const lgcn_emu_row_t* rows, int32_t n_rows, const uint32_t* x_nz, int32_t d,
                 float x_div, const lgcn_epilogue_t* epi_host, float* y, int64_t ldy,
                 const void* x_p0, int32_t live_min, int32_t max_live, void* scratch,
                 hipStream_t s) {
    if (n_rows < 0 || n_blocks < 0 || !lgcn_chain_supported(d) || d > 2048 || !x_nz ||
        !(x_div > 0.f) || !epi_host)
        return LGCN_EINVAL;
    if (n_rows == 0) return 0;
    if (!edges || !blocks || !rows || !y || !scratch || ldy < d || !x_p0 || n_blocks < n_rows)
        return LGCN_EINVAL;
    // compacted spans are indexed by first_block * LGCN_EMU_BLOCK in int32 edge offsets
    if ((int64_t)n_blocks * LGCN_EMU_BLOCK > INT32_MAX) return LGCN_EINVAL;
    if (reinterpret_cast<uintptr_t>(scratch) & 255) return LGCN_EALIGN;
    const LiveScratch ls = live_layout(scratch, n_rows, n_blocks);
    hipLaunchKernelGGL(k_live_count, dim3((uint32_t)n_blocks), dim3(64), 0, s, edges, blocks, x_nz,
                       ls.off);
    if (int e = herr_x(hipGetLastError())) return e;
    hipLaunchKernelGGL(k_live_scan, dim3((uint32_t)n_rows), dim3(256), 0, s, rows, ls.off,
                       ls.lrows, ls.lblocks, live_min, max_live);
    if (int e = herr_x(hipGetLastError())) return e;
    hipLaunchKernelGGL(k_live_scatter, dim3((uint32_t)n_blocks), dim3(64), 0, s, edges, blocks,
                       rows, x_nz, ls.off, ls.lrows, ls.ledges);
    return herr_x(hipGetLastError());
}

int live_chains(int32_t n_blocks, int32_t n_rows, lgcn_rows_t x, float x_div, float* y,
                int64_t ldy, int32_t d, const lgcn_epilogue_t* epi_host, void* scratch,
                hipStream_t s) {
    if (n_rows <= 0) return n_rows < 0 ? LGCN_EINVAL : 0;
    const LiveScratch ls = live_layout(scratch, n_rows, n_blocks);
    return lgcn_chain_rows(ls.ledges, ls.lblocks, ls.lrows, n_rows, x, x_div, y, ldy, d, epi_host,
                           s);
}

}  // namespace lgcn_detail
