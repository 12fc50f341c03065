// lgcn_eval.hip — fused evaluation for gfx950: scores = user rows · item tableᵀ, training items
// masked to -1e10, top-K per user (the semantics of the reference's evaluate, main.py:404-439:
// matmul :420, mask loop :422-424, topk :426), without materialising the [users x items] score
// matrix (1024 x 4.4M fp32 = 18 GB per batch at Books scale).
//
//  * scores: exact-f32 MFMA v_mfma_f32_32x32x2_f32 (A = 32 users, B = 32 items, K = d): each
//    score is an ordered fmaf chain over the d features (feature order 0,32,1,33,… at d = 64);
//  * a block = 4 waves x 32 users; every wave streams the SAME item split (L1/L2 reuse), so the
//    item table is read once per 128 users; grid = user tiles x item splits;
//  * top-K: a lane keeps the current K-th best score of its 16 users in registers; only scores
//    above it are candidates (after the first few tiles, ~K·ln(items/K) per user in total): the
//    train-item mask is a binary search in the user's sorted list, done for candidates only;
//    candidates go to a per-user LDS buffer (capacity 64); users whose buffer passes 32 are
//    compacted to their K best by rank counting under the total order (score desc, index asc):
//    deterministic regardless of LDS arrival order;
//  * k_topk_merge: per user, the splits' K-th scores bound the global K-th from below, so only
//    candidates >= max_s kth_s are ranked.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "lgcn.h"

namespace {

#ifndef LGCN_EVAL_WAVES
#define LGCN_EVAL_WAVES 4
#endif
constexpr int kWaves = LGCN_EVAL_WAVES;  // waves (x 32 users) per block: they share item tiles
constexpr int kUsersPerWave = 32;
constexpr int kCap = 64;     // candidate buffer per user
constexpr int kCompact = 32; // compact when a buffer holds more than this (one tile adds <= 32)
constexpr float kMasked = -1e10f;
constexpr int kLgkm0 = 0xC07F;  // s_waitcnt lgkmcnt(0) only (vmcnt/expcnt left alone)

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ bool better(float s1, int i1, float s2, int i2) {
    return s1 > s2 || (s1 == s2 && i1 < i2);
}

__device__ __forceinline__ bool in_sorted(const int32_t* __restrict__ a, int32_t lo, int32_t hi,
                                          int32_t x) {
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        const int32_t v = a[mid];
        if (v == x) return true;
        if (v < x) lo = mid + 1; else hi = mid;
    }
    return false;
}

struct WaveState {
    float score[kUsersPerWave][kCap];
    int32_t idx[kUsersPerWave][kCap];
    int32_t cnt[kUsersPerWave];
    float thr[kUsersPerWave];
    int32_t mlo[kUsersPerWave];  // the user's train items: mask_items[mlo, mhi); mhi < mlo: no user
    int32_t mhi[kUsersPerWave];
};

// Keep the K best of user u's buffer (entries at ranks >= K dropped), set its threshold.
__device__ void compact_user(WaveState& st, int u, int K, int lane) {
    const int n = st.cnt[u];
    float s0 = 0.f;
    int i0 = 0, r0 = kCap;
    static_assert(kCap <= 64, "one buffer entry per lane");
    if (lane < n) { s0 = st.score[u][lane]; i0 = st.idx[u][lane]; r0 = 0; }
    for (int m = 0; m < n; ++m) {
        const float sm = st.score[u][m];
        const int im = st.idx[u][m];
        if (lane < n && better(sm, im, s0, i0)) ++r0;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(kLgkm0);  // every lane has read the old buffer
    __builtin_amdgcn_wave_barrier();
    if (lane < n && r0 < K) { st.score[u][r0] = s0; st.idx[u][r0] = i0; }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        const int keep = n < K ? n : K;
        st.cnt[u] = keep;
        st.thr[u] = keep == K ? st.score[u][K - 1] : -INFINITY;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_wave_barrier();
}

template <int D>
__global__ __launch_bounds__(kWaves * 64) void k_score_topk(
    const float* __restrict__ uemb, int64_t ld_u, const int32_t* __restrict__ users,
    int32_t n_users, const float* __restrict__ iemb, int64_t ld_i, int32_t n_items,
    int32_t split_len, const int32_t* __restrict__ mrow, const int32_t* __restrict__ mitems, int K,
    float* __restrict__ part_s, int32_t* __restrict__ part_i) {
    constexpr int DH = D / 2;  // features per lane half
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int col = lane & 31;
    WaveState& st = reinterpret_cast<WaveState*>(smem)[wave];
    const int32_t ub = (blockIdx.x * kWaves + wave) * kUsersPerWave;  // first user slot
    const int32_t split = blockIdx.y;
    const int32_t it0 = split * split_len;
    const int32_t it1 = min(n_items, it0 + split_len);

    if (lane < kUsersPerWave) {
        st.cnt[lane] = 0;
        st.thr[lane] = -INFINITY;
    }
    // A operand: user (ub + col), features [h*DH, h*DH + DH)
    float a[DH];
    {
        const bool ok = ub + col < n_users;
        const float* ur = uemb + (ok ? (int64_t)users[ub + col] * ld_u : 0) + h * DH;
#pragma unroll
        for (int q = 0; q < DH / 4; ++q) {
            const float4 v = ok ? *reinterpret_cast<const float4*>(ur + 4 * q)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
            a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
        }
    }
    if (lane < kUsersPerWave) {
        const bool ok = ub + lane < n_users;
        const int32_t u = ok ? users[ub + lane] : 0;
        st.mlo[lane] = ok ? mrow[u] : 0;
        st.mhi[lane] = ok ? mrow[u + 1] : -1;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_wave_barrier();
    // rows of the C/D tile this lane holds: user (ub + row(r)), row(r) = (r&3)+8(r>>2)+4h.
    // The B operand (32 items x this lane's feature half) is double-buffered: the next tile's
    // loads are in flight during the current tile's MFMA chain.
    float4 bcur[DH / 4], bnxt[DH / 4];
    auto load_tile = [&](int32_t t0, float4 (&b)[DH / 4]) {
        const int32_t item = t0 + col;
        const bool iok = item < it1;
        const float* ir = iemb + (iok ? (int64_t)item * ld_i : 0) + h * DH;
#pragma unroll
        for (int q = 0; q < DH / 4; ++q)
            b[q] = iok ? *reinterpret_cast<const float4*>(ir + 4 * q)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    if (it0 < it1) load_tile(it0, bcur);

    for (int32_t t0 = it0; t0 < it1; t0 += 32) {
        if (t0 + 32 < it1) load_tile(t0 + 32, bnxt);
        const int32_t item = t0 + col;
        const bool iok = item < it1;
        f32x16 acc = {};
#pragma unroll
        for (int q = 0; q < DH / 4; ++q) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * q], bcur[q].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * q + 1], bcur[q].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * q + 2], bcur[q].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * q + 3], bcur[q].w, acc, 0, 0, 0);
        }
        bool any = false;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            float sc = acc[r];
            const float thr = st.thr[row];
            if (iok && sc > thr) {
                const int32_t lo = st.mlo[row], hi = st.mhi[row];
                if (hi >= lo) {
                    if (in_sorted(mitems, lo, hi, item)) sc = kMasked;  // main.py:422-424
                    if (sc > thr) {
                        const int pos = atomicAdd(&st.cnt[row], 1);
                        st.score[row][pos] = sc;
                        st.idx[row][pos] = item;
                        any = true;
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(kLgkm0);
        __builtin_amdgcn_wave_barrier();
        if (__any(any)) {
            // compact every user whose buffer could overflow on the next tile
            uint64_t need = __ballot(lane < kUsersPerWave && st.cnt[lane] > kCompact);
            while (need) {
                const int u = __builtin_ctzll(need);
                need &= need - 1;
                compact_user(st, u, K, lane);
            }
        }
#pragma unroll
        for (int q = 0; q < DH / 4; ++q) bcur[q] = bnxt[q];
    }
    // final: every buffer to its K best in rank order, written to this split's partial list
    for (int u = 0; u < kUsersPerWave; ++u) {
        if (ub + u >= n_users) break;
        compact_user(st, u, K, lane);
        const int n = st.cnt[u];
        if (lane < K) {
            const int64_t o = ((int64_t)split * n_users + ub + u) * K + lane;
            part_s[o] = lane < n ? st.score[u][lane] : -INFINITY;
            part_i[o] = lane < n ? st.idx[u][lane] : -1;
        }
    }
}

// One wave per user: merge the splits' K-best lists. The global K-th score is >= every split's
// K-th score, so only candidates >= max_s kth_s are ranked (always >= K of them exist).
__global__ __launch_bounds__(64) void k_topk_merge(const float* __restrict__ part_s,
                                                   const int32_t* __restrict__ part_i,
                                                   int32_t n_users, int32_t n_splits, int K,
                                                   float* __restrict__ top_s,
                                                   int32_t* __restrict__ top_i) {
    extern __shared__ __attribute__((aligned(16))) char msm[];  // n_splits*K (score, idx) pairs
    float* cs = reinterpret_cast<float*>(msm);
    int32_t* ci = reinterpret_cast<int32_t*>(msm) + n_splits * K;
    __shared__ int ncand;
    const int u = blockIdx.x;
    const int lane = threadIdx.x;
    float t = -INFINITY;
    for (int s = lane; s < n_splits; s += 64) {
        const float v = part_s[((int64_t)s * n_users + u) * K + K - 1];
        t = fmaxf(t, v);
    }
    for (int off = 32; off > 0; off >>= 1) t = fmaxf(t, __shfl_xor(t, off));
    if (lane == 0) ncand = 0;
    __syncthreads();
    const int total = n_splits * K;
    for (int e = lane; e < total; e += 64) {
        const int s = e / K, j = e - s * K;
        const int64_t o = ((int64_t)s * n_users + u) * K + j;
        const float v = part_s[o];
        const int32_t id = part_i[o];
        if (id >= 0 && v >= t) {
            const int p = atomicAdd(&ncand, 1);
            cs[p] = v;
            ci[p] = id;
        }
    }
    __syncthreads();
    const int n = ncand;
    for (int e = lane; e < n; e += 64) {
        int rank = 0;
        for (int m = 0; m < n; ++m) rank += better(cs[m], ci[m], cs[e], ci[e]) ? 1 : 0;
        if (rank < K) {
            top_s[(int64_t)u * K + rank] = cs[e];
            top_i[(int64_t)u * K + rank] = ci[e];
        }
    }
    for (int r = n + lane; r < K; r += 64) {  // fewer than K items in total
        top_s[(int64_t)u * K + r] = -INFINITY;
        top_i[(int64_t)u * K + r] = -1;
    }
}

}  // namespace

extern "C" {

int lgcn_eval_splits(int32_t n_users, int32_t n_items, int32_t n_cu) {
    // enough (user tile x split) blocks for ~2 per CU, splits of >= 2048 items, <= 256 splits
    const int64_t tiles = ((int64_t)n_users + kWaves * kUsersPerWave - 1) / (kWaves * kUsersPerWave);
    int64_t s = (2LL * (n_cu > 0 ? n_cu : 256) + tiles - 1) / (tiles > 0 ? tiles : 1);
    const int64_t max_by_len = ((int64_t)n_items + 2047) / 2048;
    if (s > max_by_len) s = max_by_len;
    if (s > 256) s = 256;
    if (s < 1) s = 1;
    return (int)s;
}

int lgcn_score_topk(const float* user_emb, int64_t ld_u, const int32_t* users, int32_t n_users,
                    const float* item_emb, int64_t ld_i, int32_t n_items, int32_t d,
                    const int32_t* mask_rowptr, const int32_t* mask_items, int32_t k,
                    int32_t n_splits, float* part_scores, int32_t* part_idx, float* top_scores,
                    int32_t* top_idx, void* stream) {
    if (n_users < 0 || n_items < 0 || k < 1 || k > kCompact || n_splits < 1 || n_splits > 256)
        return LGCN_EINVAL;
    if (d != 32 && d != 64 && d != 128 && d != 256) return LGCN_EINVAL;
    if (ld_u % 4 || ld_i % 4 || (reinterpret_cast<uintptr_t>(user_emb) & 15) ||
        (reinterpret_cast<uintptr_t>(item_emb) & 15))
        return LGCN_EALIGN;
    if (n_users == 0) return 0;
    if (!user_emb || !users || !item_emb || !mask_rowptr || !part_scores || !part_idx ||
        !top_scores || !top_idx)
        return LGCN_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int32_t split_len = (int32_t)(((int64_t)n_items + n_splits - 1) / n_splits);
    split_len = ((split_len + 31) / 32) * 32;
    if (split_len == 0) split_len = 32;
    const dim3 grid((n_users + kWaves * kUsersPerWave - 1) / (kWaves * kUsersPerWave), n_splits);
    const size_t lds = sizeof(WaveState) * kWaves;
    const void* fn = d == 32    ? reinterpret_cast<const void*>(k_score_topk<32>)
                     : d == 64  ? reinterpret_cast<const void*>(k_score_topk<64>)
                     : d == 128 ? reinterpret_cast<const void*>(k_score_topk<128>)
                                : reinterpret_cast<const void*>(k_score_topk<256>);
    {
        const hipError_t ea =
            hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ea != hipSuccess) return (int)ea;
    }
#define LGCN_SCORE_LAUNCH(D_)                                                                   \
    hipLaunchKernelGGL(k_score_topk<D_>, grid, dim3(kWaves * 64), lds, s, user_emb, ld_u, users, \
                       n_users, item_emb, ld_i, n_items, split_len, mask_rowptr, mask_items, k,  \
                       part_scores, part_idx)
    switch (d) {
        case 32: LGCN_SCORE_LAUNCH(32); break;
        case 64: LGCN_SCORE_LAUNCH(64); break;
        case 128: LGCN_SCORE_LAUNCH(128); break;
        default: LGCN_SCORE_LAUNCH(256); break;
    }
#undef LGCN_SCORE_LAUNCH
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    const size_t mlds = (size_t)n_splits * k * 8;
    hipLaunchKernelGGL(k_topk_merge, dim3(n_users), dim3(64), mlds, s, part_scores, part_idx,
                       n_users, n_splits, k, top_scores, top_idx);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"
