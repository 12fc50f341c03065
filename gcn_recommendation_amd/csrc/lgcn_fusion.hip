// lgcn_fusion.hip — the LightGCN_Fusion item pre-layer for gfx950 (reference
// models/lightgcn_fusion.py:45-49):
//     fused = leaky_relu(Linear(cat([item_id_emb, item_content_emb], 1)))
// as ONE kernel: the [I x (d+C)] concatenation is never written (each lane reads its half of a
// row straight from the two tables), the GEMM runs on exact-f32 MFMA (v_mfma_f32_32x32x2_f32),
// and bias + leaky_relu are applied to the accumulators before the single store of [I x d].
//
//  * block = 4 waves (one per SIMD), persistent over 32-row tiles, the next tile's rows loaded
//    during the current tile's MFMAs; the Linear weight W [d x (d+C)] is staged
//    once per block into LDS transposed (k-major, the two k halves 32 banks apart: conflict-free
//    reads of 32 consecutive output columns per half-wave);
//  * a wave's A operand is its tile's input rows: lane (col, h) holds row r0+col, features
//    [h*KH, h*KH + KH) of [id | content] in registers (KH = (d+C)/2); MFMA step s consumes the
//    feature pair (s, KH+s); d/32 accumulators cover the d output columns (two sets by step
//    parity at d = 64, so 4 independent MFMA chains are always in flight);
//  * epilogue: z = acc + bias[o], out = z > 0 ? z : slope * z (torch leaky_relu), 128-B stores.
// Work: 2·I·(d+C)·d flop (C5: 216 GFLOP, MFMA-bound); bytes: I·(d+C)·4 read + I·d·4 written.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "lgcn.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kFusionWaves = 4;  // one wave per SIMD: the whole 512-register file per lane

template <int D, int KH>
__device__ __forceinline__ void load_a(const float* __restrict__ idw, int64_t ld_id,
                                       const float* __restrict__ content, int64_t ld_c,
                                       int64_t row, bool ok, int h, float (&a)[KH]) {
#pragma unroll
    for (int q = 0; q < KH / 4; ++q) {
        const int k = h * KH + 4 * q;  // [id | content] feature of this lane's float4
        const float* src = k < D ? idw + row * ld_id + k : content + row * ld_c + (k - D);
        const float4 v = ok ? *reinterpret_cast<const float4*>(src)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
    }
}

template <int D, int KH>
__global__ __launch_bounds__(kFusionWaves * 64) void k_fusion_prelayer(
    const float* __restrict__ idw, int64_t ld_id, const float* __restrict__ content, int64_t ld_c,
    int32_t n, const float* __restrict__ w, const float* __restrict__ bias, float slope,
    float* __restrict__ out, int64_t ld_out) {
    constexpr int K = 2 * KH;
    constexpr int NT = D / 32;
    constexpr int NS = NT >= 4 ? 1 : 4 / NT;  // accumulator sets (by step parity): 4 MFMA chains
    constexpr int HALF = KH * D + 32;  // LDS offset of the second k half
    static_assert(K > D && KH % 4 == 0 && KH % NS == 0 && D % 32 == 0, "shape");
    extern __shared__ __attribute__((aligned(16))) float wt[];  // wt[h*HALF + s*D + o] = W[o][h*KH+s]
    for (int e = threadIdx.x; e < D * K; e += blockDim.x) {
        const int o = e / K, k = e - o * K;
        const int h = k >= KH ? 1 : 0;
        wt[h * HALF + (k - h * KH) * D + o] = w[e];
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int col = lane & 31;
    float bo[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bo[nt] = bias ? bias[nt * 32 + col] : 0.f;
    const float* wl = wt + h * HALF + col;
    const int64_t n_tiles = ((int64_t)n + 31) / 32;
    const int64_t stride = (int64_t)gridDim.x * kFusionWaves;
    int64_t t = (int64_t)blockIdx.x * kFusionWaves + wave;
    // the next tile's A rows are in flight while the current tile's MFMA chain runs
    float a[KH], an[KH];
    if (t < n_tiles) load_a<D, KH>(idw, ld_id, content, ld_c, t * 32 + col, t * 32 + col < n, h, a);
    for (; t < n_tiles; t += stride) {
        const int64_t r0 = t * 32;
        const int64_t tn = t + stride;
        if (tn < n_tiles)
            load_a<D, KH>(idw, ld_id, content, ld_c, tn * 32 + col, tn * 32 + col < n, h, an);
        f32x16 acc[NS][NT];
#pragma unroll
        for (int p = 0; p < NS; ++p)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[p][nt] = f32x16{};
#pragma unroll
        for (int s = 0; s < KH; ++s) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                acc[s % NS][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                    a[s], wl[s * D + nt * 32], acc[s % NS][nt], 0, 0, 0);
            // bound the scheduler's LDS read-ahead (it would hoist all KH*NT weight reads)
            if ((s & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        }
        // lane holds rows (r&3) + 8(r>>2) + 4h of the tile, column nt*32 + col
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t i = r0 + (r & 3) + 8 * (r >> 2) + 4 * h;
                float z = acc[0][nt][r];
#pragma unroll
                for (int p = 1; p < NS; ++p) z += acc[p][nt][r];
                z += bo[nt];
                if (i < n) out[i * ld_out + nt * 32 + col] = z > 0.f ? z : z * slope;
            }
        }
#pragma unroll
        for (int q = 0; q < KH; ++q) a[q] = an[q];
    }
}

template <int D, int KH>
int launch_fusion(const float* idw, int64_t ld_id, const float* content, int64_t ld_c, int32_t n,
                  const float* w, const float* bias, float slope, float* out, int64_t ld_out,
                  hipStream_t s) {
    constexpr size_t lds = sizeof(float) * (2 * (KH * D + 32));
    auto kern = k_fusion_prelayer<D, KH>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    int dev = 0, n_cu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n_cu = 256;
    const int64_t tiles = ((int64_t)n + 31) / 32;
    int64_t grid = (tiles + kFusionWaves - 1) / kFusionWaves;
    if (grid > n_cu) grid = n_cu;  // persistent: one block (96-128 KB of LDS) per CU
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(kFusionWaves * 64), lds, s, idw, ld_id,
                       content, ld_c, n, w, bias, slope, out, ld_out);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" {

int lgcn_fusion_prelayer(const float* id_emb, int64_t ld_id, const float* content, int64_t ld_c,
                         int32_t n_items, int32_t d, int32_t c_dim, const float* weight,
                         const float* bias, float slope, float* out, int64_t ld_out,
                         void* stream) {
    if (n_items < 0 || (d != 64 && d != 128)) return LGCN_EINVAL;
    if (c_dim != 32 && c_dim != 64 && c_dim != 128) return LGCN_EINVAL;
    if (ld_id < d || ld_c < c_dim || ld_out < d) return LGCN_EINVAL;
    if (n_items == 0) return 0;
    if (!id_emb || !content || !weight || !out) return LGCN_EINVAL;
    if (!al16(id_emb) || !al16(content) || !al16(out) || ld_id % 4 || ld_c % 4 || ld_out % 4)
        return LGCN_EALIGN;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define LGCN_F(D_, C_)                                                                          \
    if (d == D_ && c_dim == C_)                                                                 \
        return launch_fusion<D_, (D_ + C_) / 2>(id_emb, ld_id, content, ld_c, n_items, weight,   \
                                                bias, slope, out, ld_out, s);
    LGCN_F(64, 32) LGCN_F(64, 64) LGCN_F(64, 128) LGCN_F(128, 32) LGCN_F(128, 64) LGCN_F(128, 128)
#undef LGCN_F
    return LGCN_EINVAL;
}

}  // extern "C"
