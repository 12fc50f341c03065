// lgcn_bpr.hip — fused BPR loss + regulariser of one training batch (main.py:366-402 on the
// device): the two dot products, log-sigmoid, the L2 term of the layer-0 rows, and every input
// gradient, in one pass over the 6 x B gathered rows; the batch mean is a fixed-order reduction
// (deterministic, run to run). Declared in include/lgcn.h (lgcn_bpr_loss).
//
//   loss = -mean_b log(sigmoid(<u_b,p_b> - <u_b,n_b>) + 1e-8)
//          + lambda * (|U0|^2 + |P0|^2 + |N0|^2) / B
//
// Gradients follow autograd's chain for that expression: c_b = ((-1/B) / (s_b + 1e-8)) *
// (1 - s_b) * s_b (NegBackward, MeanBackward, LogBackward, SigmoidBackward), du = c*p + (-c)*n,
// dp = c*u, dn = (-c)*u, d(row0) = (2*lambda/B) * row0.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "lgcn.h"

namespace {

constexpr int kWave = 64;
constexpr int kRowsPerBlock = 4;  // one wave per batch row

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__global__ __launch_bounds__(kWave * kRowsPerBlock) void k_bpr_rows(
    const float* __restrict__ u, int64_t ldu, const float* __restrict__ p, int64_t ldp,
    const float* __restrict__ n, int64_t ldn, const float* __restrict__ u0, int64_t ldu0,
    const float* __restrict__ p0, int64_t ldp0, const float* __restrict__ n0, int64_t ldn0,
    int32_t B, int32_t d, float lambda, float* __restrict__ terms, float* __restrict__ gu,
    float* __restrict__ gp, float* __restrict__ gn, float* __restrict__ gu0,
    float* __restrict__ gp0, float* __restrict__ gn0) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t b = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kWave;
    if (b >= B) return;
    const float* ub = u + b * ldu;
    const float* pb = p + b * ldp;
    const float* nb = n + b * ldn;
    const float* ub0 = u0 + b * ldu0;
    const float* pb0 = p0 + b * ldp0;
    const float* nb0 = n0 + b * ldn0;
    float sp = 0.f, sn = 0.f, sq = 0.f;
    for (int k = lane; k < d; k += kWave) {
        const float x = ub[k];
        sp = __builtin_fmaf(x, pb[k], sp);
        sn = __builtin_fmaf(x, nb[k], sn);
        sq = __builtin_fmaf(ub0[k], ub0[k], sq);
        sq = __builtin_fmaf(pb0[k], pb0[k], sq);
        sq = __builtin_fmaf(nb0[k], nb0[k], sq);
    }
    sp = wave_sum(sp);
    sn = wave_sum(sn);
    sq = wave_sum(sq);
    const float x = sp - sn;
    const float s = 1.f / (1.f + expf(-x));
    const float c = ((-1.f / (float)B) / (s + 1e-8f)) * (1.f - s) * s;
    const float r = 2.f * lambda / (float)B;
    for (int k = lane; k < d; k += kWave) {
        const int64_t o = b * (int64_t)d + k;
        gu[o] = c * pb[k] + (-c) * nb[k];
        gp[o] = c * ub[k];
        gn[o] = (-c) * ub[k];
        gu0[o] = r * ub0[k];
        gp0[o] = r * pb0[k];
        gn0[o] = r * nb0[k];
    }
    if (lane == 0) {
        terms[b] = logf(s + 1e-8f);
        terms[B + b] = sq;
    }
}

// loss = -(sum log terms) / B + lambda * (sum squares) / B, summed in a fixed order
__global__ __launch_bounds__(256) void k_bpr_reduce(const float* __restrict__ terms, int32_t B,
                                                    float lambda, float* __restrict__ loss) {
    __shared__ float sl[256], sr[256];
    float a = 0.f, q = 0.f;
    for (int i = threadIdx.x; i < B; i += 256) {
        a += terms[i];
        q += terms[B + i];
    }
    sl[threadIdx.x] = a;
    sr[threadIdx.x] = q;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sl[threadIdx.x] += sl[threadIdx.x + w];
            sr[threadIdx.x] += sr[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = -(sl[0] / (float)B) + lambda * sr[0] / (float)B;
}

}  // namespace

extern "C" int lgcn_bpr_loss(const float* u, int64_t ldu, const float* p, int64_t ldp,
                             const float* n, int64_t ldn, const float* u0, int64_t ldu0,
                             const float* p0, int64_t ldp0, const float* n0, int64_t ldn0,
                             int32_t B, int32_t d, float lambda, float* terms, float* loss,
                             float* grads, void* stream) {
    if (B < 1 || d < 1 || !loss || !terms || !grads) return LGCN_EINVAL;
    if (!u || !p || !n || !u0 || !p0 || !n0) return LGCN_EINVAL;
    if (ldu < d || ldp < d || ldn < d || ldu0 < d || ldp0 < d || ldn0 < d) return LGCN_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t bd = (int64_t)B * d;
    const int64_t grid = ((int64_t)B + kRowsPerBlock - 1) / kRowsPerBlock;
    hipLaunchKernelGGL(k_bpr_rows, dim3((uint32_t)grid), dim3(kWave * kRowsPerBlock), 0, s, u,
                       ldu, p, ldp, n, ldn, u0, ldu0, p0, ldp0, n0, ldn0, B, d, lambda, terms,
                       grads, grads + bd, grads + 2 * bd, grads + 3 * bd, grads + 4 * bd,
                       grads + 5 * bd);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_bpr_reduce, dim3(1), dim3(256), 0, s, terms, B, lambda, loss);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}
