// Micro-benchmark (design tool): one wave's dependent fp32 fma chain latency on gfx950, and the
// issue cost when 2 or 4 independent chains are interleaved in the same wave; also a 16-step-
// per-lane chain handed down 16 lanes by DPP (the walk's seq_block<16> shape).
// hipcc --offload-arch=gfx950 -O3 -o /tmp/fma_dep tools/micro/fma_dep.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NC>
__global__ void k_chains(float* out, int n, float v0, float x0) {
    float a[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) a[c] = c * 1e-3f;
    float v = v0 + threadIdx.x * 1e-7f, x = x0;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 64; ++k) {
#pragma unroll
            for (int c = 0; c < NC; ++c) a[c] = __builtin_fmaf(v, x, a[c]);
        }
        x = x * 1.0000001f;
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += a[c];
    out[threadIdx.x] = s;
}

__device__ __forceinline__ float shr1(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x138, 0xf, 0xf, false));
}

__global__ void k_lanes(float* out, int n, float v0) {
    float vv[16], xv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) vv[k] = v0 + k * 1e-6f + threadIdx.x * 1e-7f, xv[k] = 1.f - k * 1e-6f;
    float acc = 0.f;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int L = 0; L < 16; ++L) {
            if (L > 0) acc = shr1(acc);
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = __builtin_fmaf(vv[k], xv[k], acc);
        }
    }
    out[threadIdx.x] = acc;
}

int main() {
    float* out;
    hipMalloc(&out, 1024 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int n = 20000;
    float ms;
    for (int rep = 0; rep < 2; ++rep) {
#define RUN(NC)                                                                                 \
        hipEventRecord(e0);                                                                       \
        hipLaunchKernelGGL(k_chains<NC>, dim3(1), dim3(64), 0, 0, out, n, 1.0001f, 0.5f);         \
        hipEventRecord(e1);                                                                       \
        hipEventSynchronize(e1);                                                                  \
        hipEventElapsedTime(&ms, e0, e1);                                                         \
        printf("%d chain(s): %.3f ns per fma step of each chain (one wave)\n", NC, ms * 1e6 / (n * 64.0));
        RUN(1) RUN(2) RUN(4) RUN(8)
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_lanes, dim3(1), dim3(64), 0, 0, out, n / 4, 1.0001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("16 lanes x 16 steps + DPP: %.3f ns per step\n", ms * 1e6 / ((n / 4) * 256.0));
    }
    return 0;
}
