// Micro-benchmark: cost per step of one wave's dependent fp32 fma chain on gfx950, with the
// operands (a) in registers, (b) broadcast from LDS (ds_read_b128, 2 steps per read).
// hipcc --offload-arch=gfx950 -O3 -o chain_latency chain_latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_regs(float* out, int n, float v0, float x0) {
    float a = 0.f, v = v0, x = x0;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 64; ++k) a = __builtin_fmaf(v, x, a);
        v = v * 1.0000001f;
    }
    out[threadIdx.x] = a;
}

__global__ void k_lds(float* out, int n, float v0) {
    __shared__ float2 sq[256];
    for (int i = threadIdx.x; i < 256; i += 64) sq[i] = make_float2(v0 + i * 1e-7f, 1.f - i * 1e-7f);
    __syncthreads();
    float a = 0.f;
    for (int it = 0; it < n; ++it) {
#pragma unroll 32
        for (int i = 0; i < 256; i += 2) {
            const float4 w = reinterpret_cast<const float4*>(sq)[i / 2];
            a = __builtin_fmaf(w.x, w.y, a);
            a = __builtin_fmaf(w.z, w.w, a);
        }
    }
    out[threadIdx.x] = a;
}

int main() {
    float* out;
    hipMalloc(&out, 1024 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int n = 20000;
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_regs, dim3(1), dim3(64), 0, 0, out, n, 1.0001f, 0.5f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("regs: %.3f ns per dependent fma (one wave)\n", ms * 1e6 / (n * 64.0));
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, out, n / 4, 1.0001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("lds : %.3f ns per step (one wave, ds_read_b128 per 2 steps)\n",
               ms * 1e6 / ((n / 4) * 256.0));
    }
    return 0;
}
