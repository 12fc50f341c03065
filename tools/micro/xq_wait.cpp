// Cross-queue wait latency vs how long the waiting queue has been blocked: stream A
// runs a spin kernel of T us and records an event; stream B, enqueued before A's kernel starts,
// waits on it and runs a stamp kernel. Gap = B's first instruction - A's last (s_memrealtime,
// 100 MHz). Variant "mid": B first waits on an event recorded after a first half-length spin.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/xq_wait.cpp -o tools/micro/xq_wait
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void spin(unsigned long long us, unsigned long long* t_end) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < us * 100) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0 && blockIdx.x == 0) *t_end = __builtin_amdgcn_s_memrealtime();
}
__global__ void stamp(unsigned long long* t) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *t = __builtin_amdgcn_s_memrealtime();
}
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("err %d line %d\n", e_, __LINE__); return 1; } } while (0)

int main() {
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    hipEvent_t ev, mid;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&mid, hipEventDisableTiming));
    unsigned long long* t;
    CK(hipMalloc(&t, 64));
    const unsigned long long Ts[] = {20, 100, 300, 1000, 2000, 4000};
    for (int variant = 0; variant < 2; ++variant) {
        for (unsigned long long T : Ts) {
            double g[5];
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipDeviceSynchronize());
                if (variant == 1) {
                    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, T / 2, t + 2);
                    CK(hipEventRecord(mid, a));
                    CK(hipStreamWaitEvent(b, mid, 0));
                    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, T - T / 2, t);
                } else {
                    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, T, t);
                }
                CK(hipEventRecord(ev, a));
                CK(hipStreamWaitEvent(b, ev, 0));
                hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, b, t + 1);
                CK(hipDeviceSynchronize());
                unsigned long long h[2];
                CK(hipMemcpy(h, t, 16, hipMemcpyDeviceToHost));
                g[rep] = (double)(h[1] - h[0]) / 100.0;
            }
            printf("%s T=%5llu us: gap us %.1f %.1f %.1f %.1f %.1f\n", variant ? "mid " : "plain", T,
                   g[0], g[1], g[2], g[3], g[4]);
        }
    }
    return 0;
}
