// HIP-only reproduction of the stream pattern the sided propagation records while a stream is
// captured into a HIP graph (no engine code): origin stream s, a second lane L forked from s, and
// aux streams A[0..na) that L forks and joins once per "half-layer", then everything joined back
// into s. Mode (argv[1]):
//   flat   — the aux streams are forked from s and joined into s only (the engine's default
//            under a capture: lane 1 runs on L alone, lane 0's aux streams fork from s)
//   nested — L forks A[i] and joins them back into L every half-layer (lane 1 with its own aux
//            streams under a capture: LGCN_SCHED_CAPTURE_AUX=1), A[i] also joined into s at the
//            end, as lgcn_engine.hip's join_lanes does
// argv[3] (priorities, as engine.py creates lane 1's streams): "high" = L and A[i] created at
// high priority, "aux" = A[i] only, default none
// Every record uses its own event. Prints "replay ok" after capturing, instantiating and
// launching the graph twice and checking the result; a crash in hipStreamEndCapture is the ROCm
// behaviour the engine guards against.
//   hipcc --offload-arch=gfx950 -O2 -o tools/capture_repro tools/capture_repro.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__global__ void k_add(float* p, int n, float v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += v;
}

int main(int argc, char** argv) {
    const bool nested = argc > 1 && strcmp(argv[1], "nested") == 0;
    const int layers = argc > 2 ? atoi(argv[2]) : 3;
    const char* prio = argc > 3 ? argv[3] : "none";
    const bool hi_l = strcmp(prio, "high") == 0, hi_a = hi_l || strcmp(prio, "aux") == 0;
    int lo_p = 0, hi_p = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo_p, &hi_p));
    const int na = 3, n = 1 << 16;
    hipStream_t s, L, A[na];
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&L, hipStreamNonBlocking, hi_l ? hi_p : lo_p));
    for (int i = 0; i < na; ++i)
        CK(hipStreamCreateWithPriority(&A[i], hipStreamNonBlocking, hi_a ? hi_p : lo_p));
    std::vector<hipEvent_t> pool(512);
    for (auto& e : pool) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    size_t next = 0;
    auto ev = [&]() { return pool[next++]; };
    float* buf;
    CK(hipMalloc(&buf, sizeof(float) * n * (na + 2)));
    CK(hipMemset(buf, 0, sizeof(float) * n * (na + 2)));
    auto add = [&](hipStream_t st, int slot) {
        hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, st, buf + (size_t)slot * n, n, 1.f);
        return hipGetLastError();
    };
    auto link = [&](hipStream_t from, hipStream_t to) {
        hipEvent_t e = ev();
        hipError_t r = hipEventRecord(e, from);
        return r != hipSuccess ? r : hipStreamWaitEvent(to, e, 0);
    };
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    CK(link(s, L));
    if (!nested)
        for (int i = 0; i < na; ++i) CK(link(s, A[i]));
    for (int k = 0; k < layers; ++k) {
        CK(add(s, 0));  // lane 0's work
        if (nested) {   // one half-layer of lane 1: fork the aux streams from L, join them back
            for (int i = 0; i < na; ++i) CK(link(L, A[i]));
            for (int i = 0; i < na; ++i) CK(add(A[i], 2 + i));
            CK(add(L, 1));
            for (int i = 0; i < na; ++i) CK(link(A[i], L));
        } else {
            CK(add(L, 1));
            for (int i = 0; i < na; ++i) CK(add(A[i], 2 + i));
        }
    }
    CK(link(L, s));
    for (int i = 0; i < na; ++i) CK(link(A[i], s));
    printf("ending capture (%s, %d layers, priorities %s: %d..%d)\n", nested ? "nested" : "flat",
           layers, prio, lo_p, hi_p);
    fflush(stdout);
    hipGraph_t g;
    CK(hipStreamEndCapture(s, &g));
    printf("captured\n");
    fflush(stdout);
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 2; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    std::vector<float> h((size_t)n * (na + 2));
    CK(hipMemcpy(h.data(), buf, sizeof(float) * h.size(), hipMemcpyDeviceToHost));
    bool ok = true;
    for (int slot = 0; slot < na + 2; ++slot) ok = ok && h[(size_t)slot * n] == 2.f * layers;
    printf(ok ? "replay ok\n" : "replay WRONG\n");
    return ok ? 0 : 2;
}
