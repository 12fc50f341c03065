// HIP-only reproduction of the stream pattern the sided propagation records while a stream is
// captured into a HIP graph (no engine code): origin stream s, a second lane L forked from s, and
// aux streams A[0..na) that L forks and joins once per "half-layer", then everything joined back
// into s. Mode (argv[1]):
//   flat   — the aux streams are forked from s and joined into s only (the engine's default
//            under a capture: lane 1 runs on L alone, lane 0's aux streams fork from s)
//   nested — L forks A[i] and joins them back into L every half-layer (lane 1 with its own aux
//            streams under a capture: the library built with LGCN_CAPTURE_AUX_EXP), A[i] also joined into s at the
//            end, as lgcn_engine.hip's join_lanes does
// argv[3] (priorities, as engine.py creates lane 1's streams): "high" = L and A[i] created at
// high priority, "aux" = A[i] only, default none
// file <ops> replays a capture extracted from a HIP API log (tools/capture_ops.py).
// lanes / lanes1 (argv[2] = K): the sided schedule's pattern with cross-lane waits (below).
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

__global__ void k_nop(float* p) {
    extern __shared__ float sh[];
    if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && p) sh[0] = p[0];
}

// file mode: replay a capture's operations extracted from a HIP API log (tools/capture_ops.py):
// "streams N", "prio i p", "R ev st", "W ev st", "K st gx gy gz bx shmem"
static int replay_file(const char* path) {
    FILE* f = fopen(path, "r");
    if (!f) { perror(path); return 1; }
    int ns = 0;
    if (fscanf(f, "streams %d\n", &ns) != 1 || ns < 1 || ns > 64) return 1;
    std::vector<int> prio(ns, 0);
    for (int i = 0; i < ns; ++i) {
        int a, b;
        if (fscanf(f, "prio %d %d\n", &a, &b) != 2) return 1;
        prio[a] = b;
    }
    std::vector<hipStream_t> st(ns);
    for (int i = 0; i < ns; ++i)
        CK(hipStreamCreateWithPriority(&st[i], hipStreamNonBlocking, prio[i]));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_nop),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
    std::vector<hipEvent_t> ev;
    char op[16];
    int nk = 0, nr = 0, nw = 0;
    bool capturing = false;
    auto event = [&](int e) -> hipEvent_t {
        while ((int)ev.size() <= e) {
            hipEvent_t x;
            if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) return nullptr;
            ev.push_back(x);
        }
        return ev[e];
    };
    // lower-case ops run before the capture (the warm-up call on the same streams and events),
    // "capture" begins it on stream 0, upper-case ops are captured
    while (fscanf(f, "%15s", op) == 1) {
        if (strcmp(op, "capture") == 0) {
            CK(hipDeviceSynchronize());
            CK(hipStreamBeginCapture(st[0], hipStreamCaptureModeGlobal));
            capturing = true;
            continue;
        }
        const char c = op[0] | 0x20;
        if (c == 'r' || c == 'w') {
            int e, s;
            if (fscanf(f, "%d %d", &e, &s) != 2) return 1;
            hipEvent_t x = event(e);
            if (!x) return 1;
            if (c == 'r') { CK(hipEventRecord(x, st[s])); nr += capturing; }
            else { CK(hipStreamWaitEvent(st[s], x, 0)); nw += capturing; }
        } else if (c == 'k') {
            int s, gx, gy, gz, bx, sh;
            if (fscanf(f, "%d %d %d %d %d %d", &s, &gx, &gy, &gz, &bx, &sh) != 6) return 1;
            hipLaunchKernelGGL(k_nop, dim3(gx, gy, gz), dim3(bx), sh, st[s], (float*)nullptr);
            CK(hipGetLastError());
            nk += capturing;
        }
    }
    if (!capturing) CK(hipStreamBeginCapture(st[0], hipStreamCaptureModeGlobal));
    fclose(f);
    printf("replayed %d records, %d waits, %d launches on %d streams; ending capture\n", nr, nw,
           nk, ns);
    fflush(stdout);
    hipGraph_t g;
    CK(hipStreamEndCapture(st[0], &g));
    printf("captured\n");
    fflush(stdout);
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 2; ++r) CK(hipGraphLaunch(ge, st[0]));
    CK(hipStreamSynchronize(st[0]));
    printf("replay ok\n");
    return 0;
}

__global__ void k_add(float* p, int n, float v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += v;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: capture_repro flat|nested|lanes|lanes1 [layers] [none|aux|high]\n");
        return 1;
    }
    if (strcmp(argv[1], "file") == 0) return argc > 2 ? replay_file(argv[2]) : 1;
    const bool nested = strcmp(argv[1], "nested") == 0;
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
    if (strcmp(argv[1], "lanes") == 0 || strcmp(argv[1], "lanes1") == 0) {
        // the sided schedule's pattern (lgcn_engine.hip run_sides / plan_layer under a capture):
        // lane 0 = s + aux A (forked from s and joined into s every half-layer), lane 1 = L +
        // aux B (forked from L and joined into L every half-layer; "lanes1": lane 1 without aux,
        // what the library runs under a capture by default), half-layer (k, side) on lane
        // (k + side + K) % 2, the mean half-layers (k = K) waiting for the other lane's k-1
        hipStream_t B[na];
        for (int i = 0; i < na; ++i)
            CK(hipStreamCreateWithPriority(&B[i], hipStreamNonBlocking, hi_a ? hi_p : lo_p));
        const bool l1aux = strcmp(argv[1], "lanes") == 0;
        const int K = layers;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        CK(link(s, L));
        hipEvent_t rest[16] = {}, cls[16] = {};
        auto half = [&](hipStream_t M, hipStream_t* X, int nx, int slot, hipEvent_t late)
            -> hipError_t {
            hipError_t r = hipSuccess;
            if (late && (r = hipStreamWaitEvent(M, late, 0)) != hipSuccess) return r;
            for (int i = 0; i < nx; ++i)
                if ((r = link(M, X[i])) != hipSuccess) return r;
            for (int i = 0; i < nx; ++i)
                if ((r = add(X[i], 2 + i)) != hipSuccess) return r;
            if ((r = add(M, slot)) != hipSuccess) return r;
            for (int i = 0; i < nx; ++i)
                if ((r = link(X[i], M)) != hipSuccess) return r;
            return r;
        };
        for (int k = 1; k <= K; ++k) {
            for (int side = 1; side >= 0; --side) {
                const int lane = (k + side + K) & 1;
                hipStream_t M = lane ? L : s;
                hipStream_t* X = lane ? B : A;
                const int nx = lane && !l1aux ? 0 : na;
                hipEvent_t late = k == K && k >= 2 ? (side ? rest[k - 1] : cls[k - 1]) : nullptr;
                CK(half(M, X, nx, side, late));
                hipEvent_t e = ev();
                CK(hipEventRecord(e, M));
                (side ? rest : cls)[k] = e;
            }
        }
        CK(link(L, s));
        if (l1aux)
            for (int i = 0; i < na; ++i) CK(link(B[i], s));
        printf("ending capture (%s, K=%d, priorities %s)\n", argv[1], K, prio);
        fflush(stdout);
        hipGraph_t g;
        CK(hipStreamEndCapture(s, &g));
        printf("captured\n");
        fflush(stdout);
        hipGraphExec_t ge;
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 2; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        printf("replay ok\n");
        return 0;
    }
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
