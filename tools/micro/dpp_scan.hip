#include <hip/hip_runtime.h>
__device__ __forceinline__ int wave_incl_scan(int x) {
    // inclusive prefix sum over the 64 lanes of a wave by DPP (no LDS round trips)
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
__global__ void k(const int* in, int* out) { out[threadIdx.x] = wave_incl_scan(in[threadIdx.x]); }
int main() {
    int h[64], r[64]; for (int i = 0; i < 64; ++i) h[i] = i * 7 + 1 - (i % 5) * 3;
    int *di, *dout; hipMalloc(&di, 256); hipMalloc(&dout, 256);
    hipMemcpy(di, h, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout);
    hipMemcpy(r, dout, 256, hipMemcpyDeviceToHost);
    int s = 0, bad = 0; for (int i = 0; i < 64; ++i) { s += h[i]; if (r[i] != s) { bad++; printf("lane %d got %d want %d\n", i, r[i], s); } }
    printf("dpp scan: %s\n", bad ? "FAIL" : "OK");
    return bad;
}
