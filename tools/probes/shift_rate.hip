// VALU rate of 64-bit vs 32-bit shifts on gfx950: 8 independent chains per
// thread, a runtime shift amount, enough waves to fill every SIMD.
// hipcc -O3 --offload-arch=gfx950 shift_rate.hip -o shift_rate && ./shift_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int KIND>
__global__ __launch_bounds__(256) void k(uint64_t *out, int s, int iters) {
    uint64_t x[8];
    uint32_t y[8];
    for (int j = 0; j < 8; j++) { x[j] = threadIdx.x * 0x9E3779B97F4A7C15ull + j; y[j] = (uint32_t)x[j]; }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (KIND == 0) x[j] = (x[j] >> s) ^ (x[j] << 7);          // 2 x 64-bit shift + xor
            if (KIND == 1) y[j] = (y[j] >> s) ^ (y[j] << 7);          // 2 x 32-bit shift + xor
            if (KIND == 2) y[j] = __builtin_amdgcn_alignbit(y[j], y[(j + 1) & 7], s) ^ (y[j] << 7);  // alignbit
        }
    }
    uint64_t a = 0;
    for (int j = 0; j < 8; j++) a ^= x[j] ^ y[j];
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

int main() {
    uint64_t *d;
    const int blocks = 256 * 8 * 4, iters = 4096;
    hipMalloc(&d, (size_t)blocks * 256 * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[3] = {"64-bit shifts", "32-bit shifts", "alignbit"};
    for (int rep = 0; rep < 2; rep++)
        for (int kind = 0; kind < 3; kind++) {
            hipEventRecord(a);
            if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, 13, iters);
            if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, 13, iters);
            if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, d, 13, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            // wave-instructions: 3 ops per chain step (2 shifts + xor) x 8 chains x iters per thread
            const double winst = (double)blocks * 4 * iters * 8 * 3;
            printf("%-14s %.3f ms  %.2f wave-inst / cycle / CU (2.4 GHz, 256 CUs)\n", names[kind], ms,
                   winst / (ms * 1e-3 * 2.4e9 * 256));
        }
    hipFree(d);
    return 0;
}
