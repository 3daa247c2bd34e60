// VALU issue rates on gfx950 for the digit extractions of rg_finish
// (VERDICT r05 item 3): 8 independent chains per thread, a runtime shift
// amount, 8 blocks of 256 threads per CU (16 waves per CU, 4 per SIMD).
// Each kind's loop body is 3 VALU ops per chain step; the in-kernel clock is
// read with s_memtime / s_memrealtime (100 MHz) so the rate is per cycle of
// the clock the chip actually held.
// hipcc -O3 --offload-arch=gfx950 shift_rate.hip -o shift_rate && ./shift_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int KIND>
__global__ __launch_bounds__(256) void k(uint64_t *out, uint64_t *clk, int s, int iters) {
    uint64_t x[8];
    uint32_t y[8];
    for (int j = 0; j < 8; j++) {
        x[j] = threadIdx.x * 0x9E3779B97F4A7C15ull + j;
        y[j] = (uint32_t)x[j];
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (KIND == 0) x[j] = (x[j] >> s) ^ (x[j] << 7);  // 2 x 64-bit shift + 64-bit xor (2 VALU)
            if (KIND == 1) y[j] = (y[j] >> s) ^ (y[j] << 7);  // 2 x 32-bit shift + xor
            if (KIND == 2) y[j] = __builtin_amdgcn_alignbit(y[j], y[(j + 1) & 7], s) ^ (y[j] << 7);  // alignbit
            if (KIND == 3) y[j] = (y[j] + (uint32_t)s) ^ (y[j] + 7u);  // 32-bit adds + xor
            if (KIND == 4) y[j] = __builtin_amdgcn_ubfe(y[j], s, 9) ^ (y[j] << 7);  // v_bfe_u32
            if (KIND == 5) y[j] = (uint32_t)(x[j] >> s) & 511u, x[j] ^= y[j];  // a digit from a u64 (the finish's form)
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint64_t a = 0;
    for (int j = 0; j < 8; j++) a ^= x[j] ^ y[j];
    out[blockIdx.x * 256 + threadIdx.x] = a;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main() {
    uint64_t *d, *c;
    const int blocks = 256 * 8 * 4, iters = 4096;
    hipMalloc(&d, (size_t)blocks * 256 * 8);
    hipMalloc(&c, (size_t)blocks * 16);
    std::vector<uint64_t> h(2 * blocks);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[6] = {"64-bit shifts", "32-bit shifts", "alignbit", "32-bit adds", "v_bfe_u32", "u64 digit"};
    for (int rep = 0; rep < 2; rep++)
        for (int kind = 0; kind < 6; kind++) {
            hipEventRecord(a);
            auto fn = kind == 0 ? k<0> : kind == 1 ? k<1> : kind == 2 ? k<2> : kind == 3 ? k<3> : kind == 4 ? k<4> : k<5>;
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, d, c, 13, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            hipMemcpy(h.data(), c, h.size() * 8, hipMemcpyDeviceToHost);
            std::vector<double> ghz;
            for (int i = 0; i < blocks; i++)
                if (h[2 * i + 1]) ghz.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 0.1);
            std::sort(ghz.begin(), ghz.end());
            const double clock = ghz.empty() ? 2.4 : ghz[ghz.size() / 2];
            // VALU wave-instructions of the loop body (gfx950 ISA): 4 per chain
            // step for the 64-bit form (two 64-bit shifts + two 32-bit xors),
            // 3 for the others; x 8 chains x iters per wave; 4 waves per block
            const double ops = (double)blocks * 4 * iters * 8 * (kind == 0 ? 4 : 3);
            const double rate = ops / (ms * 1e-3 * clock * 1e9 * 256);
            if (rep)
                printf("%-14s %8.3f ms  clock %.2f GHz  %.2f VALU wave-instructions / cycle / CU\n", names[kind], ms,
                       clock, rate);
        }
    hipFree(d);
    hipFree(c);
    return 0;
}
