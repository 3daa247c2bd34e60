// Micro-benchmark of the kman_finish wave-per-segment LDS sort in isolation:
// every block holds FR keys in LDS split into NSEG segments and sorts them
// REPS times (low 21 bits, 3 x 7-bit passes, packed (low << 13 | pos) items),
// timing with s_memrealtime.  Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/wsb wavesort_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int FT = 512, FW = 8, FR = 6144, WI = 12;

__device__ __forceinline__ uint32_t wscan(uint32_t v) {
    const int lane = __lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// DPP inclusive scan across 64 lanes (row_shr 1,2,4,8 then row_bcast 15 / 31)
__device__ __forceinline__ uint32_t wscan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    return x;
}

template <int MODE>
__global__ __launch_bounds__(FT) void bench(const uint64_t *in, uint64_t *out, int nseg, int reps, uint64_t *cycles) {
    __shared__ uint64_t skey[FR];
    __shared__ uint32_t spk[FR];
    __shared__ uint32_t whist[FW][128];
    const int t = threadIdx.x, lane = __lane_id(), w = t >> 6;
    const int segsz = 5120 / nseg;
    for (int i = t; i < FR; i += FT) skey[i] = in[(uint64_t)blockIdx.x * FR + i];
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t lmask = (1ull << 21) - 1;
    for (int rep = 0; rep < reps; rep++) {
        for (int sg = w; sg < nseg; sg += FW) {
            const uint32_t sa = sg * segsz, sz = segsz;
            const uint64_t pfx_hi = skey[sa] & ~lmask;
            uint64_t pw[WI];
#pragma unroll
            for (int i = 0; i < WI; i++) {
                if ((uint32_t)(i * 64) >= sz) break;
                const uint32_t p = i * 64 + lane;
                pw[i] = p < sz ? ((skey[sa + p] & lmask) << 13) | (sa + p) : 0;
            }
            for (int pp = 0; pp < 3; pp++) {
                const uint32_t sh = 13 + 7 * pp, dm = 127;
                whist[w][lane] = 0;
                whist[w][lane + 64] = 0;
                __builtin_amdgcn_wave_barrier();
                uint32_t r[WI], d[WI];
#pragma unroll
                for (int i = 0; i < WI; i++) {
                    if ((uint32_t)(i * 64) >= sz) break;
                    const uint32_t p = i * 64 + lane;
                    d[i] = (uint32_t)(pw[i] >> sh) & dm;
                    if (MODE == 1) r[i] = 0;
                    else r[i] = p < sz ? atomicAdd(&whist[w][d[i]], 1u) : 0u;
                }
                __builtin_amdgcn_wave_barrier();
                const uint32_t c0 = whist[w][2 * lane], c1 = whist[w][2 * lane + 1];
                const uint32_t inc = MODE == 3 ? wscan_dpp(c0 + c1) : wscan(c0 + c1);
                whist[w][2 * lane] = inc - c0 - c1;
                whist[w][2 * lane + 1] = inc - c1;
                __builtin_amdgcn_wave_barrier();
                const bool last = pp == 2;
#pragma unroll
                for (int i = 0; i < WI; i++) {
                    if ((uint32_t)(i * 64) >= sz) break;
                    const uint32_t p = i * 64 + lane;
                    if (p < sz) {
                        const uint32_t dst = sa + ((MODE == 2) ? p : whist[w][d[i]] + r[i]);
                        if (last) {
                            skey[dst] = pfx_hi | (pw[i] >> 13);
                            spk[dst] = (uint32_t)(pw[i] & 8191u);
                        } else {
                            skey[dst] = pw[i];
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                if (!last) {
#pragma unroll
                    for (int i = 0; i < WI; i++) {
                        if ((uint32_t)(i * 64) >= sz) break;
                        const uint32_t p = i * 64 + lane;
                        if (p < sz) pw[i] = skey[sa + p];
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        __syncthreads();
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    for (int i = t; i < FR; i += FT) out[(uint64_t)blockIdx.x * FR + i] = skey[i] ^ spk[i];
    if (t == 0) cycles[blockIdx.x] = t1 - t0;
}

__global__ void scan_check(uint32_t *o) {
    const uint32_t v = (threadIdx.x * 7 + 3) % 11;
    o[threadIdx.x] = wscan_dpp(v) - wscan(v);
}

int main(int argc, char **argv) {
    {
        uint32_t *d, h[64];
        (void)hipMalloc(&d, 256);
        hipLaunchKernelGGL(scan_check, dim3(1), dim3(64), 0, 0, d);
        (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 64; i++) bad += h[i] != 0;
        printf("dpp scan mismatches: %d\n", bad);
    }
    const int blocks = argc > 1 ? atoi(argv[1]) : 256;
    const int nseg = argc > 2 ? atoi(argv[2]) : 11;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    const int reps = 200;
    size_t n = (size_t)blocks * FR;
    uint64_t *h = (uint64_t *)malloc(n * 8);
    uint64_t x = 88172645463325252ull;
    for (size_t i = 0; i < n; i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        h[i] = x & ((1ull << 42) - 1);
    }
    uint64_t *din, *dout, *dc;
    (void)hipMalloc(&din, n * 8);
    (void)hipMalloc(&dout, n * 8);
    (void)hipMalloc(&dc, blocks * 8);
    (void)hipMemcpy(din, h, n * 8, hipMemcpyHostToDevice);
    auto k = mode == 0 ? bench<0> : mode == 1 ? bench<1> : mode == 2 ? bench<2> : bench<3>;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(FT), 0, 0, din, dout, nseg, reps, dc);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(FT), 0, 0, din, dout, nseg, reps, dc);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t *hc = (uint64_t *)malloc(blocks * 8);
    (void)hipMemcpy(hc, dc, blocks * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; i++) avg += hc[i];
    avg /= blocks;
    printf("blocks %d nseg %d mode %d: %.3f ms total, per block-rep %.2f us (memrealtime), keys/s %.1f G\n", blocks,
           nseg, mode, ms, avg * 10.0 / 1000.0 / reps, (double)blocks * 5120 * reps / (ms / 1e3) / 1e9);
    return 0;
}
