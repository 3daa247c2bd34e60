// Scattered line writes on MI355X: how fast HBM takes a digit pass's output
// when each destination region receives runs of L contiguous bytes (L = 64,
// 128, 256, 512) -- rg_pass writes whole 128-byte lines into 512 regions per
// chain.  Each 1024-thread block (one per CU, persistent like rg_pass) reads
// its input tile sequentially (64 KiB per tile) and writes the tile as
// 64 KiB / L runs, run j of tile t going to region (j * 97 + t) % NREG of the
// block at that region's next free offset (regions advance sequentially, as a
// pass's sub-regions do).  Reports GB/s of reads + writes.
// hipcc -O3 --offload-arch=gfx950 scatter_lines.hip -o scatter_lines && ./scatter_lines
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int NT = 1024, TILE = 64 << 10;

template <int L>
__global__ __launch_bounds__(NT) void k(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t tiles_per_block,
                                        uint32_t nreg, uint64_t reg_bytes) {
    constexpr int RUNS = TILE / L, U4_PER_RUN = L / 16;
    const uint64_t b = blockIdx.x;
    const uint4 *src = in + b * tiles_per_block * (TILE / 16);
    uint4 *dst = out + b * (uint64_t)nreg * (reg_bytes / 16);
    for (uint64_t t = 0; t < tiles_per_block; t++) {
        // 4096 uint4 per tile, 4 per thread
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = src[t * (TILE / 16) + threadIdx.x + i * NT];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t q = threadIdx.x + i * NT;  // uint4 index in the tile
            const uint32_t run = q / U4_PER_RUN, w = q % U4_PER_RUN;
            // the block's g-th run goes to region (97 g) mod nreg at that
            // region's slot g / nreg (every nreg consecutive runs hit every
            // region once: each region fills sequentially)
            const uint64_t g = t * RUNS + run;
            const uint32_t reg = (uint32_t)((g * 97u) % nreg);
            const uint64_t off = (g / nreg) * (L / 16) + w;
            dst[(uint64_t)reg * (reg_bytes / 16) + off] = v[i];
        }
    }
}

int main() {
    const int blocks = 256;
    const uint64_t tiles = 64;  // 4 MiB per block, 1 GiB total
    const uint64_t bytes = (uint64_t)blocks * tiles * TILE;
    uint4 *in, *out;
    hipMalloc(&in, bytes);
    hipMalloc(&out, bytes * 2);
    hipMemset(in, 1, bytes);
    hipMemset(out, 0, bytes * 2);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const uint32_t nreg = 512;
    const uint64_t reg_bytes = ((tiles * TILE / nreg) + 4095) & ~4095ull;  // a region's runs, rounded up
    for (int rep = 0; rep < 3; rep++) {
        for (int L : {64, 128, 256, 512}) {
            hipEventRecord(a);
            if (L == 64) hipLaunchKernelGGL(k<64>, dim3(blocks), dim3(NT), 0, 0, in, out, tiles, nreg, reg_bytes);
            if (L == 128) hipLaunchKernelGGL(k<128>, dim3(blocks), dim3(NT), 0, 0, in, out, tiles, nreg, reg_bytes);
            if (L == 256) hipLaunchKernelGGL(k<256>, dim3(blocks), dim3(NT), 0, 0, in, out, tiles, nreg, reg_bytes);
            if (L == 512) hipLaunchKernelGGL(k<512>, dim3(blocks), dim3(NT), 0, 0, in, out, tiles, nreg, reg_bytes);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep)
                printf("runs of %3d B into %u regions per block: %.3f ms  %.2f TB/s (read + write)\n", L, nreg, ms,
                       2.0 * bytes / (ms * 1e-3) / 1e12);
        }
    }
    hipFree(in);
    hipFree(out);
    return 0;
}
