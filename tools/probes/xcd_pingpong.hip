// Probe: which XCD runs each block (s_getreg XCC_ID), and the round-trip
// latency of a flag ping-pong between two blocks with (a) agent-scope atomics
// (sc1 loads) and (b) L2-only loads (sc0) + plain stores, same XCD vs not.
// Build: hipcc -O3 --offload-arch=gfx950 -o xcd_pingpong xcd_pingpong.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void xcc_map(uint32_t *out) {
    if (threadIdx.x == 0) {
        uint32_t v;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
        out[blockIdx.x] = v;
    }
}

__device__ __forceinline__ uint64_t ld_sc0(const uint64_t *p) {
    uint64_t v;
    asm volatile("global_load_dwordx2 %0, %1, off sc0\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void st_plain(uint64_t *p, uint64_t v) {
    asm volatile("global_store_dwordx2 %0, %1, off sc0\n s_waitcnt vmcnt(0)" ::"v"(p), "v"(v) : "memory");
}

// blocks a and b ping-pong `iters` times; mode 0 agent atomics, 1 sc0 loads
__global__ void pingpong(uint64_t *flags, int a, int b, int iters, int mode, uint64_t *cycles) {
    if (threadIdx.x != 0) return;
    const int me = blockIdx.x;
    if (me != a && me != b) return;
    uint64_t *mine = flags + (me == a ? 0 : 16), *other = flags + (me == a ? 16 : 0);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= iters; i++) {
        if (me == a) {
            if (mode == 0) __hip_atomic_store(mine, (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else st_plain(mine, (uint64_t)i);
            uint32_t spins = 0;
            while ((mode == 0 ? __hip_atomic_load(other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ld_sc0(other)) !=
                   (uint64_t)i)
                if (++spins > (1u << 22)) return;
        } else {
            uint32_t spins = 0;
            while ((mode == 0 ? __hip_atomic_load(other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ld_sc0(other)) !=
                   (uint64_t)i)
                if (++spins > (1u << 22)) return;
            if (mode == 0) __hip_atomic_store(mine, (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else st_plain(mine, (uint64_t)i);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (me == a) cycles[0] = t1 - t0;
}

int main() {
    const int nb = 64;
    uint32_t *dmap, hmap[nb];
    (void)hipMalloc(&dmap, nb * 4);
    hipLaunchKernelGGL(xcc_map, dim3(nb), dim3(64), 0, 0, dmap);
    (void)hipMemcpy(hmap, dmap, nb * 4, hipMemcpyDeviceToHost);
    printf("block -> xcc:");
    for (int i = 0; i < nb; i++) printf(" %u", hmap[i]);
    printf("\n");
    uint64_t *flags, *cyc, hc;
    (void)hipMalloc(&flags, 4096);
    (void)hipMalloc(&cyc, 8);
    const int iters = 2000;
    int pairs[3][2] = {{0, 0}, {0, 0}, {0, 0}};
    // same xcc pair and different xcc pair from the map
    for (int j = 1; j < nb; j++)
        if (hmap[j] == hmap[0]) { pairs[0][0] = 0; pairs[0][1] = j; break; }
    for (int j = 1; j < nb; j++)
        if (hmap[j] != hmap[0]) { pairs[1][0] = 0; pairs[1][1] = j; break; }
    for (int pi = 0; pi < 2; pi++) {
        for (int mode = 0; mode < 2; mode++) {
            (void)hipMemset(flags, 0, 4096);
            (void)hipMemset(cyc, 0, 8);
            hipLaunchKernelGGL(pingpong, dim3(nb), dim3(64), 0, 0, flags, pairs[pi][0], pairs[pi][1], iters, mode, cyc);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
            printf("%s xcc pair (%d,%d) mode %s: %.0f ns per round trip%s\n", pi == 0 ? "same" : "diff", pairs[pi][0],
                   pairs[pi][1], mode ? "sc0" : "agent", hc * 10.0 / iters, hc == 0 ? " (timed out)" : "");
        }
    }
    return 0;
}
