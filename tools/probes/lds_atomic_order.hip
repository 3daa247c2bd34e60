// Probe: do same-address LDS atomics of one wave return values in lane order?
// (If yes, an LDS-atomic rank is stable; the engine only relies on it after
// this probe passes on the device.)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void probe(uint32_t *out, int groups) {
    __shared__ uint32_t c[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) c[i] = 0;
    __syncthreads();
    uint32_t bad = 0;
    for (int it = 0; it < 64; it++) {
        const int lane = threadIdx.x & 63;
        const int w = threadIdx.x >> 6;
        // pseudo-random digit per lane and iteration
        uint32_t h = (lane * 2654435761u) ^ (it * 40503u) ^ (blockIdx.x * 97u);
        h ^= h >> 13;
        const uint32_t d = (h % groups) + w * 64 % 256;
        const uint32_t old = atomicAdd(&c[d % 256], 1u);
        // lanes with the same digit: earlier lane must get a smaller value
        for (int o = 0; o < 64; o++) {
            const uint32_t od = __shfl((int)d, o, 64);
            const uint32_t ov = __shfl((int)old, o, 64);
            if (od == d && o < lane && ov > old) bad++;
        }
    }
    atomicAdd(out, bad);
}
int main() {
    uint32_t *d, h = 0;
    hipMalloc(&d, 4);
    for (int g : {2, 7, 33, 128}) {
        hipMemset(d, 0, 4);
        hipLaunchKernelGGL(probe, dim3(1024), dim3(256), 0, 0, d, g);
        hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
        printf("groups %d: out-of-lane-order pairs %u\n", g, h);
    }
    return 0;
}
