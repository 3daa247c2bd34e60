// H2D probe (diagnostic, not part of the library): pinned host -> HBM rates of
// one hipMemcpyAsync, several concurrent copies on separate streams, and a
// kernel that reads the pinned pages directly (zero-copy) into HBM.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void pull(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main() {
    const size_t B = 1ull << 30;
    void *h, *d;
    CK(hipHostMalloc(&h, B, hipHostMallocDefault));
    CK(hipMalloc(&d, B));
    std::memset(h, 1, B);
    hipStream_t st[8];
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto t = [] { return std::chrono::steady_clock::now(); };
    auto rate = [&](const char *what, auto fn) -> int {
        for (int w = 0; w < 2; w++) { fn(); CK(hipDeviceSynchronize()); }
        const auto a = t();
        for (int r = 0; r < 5; r++) fn();
        CK(hipDeviceSynchronize());
        const double s = std::chrono::duration<double>(t() - a).count() / 5;
        printf("%-40s %.1f GB/s\n", what, B / s / 1e9);
        return 0;
    };
    rate("one hipMemcpyAsync", [&] { (void)hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, st[0]); });
    for (int ns : {2, 4, 8}) {
        char nm[64];
        snprintf(nm, sizeof nm, "%d concurrent copies", ns);
        rate(nm, [&] {
            for (int i = 0; i < ns; i++)
                (void)hipMemcpyAsync((char *)d + i * (B / ns), (char *)h + i * (B / ns), B / ns, hipMemcpyHostToDevice, st[i]);
        });
    }
    void *hd;
    CK(hipHostGetDevicePointer(&hd, h, 0));
    for (int g : {256, 1024, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "zero-copy kernel, %d blocks", g);
        rate(nm, [&] { hipLaunchKernelGGL(pull, dim3(g), dim3(256), 0, st[0], (const uint4 *)hd, (uint4 *)d, B / 16); });
    }
    return 0;
}
