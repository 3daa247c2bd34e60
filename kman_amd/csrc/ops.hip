// ops.hip — small device helpers used by the host API around the hot path.
//
//   kman_tag_batches  keys[i] |= ((first + i) / batch_size) << key_bits
//                     makes one stable sort over (batch, key) equal to a stable
//                     sort of every batch on its own — the per-batch
//                     Batch.sorted of the reference (batch.py:156-168) for all
//                     batches in one pass sequence.
//   kman_or_u64       v[i] |= value (tags payloads with a source id).
//   kman_memcpy_d2d   device-to-device copy on the context stream.
#include "common.h"

namespace {

__global__ void tag_kernel(uint64_t *__restrict__ keys, uint64_t n, uint32_t key_bits, uint64_t first,
                           uint64_t batch_size) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        keys[i] |= ((first + i) / batch_size) << key_bits;
}

__global__ void or_kernel(uint64_t *__restrict__ v, uint64_t n, uint64_t value) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        v[i] |= value;
}

__global__ void widen_kernel(const uint32_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n, uint64_t value) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint64_t)in[i] | value;
}

uint32_t grid_for(uint64_t n) {
    const uint64_t b = ceil_div(n, 256);
    return (uint32_t)(b < 8192 ? (b ? b : 1) : 8192);
}

}  // namespace

extern "C" int kman_tag_batches(kman_ctx *ctx, uint64_t *d_keys, uint64_t n, uint32_t key_bits, uint64_t first_index,
                                uint64_t batch_size) {
    if (!ctx) return KMAN_EINVAL;
    if (batch_size == 0 || key_bits >= 64) return kman_fail(ctx, KMAN_EINVAL, "bad batch tagging arguments");
    const uint64_t last = n ? (first_index + n - 1) / batch_size : 0;
    if (key_bits + (uint32_t)(64 - __builtin_clzll(last | 1)) > 64)
        return kman_fail(ctx, KMAN_EINVAL, "batch tag does not fit above %u key bits", key_bits);
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(tag_kernel, dim3(grid_for(n)), dim3(256), 0, ctx->stream, d_keys, n, key_bits, first_index,
                       batch_size);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}

extern "C" int kman_or_u64(kman_ctx *ctx, uint64_t *d_v, uint64_t n, uint64_t value) {
    if (!ctx) return KMAN_EINVAL;
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(or_kernel, dim3(grid_for(n)), dim3(256), 0, ctx->stream, d_v, n, value);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}

extern "C" int kman_widen_u32(kman_ctx *ctx, const uint32_t *d_in, uint64_t *d_out, uint64_t n, uint64_t value) {
    if (!ctx) return KMAN_EINVAL;
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(widen_kernel, dim3(grid_for(n)), dim3(256), 0, ctx->stream, d_in, d_out, n, value);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}

extern "C" int kman_memcpy_d2d(kman_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return KMAN_EINVAL;
    if (!bytes) return KMAN_OK;
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return KMAN_OK;
}
