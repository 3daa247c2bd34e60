// ops.hip — small device helpers used by the host API around the hot path.
//
//   kman_tag_batches  keys[i] |= ((first + i) / batch_size) << key_bits
//                     makes one stable sort over (batch, key) equal to a stable
//                     sort of every batch on its own — the per-batch
//                     Batch.sorted of the reference (batch.py:156-168) for all
//                     batches in one pass sequence.
//   kman_or_u64       v[i] |= value (tags payloads with a source id).
//   kman_memcpy_d2d   device-to-device copy on the context stream.
//   kman_rebase_pos   (source << 56 | local pos) -> global pos, per-source
//                     base offsets (byte-range shards, kman_amd/dist.py).
//   kman_synth_fasta  bytes [lo, lo + n) of the synthetic benchmark FASTA
//                     (records syn<i>, fixed-width lines, base = hash(seed,
//                     base index)), so each rank generates its own byte range
//                     of ONE global file (tests/golden/inputs.py synth_np).
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

__global__ void rebase_kernel(uint64_t *__restrict__ v, uint64_t n, const uint64_t *__restrict__ off) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = v[i];
        v[i] = (p & ((1ull << 56) - 1)) + (off[p >> 56] << 1);
    }
}

KMAN_DEV uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct SynthRec {  // record r: header at byte hb, first base index bb, L bases
    uint64_t hb, bb, L;
};

// one thread = 16 output bytes; records in a small table (binary search)
__global__ void synth_kernel(uint8_t *__restrict__ out, uint64_t lo, uint64_t n, uint64_t seed,
                             const SynthRec *__restrict__ rec, uint32_t nrec, uint32_t line) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t o0 = t * 16;
    if (o0 >= n) return;
    uint32_t a = 0, b = nrec;  // last record with hb <= lo + o0
    while (b - a > 1) {
        const uint32_t m = (a + b) / 2;
        if (rec[m].hb <= lo + o0) a = m;
        else b = m;
    }
    uint32_t r = a;
    uint8_t c[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint64_t g = lo + o0 + j;
        while (r + 1 < nrec && rec[r + 1].hb <= g) r++;
        // header ">syn<r>\n"
        uint32_t nd = 1;
        for (uint32_t x = r; x >= 10; x /= 10) nd++;
        const uint64_t hl = 5 + nd;
        const uint64_t rel = g - rec[r].hb;
        uint8_t ch;
        if (rel < hl) {
            if (rel == 0) ch = '>';
            else if (rel < 4) ch = "syn"[rel - 1];
            else if (rel == hl - 1) ch = '\n';
            else {
                uint32_t x = r;
                for (uint64_t q = hl - 2; q > rel; q--) x /= 10;
                ch = (uint8_t)('0' + x % 10);
            }
        } else {
            const uint64_t rel2 = rel - hl, ln = rel2 / (line + 1), col = rel2 % (line + 1);
            const uint64_t bi = ln * line + col;  // base index in the record
            if (col == line || bi >= rec[r].L) ch = '\n';
            else ch = "ACGT"[splitmix64(seed * 0xD1B54A32D192ED03ull + rec[r].bb + bi) >> 62];
        }
        c[j] = ch;
    }
    if (o0 + 16 <= n) {
        uint4 v;
        v.x = c[0] | (c[1] << 8) | (c[2] << 16) | ((uint32_t)c[3] << 24);
        v.y = c[4] | (c[5] << 8) | (c[6] << 16) | ((uint32_t)c[7] << 24);
        v.z = c[8] | (c[9] << 8) | (c[10] << 16) | ((uint32_t)c[11] << 24);
        v.w = c[12] | (c[13] << 8) | (c[14] << 16) | ((uint32_t)c[15] << 24);
        *reinterpret_cast<uint4 *>(out + o0) = v;
    } else {
        for (int j = 0; j < 16; j++)
            if (o0 + j < n) out[o0 + j] = c[j];
    }
}

__global__ void iota_kernel(uint64_t *__restrict__ v, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        v[i] = i;
}

template <typename T>
__global__ void gather_kernel(const T *__restrict__ src, const uint64_t *__restrict__ idx, uint64_t n,
                              T *__restrict__ dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[idx[i]];
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

extern "C" int kman_rebase_pos(kman_ctx *ctx, uint64_t *d_pos, uint64_t n, const uint64_t *offsets, uint32_t nsrc) {
    if (!ctx || (nsrc && !offsets) || nsrc > 256) return KMAN_EINVAL;
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    void *tab;
    KMAN_TRY(kman_scratch(ctx, 256 * 8, &tab));
    uint64_t h[256] = {0};
    for (uint32_t i = 0; i < nsrc; i++) h[i] = offsets[i];
    HIP_TRY(ctx, hipMemcpyAsync(tab, h, sizeof h, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(rebase_kernel, dim3(grid_for(n)), dim3(256), 0, ctx->stream, d_pos, n, (const uint64_t *)tab);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // (h must outlive the copy)
    return KMAN_OK;
}

extern "C" int kman_synth_fasta(kman_ctx *ctx, uint8_t *d_out, uint64_t byte_lo, uint64_t n_bytes, uint64_t seed,
                                const uint64_t *rec_tab, uint32_t n_records, uint32_t line) {
    if (!ctx || !rec_tab || n_records == 0 || line == 0) return KMAN_EINVAL;
    if (((uintptr_t)d_out & 15) != 0) return kman_fail(ctx, KMAN_EINVAL, "output must be 16-byte aligned");
    if (n_bytes == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    void *tab;
    KMAN_TRY(kman_aux(ctx, (size_t)n_records * sizeof(SynthRec), &tab));
    HIP_TRY(ctx, hipMemcpyAsync(tab, rec_tab, (size_t)n_records * sizeof(SynthRec), hipMemcpyHostToDevice,
                                ctx->stream));
    const uint64_t threads = ceil_div(n_bytes, 16);
    hipLaunchKernelGGL(synth_kernel, dim3((uint32_t)ceil_div(threads, 256)), dim3(256), 0, ctx->stream, d_out, byte_lo,
                       n_bytes, seed, (const SynthRec *)tab, n_records, line);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KMAN_OK;
}

extern "C" int kman_iota_u64(kman_ctx *ctx, uint64_t *d_v, uint64_t n) {
    if (!ctx) return KMAN_EINVAL;
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(iota_kernel, dim3(grid_for(n)), dim3(256), 0, ctx->stream, d_v, n);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}

extern "C" int kman_gather(kman_ctx *ctx, const void *d_src, const uint64_t *d_idx, uint64_t n, void *d_dst,
                           uint32_t elem_bytes) {
    if (!ctx) return KMAN_EINVAL;
    if (elem_bytes != 4 && elem_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "elem_bytes must be 4 or 8");
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (elem_bytes == 8)
        hipLaunchKernelGGL(gather_kernel<uint64_t>, dim3(grid_for(n)), dim3(256), 0, ctx->stream,
                           (const uint64_t *)d_src, d_idx, n, (uint64_t *)d_dst);
    else
        hipLaunchKernelGGL(gather_kernel<uint32_t>, dim3(grid_for(n)), dim3(256), 0, ctx->stream,
                           (const uint32_t *)d_src, d_idx, n, (uint32_t *)d_dst);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}
