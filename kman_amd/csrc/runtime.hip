// runtime.hip — context, memory, errors and look-back scratch of libkman.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

int kman_fail(kman_ctx *ctx, int code, const char *fmt, ...) {
    if (ctx) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}

int kman_hip_fail(kman_ctx *ctx, hipError_t e, const char *what) {
    const int code = (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? KMAN_ENOMEM : KMAN_EHIP;
    return kman_fail(ctx, code, "%s: %s (%s)", what, hipGetErrorName(e), hipGetErrorString(e));
}

int kman_scratch(kman_ctx *ctx, size_t bytes, void **p) {
    if (bytes > ctx->scratch_bytes) {
        if (ctx->d_scratch) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            HIP_TRY(ctx, hipFree(ctx->d_scratch));
            ctx->d_scratch = nullptr;
            ctx->scratch_bytes = 0;
        }
        size_t nb = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
        HIP_TRY(ctx, hipMalloc(&ctx->d_scratch, nb));
        ctx->scratch_bytes = nb;
    }
    *p = ctx->d_scratch;
    return KMAN_OK;
}

uint32_t kman_seg_fit(uint32_t np, const uint32_t *bits, uint32_t want, uint32_t copies, size_t lds_bytes) {
    for (uint32_t s = want; s > 1; s--) {
        size_t c = 0;
        for (uint32_t p = 0; p < np; p++) c += (size_t)s << bits[p];
        if (c * copies * 4 <= lds_bytes) return s;
    }
    return 1;
}

int kman_persistent_grid(kman_ctx *ctx, const void *fn, int threads, uint64_t n_tiles, size_t dyn_lds) {
    int per_cu = 1, cus = 256;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, dyn_lds);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
    uint64_t g = (uint64_t)(per_cu > 0 ? per_cu : 1) * (uint64_t)(cus > 0 ? cus : 1);
    if (g > n_tiles) g = n_tiles;
    return (int)(g ? g : 1);
}

int kman_aux(kman_ctx *ctx, size_t bytes, void **p) {
    if (bytes > ctx->aux_bytes) {
        if (ctx->d_aux) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            HIP_TRY(ctx, hipFree(ctx->d_aux));
            ctx->d_aux = nullptr;
            ctx->aux_bytes = 0;
        }
        size_t nb = bytes < (1u << 16) ? (1u << 16) : bytes + bytes / 4;
        HIP_TRY(ctx, hipMalloc(&ctx->d_aux, nb));
        ctx->aux_bytes = nb;
    }
    *p = ctx->d_aux;
    return KMAN_OK;
}

int kman_lookback_begin(kman_ctx *ctx, size_t words, uint32_t *epoch, uint32_t **counter) {
    if (words > ctx->status_words) {
        if (ctx->d_status) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            HIP_TRY(ctx, hipFree(ctx->d_status));
            ctx->d_status = nullptr;
            ctx->status_words = 0;
        }
        size_t nw = words < (1u << 16) ? (1u << 16) : words + words / 4;
        HIP_TRY(ctx, hipMalloc(&ctx->d_status, nw * sizeof(uint64_t)));
        ctx->status_words = nw;
        ctx->epoch = 63;  // force a reset below
    }
    if (ctx->epoch >= 63) {
        // a fresh epoch range: every status word and tile counter back to zero
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_status, 0, ctx->status_words * sizeof(uint64_t), ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_counters, 0, 64 * sizeof(uint32_t), ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_xcounters, 0, 64 * 8 * sizeof(uint32_t), ctx->stream));
        ctx->epoch = 0;
    }
    ctx->epoch++;
    *epoch = ctx->epoch;
    *counter = ctx->d_counters + ctx->epoch;
    return KMAN_OK;
}

int kman_check_device_error(kman_ctx *ctx) {
    uint32_t e = 0;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_small + 8, ctx->d_err, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    memcpy(&e, ctx->h_small + 8, sizeof e);
    if (e) {
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_err, 0, sizeof(uint32_t), ctx->stream));
        return kman_fail(ctx, KMAN_ETIMEOUT, "device look-back wait exceeded its bound (code %u)", e);
    }
    return KMAN_OK;
}

int kman_lookback_total(kman_ctx *ctx, uint64_t n_tiles, uint64_t *total) {
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_small + 4, ctx->d_status + (n_tiles - 1), sizeof(uint64_t),
                                hipMemcpyDeviceToHost, ctx->stream));
    KMAN_TRY(kman_check_device_error(ctx));  // synchronises
    const uint64_t w = ctx->h_small[4];
    const uint32_t ep = (uint32_t)((w >> 56) & 63u);
    if (ep != ctx->epoch || (w >> 62) != ST_INCL)
        return kman_fail(ctx, KMAN_EHIP, "look-back total not published (word %016llx, epoch %u)",
                         (unsigned long long)w, ctx->epoch);
    *total = w & ST_VMASK;
    return KMAN_OK;
}

// Probe: do same-address LDS atomics of one wave return old values in lane
// order?  (Stable atomic ranking in sort.hip depends on it.)
__global__ void lds_order_probe(uint32_t *bad) {
    __shared__ uint32_t c[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) c[i] = 0;
    __syncthreads();
    uint32_t nbad = 0;
    const int lane = threadIdx.x & 63;
    for (int it = 0; it < 32; it++) {
        uint32_t h = (lane * 2654435761u) ^ (it * 40503u) ^ (blockIdx.x * 97u) ^ (threadIdx.x >> 6);
        h ^= h >> 13;
        const uint32_t d = h % (1u + (it & 127));
        const uint32_t old = atomicAdd(&c[d], 1u);
        for (int o = 0; o < lane; o++) {
            const uint32_t od = (uint32_t)__shfl((int)d, o, 64);
            const uint32_t ov = (uint32_t)__shfl((int)old, o, 64);
            nbad += (od == d && ov > old);
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

static bool probe_lds_order(kman_ctx *ctx) {
    uint32_t *d = nullptr, h = 1;
    if (hipMalloc(&d, 4) != hipSuccess) return false;
    bool ok = hipMemsetAsync(d, 0, 4, ctx->stream) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(lds_order_probe, dim3(512), dim3(256), 0, ctx->stream, d);
        ok = hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess &&
             hipStreamSynchronize(ctx->stream) == hipSuccess;
    }
    (void)hipFree(d);
    return ok && h == 0;
}

static hipEvent_t pool_event(kman_ctx *ctx) {
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

KTimer::KTimer(kman_ctx *c, const char *tag) : ctx(c), idx((size_t)-1) {
    if (!ctx->timing) return;
    kman_ctx::TimedLaunch t{tag, pool_event(ctx), pool_event(ctx)};
    (void)hipEventRecord(t.a, ctx->stream);
    idx = ctx->launches.size();
    ctx->launches.push_back(t);
}

KTimer::~KTimer() {
    if (idx != (size_t)-1) (void)hipEventRecord(ctx->launches[idx].b, ctx->stream);
}

static void timing_clear(kman_ctx *ctx) {
    for (auto &t : ctx->launches) {
        ctx->event_pool.push_back(t.a);
        ctx->event_pool.push_back(t.b);
    }
    ctx->launches.clear();
}

extern "C" {

int kman_timing_enable(kman_ctx *ctx, int enable) {
    if (!ctx) return KMAN_EINVAL;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    timing_clear(ctx);
    ctx->timing = enable != 0;
    return KMAN_OK;
}

int kman_timing_query(kman_ctx *ctx, const char *tag, uint64_t *launches, double *total_ms) {
    if (!ctx || !tag || !launches || !total_ms) return KMAN_EINVAL;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t n = 0;
    double ms = 0;
    for (auto &t : ctx->launches) {
        if (strcmp(t.tag, tag) != 0) continue;
        float f = 0;
        HIP_TRY(ctx, hipEventElapsedTime(&f, t.a, t.b));
        ms += f;
        n++;
    }
    *launches = n;
    *total_ms = ms;
    return KMAN_OK;
}

int kman_abi_version(void) { return KMAN_ABI_VERSION; }

int kman_device_count(int *n) {
    if (!n) return KMAN_EINVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return KMAN_OK;
}

int kman_create(int device, kman_ctx **out) {
    if (!out) return KMAN_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return KMAN_EHIP;
    if (device < 0 || device >= n) return KMAN_EINVAL;
    kman_ctx *ctx = new kman_ctx();
    ctx->device = device;
    auto bail = [&](hipError_t e, const char *what) {
        kman_hip_fail(ctx, e, what);
        kman_destroy(ctx);
        return (e == hipErrorOutOfMemory) ? KMAN_ENOMEM : KMAN_EHIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return bail(e, "hipSetDevice");
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess)
        return bail(e, "hipStreamCreate");
    if ((e = hipMalloc(&ctx->d_counters, 64 * sizeof(uint32_t) + 256)) != hipSuccess) return bail(e, "hipMalloc");
    ctx->d_err = ctx->d_counters + 64;
    if ((e = hipMemset(ctx->d_counters, 0, 64 * sizeof(uint32_t) + 256)) != hipSuccess) return bail(e, "hipMemset");
    if ((e = hipMalloc(&ctx->d_xcounters, 64 * 8 * sizeof(uint32_t))) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMemset(ctx->d_xcounters, 0, 64 * 8 * sizeof(uint32_t))) != hipSuccess) return bail(e, "hipMemset");
    if ((e = hipMalloc(&ctx->d_cursors, 256 * 64 * sizeof(uint32_t))) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipHostMalloc(&ctx->h_small, 4096, hipHostMallocDefault)) != hipSuccess) return bail(e, "hipHostMalloc");
    const char *force = getenv("KMAN_RANK");  // "ballot" forces the probe-free ranking
    ctx->lds_atomic_ordered = !(force && strcmp(force, "ballot") == 0) && probe_lds_order(ctx);
    *out = ctx;
    return KMAN_OK;
}

void kman_destroy(kman_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->comm) kman_comm_destroy(ctx);
    timing_clear(ctx);
    for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
    if (ctx->d_status) (void)hipFree(ctx->d_status);
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    if (ctx->d_aux) (void)hipFree(ctx->d_aux);
    if (ctx->d_hv) (void)hipFree(ctx->d_hv);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    if (ctx->d_xcounters) (void)hipFree(ctx->d_xcounters);
    if (ctx->d_cursors) (void)hipFree(ctx->d_cursors);
    if (ctx->d_mapbits) (void)hipFree(ctx->d_mapbits);
    if (ctx->h_small) (void)hipHostFree(ctx->h_small);
    if (ctx->copy_stream) {
        (void)hipStreamSynchronize(ctx->copy_stream);
        (void)hipStreamDestroy(ctx->copy_stream);
    }
    for (auto e : ctx->d2h_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->work_ev) (void)hipEventDestroy(ctx->work_ev);
    for (auto e : ctx->copy_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->comm_stream) {
        (void)hipStreamSynchronize(ctx->comm_stream);
        (void)hipStreamDestroy(ctx->comm_stream);
    }
    if (ctx->comm_pre) (void)hipEventDestroy(ctx->comm_pre);
    for (auto e : ctx->comm_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *kman_last_error(const kman_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int kman_sync(kman_ctx *ctx) {
    if (!ctx) return KMAN_EINVAL;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return kman_check_device_error(ctx);
}

int kman_malloc(kman_ctx *ctx, void **dptr, size_t bytes) {
    if (!ctx || !dptr) return KMAN_EINVAL;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipMalloc(dptr, bytes ? bytes : 1));
    return KMAN_OK;
}

int kman_mem_info(kman_ctx *ctx, size_t *free_bytes, size_t *total_bytes) {
    if (!ctx || !free_bytes || !total_bytes) return KMAN_EINVAL;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipMemGetInfo(free_bytes, total_bytes));
    return KMAN_OK;
}

int kman_free(kman_ctx *ctx, void *dptr) {
    if (!ctx) return KMAN_EINVAL;
    if (!dptr) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(dptr));
    return KMAN_OK;
}

int kman_host_alloc(kman_ctx *ctx, void **hptr, size_t bytes) {
    if (!ctx || !hptr) return KMAN_EINVAL;
    HIP_TRY(ctx, hipHostMalloc(hptr, bytes ? bytes : 1, hipHostMallocDefault));
    return KMAN_OK;
}

int kman_host_free(kman_ctx *ctx, void *hptr) {
    if (!ctx) return KMAN_EINVAL;
    if (hptr) HIP_TRY(ctx, hipHostFree(hptr));
    return KMAN_OK;
}

int kman_memcpy_h2d(kman_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return KMAN_EINVAL;
    if (!bytes) return KMAN_OK;
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KMAN_OK;
}

int kman_memcpy_d2h(kman_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return KMAN_EINVAL;
    if (!bytes) return KMAN_OK;
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KMAN_OK;
}

int kman_copy_h2d_async(kman_ctx *ctx, void *dst, const void *src, size_t bytes, int slot) {
    if (!ctx || slot < 0 || slot >= 4) return KMAN_EINVAL;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->copy_stream) HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    if (!ctx->copy_ev[slot]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->copy_ev[slot], hipEventDisableTiming));
    if (bytes) HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->copy_stream));
    HIP_TRY(ctx, hipEventRecord(ctx->copy_ev[slot], ctx->copy_stream));
    return KMAN_OK;
}

int kman_copy_wait(kman_ctx *ctx, int slot) {
    if (!ctx || slot < 0 || slot >= 4 || !ctx->copy_ev[slot]) return KMAN_EINVAL;
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->copy_ev[slot], 0));
    return KMAN_OK;
}

// D2H on the copy stream after the work already queued on the work stream
// (the text formatted into `src`), completion marked in d2h slot 0..3; the
// work stream keeps going (the next slice is formatted meanwhile)
int kman_copy_d2h_async(kman_ctx *ctx, void *dst, const void *src, size_t bytes, int slot) {
    if (!ctx || slot < 0 || slot >= 4) return KMAN_EINVAL;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->copy_stream) HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    if (!ctx->work_ev) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->work_ev, hipEventDisableTiming));
    if (!ctx->d2h_ev[slot]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->d2h_ev[slot], hipEventDisableTiming));
    HIP_TRY(ctx, hipEventRecord(ctx->work_ev, ctx->stream));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->copy_stream, ctx->work_ev, 0));
    if (bytes) HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->copy_stream));
    HIP_TRY(ctx, hipEventRecord(ctx->d2h_ev[slot], ctx->copy_stream));
    return KMAN_OK;
}

// the host waits for the D2H marked in `slot` (callable from any host thread)
int kman_copy_d2h_wait(kman_ctx *ctx, int slot) {
    if (!ctx || slot < 0 || slot >= 4 || !ctx->d2h_ev[slot]) return KMAN_EINVAL;
    HIP_TRY(ctx, hipEventSynchronize(ctx->d2h_ev[slot]));
    return KMAN_OK;
}

int kman_copy_sync(kman_ctx *ctx) {
    if (!ctx) return KMAN_EINVAL;
    if (ctx->copy_stream) HIP_TRY(ctx, hipStreamSynchronize(ctx->copy_stream));
    return KMAN_OK;
}

int kman_memset(kman_ctx *ctx, void *dst, int value, size_t bytes) {
    if (!ctx) return KMAN_EINVAL;
    if (!bytes) return KMAN_OK;
    HIP_TRY(ctx, hipMemsetAsync(dst, value, bytes, ctx->stream));
    return KMAN_OK;
}

}  // extern "C"
