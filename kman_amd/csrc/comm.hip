// comm.hip — multi-GPU exchange over RCCL (xGMI), one process per GPU.
//
// The reference has no collective at all (its "parallelism" is joblib process
// pools over temp files); the exchange below is the single step
// the MI355X design needs to split the global join across GPUs:
//   1. every rank histograms the top bits of its keys (kman_prefix_hist),
//   2. kman_allreduce_u64 sums the histograms, the host picks contiguous
//      prefix ranges balanced to ~N/G keys per rank (kman_amd/dist.py),
//   3. kman_partition (sort.hip) groups each rank's keys by destination,
//   4. kman_alltoallv moves every group to its rank (grouped send/recv; on
//      xGMI every peer pair has its own link),
//   5. each rank sorts + run-length-groups what it received; rank order of
//      the prefix ranges makes the concatenated outputs globally sorted.
#include <rccl/rccl.h>

#include "common.h"

namespace {

struct Comm {
    ncclComm_t comm = nullptr;
    // a second communicator (ncclCommSplit of the first, same ranks) for the
    // all-to-alls queued on the communication stream: the two streams never
    // issue work on one communicator, so RCCL's per-communicator ordering
    // cannot interleave the overlapped exchanges with the compute stream's
    // all-reduces and all-gathers
    ncclComm_t comm2 = nullptr;
    int rank = 0, nranks = 1;
};

// one communicator per context (contexts are per GPU / per process)
Comm *comm_of(kman_ctx *ctx) { return reinterpret_cast<Comm *>(ctx->comm); }

int nccl_fail(kman_ctx *ctx, ncclResult_t r, const char *what) {
    return kman_fail(ctx, KMAN_ECOMM, "%s: %s", what, ncclGetErrorString(r));
}

#define NCCL_TRY(ctx, expr)                                   \
    do {                                                      \
        ncclResult_t _r = (expr);                             \
        if (_r != ncclSuccess) return nccl_fail(ctx, _r, #expr); \
    } while (0)

__global__ __launch_bounds__(256) void prefix_hist_kernel(const uint64_t *__restrict__ keys, uint64_t n,
                                                          uint32_t shift, uint32_t bits,
                                                          unsigned long long *__restrict__ hist) {
    extern __shared__ uint32_t lh[];
    const uint32_t nb = 1u << bits;
    for (uint32_t i = threadIdx.x; i < nb; i += 256) lh[i] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        atomicAdd(&lh[(uint32_t)(keys[i] >> shift) & (nb - 1)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += 256)
        if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
}

}  // namespace

extern "C" int kman_comm_unique_id(uint8_t *out128) {
    if (!out128) return KMAN_EINVAL;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return KMAN_ECOMM;
    memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return KMAN_OK;
}

extern "C" int kman_comm_init(kman_ctx *ctx, const uint8_t *id128, int nranks, int rank) {
    if (!ctx || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return KMAN_EINVAL;
    if (ctx->comm) return kman_fail(ctx, KMAN_EINVAL, "communicator already initialised");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    ncclUniqueId id;
    memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    Comm *c = new Comm();
    c->rank = rank;
    c->nranks = nranks;
    const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail(ctx, r, "ncclCommInitRank");
    }
    const ncclResult_t r2 = ncclCommSplit(c->comm, 0, rank, &c->comm2, nullptr);
    if (r2 != ncclSuccess) {
        ncclCommDestroy(c->comm);
        delete c;
        return nccl_fail(ctx, r2, "ncclCommSplit");
    }
    ctx->comm = c;
    return KMAN_OK;
}

extern "C" int kman_comm_count(kman_ctx *ctx, int *nranks, int *rank) {
    if (!ctx || !nranks || !rank) return KMAN_EINVAL;
    Comm *c = comm_of(ctx);
    if (!c) return kman_fail(ctx, KMAN_EINVAL, "no communicator");
    NCCL_TRY(ctx, ncclCommCount(c->comm, nranks));
    NCCL_TRY(ctx, ncclCommUserRank(c->comm, rank));
    return KMAN_OK;
}

extern "C" int kman_comm_destroy(kman_ctx *ctx) {
    if (!ctx) return KMAN_EINVAL;
    Comm *c = comm_of(ctx);
    if (!c) return KMAN_OK;
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->comm_stream) (void)hipStreamSynchronize(ctx->comm_stream);
    if (c->comm2) ncclCommDestroy(c->comm2);
    ncclCommDestroy(c->comm);
    delete c;
    ctx->comm = nullptr;
    return KMAN_OK;
}

extern "C" int kman_allreduce_u64(kman_ctx *ctx, uint64_t *d_buf, uint64_t n) {
    if (!ctx) return KMAN_EINVAL;
    Comm *c = comm_of(ctx);
    if (!c) return kman_fail(ctx, KMAN_EINVAL, "no communicator");
    NCCL_TRY(ctx, ncclAllReduce(d_buf, d_buf, n, ncclUint64, ncclSum, c->comm, ctx->stream));
    return KMAN_OK;
}

extern "C" int kman_allgather_u64(kman_ctx *ctx, const uint64_t *d_send, uint64_t *d_recv, uint64_t n) {
    if (!ctx) return KMAN_EINVAL;
    Comm *c = comm_of(ctx);
    if (!c) return kman_fail(ctx, KMAN_EINVAL, "no communicator");
    NCCL_TRY(ctx, ncclAllGather(d_send, d_recv, n, ncclUint64, c->comm, ctx->stream));
    return KMAN_OK;
}

// All-to-all-v of elem_bytes elements: send_counts/offsets and
// recv_counts/offsets are host arrays of nranks elements (in elements).
namespace {
int alltoallv_on(kman_ctx *ctx, hipStream_t st, bool second, const void *d_send, const uint64_t *send_counts,
                 const uint64_t *send_offsets, void *d_recv, const uint64_t *recv_counts,
                 const uint64_t *recv_offsets, uint32_t elem_bytes) {
    if (!ctx || !send_counts || !send_offsets || !recv_counts || !recv_offsets) return KMAN_EINVAL;
    if (elem_bytes != 4 && elem_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "elem_bytes must be 4 or 8");
    Comm *c = comm_of(ctx);
    if (!c) return kman_fail(ctx, KMAN_EINVAL, "no communicator");
    ncclComm_t cm = second ? c->comm2 : c->comm;
    const ncclDataType_t t = elem_bytes == 8 ? ncclUint64 : ncclUint32;
    // messages in chunks of <= 512 MiB: a single multi-GiB send/recv pair
    // was observed to move only part of its bytes (RCCL 2.27, 2.4 GB to self);
    // both ends derive the same chunk sequence from the same count
    const uint64_t CH = (512ull << 20) / elem_bytes;
    // the rank's own part is a device copy on the same stream (RCCL's
    // send/recv to self moved 8 GB at 1.34 TB/s, `profiles/r06b_bench_d1_on.json`)
    // (KMAN_RCCL_SELF=1: through RCCL as every other peer -- tests of the
    // chunked send/recv at world size 1)
    const char *rs = getenv("KMAN_RCCL_SELF");
    const bool rccl_self = rs && rs[0] == '1';
    const int me = rccl_self ? -1 : c->rank;
    if (me >= 0 && send_counts[me] != recv_counts[me])
        return kman_fail(ctx, KMAN_EINVAL, "alltoallv: %llu items sent to self, %llu expected",
                         (unsigned long long)send_counts[me], (unsigned long long)recv_counts[me]);
    if (me >= 0 && send_counts[me])
        HIP_TRY(ctx, hipMemcpyAsync((char *)d_recv + recv_offsets[me] * elem_bytes,
                                    (const char *)d_send + send_offsets[me] * elem_bytes, send_counts[me] * elem_bytes,
                                    hipMemcpyDeviceToDevice, st));
    uint64_t rounds = 0;
    for (int p = 0; p < c->nranks; p++) {
        if (p == me) continue;
        const uint64_t a = (send_counts[p] + CH - 1) / CH, b = (recv_counts[p] + CH - 1) / CH;
        rounds = a > rounds ? a : rounds;
        rounds = b > rounds ? b : rounds;
    }
    for (uint64_t r = 0; r < rounds; r++) {
        NCCL_TRY(ctx, ncclGroupStart());
        for (int p = 0; p < c->nranks; p++) {
            if (p == me) continue;
            const uint64_t o = r * CH;
            if (send_counts[p] > o) {
                const uint64_t n = send_counts[p] - o < CH ? send_counts[p] - o : CH;
                NCCL_TRY(ctx, ncclSend((const char *)d_send + (send_offsets[p] + o) * elem_bytes, n, t, p, cm, st));
            }
            if (recv_counts[p] > o) {
                const uint64_t n = recv_counts[p] - o < CH ? recv_counts[p] - o : CH;
                NCCL_TRY(ctx, ncclRecv((char *)d_recv + (recv_offsets[p] + o) * elem_bytes, n, t, p, cm, st));
            }
        }
        NCCL_TRY(ctx, ncclGroupEnd());
    }
    return KMAN_OK;
}
}  // namespace

extern "C" int kman_alltoallv(kman_ctx *ctx, const void *d_send, const uint64_t *send_counts,
                              const uint64_t *send_offsets, void *d_recv, const uint64_t *recv_counts,
                              const uint64_t *recv_offsets, uint32_t elem_bytes) {
    if (!ctx) return KMAN_EINVAL;
    KTimer kt_(ctx, "exchange");  // (the grouped send/recv on the compute stream, between HIP events)
    return alltoallv_on(ctx, ctx->stream, false, d_send, send_counts, send_offsets, d_recv, recv_counts, recv_offsets,
                        elem_bytes);
}

// The same on the context's communication stream, after the work already
// queued on its compute stream (which produced d_send); completion is
// recorded in event `slot` (0..7) for kman_comm_wait.  The compute stream
// keeps going meanwhile: the exchange of one part overlaps the work on the
// parts already received.
extern "C" int kman_alltoallv_async(kman_ctx *ctx, const void *d_send, const uint64_t *send_counts,
                                    const uint64_t *send_offsets, void *d_recv, const uint64_t *recv_counts,
                                    const uint64_t *recv_offsets, uint32_t elem_bytes, int slot) {
    if (!ctx || slot < 0 || slot >= 8) return KMAN_EINVAL;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->comm_stream) HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking));
    if (!ctx->comm_pre) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->comm_pre, hipEventDisableTiming));
    if (!ctx->comm_ev[slot]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->comm_ev[slot], hipEventDisableTiming));
    HIP_TRY(ctx, hipEventRecord(ctx->comm_pre, ctx->stream));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->comm_stream, ctx->comm_pre, 0));
    KMAN_TRY(alltoallv_on(ctx, ctx->comm_stream, true, d_send, send_counts, send_offsets, d_recv, recv_counts, recv_offsets,
                          elem_bytes));
    HIP_TRY(ctx, hipEventRecord(ctx->comm_ev[slot], ctx->comm_stream));
    return KMAN_OK;
}

// the compute stream waits for the exchange recorded in `slot`
extern "C" int kman_comm_wait(kman_ctx *ctx, int slot) {
    if (!ctx || slot < 0 || slot >= 8) return KMAN_EINVAL;
    if (!ctx->comm_ev[slot]) return KMAN_OK;
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->comm_ev[slot], 0));
    return KMAN_OK;
}

extern "C" int kman_prefix_hist(kman_ctx *ctx, const uint64_t *d_keys, uint64_t n, uint32_t shift, uint32_t bits,
                                uint64_t *d_hist) {
    if (!ctx || bits < 1 || bits > 14) return ctx ? kman_fail(ctx, KMAN_EINVAL, "hist bits must be 1..14") : KMAN_EINVAL;
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t blocks = ceil_div(n, 256 * 32);
    KTimer kt_(ctx, "prefix_hist");
    hipLaunchKernelGGL(prefix_hist_kernel, dim3((uint32_t)(blocks < 2048 ? blocks : 2048)), dim3(256),
                       (size_t)(4u << bits), ctx->stream, d_keys, n, shift, bits, (unsigned long long *)d_hist);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}
