// rle.hip — run-length grouping of sorted keys: count and uniq.
//
// Replaces the group loop of Crawler.do_batch (kmermaid/join.py:95-130) fed
// by the heap merge, and the two join functions on the hot path:
//   join_sequence_count (join.py:266-285): one (key, group size) per group;
//   join_unique         (join.py:244-263): the group only if it has exactly one
//                                          member, with that member's header.
// Both are single-pass tile kernels (256 threads x 16 keys) with decoupled
// look-back: count needs the number of groups before the tile (sum) and, for
// a tile that starts inside a group, the position of that group's head (max
// of head positions; a tile holding any head publishes it as inclusive at
// once, so the chain is short).  uniq keeps keys that differ from both
// neighbours and needs only the sum.
//
// Algorithmic bytes: count 8 B read + (8 + 4|8) B per group written;
// uniq 8 B key read (+ payload of kept keys) + (8 + 4|8) B per kept key.
#include "common.h"

#include <vector>

namespace {

constexpr int RT = 256;
constexpr int RI = 16;
constexpr int RTILE = RT * RI;

struct MaxU64 {
    KMAN_DEV uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; }
};

KMAN_DEV void stage_keys(const uint64_t *__restrict__ keys, uint64_t n, uint64_t tb, uint64_t *s) {
    for (int i = threadIdx.x; i < RTILE; i += RT) {
        const uint64_t idx = tb + i;
        s[i] = idx < n ? keys[idx] : 0;
    }
}

// look-back for "position of the last group head + 1" (max); a tile with a head
// publishes its own value as inclusive immediately.
KMAN_DEV uint64_t wave_lookback_lasthead(uint64_t *status, int64_t tile, uint64_t agg, bool need, uint32_t epoch,
                                         uint32_t *err) {
    const int lane = lane_id();
    if (agg != 0 || tile == 0) {
        if (lane == 0) st_store(&status[tile], st_make(ST_INCL, epoch, agg));
        if (!need || tile == 0) return 0;
    }
    if (agg == 0 && lane == 0) st_store(&status[tile], st_make(ST_AGG, epoch, 0));
    uint64_t best = 0;
    int64_t end = tile;
    uint32_t spins = 0;
    for (;;) {
        const int64_t j = end - 1 - lane;
        uint64_t w = 0, f = ST_INCL;
        if (j >= 0) {
            w = st_load(&status[j]);
            f = st_flag(w, epoch);
        }
        const uint64_t v = j >= 0 ? (w & ST_VMASK) : 0;
        const uint64_t notready = __ballot(j >= 0 && f == 0);
        // stop at the nearest tile whose value is final: INCL, or AGG with a head
        const uint64_t fin = __ballot(j >= 0 && (f == ST_INCL || (f == ST_AGG && v != 0)));
        const int first = fin ? __ffsll((unsigned long long)fin) - 1 : 64;
        const uint64_t need_m = first == 64 ? ~0ull : (~0ull >> (63 - first));
        if (notready & need_m) {
            if (spin_give_up(spins, err, 4u)) break;
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        if (first < 64) {
            best = shfl_any(v, first);
            break;
        }
        if (end - 64 <= 0) break;
        end -= 64;
    }
    if (agg == 0 && lane == 0) st_store(&status[tile], st_make(ST_INCL, epoch, best));
    return best;
}

template <typename C>
__global__ __launch_bounds__(RT) void rle_count_kernel(const uint64_t *__restrict__ keys, uint64_t n,
                                                       uint64_t *__restrict__ ukeys, C *__restrict__ counts,
                                                       uint64_t *__restrict__ st_sum, uint64_t *__restrict__ st_max,
                                                       uint32_t *__restrict__ counter, uint32_t epoch,
                                                       uint32_t *__restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint64_t s[RTILE];
    __shared__ __attribute__((aligned(16))) C sc[RTILE];
    __shared__ uint32_t lds_scan[RT / 64];
    __shared__ uint64_t lds_scan64[RT / 64];
    __shared__ uint64_t lds_base, lds_head;
    __shared__ uint32_t lds_tile;
    const int64_t tile = grab_tile(counter, &lds_tile);
    const uint64_t tb = (uint64_t)tile * RTILE;
    stage_keys(keys, n, tb, s);
    const uint64_t prev_key = tb ? keys[tb - 1] : 0;
    const uint64_t next_key = tb + RTILE < n ? keys[tb + RTILE] : 0;
    __syncthreads();
    const uint32_t t0 = threadIdx.x * RI;
    uint64_t k[RI];
#pragma unroll
    for (int j = 0; j < RI; j++) k[j] = s[t0 + j];
    uint32_t heads = 0, tails = 0;
#pragma unroll
    for (int j = 0; j < RI; j++) {
        const uint64_t i = tb + t0 + j;
        const uint64_t pk = j ? k[j - 1] : (t0 ? s[t0 - 1] : prev_key);
        const uint64_t nk = j + 1 < RI ? k[j + 1] : (t0 + RI < (uint32_t)RTILE ? s[t0 + RI] : next_key);
        const bool in = i < n;
        heads |= (uint32_t)(in && (i == 0 || k[j] != pk)) << j;
        tails |= (uint32_t)(in && (i == n - 1 || k[j] != nk)) << j;
    }
    const uint32_t nh = __popc(heads);
    // last head position + 1 within this thread (0 = none)
    const uint64_t lh = heads ? tb + t0 + (31 - __clz(heads)) + 1 : 0;
    uint32_t tile_heads;
    const uint32_t hoff = block_exclusive_scan<RT>(nh, SumU32(), 0u, lds_scan, &tile_heads);
    uint64_t tile_lh;
    const uint64_t lh_before = block_exclusive_scan<RT>(lh, MaxU64(), (uint64_t)0, lds_scan64, &tile_lh);
    if (threadIdx.x < 64) {
        const uint64_t b = wave_lookback<0>(st_sum, tile, tile_heads, epoch, err);
        const bool first_is_head = tb == 0 || s[0] != prev_key;
        const uint64_t h = wave_lookback_lasthead(st_max, tile, tile_lh, !first_is_head, epoch, err);
        if (threadIdx.x == 0) {
            lds_base = b;
            lds_head = h;
        }
    }
    __syncthreads();
    const uint64_t base = lds_base;
    uint64_t cur_head = lh_before ? lh_before : lds_head;  // head position + 1 of the open group
    uint64_t slot = base + hoff;                           // groups opened before this key
    // the tile's tails fill global slots [out0, out0 + tile_tails): stage them
    // in LDS (keys over s, counts in sc) and write both out coalesced
    const bool first_is_head = tb == 0 || s[0] != prev_key;
    const uint64_t out0 = base - (first_is_head ? 0 : 1);
    uint32_t tile_tails;
    block_exclusive_scan<RT>((uint32_t)__popc(tails), SumU32(), 0u, lds_scan, &tile_tails);
#pragma unroll
    for (int j = 0; j < RI; j++) {
        const uint64_t i = tb + t0 + j;
        if ((heads >> j) & 1u) {
            cur_head = i + 1;
            slot++;
        }
        if ((tails >> j) & 1u) {
            const uint32_t q = (uint32_t)(slot - 1 - out0);
            s[q] = k[j];
            sc[q] = (C)(i + 2 - cur_head);
        }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < tile_tails; q += RT) {
        ukeys[out0 + q] = s[q];
        counts[out0 + q] = sc[q];
    }
}

template <typename V>
__global__ __launch_bounds__(RT) void rle_uniq_kernel(const uint64_t *__restrict__ keys, const V *__restrict__ vals,
                                                      uint64_t n, uint64_t *__restrict__ okeys, V *__restrict__ ovals,
                                                      uint64_t *__restrict__ st_sum, uint32_t *__restrict__ counter,
                                                      uint32_t epoch, uint32_t *__restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint64_t s[RTILE];
    __shared__ __attribute__((aligned(16))) V sv[RTILE];
    __shared__ uint32_t lds_scan[RT / 64];
    __shared__ uint64_t lds_base;
    __shared__ uint32_t lds_tile;
    const int64_t tile = grab_tile(counter, &lds_tile);
    const uint64_t tb = (uint64_t)tile * RTILE;
    stage_keys(keys, n, tb, s);
    for (int i = threadIdx.x; i < RTILE; i += RT) {
        const uint64_t idx = tb + i;
        sv[i] = idx < n ? vals[idx] : (V)0;
    }
    const uint64_t prev_key = tb ? keys[tb - 1] : 0;
    const uint64_t next_key = tb + RTILE < n ? keys[tb + RTILE] : 0;
    __syncthreads();
    const uint32_t t0 = threadIdx.x * RI;
    uint64_t k[RI];
    V v[RI];
#pragma unroll
    for (int j = 0; j < RI; j++) {
        k[j] = s[t0 + j];
        v[j] = sv[t0 + j];
    }
    uint32_t single = 0;
#pragma unroll
    for (int j = 0; j < RI; j++) {
        const uint64_t i = tb + t0 + j;
        const uint64_t pk = j ? k[j - 1] : (t0 ? s[t0 - 1] : prev_key);
        const uint64_t nk = j + 1 < RI ? k[j + 1] : (t0 + RI < (uint32_t)RTILE ? s[t0 + RI] : next_key);
        const bool in = i < n;
        const bool h = i == 0 || k[j] != pk;
        const bool t = i == n - 1 || k[j] != nk;
        single |= (uint32_t)(in && h && t) << j;
    }
    uint32_t tile_cnt;
    const uint32_t off = block_exclusive_scan<RT>((uint32_t)__popc(single), SumU32(), 0u, lds_scan, &tile_cnt);
    if (threadIdx.x < 64) {
        const uint64_t b = wave_lookback<0>(st_sum, tile, tile_cnt, epoch, err);
        if (threadIdx.x == 0) lds_base = b;
    }
    // stage the kept keys / payloads at their tile-local slots (the scan's
    // barriers ordered every read of s / sv above before these writes)
    uint32_t o = off;
#pragma unroll
    for (int j = 0; j < RI; j++) {
        if ((single >> j) & 1u) {
            s[o] = k[j];
            sv[o] = v[j];
            o++;
        }
    }
    __syncthreads();
    const uint64_t base = lds_base;
    for (uint32_t q = threadIdx.x; q < tile_cnt; q += RT) {
        okeys[base + q] = s[q];
        ovals[base + q] = sv[q];
    }
}

// Wide keys (k > 32): (hi, lo) pairs, sorted lexicographically; count or
// uniq in one tile pass like the kernels above (keys read straight from HBM,
// outputs written in place).  MODE 1: (hi, lo, group size); 2: the keys of
// groups of one with their payload.
template <int MODE, typename V>
__global__ __launch_bounds__(RT) void rle_wide_kernel(const uint64_t *__restrict__ hi, const uint64_t *__restrict__ lo,
                                                      const V *__restrict__ vals, uint64_t n,
                                                      uint64_t *__restrict__ ohi, uint64_t *__restrict__ olo,
                                                      V *__restrict__ ovals, uint64_t *__restrict__ st_sum,
                                                      uint64_t *__restrict__ st_max, uint32_t *__restrict__ counter,
                                                      uint32_t epoch, uint32_t *__restrict__ err) {
    __shared__ uint32_t lds_scan[RT / 64];
    __shared__ uint64_t lds_scan64[RT / 64];
    __shared__ uint64_t lds_base, lds_head;
    __shared__ uint32_t lds_tile;
    const int64_t tile = grab_tile(counter, &lds_tile);
    const uint64_t tb = (uint64_t)tile * RTILE;
    const uint64_t t0 = tb + (uint64_t)threadIdx.x * RI;
    uint64_t kh[RI + 2], kl[RI + 2];  // [0] = previous key, [RI + 1] = next key
#pragma unroll
    for (int j = 0; j < RI + 2; j++) {
        const uint64_t i = t0 + j - 1;
        const bool in = t0 + j >= 1 && i < n;
        kh[j] = in ? hi[i] : ~0ull;
        kl[j] = in ? lo[i] : ~0ull;
    }
    uint32_t heads = 0, tails = 0;
#pragma unroll
    for (int j = 1; j <= RI; j++) {
        const uint64_t i = t0 + j - 1;
        const bool in = i < n;
        const bool dp = kh[j] != kh[j - 1] || kl[j] != kl[j - 1];
        const bool dn = kh[j] != kh[j + 1] || kl[j] != kl[j + 1];
        heads |= (uint32_t)(in && (i == 0 || dp)) << (j - 1);
        tails |= (uint32_t)(in && (i + 1 == n || dn)) << (j - 1);
    }
    if constexpr (MODE == 2) {
        const uint32_t single = heads & tails;
        uint32_t tile_cnt;
        const uint32_t off = block_exclusive_scan<RT>((uint32_t)__popc(single), SumU32(), 0u, lds_scan, &tile_cnt);
        if (threadIdx.x < 64) {
            const uint64_t b = wave_lookback<0>(st_sum, tile, tile_cnt, epoch, err);
            if (threadIdx.x == 0) lds_base = b;
        }
        __syncthreads();
        uint64_t o = lds_base + off;
#pragma unroll
        for (int j = 0; j < RI; j++) {
            if ((single >> j) & 1u) {
                ohi[o] = kh[j + 1];
                olo[o] = kl[j + 1];
                ovals[o] = vals[t0 + j];
                o++;
            }
        }
    } else {
        const uint32_t nh = __popc(heads);
        const uint64_t lh = heads ? t0 + (31 - __clz(heads)) + 1 : 0;
        uint32_t tile_heads;
        const uint32_t hoff = block_exclusive_scan<RT>(nh, SumU32(), 0u, lds_scan, &tile_heads);
        uint64_t tile_lh;
        const uint64_t lh_before = block_exclusive_scan<RT>(lh, MaxU64(), (uint64_t)0, lds_scan64, &tile_lh);
        // does the tile start with a group head?
        const bool first_is_head = tb == 0 || hi[tb] != hi[tb - 1] || lo[tb] != lo[tb - 1];
        if (threadIdx.x < 64) {
            const uint64_t b = wave_lookback<0>(st_sum, tile, tile_heads, epoch, err);
            const uint64_t h = wave_lookback_lasthead(st_max, tile, tile_lh, !first_is_head, epoch, err);
            if (threadIdx.x == 0) {
                lds_base = b;
                lds_head = h;
            }
        }
        __syncthreads();
        uint64_t cur_head = lh_before ? lh_before : lds_head;
        uint64_t slot = lds_base + hoff;
#pragma unroll
        for (int j = 0; j < RI; j++) {
            const uint64_t i = t0 + j;
            if ((heads >> j) & 1u) {
                cur_head = i + 1;
                slot++;
            }
            if ((tails >> j) & 1u) {
                ohi[slot - 1] = kh[j + 1];
                olo[slot - 1] = kl[j + 1];
                ovals[slot - 1] = (V)(i + 2 - cur_head);
            }
        }
    }
}

}  // namespace

extern "C" int kman_rle_count(kman_ctx *ctx, const uint64_t *d_keys, uint64_t n, uint64_t *d_ukeys, void *d_counts,
                              uint32_t count_bytes, uint64_t *n_unique) {
    if (!ctx || !n_unique) return KMAN_EINVAL;
    if (count_bytes != 4 && count_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "count_bytes must be 4 or 8");
    if (count_bytes == 4 && n > 0xffffffffull)
        return kman_fail(ctx, KMAN_EINVAL, "u32 counts cannot hold groups of %llu keys", (unsigned long long)n);
    *n_unique = 0;
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t T = ceil_div(n, RTILE);
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, 2 * T, &epoch, &counter));
    KTimer kt_(ctx, "rle_count");
    if (count_bytes == 4)
        hipLaunchKernelGGL(rle_count_kernel<uint32_t>, dim3((uint32_t)T), dim3(RT), 0, ctx->stream, d_keys, n, d_ukeys,
                           (uint32_t *)d_counts, ctx->d_status, ctx->d_status + T, counter, epoch, ctx->d_err);
    else
        hipLaunchKernelGGL(rle_count_kernel<uint64_t>, dim3((uint32_t)T), dim3(RT), 0, ctx->stream, d_keys, n, d_ukeys,
                           (uint64_t *)d_counts, ctx->d_status, ctx->d_status + T, counter, epoch, ctx->d_err);
    HIP_TRY(ctx, hipGetLastError());
    return kman_lookback_total(ctx, T, n_unique);
}

extern "C" int kman_rle_uniq(kman_ctx *ctx, const uint64_t *d_keys, const void *d_vals, uint32_t val_bytes, uint64_t n,
                             uint64_t *d_okeys, void *d_ovals, uint64_t *n_out) {
    if (!ctx || !n_out) return KMAN_EINVAL;
    if (val_bytes != 4 && val_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "val_bytes must be 4 or 8");
    *n_out = 0;
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t T = ceil_div(n, RTILE);
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, T, &epoch, &counter));
    KTimer kt_(ctx, "rle_uniq");
    if (val_bytes == 4)
        hipLaunchKernelGGL(rle_uniq_kernel<uint32_t>, dim3((uint32_t)T), dim3(RT), 0, ctx->stream, d_keys,
                           (const uint32_t *)d_vals, n, d_okeys, (uint32_t *)d_ovals, ctx->d_status, counter, epoch,
                           ctx->d_err);
    else
        hipLaunchKernelGGL(rle_uniq_kernel<uint64_t>, dim3((uint32_t)T), dim3(RT), 0, ctx->stream, d_keys,
                           (const uint64_t *)d_vals, n, d_okeys, (uint64_t *)d_ovals, ctx->d_status, counter, epoch,
                           ctx->d_err);
    HIP_TRY(ctx, hipGetLastError());
    return kman_lookback_total(ctx, T, n_out);
}

extern "C" int kman_rle_wide(kman_ctx *ctx, int mode, const uint64_t *d_hi, const uint64_t *d_lo, const void *d_vals,
                             uint32_t val_bytes, uint64_t n, uint64_t *d_ohi, uint64_t *d_olo, void *d_ovals,
                             uint64_t *n_out) {
    if (!ctx || !n_out) return KMAN_EINVAL;
    if (mode != KMAN_FINISH_COUNT && mode != KMAN_FINISH_UNIQ) return kman_fail(ctx, KMAN_EINVAL, "bad mode");
    if (val_bytes != 4 && val_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "val_bytes must be 4 or 8");
    if (mode == KMAN_FINISH_COUNT && val_bytes == 4 && n > 0xffffffffull)
        return kman_fail(ctx, KMAN_EINVAL, "u32 counts cannot hold groups of %llu keys", (unsigned long long)n);
    *n_out = 0;
    if (n == 0) return KMAN_OK;
    if (!d_hi || !d_lo || !d_ohi || !d_olo || !d_ovals || (mode == KMAN_FINISH_UNIQ && !d_vals))
        return kman_fail(ctx, KMAN_EINVAL, "null buffer");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t T = ceil_div(n, RTILE);
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, 2 * T, &epoch, &counter));
    KTimer kt_(ctx, mode == KMAN_FINISH_COUNT ? "rle_count" : "rle_uniq");
#define KW(M, V)                                                                                                     \
    hipLaunchKernelGGL((rle_wide_kernel<M, V>), dim3((uint32_t)T), dim3(RT), 0, ctx->stream, d_hi, d_lo,            \
                       (const V *)d_vals, n, d_ohi, d_olo, (V *)d_ovals, ctx->d_status, ctx->d_status + T, counter, \
                       epoch, ctx->d_err)
    if (mode == KMAN_FINISH_COUNT && val_bytes == 4) KW(1, uint32_t);
    else if (mode == KMAN_FINISH_COUNT) KW(1, uint64_t);
    else if (val_bytes == 4) KW(2, uint32_t);
    else KW(2, uint64_t);
#undef KW
    HIP_TRY(ctx, hipGetLastError());
    return kman_lookback_total(ctx, T, n_out);
}

// ================================================================ merge
// n-way merge of sorted runs (Crawler.do_records' heapq.merge over sorted
// batches, kmermaid/join.py:63-93): a tree of stable 2-way merges (run order
// kept, so ties go to the lower run index, then in-run order -- heapq.merge
// over (key, batch) with batches in order).  Each 2-way merge is merge-path
// in tiles: a block's MT * MI outputs start at its diagonal's split (two
// binary searches in HBM), its A and B slices are loaded coalesced into LDS,
// each thread merges MI outputs from LDS (its own diagonal searched there),
// and the tile is staged back through LDS and stored coalesced.
namespace {

constexpr int MT = 256, MI = 8;

template <typename V>
__global__ __launch_bounds__(MT) void merge2_kernel(const uint64_t *__restrict__ ak, const V *__restrict__ av,
                                                    uint64_t na, const uint64_t *__restrict__ bk,
                                                    const V *__restrict__ bv, uint64_t nb,
                                                    uint64_t *__restrict__ ok, V *__restrict__ ov) {
    constexpr int TILE = MT * MI;
    __shared__ uint64_t sk[TILE];
    __shared__ V sv[TILE];
    __shared__ uint64_t split[2];
    const uint64_t n = na + nb;
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
    if (t0 >= n) return;  // (block-uniform)
    const uint64_t t1 = t0 + TILE < n ? t0 + TILE : n;
    // A elements among the first d outputs (A first on ties), d = t0 and t1
    if (threadIdx.x < 2) {
        const uint64_t d = threadIdx.x ? t1 : t0;
        uint64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (ak[mid] <= bk[d - 1 - mid]) lo = mid + 1;
            else hi = mid;
        }
        split[threadIdx.x] = lo;
    }
    __syncthreads();
    const uint64_t a0 = split[0], b0 = t0 - a0;
    const uint32_t nA = (uint32_t)(split[1] - a0), nt = (uint32_t)(t1 - t0), nB = nt - nA;
    for (uint32_t q = threadIdx.x; q < nt; q += MT) {
        const bool isA = q < nA;
        sk[q] = isA ? ak[a0 + q] : bk[b0 + (q - nA)];
        if (av) sv[q] = isA ? av[a0 + q] : bv[b0 + (q - nA)];
    }
    __syncthreads();
    const uint32_t d = threadIdx.x * MI < nt ? threadIdx.x * MI : nt;
    uint32_t lo = d > nB ? d - nB : 0, hi = d < nA ? d : nA;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sk[mid] <= sk[nA + d - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    uint32_t i = lo, j = d - lo;
    uint64_t rk[MI];
    V rv[MI];
#pragma unroll
    for (int o = 0; o < MI; o++) {
        if (d + o < nt) {
            const bool takeA = j >= nB || (i < nA && sk[i] <= sk[nA + j]);
            const uint32_t src = takeA ? i : nA + j;
            rk[o] = sk[src];
            if (av) rv[o] = sv[src];
            i += takeA;
            j += !takeA;
        }
    }
    __syncthreads();  // every LDS read above before the outputs overwrite it
#pragma unroll
    for (int o = 0; o < MI; o++) {
        if (d + o < nt) {
            sk[d + o] = rk[o];
            if (av) sv[d + o] = rv[o];
        }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nt; q += MT) {
        ok[t0 + q] = sk[q];
        if (av) ov[t0 + q] = sv[q];
    }
}

__global__ __launch_bounds__(256) void descents_kernel(const uint64_t *__restrict__ k, uint64_t n,
                                                       unsigned long long *__restrict__ out) {
    uint32_t c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x + 1; i < n; i += (uint64_t)gridDim.x * 256)
        c += k[i] < k[i - 1];
    if (c) atomicAdd(out, (unsigned long long)c);
}

// a position-keyed digest of n rows (key, value): sum and xor of
// mix(key ^ mix(value + (first + i) * PHI)), the values' sum and the number of
// i >= 1 with keys[i] <= keys[i-1]; sums mod 2^64 and xors combine over slices
KMAN_DEV uint64_t dg_mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    return x ^ (x >> 33);
}

template <typename V>
__global__ __launch_bounds__(256) void digest_kernel(const uint64_t *__restrict__ k, const V *__restrict__ v,
                                                     uint64_t n, uint64_t first, unsigned long long *__restrict__ out) {
    uint64_t hs = 0, hx = 0, vs = 0;
    uint32_t nd = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t key = k[i], val = v ? (uint64_t)v[i] : 0;
        const uint64_t h = dg_mix(key ^ dg_mix(val + (first + i) * 0x9E3779B97F4A7C15ull));
        hs += h;
        hx ^= h;
        vs += val;
        nd += i && key <= k[i - 1];
    }
    __shared__ uint64_t r[4][256];
    r[0][threadIdx.x] = hs;
    r[1][threadIdx.x] = hx;
    r[2][threadIdx.x] = vs;
    r[3][threadIdx.x] = nd;
    __syncthreads();
    for (uint32_t s = 128; s; s >>= 1) {
        if (threadIdx.x < s) {
            r[0][threadIdx.x] += r[0][threadIdx.x + s];
            r[1][threadIdx.x] ^= r[1][threadIdx.x + s];
            r[2][threadIdx.x] += r[2][threadIdx.x + s];
            r[3][threadIdx.x] += r[3][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicAdd(&out[0], (unsigned long long)r[0][0]);
        atomicXor(&out[1], (unsigned long long)r[1][0]);
        atomicAdd(&out[2], (unsigned long long)r[2][0]);
        atomicAdd(&out[3], (unsigned long long)r[3][0]);
    }
}

}  // namespace

// ================================================================ vectors
// VEC_COUNT / VEC_COUNT_MASKED (KJoiner.join_vector_count[_masked],
// kmermaid/join.py:288-335 -> AbundanceVector.add_count, abundance.py:103-130):
// one thread per item of a key-sorted, stream-stable array; its key run (and,
// MASKED, the sub-run of its record) found by galloping + binary search, so
// runs of any length cost O(log run) per item.
namespace {

template <typename F>
KMAN_DEV uint64_t run_first(uint64_t i, F same) {  // smallest j <= i with same(j) (same: an interval around i)
    uint64_t good = i, step = 1;
    int64_t bad = -1;
    for (;;) {
        if (good < step) break;
        const uint64_t c = good - step;
        if (same(c)) {
            good = c;
            step <<= 1;
        } else {
            bad = (int64_t)c;
            break;
        }
    }
    while ((int64_t)good - bad > 1) {
        const uint64_t mid = (uint64_t)((bad + (int64_t)good) / 2);
        if (same(mid)) good = mid;
        else bad = (int64_t)mid;
    }
    return good;
}

template <typename F>
KMAN_DEV uint64_t run_last(uint64_t i, uint64_t n, F same) {  // largest j >= i with same(j)
    uint64_t good = i, step = 1, bad = n;
    for (;;) {
        if (good + step >= n) break;
        const uint64_t c = good + step;
        if (same(c)) {
            good = c;
            step <<= 1;
        } else {
            bad = c;
            break;
        }
    }
    while (bad - good > 1) {
        const uint64_t mid = good + (bad - good) / 2;
        if (same(mid)) good = mid;
        else bad = mid;
    }
    return good;
}

template <typename P>
__global__ __launch_bounds__(256) void vec_fill_kernel(const uint64_t *__restrict__ keys, const P *__restrict__ pos,
                                                       uint64_t n, int masked, const uint64_t *__restrict__ src_base,
                                                       uint32_t tagged, const uint64_t *__restrict__ rec_start,
                                                       const uint32_t *__restrict__ rec_id, uint64_t nrec,
                                                       uint32_t *__restrict__ vec) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    auto index = [&](uint64_t j) -> uint64_t {
        const uint64_t p = (uint64_t)pos[j];
        return tagged ? src_base[p >> 56] + (p & ((1ull << 56) - 1)) : p;
    };
    auto record = [&](uint64_t j) -> uint32_t {  // the record identity of item j (last rec_start <= index)
        const uint64_t x = index(j);
        uint64_t lo = 0, hi = nrec;  // first rec_start > x
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (rec_start[mid] <= x) lo = mid + 1;
            else hi = mid;
        }
        return rec_id[lo ? lo - 1 : 0];
    };
    const uint64_t key = keys[i];
    auto same_key = [&](uint64_t j) { return keys[j] == key; };
    const uint64_t a = run_first(i, same_key), b = run_last(i, n, same_key);
    const uint64_t cnt = b - a + 1;
    uint64_t v = cnt;
    if (masked) {
        // occurrences in other records (the run's records are contiguous:
        // stream order inside the run); nothing when it has one record only
        const uint32_t me = record(i);
        auto same_rec = [&](uint64_t j) { return keys[j] == key && record(j) == me; };
        const uint64_t sa = run_first(i, same_rec), sb = run_last(i, n, same_rec);
        v = cnt - (sb - sa + 1);
        if (v == 0) return;
    }
    vec[index(i)] = (uint32_t)(v < 0xffffffffull ? v : 0xffffffffull);
}

}  // namespace

extern "C" int kman_vec_fill(kman_ctx *ctx, const uint64_t *d_keys, const void *d_pos, uint32_t pos_bytes, uint64_t n,
                             int masked, const uint64_t *d_src_base, uint32_t tagged, const uint64_t *d_rec_start,
                             const uint32_t *d_rec_id, uint64_t nrec, uint32_t *d_vec) {
    if (!ctx || (pos_bytes != 4 && pos_bytes != 8)) return KMAN_EINVAL;
    if (n == 0) return KMAN_OK;
    if (!d_keys || !d_pos || !d_vec || (tagged && !d_src_base) || (masked && (!d_rec_start || !d_rec_id || !nrec)))
        return kman_fail(ctx, KMAN_EINVAL, "kman_vec_fill: null buffer");
    if (tagged && pos_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "tagged pos are u64");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const dim3 g((uint32_t)ceil_div(n, 256));
    if (pos_bytes == 8)
        hipLaunchKernelGGL(vec_fill_kernel<uint64_t>, g, dim3(256), 0, ctx->stream, d_keys, (const uint64_t *)d_pos, n,
                           masked, d_src_base, tagged, d_rec_start, d_rec_id, nrec, d_vec);
    else
        hipLaunchKernelGGL(vec_fill_kernel<uint32_t>, g, dim3(256), 0, ctx->stream, d_keys, (const uint32_t *)d_pos, n,
                           masked, d_src_base, tagged, d_rec_start, d_rec_id, nrec, d_vec);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}

extern "C" int kman_count_descents(kman_ctx *ctx, const uint64_t *d_keys, uint64_t n, uint64_t *descents) {
    if (!ctx || !descents) return KMAN_EINVAL;
    *descents = 0;
    if (n < 2) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    void *scr;
    KMAN_TRY(kman_scratch(ctx, 256, &scr));
    HIP_TRY(ctx, hipMemsetAsync(scr, 0, 8, ctx->stream));
    const uint64_t b = ceil_div(n, 256 * 16);
    hipLaunchKernelGGL(descents_kernel, dim3((uint32_t)(b < 4096 ? b : 4096)), dim3(256), 0, ctx->stream, d_keys, n,
                       (unsigned long long *)scr);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_small, scr, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *descents = ctx->h_small[0];
    return KMAN_OK;
}

extern "C" int kman_row_digest(kman_ctx *ctx, const uint64_t *d_keys, const void *d_vals, uint32_t val_bytes, uint64_t n,
                               uint64_t first_index, uint64_t *out4) {
    if (!ctx || !out4) return KMAN_EINVAL;
    if (val_bytes != 0 && val_bytes != 4 && val_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "val_bytes 0, 4 or 8");
    out4[0] = out4[1] = out4[2] = out4[3] = 0;
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    void *scr;
    KMAN_TRY(kman_scratch(ctx, 256, &scr));
    HIP_TRY(ctx, hipMemsetAsync(scr, 0, 32, ctx->stream));
    const uint64_t b = ceil_div(n, 256 * 16);
    const dim3 g((uint32_t)(b < 4096 ? b : 4096));
    if (val_bytes == 8)
        hipLaunchKernelGGL(digest_kernel<uint64_t>, g, dim3(256), 0, ctx->stream, d_keys, (const uint64_t *)d_vals, n,
                           first_index, (unsigned long long *)scr);
    else
        hipLaunchKernelGGL(digest_kernel<uint32_t>, g, dim3(256), 0, ctx->stream, d_keys,
                           val_bytes ? (const uint32_t *)d_vals : (const uint32_t *)nullptr, n, first_index,
                           (unsigned long long *)scr);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_small, scr, 32, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < 4; i++) out4[i] = ctx->h_small[i];
    return KMAN_OK;
}

extern "C" int kman_merge_runs(kman_ctx *ctx, const kman_run *runs, int nruns, uint32_t val_bytes,
                               uint64_t *d_okeys, void *d_ovals, uint64_t *d_tmp_keys, void *d_tmp_vals) {
    if (!ctx || nruns < 0 || (nruns && !runs)) return KMAN_EINVAL;
    if (val_bytes != 0 && val_bytes != 4 && val_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "val_bytes 0, 4 or 8");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    struct R {
        const uint64_t *k;
        const void *v;
        uint64_t n;
    };
    std::vector<R> cur;
    uint64_t total = 0;
    for (int r = 0; r < nruns; r++) {
        cur.push_back({runs[r].keys, runs[r].vals, runs[r].n});
        total += runs[r].n;
    }
    if (total == 0) return KMAN_OK;
    if (!d_okeys || (val_bytes && !d_ovals)) return kman_fail(ctx, KMAN_EINVAL, "null output");
    // levels of pairwise merges; the output of the last level must be d_okeys:
    // levels alternate between (out, tmp) starting so that the last is out
    int levels = 0;
    for (size_t m = cur.size(); m > 1; m = (m + 1) / 2) levels++;
    // (one level -- two runs -- writes d_okeys directly: no scratch)
    if (levels > 1 && (!d_tmp_keys || (val_bytes && !d_tmp_vals))) return kman_fail(ctx, KMAN_EINVAL, "null scratch");
    KTimer kt_(ctx, "merge");
    for (int lv = 0; lv < levels; lv++) {
        const bool to_out = ((levels - 1 - lv) & 1) == 0;
        uint64_t *dk = to_out ? d_okeys : d_tmp_keys;
        char *dv = (char *)(to_out ? d_ovals : d_tmp_vals);
        std::vector<R> nxt;
        uint64_t at = 0;
        for (size_t p = 0; p < cur.size(); p += 2) {
            const R a = cur[p];
            const R b = p + 1 < cur.size() ? cur[p + 1] : R{nullptr, nullptr, 0};
            const uint64_t n = a.n + b.n;
            uint64_t *ok = dk + at;
            void *ov = val_bytes ? (void *)(dv + (size_t)val_bytes * at) : nullptr;
            if (n) {
                const dim3 g((uint32_t)ceil_div(n, (uint64_t)MT * MI));
                if (val_bytes == 8)
                    hipLaunchKernelGGL(merge2_kernel<uint64_t>, g, dim3(MT), 0, ctx->stream, a.k, (const uint64_t *)a.v,
                                       a.n, b.k, (const uint64_t *)b.v, b.n, ok, (uint64_t *)ov);
                else if (val_bytes == 4)
                    hipLaunchKernelGGL(merge2_kernel<uint32_t>, g, dim3(MT), 0, ctx->stream, a.k, (const uint32_t *)a.v,
                                       a.n, b.k, (const uint32_t *)b.v, b.n, ok, (uint32_t *)ov);
                else
                    hipLaunchKernelGGL(merge2_kernel<uint32_t>, g, dim3(MT), 0, ctx->stream, a.k, (const uint32_t *)nullptr,
                                       a.n, b.k, (const uint32_t *)nullptr, b.n, ok, (uint32_t *)nullptr);
                HIP_TRY(ctx, hipGetLastError());
            }
            nxt.push_back({ok, ov, n});
            at += n;
        }
        cur.swap(nxt);
    }
    if (levels == 0) {  // one run: a copy
        HIP_TRY(ctx, hipMemcpyAsync(d_okeys, cur[0].k, 8 * total, hipMemcpyDeviceToDevice, ctx->stream));
        if (val_bytes)
            HIP_TRY(ctx, hipMemcpyAsync(d_ovals, cur[0].v, (size_t)val_bytes * total, hipMemcpyDeviceToDevice,
                                        ctx->stream));
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return kman_check_device_error(ctx);
}
