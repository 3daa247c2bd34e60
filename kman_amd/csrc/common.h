// common.h — shared device helpers for the kman gfx950 kernels.
//
// Everything here is wave64-native: lane masks are 64-bit, wave scans are DPP
// row shifts + row broadcasts, block scans combine wave totals through LDS.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/kman.h"

#define KMAN_DEV __device__ __forceinline__

// ---------------------------------------------------------------- context
struct kman_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // look-back scratch: status words (flag:2 | epoch:6 | value:56)
    uint64_t *d_status = nullptr;
    size_t status_words = 0;
    uint32_t *d_counters = nullptr; // one dynamic-tile counter per epoch (64)
    uint32_t *d_mapbits = nullptr;   // kman_extract_marked's coarse bitmap (2048 words)
    uint32_t *d_xcounters = nullptr; // eight per epoch: one tile counter per XCD partition (rg_extract XG)
    uint32_t *d_cursors = nullptr;   // 256 x 64 region cursors of the shard extraction (rg_extract EX + AT)
    uint32_t *d_err = nullptr;      // device-side error word (spin timeouts)
    uint32_t epoch = 63;            // last epoch handed out; wraps 63 -> 1 with a reset
    // small pinned host area for results
    uint64_t *h_small = nullptr;
    // generic device scratch
    void *d_scratch = nullptr;
    size_t scratch_bytes = 0;
    // second scratch for callers that hold a region across calls that use d_scratch
    void *d_aux = nullptr;
    size_t aux_bytes = 0;
    // optional launch timing (kman_timing_*)
    bool timing = false;
    struct TimedLaunch {
        const char *tag;
        hipEvent_t a, b;
    };
    std::vector<TimedLaunch> launches;
    std::vector<hipEvent_t> event_pool;
    // RCCL communicator (comm.hip), null on a single GPU
    void *comm = nullptr;
    // probed at kman_create: same-address LDS atomics of one wave return in
    // lane order on this device (observed on gfx950, not architectural); the
    // sort uses atomic ranking only when true
    bool lds_atomic_ordered = false;
    // H2D copies that overlap the work of `stream` (chunked FASTA uploads)
    hipStream_t copy_stream = nullptr;
    hipEvent_t copy_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // D2H copies on the copy stream (formatted text leaving while the next
    // slice is formatted): kman_copy_d2h_async / kman_copy_d2h_wait
    hipEvent_t work_ev = nullptr;
    hipEvent_t d2h_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // all-to-alls that overlap the work of `stream` (kman_alltoallv_async)
    hipStream_t comm_stream = nullptr;
    hipEvent_t comm_pre = nullptr;
    hipEvent_t comm_ev[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    // key ranges [lo, hi] (pairs) that the last kman_dround_finish left out
    // (KMAN_EPARTIAL): regions that overflowed a capacity
    std::vector<uint64_t> failed;
    // heavy keys of the last kman_dround_finish (counted apart in its pass 1)
    // and their scratch (table, drop counts, samples)
    uint32_t heavy_keys = 0, heavy_slots = 0;
    int heavy_mode = 0;
    void *d_hv = nullptr;
    size_t hv_bytes = 0;
    // the last kman_dround_finish's pass-1 output, for kman_dround_left (its
    // left-out regions' items gathered from there): valid when pass 1 lost
    // nothing; bd = the (bucket, digit) sub-buckets whose regions were left out
    struct LeftRound {
        bool valid = false;
        const void *r1 = nullptr;
        const uint32_t *c1 = nullptr;
        uint64_t C1s = 0;
        uint32_t nb = 0, G = 0, H = 0, K = 0, Q = 0, b_lo = 0, g = 0;
        const uint8_t *freg = nullptr;  // the round's left-out regions (arena A)
        bool rc = false, narrow = false;
        int mode = 0;
        std::vector<uint32_t> bd;
    } left;
    // kman_groups_begin .. kman_groups_end: pass 0 by tile ranges as the
    // codes arrive (the look-back epoch it runs in, the next tile)
    uint32_t grp_epoch = 0;
    uint32_t grp_next = 0;
    uint32_t grp_tiles = 0;
};

// RAII launch timer: records an event pair around the launches in its scope.
struct KTimer {
    kman_ctx *ctx;
    size_t idx;
    KTimer(kman_ctx *c, const char *tag);
    ~KTimer();
};

int kman_fail(kman_ctx *ctx, int code, const char *fmt, ...);
int kman_hip_fail(kman_ctx *ctx, hipError_t e, const char *what);
// status buffer with >= words entries; returns epoch to use (1..63) and the
// counter for dynamic tile ids of that epoch.
int kman_lookback_begin(kman_ctx *ctx, size_t words, uint32_t *epoch, uint32_t **counter);
int kman_scratch(kman_ctx *ctx, size_t bytes, void **p);
int kman_aux(kman_ctx *ctx, size_t bytes, void **p);
int kman_check_device_error(kman_ctx *ctx);
// blocks of `fn` resident at once on the device (occupancy x CUs), capped at n_tiles
int kman_persistent_grid(kman_ctx *ctx, const void *fn, int threads, uint64_t n_tiles, size_t dyn_lds = 0);
// internal (not in kman.h): the histogram pre-pass of kman_extract_sorted
int kman_kmer_hist(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                   uint32_t lo_bit, uint32_t nseg, uint64_t seg_w, uint64_t *d_seg, uint64_t *n_kmers);
// the most segments (<= want) whose per-pass digit tables [pass][seg][bin] x copies
// fit `lds_bytes`; radix of each pass from bits[]
uint32_t kman_seg_fit(uint32_t np, const uint32_t *bits, uint32_t want, uint32_t copies, size_t lds_bytes);
// synchronises; reads the inclusive value of the last tile of the most recent
// look-back launch (checks its epoch) and the device error word.
int kman_lookback_total(kman_ctx *ctx, uint64_t n_tiles, uint64_t *total);

#define HIP_TRY(ctx, expr)                                      \
    do {                                                        \
        hipError_t _e = (expr);                                 \
        if (_e != hipSuccess) return kman_hip_fail(ctx, _e, #expr); \
    } while (0)

#define KMAN_TRY(expr)              \
    do {                            \
        int _r = (expr);            \
        if (_r != KMAN_OK) return _r; \
    } while (0)

// ------------------------------------------------------------ status words
constexpr uint64_t ST_AGG = 1ull;
constexpr uint64_t ST_INCL = 2ull;
constexpr uint64_t ST_VMASK = (1ull << 56) - 1;
constexpr uint32_t SPIN_LIMIT = 1u << 20; // ~1 s of polling; a hit is an engine bug

// true when this waiter must give up: its own bound is spent, or another wave
// already flagged a fault (so one fault does not cascade into serial
// timeouts).  Bit 8 (region.hip's ERR_REGION, a region that would overflow)
// is not a fault: the round path keeps every other region's rows, so their
// look-backs must still complete.
KMAN_DEV bool spin_give_up(uint32_t &spins, uint32_t *err, uint32_t code) {
    ++spins;
    if ((spins & 255u) == 0 && (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~(1u << 8)) != 0)
        return true;
    if (spins > SPIN_LIMIT) {
        atomicOr(err, code);
        return true;
    }
    return false;
}

KMAN_DEV uint64_t st_make(uint64_t flag, uint32_t epoch, uint64_t v) {
    return (flag << 62) | ((uint64_t)epoch << 56) | (v & ST_VMASK);
}
KMAN_DEV void st_store(uint64_t *p, uint64_t w) {
    __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
KMAN_DEV uint64_t st_load(const uint64_t *p) {
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
KMAN_DEV uint64_t st_flag(uint64_t w, uint32_t epoch) {
    return (((w >> 56) & 63u) == epoch) ? (w >> 62) : 0ull;
}

// --------------------------------------------------------------- lanes
KMAN_DEV int lane_id() { return __lane_id(); }
KMAN_DEV uint64_t lanemask_lt() {
    const int l = lane_id();
    return l ? (~0ull >> (64 - l)) : 0ull;
}

template <typename T>
KMAN_DEV T shfl_up_any(T v, int d) {
    static_assert(sizeof(T) % 4 == 0, "32-bit granular");
    constexpr int W = sizeof(T) / 4;
    uint32_t w[W];
    memcpy(w, &v, sizeof(T));
#pragma unroll
    for (int i = 0; i < W; i++) w[i] = (uint32_t)__shfl_up((int)w[i], d, 64);
    T r;
    memcpy(&r, w, sizeof(T));
    return r;
}

template <typename T>
KMAN_DEV T shfl_any(T v, int src) {
    static_assert(sizeof(T) % 4 == 0, "32-bit granular");
    constexpr int W = sizeof(T) / 4;
    uint32_t w[W];
    memcpy(w, &v, sizeof(T));
#pragma unroll
    for (int i = 0; i < W; i++) w[i] = (uint32_t)__shfl((int)w[i], src, 64);
    T r;
    memcpy(&r, w, sizeof(T));
    return r;
}

// DPP move of a value made of 32-bit words; lanes without a source (or in
// rows outside row_mask) read `fill`
template <int CTRL, int ROWMASK, typename T>
KMAN_DEV T dpp_move(T v, T fill) {
    static_assert(sizeof(T) % 4 == 0, "32-bit granular");
    constexpr int W = sizeof(T) / 4;
    int x[W], f[W], r[W];
    memcpy(x, &v, sizeof(T));
    memcpy(f, &fill, sizeof(T));
#pragma unroll
    for (int i = 0; i < W; i++) r[i] = __builtin_amdgcn_update_dpp(f[i], x[i], CTRL, ROWMASK, 0xf, false);
    T o;
    memcpy(&o, r, sizeof(T));
    return o;
}

// Inclusive scan across the 64 lanes; op(a, b) with a the earlier element,
// `identity` its identity (op need not commute).  DPP only: row_shr 1/2/4/8
// inside rows of 16, then row_bcast 15 / 31 across rows; no LDS traffic.
template <typename T, typename Op>
KMAN_DEV T wave_inclusive_scan(T v, Op op, T identity) {
    v = op(dpp_move<0x111, 0xf>(v, identity), v);
    v = op(dpp_move<0x112, 0xf>(v, identity), v);
    v = op(dpp_move<0x114, 0xf>(v, identity), v);
    v = op(dpp_move<0x118, 0xf>(v, identity), v);
    v = op(dpp_move<0x142, 0xa>(v, identity), v);
    v = op(dpp_move<0x143, 0xc>(v, identity), v);
    return v;
}

template <typename T, typename Op>
KMAN_DEV T wave_inclusive_scan(T v, Op op) {
    return wave_inclusive_scan(v, op, T{});
}

// the previous lane's value (lane 0: fill), DPP wave_shr:1
template <typename T>
KMAN_DEV T wave_shr1(T v, T fill) {
    return dpp_move<0x138, 0xf>(v, fill);
}

// the next lane's value (lane 63: fill), DPP wave_shl:1
template <typename T>
KMAN_DEV T wave_shl1(T v, T fill) {
    return dpp_move<0x130, 0xf>(v, fill);
}

// Exclusive block scan for NT threads (NT multiple of 64, <= 1024).
// lds must hold NT/64 elements.  Returns the exclusive prefix; *total (if not
// null) receives the block aggregate in every thread.
template <int NT, typename T, typename Op>
KMAN_DEV T block_exclusive_scan(T v, Op op, T identity, T *lds, T *total) {
    constexpr int NW = NT / 64;
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    T inc = wave_inclusive_scan(v, op, identity);
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    if (w == 0) {
        T x = lane < NW ? lds[lane] : identity;
        x = wave_inclusive_scan(x, op, identity);
        if (lane < NW) lds[lane] = x;
    }
    __syncthreads();
    T ex = wave_shr1(inc, identity);
    T res = w ? op(lds[w - 1], ex) : ex;
    if (total) *total = lds[NW - 1];
    __syncthreads();
    return res;
}

// The same scan with ONE barrier: each wave's total to lds[w], a barrier,
// then every thread folds the earlier waves' totals itself (NW broadcast LDS
// reads).  The caller must order this scan's reads of `lds` before the next
// write of it (a barrier between two scans on one lds array).
template <int NT, typename T, typename Op>
KMAN_DEV T block_exclusive_scan1(T v, Op op, T identity, T *lds, T *total) {
    constexpr int NW = NT / 64;
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    const T inc = wave_inclusive_scan(v, op, identity);
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    T pre = identity, all = identity;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const T x = lds[i];
        if (i < w) pre = op(pre, x);
        all = op(all, x);
    }
    if (total) *total = all;
    return op(pre, wave_shr1(inc, identity));
}

struct SumU64 {
    KMAN_DEV uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
};
struct SumU32 {
    KMAN_DEV uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};

// ------------------------------------------------------ decoupled look-back
// the wave's sum (OP 0) or max (OP 1) of v in every lane: DPP row shifts and
// broadcasts, then lane 63's by readlane (no LDS round trips; the xor
// butterfly through ds_bpermute took six, two per step for 64 bits)
template <int OP>
KMAN_DEV uint64_t wave_reduce_lb(uint64_t v) {
    struct MaxU64 {
        KMAN_DEV uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; }
    };
    if (OP == 0) v = wave_inclusive_scan(v, SumU64(), (uint64_t)0);
    else v = wave_inclusive_scan(v, MaxU64(), (uint64_t)0);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}

// Called by ONE full wave of the tile (all 64 lanes active).  Publishes the
// tile aggregate, looks back over up to 64 predecessors per round (one status
// word per lane, sc1 loads), publishes the inclusive prefix and returns the
// exclusive prefix (wave-uniform).  op: 0 = sum, 1 = max.
template <int OP>
KMAN_DEV uint64_t wave_lookback(uint64_t *status, int64_t tile, uint64_t agg, uint32_t epoch,
                                uint32_t *err) {
    const int lane = lane_id();
    if (tile == 0) {
        if (lane == 0) st_store(&status[0], st_make(ST_INCL, epoch, agg));
        return 0;
    }
    if (lane == 0) st_store(&status[tile], st_make(ST_AGG, epoch, agg));
    uint64_t excl = 0;
    int64_t end = tile; // exclusive upper bound of the window still to fold
    uint32_t spins = 0;
    for (;;) {
        const int64_t j = end - 1 - lane;
        uint64_t w = 0, f = ST_INCL;
        if (j >= 0) {
            w = st_load(&status[j]);
            f = st_flag(w, epoch);
        }
        const uint64_t notready = __ballot(f == 0);
        const uint64_t incl = __ballot(f == ST_INCL && j >= 0);
        // lanes 0..first_incl must all be ready; fold them
        const int first_incl = incl ? __ffsll((unsigned long long)incl) - 1 : 64;
        const uint64_t need = first_incl == 64 ? ~0ull : (~0ull >> (63 - first_incl));
        if (notready & need) {
            if (spin_give_up(spins, err, 1u)) break;
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = (j >= 0 && (need >> lane) & 1ull) ? (w & ST_VMASK) : 0ull;
        // wave reduce
        v = wave_reduce_lb<OP>(v);
        excl = OP == 0 ? excl + v : (excl > v ? excl : v);
        if (first_incl < 64 || end - 64 <= 0) break;
        end -= 64;
    }
    const uint64_t inc = OP == 0 ? excl + agg : (excl > agg ? excl : agg);
    if (lane == 0) st_store(&status[tile], st_make(ST_INCL, epoch, inc));
    return excl;
}

// wave_lookback for a tile that published its aggregate earlier itself
// (publish_agg): no second AGG store; tile 0 already stored its INCL
template <int OP>
KMAN_DEV void publish_agg(uint64_t *status, int64_t tile, uint64_t agg, uint32_t epoch) {
    st_store(&status[tile], st_make(tile == 0 ? ST_INCL : ST_AGG, epoch, agg));
}
template <int OP>
KMAN_DEV uint64_t wave_lookback_published(uint64_t *status, int64_t tile, uint64_t agg, uint32_t epoch,
                                          uint32_t *err) {
    const int lane = lane_id();
    if (tile == 0) return 0;
    uint64_t excl = 0;
    int64_t end = tile;
    uint32_t spins = 0;
    for (;;) {
        const int64_t j = end - 1 - lane;
        uint64_t w = 0, f = ST_INCL;
        if (j >= 0) {
            w = st_load(&status[j]);
            f = st_flag(w, epoch);
        }
        const uint64_t notready = __ballot(f == 0);
        const uint64_t incl = __ballot(f == ST_INCL && j >= 0);
        const int first_incl = incl ? __ffsll((unsigned long long)incl) - 1 : 64;
        const uint64_t need = first_incl == 64 ? ~0ull : (~0ull >> (63 - first_incl));
        if (notready & need) {
            if (spin_give_up(spins, err, 1u)) break;
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = (j >= 0 && (need >> lane) & 1ull) ? (w & ST_VMASK) : 0ull;
        v = wave_reduce_lb<OP>(v);
        excl = OP == 0 ? excl + v : (excl > v ? excl : v);
        if (first_incl < 64 || end - 64 <= 0) break;
        end -= 64;
    }
    const uint64_t inc = OP == 0 ? excl + agg : (excl > agg ? excl : agg);
    if (lane == 0) st_store(&status[tile], st_make(ST_INCL, epoch, inc));
    return excl;
}

// dynamic tile id: tiles are numbered in the order they start, so every
// predecessor of a tile is resident or finished (forward progress).
KMAN_DEV int64_t grab_tile(uint32_t *counter, uint32_t *lds_slot) {
    if (threadIdx.x == 0) *lds_slot = atomicAdd(counter, 1u);
    __syncthreads();
    const int64_t t = *lds_slot;
    __syncthreads();
    return t;
}

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
