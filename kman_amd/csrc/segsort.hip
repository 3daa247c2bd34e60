// segsort.hip — finishing a prefix-sorted key array inside LDS: sort, count
// or uniq in one pass over HBM.
//
// kman_sort_range stably sorts keys by their top P bits only (bits
// [lo_bit, key_bits), kman_split_bits picks P so that the average run of
// equal prefixes — a "segment" — holds ~512 keys).  kman_finish then reads the
// array once in chunks of FC keys.  A chunk owns every segment that starts in
// it; it loads those segments whole (the last one may run up to FR - FC keys
// past the chunk end), sorts them in LDS by (segment index, low bits) with
// stable 7-bit LSD passes, and emits the mode's output:
//   SORT   sorted keys (+ payload) written back in place   Batch.sorted, batch.py:156-168
//   COUNT  (key, group size) per distinct key             join_sequence_count, join.py:266-285
//   UNIQ   keys that occur once, with their payload        join_unique, join.py:244-263
// (the group walk of Crawler.do_batch, join.py:95-130, is the run-length pass
// over the LDS-sorted segments).  COUNT / UNIQ outputs are compacted with one
// decoupled look-back per chunk.  Equal keys always share a segment, so every
// group is decided inside one chunk, except inside "big" segments.
//
// Big segments (longer than the owner's region, FR - start offset > FC - 1
// keys) cannot be staged.  The first run records their starts; the host then
// sorts them out of place with the full-key kman_sort (gathered contiguously:
// their prefixes ascend, so the concatenation sorts into the same order) and
// scatters them back, and a second run treats them as presorted slices that
// every chunk they overlap processes in place (a group crossing a chunk end
// inside one is measured by a galloping search for its end).
//
// Algorithmic bytes per key: 8 B key read (+ val) + output; the ~half
// segment of tail keys that the next chunk re-reads to find its first start
// is ~6% extra.
#include "common.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace {

#ifndef KMAN_FT
#define KMAN_FT 512
#endif
#ifndef KMAN_FC
#define KMAN_FC 5120
#define KMAN_FR 6144
#endif
constexpr int FT = KMAN_FT;    // threads per chunk
constexpr int FW = FT / 64;    // waves
constexpr int FC = KMAN_FC;    // chunk: segments that start here are owned
constexpr int FR = KMAN_FR;    // region capacity: chunk + tail of its last segment
constexpr int FI = FR / FT;    // items per thread
constexpr int PI = FC / FT + 1;  // rounds loaded up front: the chunk and the next FT keys
constexpr int NWORD = FR / 64;   // segment-start mask words
constexpr int FRADIX = 128;    // local LSD digit radix
constexpr int FBITS = 7;
constexpr int WI = 12;         // wave-per-segment path: items per lane (segments <= 768 keys)
static_assert(FC % FT == 0 && FR % FT == 0 && FR >= FC + FT && FT % 64 == 0, "chunk geometry");
static_assert(NWORD <= 128, "mask words: two per lane");

struct NoV {};

#if defined(KMAN_ABL) && (KMAN_ABL & 4)
// diagnostic build only: per-chunk s_memrealtime stamps (100 MHz), thread 0
__device__ uint64_t *g_fdbg;
__device__ unsigned long long g_fstat[4];  // wave-path chunks, block-path chunks, segments, sorted keys
#define FSTAMP(i)                                                                                   \
    do {                                                                                            \
        if (threadIdx.x == 0 && g_fdbg) g_fdbg[(uint64_t)tile * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define FSTAMP(i) \
    do {          \
    } while (0)
#endif

KMAN_DEV uint64_t pre_of(uint64_t x, uint32_t lo) { return lo >= 64 ? 0ull : x >> lo; }

KMAN_DEV uint64_t comp_of(uint64_t key, uint32_t seg, uint32_t lo) {
    return lo >= 64 ? key : (((uint64_t)seg << lo) | (key & ((1ull << lo) - 1)));
}

// index of the listed big segment that starts at or before pos (-1 if none);
// ov holds (start, end) pairs sorted by start
KMAN_DEV int64_t find_big(const uint64_t *ov, uint32_t n_ov, uint64_t pos) {
    int64_t lo = 0, hi = n_ov;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (ov[2 * mid] <= pos) lo = mid + 1;
        else hi = mid;
    }
    return lo - 1;
}

// first index >= from whose key differs from `key` (keys sorted, keys[from-1] == key)
KMAN_DEV uint64_t run_end(const uint64_t *keys, uint64_t n, uint64_t from, uint64_t key) {
    uint64_t lo = from, hi = n, step = 1;
    while (lo < n) {
        const uint64_t probe = lo + step - 1;
        if (probe >= n) break;
        if (keys[probe] != key) {
            hi = probe;
            break;
        }
        lo = probe + 1;
        step <<= 1;
    }
    if (lo >= n) return n;
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        if (keys[mid] == key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// One wave sorts the staged segment [sa, sa + sz) by its low bits (stable LSD,
// 7-bit digits, the wave's own 128 counters).  Items travel
// packed: IT = u32 holds (low bits << 10 | offset in the segment) when the low
// bits fit in 22 (passes bounce through spk), IT = u64 holds (low bits << 13 |
// position) (passes bounce through skey).  The last pass writes the full key to
// skey and its original position to spk.
template <typename IT, bool ATOMIC>
KMAN_DEV void wave_sort_segment(uint64_t *skey, uint32_t *spk, uint32_t *wh, uint32_t sa, uint32_t sz,
                                uint32_t low_bits) {
    constexpr bool SMALL = sizeof(IT) == 4;
    constexpr uint32_t PS = SMALL ? 10 : 13;  // position bits
    const int lane = lane_id();
    const uint32_t npl = (low_bits + FBITS - 1) / FBITS;
    const uint64_t lmask = low_bits >= 64 ? ~0ull : ((1ull << low_bits) - 1);
    {
        const uint64_t pfx_hi = skey[sa] & ~lmask;
        IT pw[WI];
#pragma unroll
        for (int i = 0; i < WI; i++) {
            if ((uint32_t)(i * 64) >= sz) break;
            const uint32_t p = (uint32_t)(i * 64 + lane);
            pw[i] = p < sz ? (IT)(((skey[sa + p] & lmask) << PS) | (SMALL ? p : sa + p)) : (IT)0;
        }
        uint32_t at = 0;
        for (uint32_t pp = 0; pp < npl; pp++) {
            const uint32_t bw = (low_bits - at + (npl - pp) - 1) / (npl - pp);
            const uint32_t sh = at + PS, dm = (1u << bw) - 1;
            at += bw;
            wh[lane] = 0;
            wh[lane + 64] = 0;
            __builtin_amdgcn_wave_barrier();
            uint32_t r[WI], d[WI];
#pragma unroll
            for (int i = 0; i < WI; i++) {
                if ((uint32_t)(i * 64) >= sz) break;
                const uint32_t p = (uint32_t)(i * 64 + lane);
                d[i] = (uint32_t)(pw[i] >> sh) & dm;
                if (ATOMIC) {
                    r[i] = p < sz ? atomicAdd(&wh[d[i]], 1u) : 0u;
                } else {
                    const bool valid = p < sz;
                    uint64_t peers = __ballot(valid);
                    for (uint32_t bb = 0; bb < bw; bb++) {
                        const bool set = (d[i] >> bb) & 1u;
                        const uint64_t mm = __ballot(set);
                        peers &= set ? mm : ~mm;
                    }
                    uint32_t before = 0;
                    if (valid) before = wh[d[i]];
                    r[i] = before + (uint32_t)__popcll(peers & lanemask_lt());
                    const int leader = __ffsll((unsigned long long)peers) - 1;
                    if (valid && lane == leader) wh[d[i]] = before + (uint32_t)__popcll(peers);
                    __builtin_amdgcn_wave_barrier();
                }
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t c0 = wh[2 * lane], c1 = wh[2 * lane + 1];
            const uint32_t inc = wave_inclusive_scan(c0 + c1, SumU32());
            wh[2 * lane] = inc - c0 - c1;
            wh[2 * lane + 1] = inc - c1;
            __builtin_amdgcn_wave_barrier();
            const bool last_pass = pp + 1 == npl;
#pragma unroll
            for (int i = 0; i < WI; i++) {
                if ((uint32_t)(i * 64) >= sz) break;
                const uint32_t p = (uint32_t)(i * 64 + lane);
                if (p < sz) {
                    const uint32_t dst = sa + wh[d[i]] + r[i];
                    if (last_pass) {
                        skey[dst] = pfx_hi | (uint64_t)(pw[i] >> PS);
                        spk[dst] = SMALL ? sa + (uint32_t)(pw[i] & 1023u) : (uint32_t)(pw[i] & 8191u);
                    } else if constexpr (SMALL) {
                        spk[dst] = (uint32_t)pw[i];
                    } else {
                        skey[dst] = (uint64_t)pw[i];
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (!last_pass) {
#pragma unroll
                for (int i = 0; i < WI; i++) {
                    if ((uint32_t)(i * 64) >= sz) break;
                    const uint32_t p = (uint32_t)(i * 64 + lane);
                    if (p < sz) {
                        if constexpr (SMALL) pw[i] = (IT)spk[sa + p];
                        else pw[i] = (IT)skey[sa + p];
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
}

// position of the n-th (0-based) set bit of x; n < popcount(x)
KMAN_DEV uint32_t nth_bit(uint64_t x, uint32_t n) {
    uint32_t pos = 0, c;
    c = (uint32_t)__popc((uint32_t)x);
    if (n >= c) { n -= c; x >>= 32; pos += 32; }
    c = (uint32_t)__popc((uint32_t)x & 0xffffu);
    if (n >= c) { n -= c; x >>= 16; pos += 16; }
    c = (uint32_t)__popc((uint32_t)x & 0xffu);
    if (n >= c) { n -= c; x >>= 8; pos += 8; }
    c = (uint32_t)__popc((uint32_t)x & 0xfu);
    if (n >= c) { n -= c; x >>= 4; pos += 4; }
    c = (uint32_t)__popc((uint32_t)x & 0x3u);
    if (n >= c) { n -= c; x >>= 2; pos += 2; }
    c = (uint32_t)(x & 1u);
    if (n >= c) pos += 1;
    return pos;
}

// bits of mask word wi (positions 64 wi ..) that lie in [a, b)
KMAN_DEV uint64_t span_bits(uint32_t wi, uint32_t a, uint32_t b) {
    auto below = [wi](uint32_t lim) -> uint64_t {
        const int32_t d = (int32_t)lim - (int32_t)(wi * 64);
        return d <= 0 ? 0ull : d >= 64 ? ~0ull : ((1ull << d) - 1);
    };
    return below(b) & ~below(a);
}

KMAN_DEV uint32_t wave_min_u32(uint32_t v) {
    v = wave_inclusive_scan(v, [](uint32_t a, uint32_t b) { return a < b ? a : b; }, 0xffffffffu);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
KMAN_DEV uint32_t wave_max_u32(uint32_t v) {
    v = wave_inclusive_scan(v, [](uint32_t a, uint32_t b) { return a > b ? a : b; }, 0u);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

enum { M_SORT = 0, M_COUNT = 1, M_UNIQ = 2 };

// One chunk per block.  Segment starts are found while the chunk loads (the
// previous key of each lane comes over DPP) and kept as a bit mask in LDS;
// every wave then derives the same plan from the mask (owned range, tail end,
// segment bounds and the longest segment) without further block barriers, and
// sorts its share of the segments (round robin) alone.
template <int MODE, typename V, typename O, bool ATOMIC>
__global__ __launch_bounds__(FT) void segfin_kernel(uint64_t *__restrict__ keys, V *__restrict__ vals, uint64_t n,
                                                    uint32_t lo_bit, const uint64_t *__restrict__ ov, uint32_t n_ov,
                                                    uint64_t *__restrict__ big, uint32_t *__restrict__ n_big,
                                                    uint32_t big_cap, uint64_t *__restrict__ okeys,
                                                    O *__restrict__ ovals, uint64_t *__restrict__ status,
                                                    uint32_t *__restrict__ counter, uint32_t epoch,
                                                    uint32_t *__restrict__ err) {
    constexpr bool HAS_V = !std::is_same<V, NoV>::value;
    constexpr bool V32 = HAS_V && sizeof(V) == 4 && MODE != M_COUNT;  // u32 payload staged through LDS
    constexpr uint32_t NONE = 0xffffffffu;
    __shared__ __attribute__((aligned(16))) uint64_t skey[FR];
    __shared__ uint32_t spk[FR];  // (segment index << 16) | position in the chunk
    __shared__ uint64_t smask[NWORD];  // bit p: a segment starts at position p
    __shared__ uint32_t whist[FW][FRADIX];
    __shared__ uint32_t lstart[FRADIX];
    __shared__ uint32_t lds_scan[FW];
    __shared__ uint64_t lds_scan64[FW];
    __shared__ uint32_t s_end, s_tile, s_flags;
    __shared__ uint64_t s_out;

    // dynamic chunk id (chunks start in id order: every predecessor of a chunk is
    // resident or done); s_tile is never rewritten, so one barrier suffices
    if (threadIdx.x == 0) s_tile = atomicAdd(counter, 1u);
    __syncthreads();
    const int64_t tile = s_tile;
    FSTAMP(0);
    const uint64_t base = (uint64_t)tile * FC;
    const uint32_t cnt = (uint32_t)(n - base < (uint64_t)FC ? n - base : (uint64_t)FC);
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    const int t = threadIdx.x;
    if (t == 0) {
        s_end = FR + 1;
        s_flags = 0;
    }

    // ---- load the chunk and the next FT keys; mark segment starts.  Every
    // load is issued before the first is consumed (one round trip, not PI)
    const uint64_t prevk = base ? keys[base - 1] : 0;
    uint64_t kk[PI], k0[PI];
#pragma unroll
    for (int r = 0; r < PI; r++) {
        const uint64_t g = base + (uint64_t)(r * FT + t);
        kk[r] = g < n ? keys[g] : 0;
    }
    // lane 0's previous key belongs to another wave
#pragma unroll
    for (int r = 0; r < PI; r++) {
        const uint32_t p = (uint32_t)(r * FT + t);
        const uint64_t g = base + p;
        k0[r] = (lane == 0 && p > 0 && g <= n) ? keys[g - 1] : prevk;
    }
#pragma unroll
    for (int r = 0; r < PI; r++) {
        const uint32_t p = (uint32_t)(r * FT + t);
        const uint64_t g = base + p;
        const bool in = g < n;
        const uint64_t k = kk[r];
        uint64_t kp = wave_shr1(k, (uint64_t)0);
        if (lane == 0) kp = k0[r];
        const bool st = in && (g == 0 || pre_of(k, lo_bit) != pre_of(kp, lo_bit));
        const uint64_t mk = __ballot(st);
        if (in) skey[p] = k;
        if (lane == 0) smask[p >> 6] = mk;
    }
    for (int wi = PI * FT / 64 + t; wi < NWORD; wi += FT) smask[wi] = 0;
    __syncthreads();
    FSTAMP(1);

    // ---- the plan, computed by every wave from the mask (lane l: words l, l + 64)
    const uint32_t wia = (uint32_t)lane, wib = (uint32_t)lane + 64;
    const uint64_t ma = wia < (uint32_t)NWORD ? smask[wia] : 0ull;
    const uint64_t mb = wib < (uint32_t)NWORD ? smask[wib] : 0ull;
    uint32_t first, lastp1, endp;
    {
        const uint64_t ia = ma & span_bits(wia, 0, cnt), ib = mb & span_bits(wib, 0, cnt);
        const uint64_t oa = ma & ~span_bits(wia, 0, cnt), ob = mb & ~span_bits(wib, 0, cnt);
        uint32_t f = NONE, l = 0, e = NONE;
        if (ia) {
            f = wia * 64 + (uint32_t)__ffsll((unsigned long long)ia) - 1;
            l = wia * 64 + 64 - (uint32_t)__clzll(ia);
        }
        if (ib) {
            f = f < NONE ? f : wib * 64 + (uint32_t)__ffsll((unsigned long long)ib) - 1;
            l = wib * 64 + 64 - (uint32_t)__clzll(ib);
        }
        if (oa) e = wia * 64 + (uint32_t)__ffsll((unsigned long long)oa) - 1;
        else if (ob) e = wib * 64 + (uint32_t)__ffsll((unsigned long long)ob) - 1;
        first = wave_min_u32(f);
        lastp1 = wave_max_u32(l);
        endp = wave_min_u32(e);
    }
    const bool has_start = first < cnt;
    const uint32_t last = lastp1 - 1;
    // listed big segments: the leading one (started before the chunk) and the
    // last one starting here are processed as presorted slices
    if (n_ov) {
        if (t == 0) {
            uint32_t f = 0;
            if (first > 0 && base > 0) {
                const int64_t i = find_big(ov, n_ov, base);
                if (i >= 0 && ov[2 * i + 1] > base) f |= 1;
            }
            if (has_start) {
                const int64_t i = find_big(ov, n_ov, base + last);
                if (i >= 0 && ov[2 * i] == base + last) f |= 2;
            }
            s_flags = f;
        }
        __syncthreads();
    }
    const bool lead_pre = s_flags & 1;
    const bool last_pre = s_flags & 2;

    // ---- end of the last owned segment
    uint32_t hi = cnt;
    bool trail_pre = last_pre;  // the last segment is a presorted (or unstaged big) slice
    if (has_start && !last_pre && base + cnt < n) {
        if (endp != NONE) {
            hi = endp;  // a start among the keys loaded with the chunk
        } else if (n - base <= (uint64_t)(PI * FT)) {
            hi = (uint32_t)(n - base);  // the array ends there
        } else {
            // longer tail: load further rounds until the prefix changes
            const uint64_t lp = pre_of(skey[last], lo_bit);
            for (uint32_t r0 = PI * FT; r0 < (uint32_t)FR; r0 += FT) {
                const uint32_t rel = r0 + t;
                const uint64_t g = base + rel;
                if (g < n) {
                    const uint64_t kk = keys[g];
                    skey[rel] = kk;
                    if (pre_of(kk, lo_bit) != lp) atomicMin(&s_end, rel);
                } else if (g == n) {
                    atomicMin(&s_end, rel);
                }
                __syncthreads();
                if (s_end < r0 + FT) break;
            }
            hi = s_end;
            if (hi > (uint32_t)FR) {
                trail_pre = true;
                // a big segment nobody listed (first run): record it; this run's
                // output is discarded by the host
                if (t == 0) {
                    const uint32_t slot = atomicAdd(n_big, 1u);
                    if (slot < big_cap) big[slot] = base + last;
                }
                hi = cnt;
            }
        }
    }
    const uint32_t lo = lead_pre ? 0u : (has_start ? first : cnt);
    if (!has_start && !lead_pre) hi = lo;
    const uint32_t m = hi - lo;
    const bool need_sort = has_start && m > 1;
    // the u32 payload of positions t + r FT in [lo, hi): in flight during the sort
    uint32_t cv[V32 ? FI : 1];
    if constexpr (V32) {
#pragma unroll
        for (int r = 0; r < FI; r++) {
            const uint32_t p = (uint32_t)(t + r * FT);
            cv[r] = (p >= lo && p < hi) ? (uint32_t)vals[base + p] : 0u;
        }
    }

    FSTAMP(2);
    // ---- stable LDS sort of [lo, hi): every owned segment by its low bits
    if (need_sort) {
        const uint32_t low_bits = lo_bit >= 64 ? 64u : lo_bit;
        // segment starts after lo (the range's first segment starts at lo)
        const uint64_t xa = ma & span_bits(wia, lo + 1, hi), xb = mb & span_bits(wib, lo + 1, hi);
        const uint32_t ca = (uint32_t)__popcll(xa), cb = (uint32_t)__popcll(xb);
        const uint32_t inca = wave_inclusive_scan(ca, SumU32()), incb = wave_inclusive_scan(cb, SumU32());
        const uint32_t tota = (uint32_t)__builtin_amdgcn_readlane((int)inca, 63);
        const uint32_t nsegs = 1 + tota + (uint32_t)__builtin_amdgcn_readlane((int)incb, 63);
        const uint32_t prea = inca - ca, preb = tota + incb - cb;
        // longest segment: gaps between consecutive starts (lo and hi included)
        uint32_t maxlen;
        {
            auto mx = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
            const uint32_t la = xa ? wia * 64 + 63 - (uint32_t)__clzll(xa) : 0u;
            const uint32_t lb = xb ? wib * 64 + 63 - (uint32_t)__clzll(xb) : 0u;
            // last start before each word (in word order a[0..63], b[0..31])
            const uint32_t pa = wave_shr1(wave_inclusive_scan(la, mx), 0u);
            const uint32_t lasta = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_scan(la, mx), 63);
            const uint32_t pb = mx(wave_shr1(wave_inclusive_scan(lb, mx), 0u), lasta);
            uint32_t g = 0;
            uint64_t x = xa;
            uint32_t prv = mx(pa, lo);
            while (x) {
                const uint32_t q = wia * 64 + (uint32_t)__ffsll((unsigned long long)x) - 1;
                g = mx(g, q - prv);
                prv = q;
                x &= x - 1;
            }
            x = xb;
            prv = mx(pb, lo);
            while (x) {
                const uint32_t q = wib * 64 + (uint32_t)__ffsll((unsigned long long)x) - 1;
                g = mx(g, q - prv);
                prv = q;
                x &= x - 1;
            }
            const uint32_t lastall = mx(mx(lasta, (uint32_t)__builtin_amdgcn_readlane(
                                                         (int)wave_inclusive_scan(lb, mx), 63)), lo);
            maxlen = mx(wave_max_u32(g), hi - lastall);
        }
        const bool wave_path = maxlen <= (uint32_t)(WI * 64) && low_bits <= 51;
        if (wave_path) {
            // start of segment j (j >= 1): the (j-1)-th set bit after lo
            auto seg_start = [&](uint32_t j) -> uint32_t {
                if (j == 0) return lo;
                if (j >= nsegs) return hi;
                const uint32_t nb = j - 1;
                const uint64_t ba = __ballot(ca && nb >= prea && nb < prea + ca);
                const uint64_t bb = __ballot(cb && nb >= preb && nb < preb + cb);
                const bool inb = ba == 0;
                const int src = __ffsll((unsigned long long)(inb ? bb : ba)) - 1;
                const uint32_t pos = inb ? wib * 64 + nth_bit(xb, nb - preb) : wia * 64 + nth_bit(xa, nb - prea);
                return (uint32_t)__builtin_amdgcn_readlane((int)pos, src);
            };
            if (lead_pre || trail_pre) {
                // identity positions for the presorted slices
                for (uint32_t q = t; q < m; q += FT) spk[lo + q] = lo + q;
                __syncthreads();
            }
            const uint32_t s0 = lead_pre ? 1u : 0u, s1 = nsegs - (trail_pre ? 1u : 0u);
#if defined(KMAN_ABL) && (KMAN_ABL & 8)
            // ablation build only: no segment sort (wrong order, measures the rest)
            if (false)
#endif
            for (uint32_t j = s0 + (uint32_t)w; j < s1; j += FW) {
                const uint32_t sa = seg_start(j), sb = seg_start(j + 1);
                if (sb - sa < 2) {
                    if (lane == 0) spk[sa] = sa;
                    continue;
                }
                if (low_bits <= 22)
                    wave_sort_segment<uint32_t, ATOMIC>(skey, spk, whist[w], sa, sb - sa, low_bits);
                else
                    wave_sort_segment<uint64_t, ATOMIC>(skey, spk, whist[w], sa, sb - sa, low_bits);
            }
            __syncthreads();
        } else {
            // many or long segments: block-wide LSD on (segment index, low bits)
            uint64_t key[FI];
            uint32_t pk[FI];
            uint32_t run = 0;
#pragma unroll
            for (int i = 0; i < FI; i++) {
                const uint32_t q = (uint32_t)(w * FI * 64 + i * 64 + lane);
                const bool valid = q < m;
                key[i] = valid ? skey[lo + q] : 0;
                const bool st = valid && q > 0 && ((smask[(lo + q) >> 6] >> ((lo + q) & 63)) & 1ull);
                const uint64_t msk = __ballot(st);
                pk[i] = run + (uint32_t)__popcll(msk & (lanemask_lt() | (1ull << lane)));
                run += (uint32_t)__popcll(msk);
            }
            if (lane == 0) lds_scan[w] = run;
            __syncthreads();
            uint32_t woff = 0;
#pragma unroll
            for (int ww = 0; ww < FW; ww++) woff += ww < w ? lds_scan[ww] : 0u;
#pragma unroll
            for (int i = 0; i < FI; i++) {
                const uint32_t q = (uint32_t)(w * FI * 64 + i * 64 + lane);
                pk[i] = ((pk[i] + woff) << 16) | (lo + q);
            }
            const uint32_t sbits = nsegs > 1 ? 32 - __clz(nsegs - 1) : 0;
            const uint32_t tb = sbits + low_bits;
            const uint32_t np = (tb + FBITS - 1) / FBITS;
            uint32_t at = 0;
            for (uint32_t p = 0; p < np; p++) {
                const uint32_t b = (tb - at + (np - p) - 1) / (np - p);
                const uint32_t sh = at;
                at += b;
                const uint32_t radix = 1u << b, dm = radix - 1;
                for (int j = t; j < FW * FRADIX; j += FT) (&whist[0][0])[j] = 0;
                __syncthreads();
                uint32_t rank[FI];
                uint32_t dg[FI];
#pragma unroll
                for (int i = 0; i < FI; i++) {
                    const uint32_t q = (uint32_t)(w * FI * 64 + i * 64 + lane);
                    dg[i] = (uint32_t)(comp_of(key[i], pk[i] >> 16, lo_bit) >> sh) & dm;
                    const bool valid = q < m;
                    if (ATOMIC) {
                        rank[i] = valid ? atomicAdd(&whist[w][dg[i]], 1u) : 0u;
                    } else {
                        uint64_t peers = __ballot(valid);
                        for (uint32_t bb = 0; bb < b; bb++) {
                            const bool set = (dg[i] >> bb) & 1u;
                            const uint64_t mm = __ballot(set);
                            peers &= set ? mm : ~mm;
                        }
                        uint32_t before = 0;
                        if (valid) before = whist[w][dg[i]];
                        rank[i] = before + (uint32_t)__popcll(peers & lanemask_lt());
                        const int leader = __ffsll((unsigned long long)peers) - 1;
                        if (valid && lane == leader) whist[w][dg[i]] = before + (uint32_t)__popcll(peers);
                    }
                }
                __syncthreads();
                uint32_t tot = 0;
                if (t < (int)radix) {
#pragma unroll
                    for (int ww = 0; ww < FW; ww++) {
                        const uint32_t c = whist[ww][t];
                        whist[ww][t] = tot;
                        tot += c;
                    }
                }
                const uint32_t ls = block_exclusive_scan<FT>(tot, SumU32(), 0u, lds_scan, (uint32_t *)nullptr);
                if (t < (int)radix) lstart[t] = ls;
                __syncthreads();
#pragma unroll
                for (int i = 0; i < FI; i++) {
                    const uint32_t q = (uint32_t)(w * FI * 64 + i * 64 + lane);
                    if (q < m) {
                        const uint32_t dst = lo + lstart[dg[i]] + whist[w][dg[i]] + rank[i];
                        skey[dst] = key[i];
                        spk[dst] = pk[i];
                    }
                }
                __syncthreads();
                if (p + 1 < np) {
#pragma unroll
                    for (int i = 0; i < FI; i++) {
                        const uint32_t q = (uint32_t)(w * FI * 64 + i * 64 + lane);
                        if (q < m) {
                            key[i] = skey[lo + q];
                            pk[i] = spk[lo + q];
                        }
                    }
                }
            }
            if (np == 0) {
                for (uint32_t q = t; q < m; q += FT) spk[lo + q] = lo + q;
                __syncthreads();
            }
        }
    } else {
        for (uint32_t q = t; q < m; q += FT) spk[lo + q] = lo + q;
        __syncthreads();
    }

    FSTAMP(3);
    if constexpr (MODE == M_SORT) {
        if (!need_sort) return;
        for (uint32_t q = t; q < m; q += FT) keys[base + lo + q] = skey[lo + q];
        if constexpr (V32) {
            // u32 payload: staged in LDS by position (over spk, once every sorted
            // position has been read) and permuted from there
            uint32_t ixr[FI];
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                ixr[r] = q < m ? spk[lo + q] & 0xffffu : 0;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t p = (uint32_t)(t + r * FT);
                if (p >= lo && p < hi) spk[p] = cv[r];
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                if (q < m) vals[base + lo + q] = (V)spk[ixr[r]];
            }
        } else if constexpr (HAS_V) {
            // gather the payload in sorted order; staging it in LDS makes every
            // gather complete before any in-place write below
            V vv[FI];
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                vv[r] = q < m ? vals[base + (spk[lo + q] & 0xffffu)] : (V)0;
            }
            __syncthreads();
            V *sval = reinterpret_cast<V *>(skey);
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                if (q < m) sval[q] = vv[r];
            }
            __syncthreads();
            for (uint32_t q = t; q < m; q += FT) vals[base + lo + q] = sval[q];
        }
        return;
    } else {
        // ---- run-length pass over the sorted range (thread t: items t*FI ..)
        const bool has_prev_g = base + lo > 0;
        const uint64_t prev_g = lo ? skey[lo - 1] : prevk;  // [0, lo) is untouched by the sort
        const bool has_next_g = base + hi < n;
        // the first key past the range (another segment) was staged by the chunk
        // load or the tail rounds
        const uint64_t next_g = has_next_g ? skey[hi] : 0;
        uint64_t k[FI];
        uint32_t ix[FI];  // UNIQ: each item's position in the chunk, for its payload
        const uint32_t q0 = (uint32_t)t * FI;
#pragma unroll
        for (int j = 0; j < FI; j++) {
            k[j] = q0 + j < m ? skey[lo + q0 + j] : 0;
            ix[j] = (MODE == M_UNIQ && q0 + j < m) ? spk[lo + q0 + j] & 0xffffu : 0;
        }
        uint32_t heads = 0, tails = 0;
#pragma unroll
        for (int j = 0; j < FI; j++) {
            const uint32_t q = q0 + j;
            if (q < m) {
                const uint64_t pk = q == 0 ? prev_g : (j ? k[j - 1] : skey[lo + q - 1]);
                const uint64_t nk = q + 1 < m ? (j + 1 < FI ? k[j + 1] : skey[lo + q + 1]) : next_g;
                const bool hp = q > 0 || has_prev_g;
                const bool hn = q + 1 < m || has_next_g;
                heads |= (uint32_t)(!hp || k[j] != pk) << j;
                tails |= (uint32_t)(!hn || k[j] != nk) << j;
            }
        }
        uint32_t emit = 0;  // items that produce an output, in item order
        uint64_t cval[FI];  // COUNT: group sizes
        if constexpr (MODE == M_UNIQ) {
            emit = heads & tails;
        } else {
            // a group is emitted by the chunk holding its head, at its tail (or at
            // the range end when it continues into a presorted slice beyond)
            const uint64_t lh = heads ? (uint64_t)(q0 + (31 - __clz(heads)) + 1) : 0;
            const uint64_t lh_before = block_exclusive_scan<FT>(
                lh, [](uint64_t a, uint64_t b) { return a > b ? a : b; }, (uint64_t)0, lds_scan64,
                (uint64_t *)nullptr);
            uint64_t cur = lh_before;  // head position + 1 of the open group, 0 = none
#pragma unroll
            for (int j = 0; j < FI; j++) {
                const uint32_t q = q0 + j;
                cval[j] = 0;
                if (q >= m) continue;
                if ((heads >> j) & 1u) cur = q + 1;
                if (cur == 0) continue;
                if ((tails >> j) & 1u) {
                    emit |= 1u << j;
                    cval[j] = q + 2 - cur;
                } else if (q + 1 == m) {
                    emit |= 1u << j;
                    cval[j] = run_end(keys, n, base + hi, k[j]) - (base + lo + cur - 1);
                }
            }
            // each emitting item closes the group of the head before it: output
            // slots follow heads, so count heads for the offsets
        }
        const uint32_t ne = (uint32_t)__popc(emit);
        uint32_t total;
        const uint32_t off = block_exclusive_scan<FT>(ne, SumU32(), 0u, lds_scan, &total);
        FSTAMP(7);
        // (the scan's barriers ordered every read of skey / spk above before the
        // writes below)
        constexpr bool LDS_V = MODE == M_UNIQ && V32;
        if (w == 0) {
            const uint64_t b = wave_lookback<0>(status, tile, total, epoch, err);
            if (lane == 0) s_out = b;
        }
        O ov_[FI];
        if constexpr (MODE == M_UNIQ && !LDS_V) {
#pragma unroll
            for (int j = 0; j < FI; j++)
                ov_[j] = ((emit >> j) & 1u) ? (O)vals[base + ix[j]] : (O)0;
        } else if constexpr (MODE == M_COUNT) {
#pragma unroll
            for (int j = 0; j < FI; j++) ov_[j] = (O)cval[j];
        }
        if constexpr (LDS_V) {
            // the range's payload by position
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t p = (uint32_t)(t + r * FT);
                if (p >= lo && p < hi) spk[p] = cv[r];
            }
        }
        FSTAMP(4);
        if constexpr (!LDS_V) __syncthreads();
        uint32_t o = off;
#pragma unroll
        for (int j = 0; j < FI; j++)
            if ((emit >> j) & 1u) skey[o++] = k[j];
        __syncthreads();
        if constexpr (LDS_V) {
#pragma unroll
            for (int j = 0; j < FI; j++) ov_[j] = ((emit >> j) & 1u) ? (O)spk[ix[j]] : (O)0;
        }
        const uint64_t ob = s_out;
        FSTAMP(5);
        for (uint32_t q = t; q < total; q += FT) okeys[ob + q] = skey[q];
        __syncthreads();
        O *so = reinterpret_cast<O *>(skey);
        o = off;
#pragma unroll
        for (int j = 0; j < FI; j++)
            if ((emit >> j) & 1u) so[o++] = ov_[j];
        __syncthreads();
        for (uint32_t q = t; q < total; q += FT) ovals[ob + q] = so[q];
        FSTAMP(6);
    }
}

// end of each listed big segment: first index whose prefix differs
__global__ void big_end_kernel(const uint64_t *__restrict__ keys, uint64_t n, uint32_t lo_bit,
                               uint64_t *__restrict__ ov, uint32_t n_ov) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_ov) return;
    const uint64_t s = ov[2 * i];
    const uint64_t p = pre_of(keys[s], lo_bit);
    uint64_t lo = s + 1, hi = n, step = 1;
    while (lo < n) {
        const uint64_t probe = lo + step - 1;
        if (probe >= n) break;
        if (pre_of(keys[probe], lo_bit) != p) {
            hi = probe;
            break;
        }
        lo = probe + 1;
        step <<= 1;
    }
    if (lo < n) {
        while (lo < hi) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            if (pre_of(keys[mid], lo_bit) == p) lo = mid + 1;
            else hi = mid;
        }
    } else {
        lo = n;
    }
    ov[2 * i + 1] = lo;
}

// copy the listed big segments between their places in the array and a
// contiguous buffer (dir 0: gather, 1: scatter back); off = exclusive prefix of lengths
template <typename T>
__global__ void big_copy_kernel(T *__restrict__ arr, T *__restrict__ packed, const uint64_t *__restrict__ ov,
                                const uint64_t *__restrict__ off, uint32_t n_ov, uint64_t total, int dir) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total;
         j += (uint64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = n_ov;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (off[mid] <= j) lo = mid + 1;
            else hi = mid;
        }
        const int64_t g = lo - 1;
        const uint64_t a = ov[2 * g] + (j - off[g]);
        if (dir == 0) packed[j] = arr[a];
        else arr[a] = packed[j];
    }
}

template <int MODE, typename V, typename O>
int launch_segfin(kman_ctx *ctx, uint64_t *keys, V *vals, uint64_t n, uint32_t lo_bit, const uint64_t *ov,
                  uint32_t n_ov, uint64_t *big, uint32_t *n_big, uint32_t big_cap, uint64_t *okeys, O *ovals,
                  uint64_t *n_out) {
    const uint64_t T = ceil_div(n, (uint64_t)FC);
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, T, &epoch, &counter));
    HIP_TRY(ctx, hipMemsetAsync(n_big, 0, sizeof(uint32_t), ctx->stream));
    {
        KTimer kt_(ctx, "finish");
        if (ctx->lds_atomic_ordered)
            hipLaunchKernelGGL((segfin_kernel<MODE, V, O, true>), dim3((uint32_t)T), dim3(FT), 0, ctx->stream, keys,
                               vals, n, lo_bit, ov, n_ov, big, n_big, big_cap, okeys, ovals, ctx->d_status, counter,
                               epoch, ctx->d_err);
        else
            hipLaunchKernelGGL((segfin_kernel<MODE, V, O, false>), dim3((uint32_t)T), dim3(FT), 0, ctx->stream, keys,
                               vals, n, lo_bit, ov, n_ov, big, n_big, big_cap, okeys, ovals, ctx->d_status, counter,
                               epoch, ctx->d_err);
        HIP_TRY(ctx, hipGetLastError());
    }
    if (MODE == M_SORT) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        *n_out = n;
        return kman_check_device_error(ctx);
    }
    return kman_lookback_total(ctx, T, n_out);
}

// the run over every chunk, the big-segment fallback when the first run found
// any, and the second run
template <int MODE, typename V, typename O>
int finish_typed(kman_ctx *ctx, uint64_t *keys, uint64_t *keys_alt, V *vals, V *vals_alt, uint32_t vb, uint64_t n,
                 uint32_t key_bits, uint32_t lo_bit, uint64_t *okeys, O *ovals, uint64_t *n_out) {
    // any big segment is longer than FR - FC keys.  Device list layout:
    // [0, 2 cap) (start, end) pairs, [2 cap, 3 cap) starts found by a run, then the count
    const uint32_t big_cap = (uint32_t)(n / (FR - FC) + 2);
    uint64_t *d_ov = nullptr;
    KMAN_TRY(kman_aux(ctx, (3 * (size_t)big_cap + 2) * 8, (void **)&d_ov));
    uint64_t *d_big = d_ov + 2 * (size_t)big_cap;
    uint32_t *d_nbig = (uint32_t *)(d_ov + 3 * (size_t)big_cap);
    KMAN_TRY((launch_segfin<MODE, V, O>(ctx, keys, vals, n, lo_bit, nullptr, 0, d_big, d_nbig, big_cap, okeys, ovals,
                                        n_out)));
    uint32_t nb = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&nb, d_nbig, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (nb == 0) return KMAN_OK;
    if (nb > big_cap) return kman_fail(ctx, KMAN_EINVAL, "big segment list overflow (%u > %u)", nb, big_cap);
    std::vector<uint64_t> starts(nb), pairs(2 * (size_t)nb);
    HIP_TRY(ctx, hipMemcpyAsync(starts.data(), d_big, 8 * (size_t)nb, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    std::sort(starts.begin(), starts.end());
    for (uint32_t i = 0; i < nb; i++) pairs[2 * i] = starts[i];
    HIP_TRY(ctx, hipMemcpyAsync(d_ov, pairs.data(), 16 * (size_t)nb, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(big_end_kernel, dim3((nb + 255) / 256), dim3(256), 0, ctx->stream, keys, n, lo_bit, d_ov, nb);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(pairs.data(), d_ov, 16 * (size_t)nb, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<uint64_t> off(nb + 1);
    uint64_t M = 0;
    for (uint32_t i = 0; i < nb; i++) {
        off[i] = M;
        M += pairs[2 * i + 1] - pairs[2 * i];
    }
    off[nb] = M;
    // the big segments, gathered contiguously, full-key sorted, scattered back
    constexpr bool HAS_V = !std::is_same<V, NoV>::value;
    const size_t vsz = HAS_V ? sizeof(V) : 0;
    char *tmp = nullptr;
    const size_t tbytes = 8 * (nb + 1) + M * 16 + M * vsz * 2 + 256;
    HIP_TRY(ctx, hipMalloc((void **)&tmp, tbytes));
    struct Free {
        kman_ctx *c;
        void *p;
        ~Free() {
            (void)hipStreamSynchronize(c->stream);
            (void)hipFree(p);
        }
    } ft_{ctx, tmp};
    uint64_t *d_off = (uint64_t *)tmp;
    uint64_t *pk0 = d_off + (nb + 1);
    uint64_t *pk1 = pk0 + M;
    V *pv0 = HAS_V ? (V *)(pk1 + M) : nullptr;
    V *pv1 = HAS_V ? pv0 + M : nullptr;
    HIP_TRY(ctx, hipMemcpyAsync(d_off, off.data(), 8 * (nb + 1), hipMemcpyHostToDevice, ctx->stream));
    const uint32_t cg = (uint32_t)(ceil_div(M, 256) < 65536 ? ceil_div(M, 256) : 65536);
    hipLaunchKernelGGL(big_copy_kernel<uint64_t>, dim3(cg), dim3(256), 0, ctx->stream, keys, pk0, d_ov, d_off, nb, M,
                       0);
    if constexpr (HAS_V)
        hipLaunchKernelGGL(big_copy_kernel<V>, dim3(cg), dim3(256), 0, ctx->stream, vals, pv0, d_ov, d_off, nb, M, 0);
    HIP_TRY(ctx, hipGetLastError());
    int in_alt = 0;
    KMAN_TRY(kman_sort(ctx, pk0, pk1, (void *)pv0, (void *)pv1, (uint32_t)vsz, M, key_bits, nullptr, &in_alt));
    hipLaunchKernelGGL(big_copy_kernel<uint64_t>, dim3(cg), dim3(256), 0, ctx->stream, keys, in_alt ? pk1 : pk0, d_ov,
                       d_off, nb, M, 1);
    if constexpr (HAS_V)
        hipLaunchKernelGGL(big_copy_kernel<V>, dim3(cg), dim3(256), 0, ctx->stream, vals, in_alt ? pv1 : pv0, d_ov,
                           d_off, nb, M, 1);
    HIP_TRY(ctx, hipGetLastError());
    // second run with the presorted list; it must find nothing new
    KMAN_TRY((launch_segfin<MODE, V, O>(ctx, keys, vals, n, lo_bit, d_ov, nb, d_big, d_nbig, big_cap, okeys, ovals,
                                        n_out)));
    uint32_t nb2 = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&nb2, d_nbig, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    (void)keys_alt;
    (void)vals_alt;
    (void)vb;
    if (nb2 != 0) {
        if (getenv("KMAN_FINISH_DEBUG")) {
            std::vector<uint64_t> s2(nb2 < big_cap ? nb2 : big_cap);
            (void)hipMemcpy(s2.data(), d_big, 8 * s2.size(), hipMemcpyDeviceToHost);
            for (uint32_t i = 0; i < nb; i++)
                fprintf(stderr, "listed %llu..%llu\n", (unsigned long long)pairs[2 * i],
                        (unsigned long long)pairs[2 * i + 1]);
            for (auto v : s2) fprintf(stderr, "unlisted start %llu\n", (unsigned long long)v);
        }
        return kman_fail(ctx, KMAN_EINVAL, "finish: %u unlisted big segments on the second run", nb2);
    }
    return KMAN_OK;
}

}  // namespace

#if defined(KMAN_ABL) && (KMAN_ABL & 4)
extern "C" int kman_debug_set_finish(kman_ctx *ctx, void *dptr) {
    HIP_TRY(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_fdbg), &dptr, sizeof(dptr)));
    unsigned long long z[4] = {0, 0, 0, 0};
    HIP_TRY(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_fstat), z, sizeof(z)));
    return KMAN_OK;
}
extern "C" int kman_debug_finish_stats(kman_ctx *ctx, unsigned long long *out4) {
    HIP_TRY(ctx, hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_fstat), 4 * sizeof(unsigned long long)));
    return KMAN_OK;
}
#endif

extern "C" int kman_split_bits(uint64_t n, uint32_t key_bits, uint32_t *lo_bit) {
    if (!lo_bit || key_bits == 0 || key_bits > 64) return KMAN_EINVAL;
    // P prefix bits so that n / 2^P <= 512 keys per segment on average
    uint32_t p = 0;
    while (p < key_bits && (n >> p) > 512) p++;
    *lo_bit = key_bits - p;
    return KMAN_OK;
}

extern "C" int kman_finish(kman_ctx *ctx, uint64_t *d_keys, uint64_t *d_keys_alt, void *d_vals, void *d_vals_alt,
                           uint32_t val_bytes, uint64_t n, uint32_t key_bits, uint32_t lo_bit, int mode,
                           uint64_t *d_okeys, void *d_ovals, uint32_t oval_bytes, uint64_t *n_out) {
    if (!ctx || !n_out) return KMAN_EINVAL;
    *n_out = 0;
    if (key_bits == 0 || key_bits > 64 || lo_bit > key_bits)
        return kman_fail(ctx, KMAN_EINVAL, "bad key bits %u / low bit %u", key_bits, lo_bit);
    if (val_bytes != 0 && val_bytes != 4 && val_bytes != 8)
        return kman_fail(ctx, KMAN_EINVAL, "val_bytes must be 0, 4 or 8");
    if (mode < KMAN_FINISH_SORT || mode > KMAN_FINISH_UNIQ) return kman_fail(ctx, KMAN_EINVAL, "bad mode %d", mode);
    if (n == 0) return KMAN_OK;
    if (!d_keys) return kman_fail(ctx, KMAN_EINVAL, "null keys");
    if (val_bytes && !d_vals) return kman_fail(ctx, KMAN_EINVAL, "null vals");
    if (mode != KMAN_FINISH_SORT && (!d_okeys || !d_ovals)) return kman_fail(ctx, KMAN_EINVAL, "null output");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (mode == KMAN_FINISH_SORT) {
        if (val_bytes == 0)
            return finish_typed<M_SORT, NoV, uint32_t>(ctx, d_keys, d_keys_alt, nullptr, nullptr, 0, n, key_bits,
                                                       lo_bit, nullptr, nullptr, n_out);
        if (val_bytes == 4)
            return finish_typed<M_SORT, uint32_t, uint32_t>(ctx, d_keys, d_keys_alt, (uint32_t *)d_vals,
                                                            (uint32_t *)d_vals_alt, 4, n, key_bits, lo_bit, nullptr,
                                                            nullptr, n_out);
        return finish_typed<M_SORT, uint64_t, uint64_t>(ctx, d_keys, d_keys_alt, (uint64_t *)d_vals,
                                                        (uint64_t *)d_vals_alt, 8, n, key_bits, lo_bit, nullptr,
                                                        nullptr, n_out);
    }
    if (mode == KMAN_FINISH_COUNT) {
        // the payload is not needed for counts; it is carried through the
        // big-segment fallback only when given
        if (oval_bytes != 4 && oval_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "count bytes must be 4 or 8");
        if (oval_bytes == 4 && n > 0xffffffffull)
            return kman_fail(ctx, KMAN_EINVAL, "u32 counts cannot hold groups of %llu keys", (unsigned long long)n);
        if (oval_bytes == 4)
            return finish_typed<M_COUNT, NoV, uint32_t>(ctx, d_keys, d_keys_alt, nullptr, nullptr, 0, n, key_bits,
                                                        lo_bit, d_okeys, (uint32_t *)d_ovals, n_out);
        return finish_typed<M_COUNT, NoV, uint64_t>(ctx, d_keys, d_keys_alt, nullptr, nullptr, 0, n, key_bits, lo_bit,
                                                    d_okeys, (uint64_t *)d_ovals, n_out);
    }
    if (val_bytes == 0 || oval_bytes != val_bytes)
        return kman_fail(ctx, KMAN_EINVAL, "uniq needs a payload and oval_bytes == val_bytes");
    if (val_bytes == 4)
        return finish_typed<M_UNIQ, uint32_t, uint32_t>(ctx, d_keys, d_keys_alt, (uint32_t *)d_vals,
                                                        (uint32_t *)d_vals_alt, 4, n, key_bits, lo_bit, d_okeys,
                                                        (uint32_t *)d_ovals, n_out);
    return finish_typed<M_UNIQ, uint64_t, uint64_t>(ctx, d_keys, d_keys_alt, (uint64_t *)d_vals, (uint64_t *)d_vals_alt,
                                                    8, n, key_bits, lo_bit, d_okeys, (uint64_t *)d_ovals, n_out);
}
