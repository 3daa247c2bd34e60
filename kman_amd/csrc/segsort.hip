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

constexpr int FT = 512;        // threads per chunk
constexpr int FW = FT / 64;    // waves
#ifndef KMAN_FC
#define KMAN_FC 5120
#define KMAN_FR 6144
#endif
constexpr int FC = KMAN_FC;    // chunk: segments that start here are owned
constexpr int FR = KMAN_FR;    // region capacity: chunk + tail of its last segment
constexpr int FI = FR / FT;    // items per thread
constexpr int FRADIX = 128;    // local LSD digit radix
constexpr int FBITS = 7;
constexpr int MAXSEG = 256;    // wave-per-segment path: segments per range
constexpr int WI = 12;         // ... and items per lane (segments <= 768 keys)

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

// One wave sorts segments sg0, sg0 + FW, ... < sg1 of the staged range by their
// low bits (stable LSD, 7-bit digits, the wave's own 128 counters).  Items travel
// packed: IT = u32 holds (low bits << 10 | offset in the segment) when the low
// bits fit in 22 (passes bounce through spk), IT = u64 holds (low bits << 13 |
// position) (passes bounce through skey).  The last pass writes the full key to
// skey and its original position to spk.
template <typename IT, bool ATOMIC>
KMAN_DEV void wave_sort_segments(uint64_t *skey, uint32_t *spk, uint32_t *wh, const uint32_t *segstart, uint32_t sg0,
                                 uint32_t sg1, uint32_t lo, uint32_t low_bits) {
    constexpr bool SMALL = sizeof(IT) == 4;
    constexpr uint32_t PS = SMALL ? 10 : 13;  // position bits
    const int lane = lane_id();
    const uint32_t npl = (low_bits + FBITS - 1) / FBITS;
    const uint64_t lmask = low_bits >= 64 ? ~0ull : ((1ull << low_bits) - 1);
    for (uint32_t sg = sg0; sg < sg1; sg += FW) {
        const uint32_t sa = lo + segstart[sg];
        const uint32_t sz = lo + segstart[sg + 1] - sa;
        if (sz < 2) continue;
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

enum { M_SORT = 0, M_COUNT = 1, M_UNIQ = 2 };

template <int MODE, typename V, typename O, bool ATOMIC>
__global__ __launch_bounds__(FT) void segfin_kernel(uint64_t *__restrict__ keys, V *__restrict__ vals, uint64_t n,
                                                    uint32_t lo_bit, const uint64_t *__restrict__ ov, uint32_t n_ov,
                                                    uint64_t *__restrict__ big, uint32_t *__restrict__ n_big,
                                                    uint32_t big_cap, uint64_t *__restrict__ okeys,
                                                    O *__restrict__ ovals, uint64_t *__restrict__ status,
                                                    uint32_t *__restrict__ counter, uint32_t epoch,
                                                    uint32_t *__restrict__ err) {
    constexpr bool HAS_V = !std::is_same<V, NoV>::value;
    __shared__ __attribute__((aligned(16))) uint64_t skey[FR];
    __shared__ uint32_t spk[FR];  // (segment index << 16) | position in the chunk
    __shared__ uint32_t whist[FW][FRADIX];
    __shared__ uint32_t lstart[FRADIX];
    __shared__ uint32_t lds_scan[FW];
    __shared__ uint64_t lds_scan64[FW];
    __shared__ uint32_t segstart[MAXSEG + 2];
    __shared__ uint32_t s_first, s_lastp1, s_end, s_tile, s_flags, s_maxseg;
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
        s_first = FC;
        s_lastp1 = 0;
        s_end = FR + 1;
        s_flags = 0;
        s_maxseg = 0;
    }
    for (uint32_t i = t; i < cnt; i += FT) skey[i] = keys[base + i];
    // the first FT keys past the chunk come with it: the last segment's tail
    // usually ends there (~half a segment), saving a dependent round trip
    if (cnt == (uint32_t)FC && base + FC + t < n) skey[FC + t] = keys[base + FC + t];
    const uint64_t prevk = base ? keys[base - 1] : 0;
    __syncthreads();

    // ---- segment starts in the chunk
    for (uint32_t i = t; i < cnt; i += FT) {
        const uint64_t pk = i ? skey[i - 1] : prevk;
        if (base + i == 0 || pre_of(skey[i], lo_bit) != pre_of(pk, lo_bit)) {
            atomicMin(&s_first, i);
            atomicMax(&s_lastp1, i + 1);
        }
    }
    __syncthreads();
    const uint32_t first = s_first;
    const bool has_start = first < (uint32_t)FC;
    const uint32_t last = s_lastp1 - 1;
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
    FSTAMP(1);

    // ---- end of the last owned segment (tail keys are staged behind the chunk)
    uint32_t hi = cnt;
    bool trail_pre = last_pre;  // the last segment is a presorted (or unstaged big) slice
    if (has_start && !last_pre && base + cnt < n) {
        const uint64_t lp = pre_of(skey[last], lo_bit);
        for (uint32_t r0 = FC; r0 < (uint32_t)FR; r0 += FT) {
            const uint32_t rel = r0 + t;
            const uint64_t g = base + rel;
            if (g < n) {
                uint64_t kk;
                if (r0 == (uint32_t)FC) {
                    kk = skey[rel];  // prefetched with the chunk
                } else {
                    kk = keys[g];
                    skey[rel] = kk;
                }
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
    const uint32_t lo = lead_pre ? 0u : (has_start ? first : cnt);
    if (!has_start && !lead_pre) hi = lo;
    const uint32_t m = hi - lo;
    const bool need_sort = has_start && m > 1;

    FSTAMP(2);
    // ---- stable LDS sort of [lo, hi): every owned segment by its low bits
    if (need_sort) {
        // segment index of every item (starts inside the range, in order)
        uint64_t key[FI];
        uint32_t pk[FI];
        uint32_t run = 0, stm = 0;
#pragma unroll
        for (int i = 0; i < FI; i++) {
            const uint32_t q = (uint32_t)(w * FI * 64 + i * 64 + lane);
            const bool valid = q < m;
            key[i] = valid ? skey[lo + q] : 0;
            const bool st = valid && q > 0 && pre_of(key[i], lo_bit) != pre_of(skey[lo + q - 1], lo_bit);
            stm |= (uint32_t)st << i;
            const uint64_t msk = __ballot(st);
            pk[i] = run + (uint32_t)__popcll(msk & (lanemask_lt() | (1ull << lane)));
            run += (uint32_t)__popcll(msk);
        }
        if (lane == 0) lds_scan[w] = run;
        __syncthreads();
        uint32_t woff = 0, nsegs = 0;
#pragma unroll
        for (int ww = 0; ww < FW; ww++) {
            const uint32_t c = lds_scan[ww];
            woff += ww < w ? c : 0;
            nsegs += c;
        }
        nsegs += 1;  // segment 0 starts at q = 0
        const uint32_t s0 = lead_pre ? 1u : 0u, s1 = nsegs - (trail_pre ? 1u : 0u);
        const uint32_t low_bits = lo_bit >= 64 ? 64u : lo_bit;
        bool wave_path = nsegs <= (uint32_t)MAXSEG && low_bits <= 51;
        if (wave_path) {
#pragma unroll
            for (int i = 0; i < FI; i++) {
                const uint32_t q = (uint32_t)(w * FI * 64 + i * 64 + lane);
                if (q == 0) segstart[0] = 0;
                else if ((stm >> i) & 1u) segstart[pk[i] + woff] = q;
            }
            if (t == 0) segstart[nsegs] = m;
            __syncthreads();
            if ((uint32_t)t + s0 < s1) {
                for (uint32_t sg = s0 + t; sg < s1; sg += FT) {
                    const uint32_t sz = segstart[sg + 1] - segstart[sg];
                    if (sz > (uint32_t)(WI * 64)) atomicMax(&s_maxseg, sz);
                }
            }
            // identity positions for the presorted slices and single-key segments
            // (the sorted segments write theirs in the last pass)
            for (uint32_t q = t; q < m; q += FT) spk[lo + q] = lo + q;
            __syncthreads();
            wave_path = s_maxseg == 0;
        }
#if defined(KMAN_ABL) && (KMAN_ABL & 16)
        if (t == 0) {
            atomicAdd(&g_fstat[wave_path ? 0 : 1], 1ull);
            atomicAdd(&g_fstat[2], (unsigned long long)nsegs);
            atomicAdd(&g_fstat[3], (unsigned long long)m);
        }
#endif
        if (wave_path) {
            // one wave per segment: stable LSD over the low bits with the
            // wave's own counters; no block barrier until every segment is done
#if defined(KMAN_ABL) && (KMAN_ABL & 8)
            // ablation build only: no segment sort (wrong order, measures the rest)
            if (false)
#endif
            {
                if (low_bits <= 22)
                    wave_sort_segments<uint32_t, ATOMIC>(skey, spk, whist[w], segstart, s0 + w, s1, lo, low_bits);
                else
                    wave_sort_segments<uint64_t, ATOMIC>(skey, spk, whist[w], segstart, s0 + w, s1, lo, low_bits);
            }
            __syncthreads();
        } else {
            // many or long segments: block-wide LSD on (segment index, low bits)
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
        if constexpr (HAS_V && sizeof(V) == 4) {
            // u32 payload: read the range coalesced into LDS (over spk, once every
            // sorted position has been read), then permute it from there
            uint32_t ixr[FI];
            V vl[FI];
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                ixr[r] = q < m ? (spk[lo + q] & 0xffffu) - lo : 0;
                vl[r] = q < m ? vals[base + lo + q] : (V)0;
            }
            __syncthreads();
            V *sv = reinterpret_cast<V *>(spk);
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                if (q < m) sv[q] = vl[r];
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                if (q < m) vals[base + lo + q] = sv[ixr[r]];
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
        const uint64_t next_g = has_next_g ? keys[base + hi] : 0;
        uint64_t k[FI];
        uint32_t ix[FI];  // UNIQ: each item's position in the range, for its payload
        const uint32_t q0 = (uint32_t)t * FI;
#pragma unroll
        for (int j = 0; j < FI; j++) {
            k[j] = q0 + j < m ? skey[lo + q0 + j] : 0;
            ix[j] = (MODE == M_UNIQ && q0 + j < m) ? (spk[lo + q0 + j] & 0xffffu) - lo : 0;
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
        constexpr bool LDS_V = MODE == M_UNIQ && sizeof(V) == 4;
        V vl[LDS_V ? FI : 1];
        if constexpr (LDS_V) {
            // the range's payload, coalesced; in flight during the look-back
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                vl[r] = q < m ? vals[base + lo + q] : (V)0;
            }
        }
        if (w == 0) {
            const uint64_t b = wave_lookback<0>(status, tile, total, epoch, err);
            if (lane == 0) s_out = b;
        }
        O ov_[FI];
        if constexpr (MODE == M_UNIQ && !LDS_V) {
#pragma unroll
            for (int j = 0; j < FI; j++)
                ov_[j] = ((emit >> j) & 1u) ? (O)vals[base + lo + ix[j]] : (O)0;
        } else if constexpr (MODE == M_COUNT) {
#pragma unroll
            for (int j = 0; j < FI; j++) ov_[j] = (O)cval[j];
        }
        if constexpr (LDS_V) {
            V *sv = reinterpret_cast<V *>(spk);
#pragma unroll
            for (int r = 0; r < FI; r++) {
                const uint32_t q = t + r * FT;
                if (q < m) sv[q] = vl[r];
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
            const V *sv = reinterpret_cast<const V *>(spk);
#pragma unroll
            for (int j = 0; j < FI; j++) ov_[j] = ((emit >> j) & 1u) ? (O)sv[ix[j]] : (O)0;
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
