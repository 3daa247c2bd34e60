// sort.hip — stable LSD radix sort of packed k-mer keys (+ optional payload).
//
// Replaces Batch.sorted (kmermaid/batch.py:156-168: a stable Timsort by .seq)
// as forced for every batch by BatcherBase.write_all (batcher.py:133-153,392).
// Stable because tied keys must keep stream order, exactly as Timsort keeps
// them (this is what makes `kmer batch` files and Crawler group member order
// match the reference).
//
// One "onesweep" pass per digit (Adinets & Merrill's single-pass LSD scheme,
// re-derived for wave64 / gfx950):
//   1. a tile of 4096 keys is read coalesced (wave-striped: item i of lane l of
//      wave w is key tile*4096 + w*1024 + i*64 + l);
//   2. each wave ranks its 16 items stably with 64-bit ballot match-any over
//      the digit bits and per-wave LDS counters (no LDS atomics);
//   3. the tile's per-digit counts are published and every digit looks back
//      across predecessor tiles (decoupled look-back, agent-scope sc1 status
//      words flag:2|epoch:6|count:56) for its exclusive global offset;
//   4. keys are scattered into LDS in tile-sorted order and written out so
//      consecutive lanes write consecutive addresses of one digit run.
// The digit histograms of all passes come from kman_extract (fused) or from
// one histogram pass, so a pass reads and writes every key exactly once:
// 16 B/key (+ 2x payload bytes) — the figure the roofline is quoted against.
#include "common.h"
#include "kmer.h"
#include "onesweep.h"

namespace {

constexpr int MAXPASS = 8;
struct NoVal {};

// A pass's input is cut into NSEG segments of contiguous tiles, each with its
// own look-back chain; tile ids are handed out round robin over the segments
// so the chains advance side by side.  A segment's bucket bases include the
// digit counts of the segments before it (known before the pass), so no chain
// ever waits on another.  With one chain, every tile in flight lies on it and
// the inclusive-prefix frontier (TPD x LB tiles per look-back round) bounds
// the pass.
constexpr int NSEG = 8;
struct SegDesc {
    uint64_t start, end;  // input range (keys; windows for the extraction pass)
    uint32_t tile0;       // status index of the segment's first tile
    uint32_t ntiles;
};

#if defined(KMAN_ABL) && (KMAN_ABL & 4)
// diagnostic build only: per-tile s_memrealtime stamps (100 MHz) at phase
// boundaries, thread 0, into a buffer set with kman_debug_set
__device__ uint64_t *g_dbg;
#define STAMP(i)                                                                         \
    do {                                                                                 \
        if (threadIdx.x == 0 && g_dbg) g_dbg[(uint64_t)tile * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define STAMP(i) \
    do {         \
    } while (0)
#endif

// one thread per digit walks back along that digit's tile chain, LB
// predecessors per round (independent sc1 loads in flight), summing AGG
// counts until it meets an INCL prefix
template <bool PUBLISHED>
KMAN_DEV uint64_t digit_lookback(uint64_t *st, int64_t tile, int64_t first, uint64_t agg, uint32_t epoch,
                                uint32_t *err) {
    if (tile == first) {
        if (!PUBLISHED) st_store(&st[(uint64_t)tile * RADIX], st_make(ST_INCL, epoch, agg));
        return 0;
    }
    if (!PUBLISHED) st_store(&st[(uint64_t)tile * RADIX], st_make(ST_AGG, epoch, agg));
    uint64_t excl = 0;
    int64_t j = tile - 1;
    uint32_t spins = 0;
    while (j >= first) {
        uint64_t w[LB];
#pragma unroll
        for (int q = 0; q < LB; q++)
            w[q] = (j - q >= first) ? st_load(&st[(uint64_t)(j - q) * RADIX]) : st_make(ST_INCL, epoch, 0);
        bool done = false, stall = false;
        int used = 0;
#pragma unroll
        for (int q = 0; q < LB; q++) {
            if (done || stall) continue;
            const uint64_t f = st_flag(w[q], epoch);
            if (f == 0) {
                stall = true;
                continue;
            }
            excl += w[q] & ST_VMASK;
            used++;
            if (f == ST_INCL) done = true;
        }
        if (done) break;
        j -= used;
        if (stall) {
            if (spin_give_up(spins, err, 2u)) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    st_store(&st[(uint64_t)tile * RADIX], st_make(ST_INCL, epoch, excl + agg));
    return excl;
}

// One LSD digit pass over a tile of NT*SI keys.  With LUT the digit is
// lut[key >> shift] (destination rank of a prefix range: kman_partition).
template <int NT, int SI, bool EARLY, typename V, bool LUT = false, bool ATOMIC = false, int MINW = 1>
__global__ __launch_bounds__(NT, MINW) void onesweep_pass(const uint64_t *__restrict__ kin, uint64_t *__restrict__ kout,
                                                    const V *__restrict__ vin, V *__restrict__ vout,
                                                    const SegDesc *__restrict__ segs, uint32_t nseg,
                                                    uint32_t shift, uint32_t bits,
                                                    const uint64_t *__restrict__ bucket_base,
                                                    uint64_t *__restrict__ status, uint32_t *__restrict__ counter,
                                                    uint32_t epoch, uint32_t *__restrict__ err,
                                                    const uint8_t *__restrict__ lut = nullptr) {
#define DIGIT(x) (LUT ? (uint32_t)lut[(x) >> shift] : ((uint32_t)((x) >> shift) & dmask))
    constexpr bool HAS_V = !std::is_same<V, NoVal>::value;
    constexpr int TILE = NT * SI;
    constexpr int NWAVE = NT / 64;
    static_assert(NT >= RADIX, "one thread per digit");
    __shared__ __attribute__((aligned(16))) uint64_t skeys[TILE];
    __shared__ uint32_t whist[NWAVE][RADIX];
    __shared__ uint32_t thist[RADIX];
    __shared__ uint32_t lstart[RADIX];
    __shared__ uint64_t gstart[RADIX];
    __shared__ uint32_t lds_scan[NT / 64];
    __shared__ uint32_t lds_tile;

    // round-robin over the segments: id c -> tile c / nseg of segment c % nseg
    const uint32_t cid = (uint32_t)grab_tile(counter, &lds_tile);
    const uint32_t sgi = cid % nseg, jj = cid / nseg;
    const SegDesc sd = segs[sgi];
    if (jj >= sd.ntiles) return;  // (block-uniform) past a shorter segment's end
    const int64_t tile = (int64_t)sd.tile0 + jj;  // status index
    const int64_t first = sd.tile0;
    const uint64_t n = sd.end;  // this segment's end bounds the tile
    const uint64_t *__restrict__ bb = bucket_base + (uint64_t)sgi * RADIX;
    STAMP(0);
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    const uint32_t radix = 1u << bits;
    const uint32_t dmask = radix - 1;
    for (int i = threadIdx.x; i < NWAVE * RADIX; i += NT) (&whist[0][0])[i] = 0;
    if (EARLY && threadIdx.x < RADIX) thist[threadIdx.x] = 0;

    const uint64_t tb = sd.start + (uint64_t)jj * TILE;
    const uint64_t ib = tb + (uint64_t)w * (SI * 64) + lane;
    uint64_t key[SI];
    uint32_t rank[SI];
#pragma unroll
    for (int i = 0; i < SI; i++) {
        const uint64_t idx = ib + (uint64_t)i * 64;
        key[i] = idx < n ? kin[idx] : 0;
    }
    // payloads are loaded up front too, so their latency hides under the ranking
    using VL = typename std::conditional<HAS_V, V, uint8_t>::type;
    VL val[HAS_V ? SI : 1];
    if constexpr (HAS_V) {
#pragma unroll
        for (int i = 0; i < SI; i++) {
            const uint64_t idx = ib + (uint64_t)i * 64;
            val[i] = idx < n ? vin[idx] : (V)0;
        }
    }
#if defined(KMAN_ABL) && (KMAN_ABL & 4)
    {
        uint64_t x = key[0] ^ key[SI - 1];
        asm volatile("" ::"v"(x));
    }
#endif
    __syncthreads();
    STAMP(1);
    if (ATOMIC) {
        // stable in-wave ranking with LDS atomics: one ds_add_rtn per item, all
        // in flight together; items in program order, same-address lanes in
        // lane order (probed per device at kman_create)
#pragma unroll
        for (int i = 0; i < SI; i++) {
            const bool valid = ib + (uint64_t)i * 64 < n;
            rank[i] = valid ? atomicAdd(&whist[w][DIGIT(key[i])], 1u) : 0u;
        }
        __syncthreads();
        if (EARLY && threadIdx.x < radix) {
            uint32_t c = 0;
#pragma unroll
            for (int ww = 0; ww < NWAVE; ww++) c += whist[ww][threadIdx.x];
            thist[threadIdx.x] = c;
            digit_publish(status + threadIdx.x, tile, first, c, epoch);
        }
    } else {
        if (EARLY) {
            // publish this tile's digit counts as soon as its keys have landed, so
            // successors' look-backs are not held up by the ranking below
#pragma unroll
            for (int i = 0; i < SI; i++)
                if (ib + (uint64_t)i * 64 < n) atomicAdd(&thist[DIGIT(key[i])], 1u);
            __syncthreads();
            if (threadIdx.x < radix) digit_publish(status + threadIdx.x, tile, first, thist[threadIdx.x], epoch);
        }

        // stable in-wave ranking: items in order, lanes in order (ballot match-any)
#pragma unroll
        for (int i = 0; i < SI; i++) {
            const bool valid = ib + (uint64_t)i * 64 < n;
            const uint32_t d = DIGIT(key[i]);
            uint64_t peers = __ballot(valid);
            for (uint32_t b = 0; b < bits; b++) {
                const bool set = (d >> b) & 1u;
                const uint64_t m = __ballot(set);
                peers &= set ? m : ~m;
            }
            uint32_t before = 0;
            if (valid) before = whist[w][d];
            rank[i] = before + (uint32_t)__popcll(peers & lanemask_lt());
            const int leader = __ffsll((unsigned long long)peers) - 1;
            if (valid && lane == leader) whist[w][d] = before + (uint32_t)__popcll(peers);
        }
    }
    __syncthreads();
    STAMP(2);

    // per-digit tile counts and per-wave exclusive offsets (thread = digit)
    const uint32_t d0 = threadIdx.x;
    uint32_t tot = 0;
    if (d0 < RADIX) {
#pragma unroll
        for (int ww = 0; ww < NWAVE; ww++) {
            const uint32_t c = whist[ww][d0];
            whist[ww][d0] = tot;
            tot += c;
        }
    }
    uint32_t tile_total;
    const uint32_t ls = block_exclusive_scan<NT>(tot, SumU32(), 0u, lds_scan, &tile_total);
    if (d0 < RADIX) lstart[d0] = ls;
    __syncthreads();
    // scatter into LDS in tile order: tile-local offsets only, so the LDS
    // stores are in flight while the look-back below waits on other tiles
    uint32_t lp[SI];
#pragma unroll
    for (int i = 0; i < SI; i++) {
        const bool valid = ib + (uint64_t)i * 64 < n;
        const uint32_t d = DIGIT(key[i]);
        lp[i] = valid ? lstart[d] + whist[w][d] + rank[i] : 0xffffffffu;
        if (valid) skeys[lp[i]] = key[i];
    }
#if defined(KMAN_ABL) && (KMAN_ABL & 1)
    // ablation build only: no look-back (wrong offsets, measures the rest)
    if (d0 < radix) gstart[d0] = bb[d0] + (uint64_t)jj * TILE / radix - ls;
#else
    if constexpr (EARLY) {
        // several lanes per digit walk the chain (see group_lookback)
        const uint32_t tpd = NT / radix >= 4 ? 4 : (NT / radix >= 2 ? 2 : 1);
        if (threadIdx.x < radix * tpd) {
            const uint32_t d = threadIdx.x / tpd;
            uint64_t excl;
            if (tpd == 4) excl = group_lookback<4>(status + d, tile, first, thist[d], epoch, err);
            else if (tpd == 2) excl = group_lookback<2>(status + d, tile, first, thist[d], epoch, err);
            else excl = group_lookback<1>(status + d, tile, first, thist[d], epoch, err);
            if (threadIdx.x % tpd == 0) gstart[d] = bb[d] + excl - lstart[d];
        }
    } else if (d0 < radix) {
        const uint64_t excl = digit_lookback<EARLY>(status + d0, tile, first, tot, epoch, err);
        gstart[d0] = bb[d0] + excl - ls;
    }
#endif
    __syncthreads();
    STAMP(3);
    const uint32_t cnt = (uint32_t)(n - tb < (uint64_t)TILE ? n - tb : (uint64_t)TILE);
    constexpr int RQ = (TILE + NT - 1) / NT;
    uint8_t dq[HAS_V ? RQ : 1];  // digits of the tile-ordered keys, for the payload
#pragma unroll
    for (int r = 0; r < RQ; r++) {
        const uint32_t q = threadIdx.x + r * NT;
        if (q < cnt) {
            const uint64_t kk = skeys[q];
            const uint32_t d = DIGIT(kk);
#if defined(KMAN_ABL) && (KMAN_ABL & 2)
            // ablation build only: contiguous writes instead of the digit scatter
            kout[tb + q] = kk + gstart[d];
#else
            kout[gstart[d] + q] = kk;
#endif
            if constexpr (HAS_V) dq[r] = (uint8_t)d;
        }
    }
    STAMP(4);
    if constexpr (HAS_V) {
        __syncthreads();
        V *sval = reinterpret_cast<V *>(skeys);
#pragma unroll
        for (int i = 0; i < SI; i++)
            if (lp[i] != 0xffffffffu) sval[lp[i]] = val[i];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RQ; r++) {
            const uint32_t q = threadIdx.x + r * NT;
            if (q < cnt) vout[gstart[dq[r]] + q] = sval[q];
        }
    }
    STAMP(5);
}


// ---------------------------------------------------------------------------
// Fused k-mer extraction + first prefix pass (kman_extract_sorted).
// A tile of NT*EI window starts is rolled into keys exactly like extract.hip
// (stream order: window, then '+' before '-' with -r), the valid keys are
// compacted into LDS in stream order with their tile-local (window << 1 |
// strand) packed above the 2k key bits, and the tile then runs the onesweep
// body on digit 0: stable rank, early digit counts, grouped look-back,
// LDS-staged coalesced scatter.  The keys never exist in stream order in HBM:
// 1 B code read + the pass's 8 B key + payload writes per k-mer.
constexpr int XT = 512;

template <int EI, bool RC, typename V, bool ATOMIC>
__global__ __launch_bounds__(XT) void extract_pass(const uint8_t *__restrict__ codes, uint64_t n_bases, int k,
                                                   uint64_t *__restrict__ kout, V *__restrict__ vout,
                                                   const SegDesc *__restrict__ segs, uint32_t nseg, uint32_t shift,
                                                   uint32_t bits, const uint64_t *__restrict__ bucket_base,
                                                   uint64_t *__restrict__ status, uint32_t *__restrict__ counter,
                                                   uint32_t epoch, uint32_t *__restrict__ err) {
    constexpr int NT = XT;
    constexpr int NWAVE = NT / 64;
    constexpr int WIN = NT * EI;          // window starts per tile
    constexpr int TILE = WIN * (RC ? 2 : 1);  // keys per tile, at most
    constexpr int SI = TILE / NT;
    constexpr bool HAS_V = !std::is_same<V, NoVal>::value;
    static_assert(WIN + 64 <= TILE * 8, "codes fit in the key staging area");
    __shared__ __attribute__((aligned(16))) uint64_t skeys[TILE];
    __shared__ uint32_t whist[NWAVE][RADIX];
    __shared__ uint32_t thist[RADIX];
    __shared__ uint32_t lstart[RADIX];
    __shared__ uint64_t gstart[RADIX];
    __shared__ uint32_t lds_scan[NWAVE];
    __shared__ uint32_t lds_tile;

    // round-robin over the window segments (see SegDesc)
    const uint32_t cid = (uint32_t)grab_tile(counter, &lds_tile);
    const uint32_t sgi = cid % nseg, jj = cid / nseg;
    const SegDesc sd = segs[sgi];
    if (jj >= sd.ntiles) return;
    const int64_t tile = (int64_t)sd.tile0 + jj;
    const int64_t first = sd.tile0;
    const uint64_t *__restrict__ bb = bucket_base + (uint64_t)sgi * RADIX;
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    const uint32_t radix = 1u << bits;
    const uint32_t dmask = radix - 1;
    const uint32_t kb = 2u * (uint32_t)k;
    const uint64_t keymask = kb >= 64 ? ~0ull : ((1ull << kb) - 1);
    const uint64_t wb = sd.start + (uint64_t)jj * WIN;
    // segments end on tile boundaries, except the last at n_bases
    uint8_t *scodes = reinterpret_cast<uint8_t *>(skeys);
    stage_codes<NT, EI>(codes, n_bases, wb, scodes);
    for (int i = threadIdx.x; i < NWAVE * RADIX; i += NT) (&whist[0][0])[i] = 0;
    if (threadIdx.x < RADIX) thist[threadIdx.x] = 0;
    __syncthreads();

    // roll this thread's EI windows; compact the valid keys in stream order
    uint64_t kf[EI], kr[EI];
    const uint32_t w0 = threadIdx.x * EI;
    const uint32_t valid = roll<EI, false>(scodes, w0, k, keymask, wb + w0, n_bases, kf, kr);
    uint32_t tcnt;
    const uint32_t off = block_exclusive_scan<NT>((uint32_t)__popc(valid) * (RC ? 2u : 1u), SumU32(), 0u, lds_scan,
                                                  &tcnt);
    {
        // (the scan's barriers ordered every read of the codes before this)
        uint32_t o = off;
#pragma unroll
        for (int j = 0; j < EI; j++) {
            if ((valid >> j) & 1u) {
                const uint64_t tag = (uint64_t)((w0 + j) << 1) << kb;
                skeys[o++] = kf[j] | tag;
                if (RC) skeys[o++] = kr[j] | tag | (1ull << kb);
            }
        }
    }
    __syncthreads();

    // ---- the onesweep body on digit 0 (items wave-striped, stream order)
    const uint32_t ib = (uint32_t)(w * (SI * 64) + lane);
    uint64_t key[SI];
    uint32_t rank[SI];
#pragma unroll
    for (int i = 0; i < SI; i++) key[i] = ib + i * 64 < tcnt ? skeys[ib + i * 64] : 0;
#define XDIGIT(x) ((uint32_t)((x) >> shift) & dmask)
    if (ATOMIC) {
#pragma unroll
        for (int i = 0; i < SI; i++) rank[i] = ib + i * 64 < tcnt ? atomicAdd(&whist[w][XDIGIT(key[i])], 1u) : 0u;
        __syncthreads();
        if (threadIdx.x < radix) {
            uint32_t c = 0;
#pragma unroll
            for (int ww = 0; ww < NWAVE; ww++) c += whist[ww][threadIdx.x];
            thist[threadIdx.x] = c;
            digit_publish(status + threadIdx.x, tile, first, c, epoch);
        }
    } else {
#pragma unroll
        for (int i = 0; i < SI; i++)
            if (ib + i * 64 < tcnt) atomicAdd(&thist[XDIGIT(key[i])], 1u);
        __syncthreads();
        if (threadIdx.x < radix) digit_publish(status + threadIdx.x, tile, first, thist[threadIdx.x], epoch);
#pragma unroll
        for (int i = 0; i < SI; i++) {
            const bool valid_i = ib + i * 64 < tcnt;
            const uint32_t d = XDIGIT(key[i]);
            uint64_t peers = __ballot(valid_i);
            for (uint32_t b = 0; b < bits; b++) {
                const bool set = (d >> b) & 1u;
                const uint64_t m = __ballot(set);
                peers &= set ? m : ~m;
            }
            uint32_t before = 0;
            if (valid_i) before = whist[w][d];
            rank[i] = before + (uint32_t)__popcll(peers & lanemask_lt());
            const int leader = __ffsll((unsigned long long)peers) - 1;
            if (valid_i && lane == leader) whist[w][d] = before + (uint32_t)__popcll(peers);
        }
    }
    __syncthreads();
    const uint32_t d0 = threadIdx.x;
    uint32_t tot = 0;
    if (d0 < RADIX) {
#pragma unroll
        for (int ww = 0; ww < NWAVE; ww++) {
            const uint32_t c = whist[ww][d0];
            whist[ww][d0] = tot;
            tot += c;
        }
    }
    const uint32_t ls = block_exclusive_scan<NT>(tot, SumU32(), 0u, lds_scan, (uint32_t *)nullptr);
    if (d0 < RADIX) lstart[d0] = ls;
    __syncthreads();
    // tile-order scatter into LDS first: in flight while the look-back waits
    uint32_t lp[SI];
#pragma unroll
    for (int i = 0; i < SI; i++) {
        const bool valid_i = ib + i * 64 < tcnt;
        const uint32_t d = XDIGIT(key[i]);
        lp[i] = valid_i ? lstart[d] + whist[w][d] + rank[i] : 0xffffffffu;
        if (valid_i) skeys[lp[i]] = key[i];
    }
    {
        const uint32_t tpd = NT / radix >= 4 ? 4 : (NT / radix >= 2 ? 2 : 1);
        if (threadIdx.x < radix * tpd) {
            const uint32_t d = threadIdx.x / tpd;
            uint64_t excl;
            if (tpd == 4) excl = group_lookback<4>(status + d, tile, first, thist[d], epoch, err);
            else if (tpd == 2) excl = group_lookback<2>(status + d, tile, first, thist[d], epoch, err);
            else excl = group_lookback<1>(status + d, tile, first, thist[d], epoch, err);
            if (threadIdx.x % tpd == 0) gstart[d] = bb[d] + excl - lstart[d];
        }
    }
    __syncthreads();
    constexpr int RQ = (TILE + NT - 1) / NT;
    uint8_t dq[HAS_V ? RQ : 1];
#pragma unroll
    for (int r = 0; r < RQ; r++) {
        const uint32_t q = threadIdx.x + r * NT;
        if (q < tcnt) {
            const uint64_t kk = skeys[q];
            const uint32_t d = XDIGIT(kk);
            kout[gstart[d] + q] = kk & keymask;
            if constexpr (HAS_V) dq[r] = (uint8_t)d;
        }
    }
    if constexpr (HAS_V) {
        __syncthreads();
        V *sval = reinterpret_cast<V *>(skeys);
#pragma unroll
        for (int i = 0; i < SI; i++) {
            if (lp[i] != 0xffffffffu) {
                const uint64_t f = key[i] >> kb;  // (window << 1 | strand)
                sval[lp[i]] = (V)(((wb + (f >> 1)) << 1) | (f & 1u));
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RQ; r++) {
            const uint32_t q = threadIdx.x + r * NT;
            if (q < tcnt) vout[gstart[dq[r]] + q] = sval[q];
        }
    }
#undef XDIGIT
}

// digit tables [pass][seg][256] of every pass: the segment of pass 0 is the
// position range (seg_len keys), of pass p >= 1 the group of digit p - 1
// ((d * nseg) >> bits, see SegDesc); counters in dynamic LDS at off[p]
struct HistPlan {
    uint32_t np, nseg;
    uint64_t seg_len;
    uint8_t shift[MAXPASS], bits[MAXPASS];
    uint32_t off[MAXPASS];
};

__global__ __launch_bounds__(256) void histogram_kernel(const uint64_t *__restrict__ keys, uint64_t n, HistPlan hp,
                                                        unsigned long long *__restrict__ hist) {
    extern __shared__ uint32_t lh[];
    const uint32_t ncnt = hp.off[hp.np - 1] + (hp.nseg << hp.bits[hp.np - 1]);
    for (uint32_t i = threadIdx.x; i < ncnt; i += 256) lh[i] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t k = keys[i];
        uint32_t sg = (uint32_t)(i / hp.seg_len);
        for (uint32_t p = 0; p < hp.np; p++) {
            const uint32_t b = hp.bits[p];
            const uint32_t d = (uint32_t)(k >> hp.shift[p]) & ((1u << b) - 1);
            atomicAdd(&lh[hp.off[p] + ((sg << b) | d)], 1u);
            sg = (d * hp.nseg) >> b;
        }
    }
    __syncthreads();
    for (uint32_t p = 0; p < hp.np; p++) {
        const uint32_t b = hp.bits[p];
        for (uint32_t i = threadIdx.x; i < (hp.nseg << b); i += 256) {
            const uint32_t c = lh[hp.off[p] + i];
            if (c) atomicAdd(&hist[((uint64_t)p * hp.nseg + (i >> b)) * RADIX + (i & ((1u << b) - 1))],
                             (unsigned long long)c);
        }
    }
}

// Segments of one pass over n keys in tiles of TILE: cut at `cut` (nseg + 1
// positions), bucket bases per segment from the global digit counts g and the
// segment tables t ([nseg][RADIX], null: one segment).  Checks every segment's
// table against its length.
int plan_pass(kman_ctx *ctx, uint64_t n, uint64_t tile, uint32_t nseg, const uint64_t *cut, const uint64_t *g,
              const uint64_t *t, SegDesc *segs, uint64_t *bases, uint32_t *tiles_total, uint32_t *max_tiles) {
    uint64_t run[RADIX];
    uint64_t acc = 0;
    for (int d = 0; d < RADIX; d++) {
        run[d] = acc;
        acc += g[d];
    }
    if (acc != n)
        return kman_fail(ctx, KMAN_EINVAL, "digit histogram sums to %llu, expected %llu", (unsigned long long)acc,
                         (unsigned long long)n);
    uint32_t t0 = 0, mx = 0;
    for (uint32_t sg = 0; sg < nseg; sg++) {
        const uint64_t len = cut[sg + 1] - cut[sg];
        if (t) {
            uint64_t sum = 0;
            for (int d = 0; d < RADIX; d++) sum += t[(uint64_t)sg * RADIX + d];
            if (sum != len)
                return kman_fail(ctx, KMAN_EINVAL, "segment %u table sums to %llu, length %llu", sg,
                                 (unsigned long long)sum, (unsigned long long)len);
        }
        for (int d = 0; d < RADIX; d++) {
            bases[(uint64_t)sg * RADIX + d] = run[d];
            run[d] += t ? t[(uint64_t)sg * RADIX + d] : g[d];
        }
        const uint32_t nt = (uint32_t)ceil_div(len, tile);
        segs[sg] = SegDesc{cut[sg], cut[sg + 1], t0, nt};
        t0 += nt;
        mx = nt > mx ? nt : mx;
    }
    *tiles_total = t0;
    *max_tiles = mx;
    return KMAN_OK;
}

// cut points of pass p's input: equal tile-aligned ranges (by_pos), or the
// groups of the previous pass's digit (global counts prev, bits pbits)
void pass_cuts(uint64_t n, uint64_t tile, uint32_t nseg, bool by_pos, const uint64_t *prev, uint32_t pbits,
               uint64_t *cut) {
    if (by_pos) {
        const uint64_t len = ceil_div(ceil_div(n, tile), nseg) * tile;
        for (uint32_t sg = 0; sg <= nseg; sg++) cut[sg] = sg * len < n ? sg * len : n;
        return;
    }
    const uint32_t r = 1u << pbits;
    uint64_t acc = 0;
    uint32_t d = 0;
    for (uint32_t sg = 0; sg <= nseg; sg++) {
        const uint32_t lim = (uint32_t)ceil_div((uint64_t)sg * r, nseg);  // first digit of group sg
        while (d < lim && d < r) acc += prev[d++];
        cut[sg] = sg == nseg ? n : acc;
    }
}

// The onesweep passes of a plan.  h_hist: global digit counts [pass][RADIX];
// h_seg: segment tables [pass][nseg][RADIX] (null: one chain per pass).  The
// first pass's input is cut by position (prev null) or by the groups of the
// previous pass's digit (prev: its global counts, pbits: its width).
template <int NT, int SI, bool EARLY, typename V, int MINW>
int run_passes(kman_ctx *ctx, uint64_t *k0, uint64_t *k1, V *v0, V *v1, uint64_t n, uint32_t np, const uint32_t *sh,
               const uint32_t *bi, const uint64_t *h_hist, const uint64_t *h_seg, uint32_t nseg, const uint64_t *prev,
               uint32_t pbits, int *result_in_alt) {
    constexpr uint64_t TILE = (uint64_t)NT * SI;
    if (!h_seg) nseg = 1;
    // per pass: the segment descriptors, then the bases [nseg][RADIX]
    constexpr size_t PER_PASS = NSEG * sizeof(SegDesc) + NSEG * RADIX * 8;
    static thread_local unsigned char tab[MAXPASS * PER_PASS];
    uint32_t tiles[MAXPASS], maxt[MAXPASS];
    bool skip[MAXPASS];
    for (uint32_t p = 0; p < np; p++) {
        const uint64_t *g = h_hist + (uint64_t)p * RADIX;
        skip[p] = false;
        for (int d = 0; d < RADIX; d++) skip[p] |= g[d] == n;
        uint64_t cut[NSEG + 1];
        if (nseg == 1) {
            cut[0] = 0;
            cut[1] = n;
        } else if (p == 0) {
            pass_cuts(n, TILE, nseg, prev == nullptr, prev, pbits, cut);
        } else {
            pass_cuts(n, TILE, nseg, false, h_hist + (uint64_t)(p - 1) * RADIX, bi[p - 1], cut);
        }
        SegDesc *segs = reinterpret_cast<SegDesc *>(tab + p * PER_PASS);
        uint64_t *bases = reinterpret_cast<uint64_t *>(tab + p * PER_PASS + NSEG * sizeof(SegDesc));
        KMAN_TRY(plan_pass(ctx, n, TILE, nseg, cut, g, h_seg ? h_seg + (uint64_t)p * nseg * RADIX : nullptr, segs,
                           bases, &tiles[p], &maxt[p]));
    }
    void *scr;
    KMAN_TRY(kman_scratch(ctx, np * PER_PASS, &scr));
    HIP_TRY(ctx, hipMemcpyAsync(scr, tab, np * PER_PASS, hipMemcpyHostToDevice, ctx->stream));
    int cur = 0;
    uint64_t *kb[2] = {k0, k1};
    V *vb[2] = {v0, v1};
    for (uint32_t p = 0; p < np; p++) {
        if (skip[p]) continue;
        const SegDesc *d_segs = reinterpret_cast<const SegDesc *>((const unsigned char *)scr + p * PER_PASS);
        const uint64_t *d_bases =
            reinterpret_cast<const uint64_t *>((const unsigned char *)scr + p * PER_PASS + NSEG * sizeof(SegDesc));
        uint32_t epoch, *counter;
        KMAN_TRY(kman_lookback_begin(ctx, (uint64_t)tiles[p] * RADIX, &epoch, &counter));
        const uint32_t grid = nseg * maxt[p];
        KTimer kt_(ctx, "sort_pass");
        if (ctx->lds_atomic_ordered)
            hipLaunchKernelGGL((onesweep_pass<NT, SI, EARLY, V, false, true, MINW>), dim3(grid), dim3(NT), 0,
                               ctx->stream, kb[cur], kb[cur ^ 1], vb[cur], vb[cur ^ 1], d_segs, nseg, sh[p], bi[p],
                               d_bases, ctx->d_status, counter, epoch, ctx->d_err, nullptr);
        else
            hipLaunchKernelGGL((onesweep_pass<NT, SI, EARLY, V, false, false, MINW>), dim3(grid), dim3(NT), 0,
                               ctx->stream, kb[cur], kb[cur ^ 1], vb[cur], vb[cur ^ 1], d_segs, nseg, sh[p], bi[p],
                               d_bases, ctx->d_status, counter, epoch, ctx->d_err, nullptr);
        HIP_TRY(ctx, hipGetLastError());
        cur ^= 1;
    }
    *result_in_alt = cur;
    return KMAN_OK;
}

template <int NT, int SI, bool EARLY = true, int MINW = 1>
int dispatch_vals(kman_ctx *ctx, uint64_t *k0, uint64_t *k1, void *v0, void *v1, uint32_t vb, uint64_t n, uint32_t np,
                  const uint32_t *sh, const uint32_t *bi, const uint64_t *h_hist, const uint64_t *h_seg, uint32_t nseg,
                  const uint64_t *prev, uint32_t pbits, int *res) {
    if (vb == 0)
        return run_passes<NT, SI, EARLY, NoVal, MINW>(ctx, k0, k1, nullptr, nullptr, n, np, sh, bi, h_hist, h_seg,
                                                      nseg, prev, pbits, res);
    if (vb == 4)
        return run_passes<NT, SI, EARLY, uint32_t, MINW>(ctx, k0, k1, (uint32_t *)v0, (uint32_t *)v1, n, np, sh, bi,
                                                         h_hist, h_seg, nseg, prev, pbits, res);
    return run_passes<NT, SI, EARLY, uint64_t, MINW>(ctx, k0, k1, (uint64_t *)v0, (uint64_t *)v1, n, np, sh, bi,
                                                     h_hist, h_seg, nseg, prev, pbits, res);
}

}  // namespace

#if defined(KMAN_ABL) && (KMAN_ABL & 4)
// diagnostic builds only (not part of include/kman.h)
extern "C" int kman_debug_set(kman_ctx *ctx, void *dptr) {
    HIP_TRY(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), &dptr, sizeof(dptr)));
    return KMAN_OK;
}
#endif

// as few passes of <= 8 bits as possible over bits [lo, hi), bits spread
// evenly (k=21 full sort: 6 x 7; the prefix [21, 42) of kman_split_bits: 3 x 7)
extern "C" int kman_sort_plan_range(uint32_t lo_bit, uint32_t hi_bit, uint32_t *npass, uint32_t *shift,
                                    uint32_t *bits) {
    if (!npass || !shift || !bits || hi_bit > 64 || lo_bit > hi_bit) return KMAN_EINVAL;
    const uint32_t nb = hi_bit - lo_bit;
    const uint32_t np = (nb + 7) / 8;
    uint32_t at = lo_bit;
    for (uint32_t p = 0; p < np; p++) {
        const uint32_t b = (hi_bit - at + (np - p) - 1) / (np - p);
        shift[p] = at;
        bits[p] = b;
        at += b;
    }
    *npass = np;
    return KMAN_OK;
}

extern "C" int kman_sort_plan(uint32_t key_bits, uint32_t *npass, uint32_t *shift, uint32_t *bits) {
    if (key_bits == 0) return KMAN_EINVAL;
    return kman_sort_plan_range(0, key_bits, npass, shift, bits);
}

extern "C" int kman_sort_range(kman_ctx *ctx, uint64_t *d_keys, uint64_t *d_keys_alt, void *d_vals,
                               void *d_vals_alt, uint32_t val_bytes, uint64_t n, uint32_t lo_bit, uint32_t hi_bit,
                               const uint64_t *d_hist, int *result_in_alt) {
    if (!ctx || !result_in_alt) return KMAN_EINVAL;
    if (val_bytes != 0 && val_bytes != 4 && val_bytes != 8)
        return kman_fail(ctx, KMAN_EINVAL, "val_bytes must be 0, 4 or 8");
    *result_in_alt = 0;
    if (n <= 1) return KMAN_OK;
    if (!d_keys || !d_keys_alt || (val_bytes && (!d_vals || !d_vals_alt)))
        return kman_fail(ctx, KMAN_EINVAL, "null buffer");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    uint32_t np, sh[MAXPASS], bi[MAXPASS];
    if (kman_sort_plan_range(lo_bit, hi_bit, &np, sh, bi) != KMAN_OK)
        return kman_fail(ctx, KMAN_EINVAL, "bad bit range [%u, %u)", lo_bit, hi_bit);
    if (np == 0) return KMAN_OK;
    // digit tables of every pass (device), then to the host for the bucket bases:
    // per segment when computed here, global only when the caller gives them
    constexpr uint64_t TILE = 512 * 16;
    uint32_t nseg = d_hist ? 1u : kman_seg_fit(np, bi, NSEG, 1, 48 * 1024);
    unsigned long long *hist = nullptr;
    void *scr = nullptr;
    const size_t hbytes = (size_t)np * nseg * RADIX * 8;
    // (in scratch, not aux: kman_finish holds its big-segment list in aux across
    // the nested full sort; run_passes reuses scratch only after the download)
    if (!d_hist) KMAN_TRY(kman_scratch(ctx, hbytes, (void **)&hist));
    static thread_local uint64_t h_hist[MAXPASS * RADIX];
    static thread_local uint64_t h_seg[MAXPASS * NSEG * RADIX];
    if (d_hist) {
        HIP_TRY(ctx, hipMemcpyAsync(h_hist, d_hist, np * RADIX * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    } else {
        HistPlan hp{};
        hp.np = np;
        hp.nseg = nseg;
        hp.seg_len = ceil_div(ceil_div(n, TILE), nseg) * TILE;
        uint32_t ncnt = 0;
        for (uint32_t p = 0; p < np; p++) {
            hp.shift[p] = (uint8_t)sh[p];
            hp.bits[p] = (uint8_t)bi[p];
            hp.off[p] = ncnt;
            ncnt += nseg << bi[p];
        }
        HIP_TRY(ctx, hipMemsetAsync(hist, 0, hbytes, ctx->stream));
        const uint64_t blocks = ceil_div(n, 256 * 16);
        KTimer kt_(ctx, "sort_hist");
        hipLaunchKernelGGL(histogram_kernel, dim3((uint32_t)(blocks < 2048 ? blocks : 2048)), dim3(256),
                           (size_t)ncnt * 4, ctx->stream, d_keys, n, hp, hist);
        HIP_TRY(ctx, hipGetLastError());
        HIP_TRY(ctx, hipMemcpyAsync(h_seg, hist, hbytes, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        for (uint32_t p = 0; p < np; p++)
            for (int d = 0; d < RADIX; d++) {
                uint64_t c = 0;
                for (uint32_t sg = 0; sg < nseg; sg++) c += h_seg[((uint64_t)p * nseg + sg) * RADIX + d];
                h_hist[p * RADIX + d] = c;
            }
    }
    (void)scr;
    const uint64_t *hs = d_hist ? nullptr : h_seg;
    static const int cfg = [] {
        const char *e = getenv("KMAN_SORT_CFG");  // tuning experiments only
        return e ? atoi(e) : 0;
    }();
    if (cfg) nseg = 1, hs = nullptr;  // (tile-size experiments: one chain, global bases)
#define KMAN_DV(NT_, SI_, ...)                                                                                     \
    KMAN_TRY((dispatch_vals<NT_, SI_, ##__VA_ARGS__>(ctx, d_keys, d_keys_alt, d_vals, d_vals_alt, val_bytes, n, np, \
                                                      sh, bi, h_hist, hs, nseg, nullptr, 0, result_in_alt)))
    switch (cfg) {
        case 1: KMAN_DV(512, 12); break;
        case 2: KMAN_DV(256, 24); break;
        case 3: KMAN_DV(1024, 8); break;
        case 4: KMAN_DV(256, 16); break;
        case 6: KMAN_DV(256, 16, false); break;
        case 7: KMAN_DV(512, 12, false); break;
        case 5: KMAN_DV(256, 8); break;
        default: KMAN_DV(512, 16); break;
    }
#undef KMAN_DV
    return kman_check_device_error(ctx);
}

extern "C" int kman_sort(kman_ctx *ctx, uint64_t *d_keys, uint64_t *d_keys_alt, void *d_vals, void *d_vals_alt,
                         uint32_t val_bytes, uint64_t n, uint32_t key_bits, const uint64_t *d_hist,
                         int *result_in_alt) {
    if (key_bits == 0 || key_bits > 64) return ctx ? kman_fail(ctx, KMAN_EINVAL, "key_bits must be 1..64") : KMAN_EINVAL;
    return kman_sort_range(ctx, d_keys, d_keys_alt, d_vals, d_vals_alt, val_bytes, n, 0, key_bits, d_hist,
                           result_in_alt);
}

namespace {
template <typename V>
int launch_partition(kman_ctx *ctx, const uint64_t *kin, uint64_t *kout, const V *vin, V *vout, uint64_t n,
                     const uint8_t *lut, uint32_t lut_shift, uint32_t bits, const uint64_t *d_base) {
    constexpr int NT = 512, SI = 12;
    const uint64_t n_tiles = ceil_div(n, (uint64_t)NT * SI);
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, n_tiles * RADIX, &epoch, &counter));
    // one chain: the segment descriptor rides behind the bases in scratch
    const SegDesc *d_seg = reinterpret_cast<const SegDesc *>(d_base + RADIX);
    KTimer kt_(ctx, "partition");
    if (ctx->lds_atomic_ordered)
        hipLaunchKernelGGL((onesweep_pass<NT, SI, true, V, true, true>), dim3((uint32_t)n_tiles), dim3(NT), 0,
                           ctx->stream, kin, kout, vin, vout, d_seg, 1u, lut_shift, bits, d_base, ctx->d_status,
                           counter, epoch, ctx->d_err, lut);
    else
        hipLaunchKernelGGL((onesweep_pass<NT, SI, true, V, true>), dim3((uint32_t)n_tiles), dim3(NT), 0, ctx->stream,
                           kin, kout, vin, vout, d_seg, 1u, lut_shift, bits, d_base, ctx->d_status, counter, epoch,
                           ctx->d_err, lut);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}
}  // namespace

extern "C" int kman_partition(kman_ctx *ctx, const uint64_t *d_keys, uint64_t *d_keys_out, const void *d_vals,
                              void *d_vals_out, uint32_t val_bytes, uint64_t n, const uint8_t *d_lut,
                              uint32_t lut_shift, uint32_t nbuckets, const uint64_t *bucket_counts) {
    if (!ctx || !bucket_counts || nbuckets < 1 || nbuckets > 256) return KMAN_EINVAL;
    if (val_bytes != 0 && val_bytes != 4 && val_bytes != 8)
        return kman_fail(ctx, KMAN_EINVAL, "val_bytes must be 0, 4 or 8");
    if (n == 0) return KMAN_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    uint64_t base[RADIX] = {0}, acc = 0;
    for (uint32_t b = 0; b < nbuckets; b++) {
        base[b] = acc;
        acc += bucket_counts[b];
    }
    if (acc != n)
        return kman_fail(ctx, KMAN_EINVAL, "bucket counts sum to %llu, expected %llu", (unsigned long long)acc,
                         (unsigned long long)n);
    uint32_t bits = 1;
    while ((1u << bits) < nbuckets) bits++;
    struct {
        uint64_t base[RADIX];
        SegDesc seg;
    } tab;
    memcpy(tab.base, base, sizeof(base));
    tab.seg = SegDesc{0, n, 0, (uint32_t)ceil_div(n, 512 * 12)};
    void *scr;
    KMAN_TRY(kman_scratch(ctx, sizeof(tab), &scr));
    HIP_TRY(ctx, hipMemcpyAsync(scr, &tab, sizeof(tab), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t *d_base = (const uint64_t *)scr;
    if (val_bytes == 0)
        KMAN_TRY(launch_partition<NoVal>(ctx, d_keys, d_keys_out, nullptr, nullptr, n, d_lut, lut_shift, bits, d_base));
    else if (val_bytes == 4)
        KMAN_TRY(launch_partition<uint32_t>(ctx, d_keys, d_keys_out, (const uint32_t *)d_vals, (uint32_t *)d_vals_out,
                                            n, d_lut, lut_shift, bits, d_base));
    else
        KMAN_TRY(launch_partition<uint64_t>(ctx, d_keys, d_keys_out, (const uint64_t *)d_vals, (uint64_t *)d_vals_out,
                                            n, d_lut, lut_shift, bits, d_base));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return kman_check_device_error(ctx);
}

namespace {
template <int EI, bool RC, typename V>
int launch_extract_pass(kman_ctx *ctx, const uint8_t *codes, uint64_t n_bases, uint32_t k, uint64_t *kout, V *vout,
                        uint32_t shift, uint32_t bits, const SegDesc *d_segs, uint32_t nseg, uint32_t n_tiles,
                        uint32_t max_tiles, const uint64_t *d_base) {
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, (uint64_t)n_tiles * RADIX, &epoch, &counter));
    KTimer kt_(ctx, "extract_pass");
    const uint32_t grid = nseg * max_tiles;
    if (ctx->lds_atomic_ordered)
        hipLaunchKernelGGL((extract_pass<EI, RC, V, true>), dim3(grid), dim3(XT), 0, ctx->stream, codes, n_bases,
                           (int)k, kout, vout, d_segs, nseg, shift, bits, d_base, ctx->d_status, counter, epoch,
                           ctx->d_err);
    else
        hipLaunchKernelGGL((extract_pass<EI, RC, V, false>), dim3(grid), dim3(XT), 0, ctx->stream, codes, n_bases,
                           (int)k, kout, vout, d_segs, nseg, shift, bits, d_base, ctx->d_status, counter, epoch,
                           ctx->d_err);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}
}  // namespace

extern "C" int kman_extract_sorted(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                                   uint32_t lo_bit, uint64_t *d_keys, uint64_t *d_keys_alt, void *d_pos,
                                   void *d_pos_alt, uint32_t pos_bytes, uint64_t cap, uint64_t *n_kmers,
                                   int *result_in_alt) {
    if (!ctx || !n_kmers || !result_in_alt) return KMAN_EINVAL;
    *n_kmers = 0;
    *result_in_alt = 0;
    if (k < 2 || k > 32) return kman_fail(ctx, KMAN_EINVAL, "k must be in [2, 32] on the GPU path, got %u", k);
    if (lo_bit > 2 * k) return kman_fail(ctx, KMAN_EINVAL, "low bit %u > 2k", lo_bit);
    const bool want_pos = flags & KMAN_WANT_POS;
    if (want_pos && pos_bytes != 4 && pos_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "pos_bytes must be 4 or 8");
    if (want_pos && pos_bytes == 4 && (n_bases << 1) > 0xffffffffull)
        return kman_fail(ctx, KMAN_EINVAL, "u32 pos payload cannot address %llu bases", (unsigned long long)n_bases);
    if (!d_keys || !d_keys_alt || (want_pos && (!d_pos || !d_pos_alt)))
        return kman_fail(ctx, KMAN_EINVAL, "null buffer");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (n_bases == 0) return KMAN_OK;
    const uint32_t vb = want_pos ? pos_bytes : 0;
    uint64_t *d_hist;
    KMAN_TRY(kman_aux(ctx, MAXPASS * RADIX * 8, (void **)&d_hist));
    // the fused path: forward / -r keys of k <= 25 (the tile-local window index
    // rides in the 14 bits above the key), u32 or no payload
    // (and at most 4 prefix passes: the histogram pre-pass's unrolled plans)
    uint32_t np0, sh0[MAXPASS], bi0[MAXPASS];
    KMAN_TRY(kman_sort_plan_range(lo_bit, 2 * k, &np0, sh0, bi0));
    const bool fused = !(flags & KMAN_CANONICAL) && k <= 25 && lo_bit < 2 * k && vb != 8 && np0 <= 4;
    if (!fused) {
        HIP_TRY(ctx, hipMemsetAsync(d_hist, 0, MAXPASS * RADIX * 8, ctx->stream));
        uint64_t n;
        KMAN_TRY(kman_extract(ctx, d_codes, n_bases, k, flags | KMAN_HIST_LO(lo_bit), d_keys, d_pos, pos_bytes, cap,
                              d_hist, &n));
        *n_kmers = n;
        return kman_sort_range(ctx, d_keys, d_keys_alt, d_pos, d_pos_alt, vb, n, lo_bit, 2 * k, d_hist,
                               result_in_alt);
    }
    const bool rc = flags & KMAN_RC;
    uint32_t np, sh[MAXPASS], bi[MAXPASS];
    KMAN_TRY(kman_sort_plan_range(lo_bit, 2 * k, &np, sh, bi));
    // window segments of the extraction pass: whole tiles, equal counts
    const uint64_t WIN = (uint64_t)XT * (rc ? 8 : 16);
    const uint32_t nseg = kman_seg_fit(np, bi, NSEG, 2, 48 * 1024);
    const uint64_t xtiles = ceil_div(n_bases, WIN);
    const uint64_t tps = ceil_div(xtiles, nseg);
    uint64_t *d_seg;
    KMAN_TRY(kman_aux(ctx, (size_t)np * nseg * RADIX * 8, (void **)&d_seg));
    uint64_t n;
    KMAN_TRY(kman_kmer_hist(ctx, d_codes, n_bases, k, rc ? KMAN_RC : 0u, lo_bit, nseg, tps * WIN, d_seg, &n));
    if (n > cap)
        return kman_fail(ctx, KMAN_ECAP, "key capacity %llu < %llu", (unsigned long long)cap, (unsigned long long)n);
    *n_kmers = n;
    if (n == 0) return KMAN_OK;
    static thread_local uint64_t h_seg[MAXPASS * NSEG * RADIX];
    static thread_local uint64_t h_hist[MAXPASS * RADIX];
    HIP_TRY(ctx, hipMemcpyAsync(h_seg, d_seg, (size_t)np * nseg * RADIX * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (uint32_t p = 0; p < np; p++)
        for (int d = 0; d < RADIX; d++) {
            uint64_t c = 0;
            for (uint32_t sg = 0; sg < nseg; sg++) c += h_seg[((uint64_t)p * nseg + sg) * RADIX + d];
            h_hist[p * RADIX + d] = c;
        }
    // pass 0 tables: segment descriptors over windows, bases per segment
    struct {
        SegDesc segs[NSEG];
        uint64_t base[NSEG][RADIX];
    } tab;
    {
        uint64_t run[RADIX], acc = 0;
        for (int d = 0; d < RADIX; d++) {
            run[d] = acc;
            acc += h_hist[d];
        }
        if (acc != n)
            return kman_fail(ctx, KMAN_EINVAL, "digit histogram sums to %llu, expected %llu", (unsigned long long)acc,
                             (unsigned long long)n);
        for (uint32_t sg = 0; sg < nseg; sg++) {
            for (int d = 0; d < RADIX; d++) {
                tab.base[sg][d] = run[d];
                run[d] += h_seg[(uint64_t)sg * RADIX + d];
            }
            const uint64_t t0 = sg * tps < xtiles ? sg * tps : xtiles;
            const uint64_t t1 = (sg + 1) * tps < xtiles ? (sg + 1) * tps : xtiles;
            tab.segs[sg] = SegDesc{t0 * WIN, t1 * WIN < n_bases ? t1 * WIN : n_bases, (uint32_t)t0,
                                   (uint32_t)(t1 - t0)};
        }
    }
    void *scr;
    KMAN_TRY(kman_scratch(ctx, sizeof(tab), &scr));
    HIP_TRY(ctx, hipMemcpyAsync(scr, &tab, sizeof(tab), hipMemcpyHostToDevice, ctx->stream));
    const SegDesc *d_segs = (const SegDesc *)scr;
    const uint64_t *d_base = (const uint64_t *)((const char *)scr + sizeof(tab.segs));
    const uint32_t nt = (uint32_t)xtiles, mt = (uint32_t)tps;
    if (rc) {
        if (vb) KMAN_TRY((launch_extract_pass<8, true, uint32_t>(ctx, d_codes, n_bases, k, d_keys, (uint32_t *)d_pos,
                                                                sh[0], bi[0], d_segs, nseg, nt, mt, d_base)));
        else KMAN_TRY((launch_extract_pass<8, true, NoVal>(ctx, d_codes, n_bases, k, d_keys, nullptr, sh[0], bi[0],
                                                           d_segs, nseg, nt, mt, d_base)));
    } else {
        if (vb) KMAN_TRY((launch_extract_pass<16, false, uint32_t>(ctx, d_codes, n_bases, k, d_keys,
                                                                  (uint32_t *)d_pos, sh[0], bi[0], d_segs, nseg, nt,
                                                                  mt, d_base)));
        else KMAN_TRY((launch_extract_pass<16, false, NoVal>(ctx, d_codes, n_bases, k, d_keys, nullptr, sh[0], bi[0],
                                                             d_segs, nseg, nt, mt, d_base)));
    }
    // the remaining prefix passes, ping-ponging from the pass-0 output; their
    // input segments are the groups of the previous digit
    if (np > 1) {
        KMAN_TRY((dispatch_vals<512, 16>(ctx, d_keys, d_keys_alt, d_pos, d_pos_alt, vb, n, np - 1, sh + 1, bi + 1,
                                         h_hist + RADIX, h_seg + (uint64_t)nseg * RADIX, nseg, h_hist, bi[0],
                                         result_in_alt)));
    }
    return kman_check_device_error(ctx);
}
