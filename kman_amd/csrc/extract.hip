// extract.hip — sliding-window k-mer enumeration on the GPU.
//
// Restates Sequence.yield_kmers (kmermaid/seq.py:285-328) over the cleaned
// codes written by kman_parse_fasta:
//   * every window [i, i+k) of a record is visited in order (seq.py:317);
//   * the window is skipped unless all k chars are in "ACGT" after upper()
//     (seq.py:313,318 -> om.check_ab; kmer.is_ab_checked, batcher.py:560);
//   * a kept window yields KMer(+) and, with -r, KMer(-) = mkrc(window) with
//     the same coordinates (seq.py:274-282), in that order.
// Keys are packed 2 bits/base MSB-first, so key order == Python str order of
// the upper-case window (A<C<G<T).  Output order == the reference's stream
// order (record, position, strand): tiles are compacted in order with a
// decoupled look-back over tile counts.
//
// Layout per tile: 256 threads x EI consecutive window starts (EI = 16, or 8
// with -r so a tile emits at most 4096 keys).  The tile's codes (+64 halo) are
// staged in LDS with 16-byte loads; each thread rolls its windows from LDS;
// keys are staged in LDS at their compacted tile offsets and written out
// coalesced.  The radix-digit histograms of every sort pass are accumulated in
// LDS across the tiles a persistent block processes and flushed once per
// block, so kman_sort needs no histogram pass over the keys.
//
// Algorithmic bytes: 1 B code read + 8 B key write (+ 4/8 B pos) per k-mer.
#include "common.h"
#include "kmer.h"

namespace {

constexpr int ET = 256;
constexpr int MAXPASS = 8;

struct Plan {
    int npass;
    uint8_t shift[MAXPASS];
    uint8_t bits[MAXPASS];
    uint32_t off[MAXPASS];  // kmer_hist: first counter of each pass's [seg][bin] table
};

struct NoPos {};

template <int EI, bool RC, int CANON, typename P>
__global__ __launch_bounds__(ET) void extract_kernel(const uint8_t *__restrict__ codes, uint64_t n_bases,
                                                     uint64_t n_tiles, int k, uint64_t *__restrict__ keys,
                                                     P *__restrict__ pos, uint64_t *__restrict__ status,
                                                     uint32_t *__restrict__ counter, uint32_t epoch,
                                                     uint32_t *__restrict__ err, uint64_t *__restrict__ hist,
                                                     Plan plan, uint64_t key_lo, uint64_t key_hi, uint64_t cap,
                                                     const uint8_t *__restrict__ pmap, uint32_t pshift,
                                                     uint32_t pval, const uint32_t *__restrict__ pcoarse,
                                                     uint32_t cshift, uint32_t cexact) {
    constexpr int TILE = ET * EI;
    constexpr int KPT = RC && !CANON ? 2 * EI : EI;  // keys per thread, max
    constexpr int MAXKEYS = ET * KPT;
    constexpr bool HAS_POS = !std::is_same<P, NoPos>::value;
    __shared__ __attribute__((aligned(16))) uint8_t scodes[TILE + 64];
    __shared__ __attribute__((aligned(16))) uint64_t skeys[MAXKEYS];
    __shared__ uint32_t lhist[MAXPASS][256];
    __shared__ uint32_t lds_scan[ET / 64];
    __shared__ uint64_t lds_base;
    __shared__ uint32_t lds_tile;

    const uint64_t mask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    if (hist) {
        for (int i = threadIdx.x; i < MAXPASS * 256; i += ET) (&lhist[0][0])[i] = 0;
    }
    // pmap (no hist then): the coarse bitmap of the map's marked prefixes
    // (top cshift..2k key bits, map_coarse) held in the histogram's LDS, so
    // most keys are rejected without reading the map in HBM; cexact: the
    // bitmap is the map itself
    const uint32_t *lbits = &lhist[0][0];
    if (pmap) {
        for (int i = threadIdx.x; i < MAXPASS * 256; i += ET) (&lhist[0][0])[i] = pcoarse[i];
        __syncthreads();
    }
    for (;;) {
        const int64_t tile = grab_tile(counter, &lds_tile);
        if ((uint64_t)tile >= n_tiles) break;
        const uint64_t tb = (uint64_t)tile * TILE;
        stage_codes<ET, EI>(codes, n_bases, tb, scodes);
        __syncthreads();
        uint64_t kf[EI], kr[EI];
        const uint64_t p0 = tb + (uint64_t)threadIdx.x * EI;
        const uint32_t valid = roll<EI, CANON>(scodes, threadIdx.x * EI, k, mask, p0, n_bases, kf, kr);
        // keys inside [key_lo, key_hi] only (kman_extract_range; the full range
        // otherwise), or with pmap[key >> pshift] == pval (kman_extract_marked)
        uint32_t vf = 0, vr = 0;
        if (pmap) {
#pragma unroll
            for (int j = 0; j < EI; j++) {
                if ((valid >> j) & 1u) {
                    const uint32_t cf = (uint32_t)(kf[j] >> cshift);
                    bool hf = (lbits[cf >> 5] >> (cf & 31u)) & 1u;
                    if (hf && !cexact) hf = pmap[kf[j] >> pshift] == pval;
                    vf |= (uint32_t)hf << j;
                    if (RC && !CANON) {
                        const uint32_t cr = (uint32_t)(kr[j] >> cshift);
                        bool hr = (lbits[cr >> 5] >> (cr & 31u)) & 1u;
                        if (hr && !cexact) hr = pmap[kr[j] >> pshift] == pval;
                        vr |= (uint32_t)hr << j;
                    }
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < EI; j++) {
                vf |= (uint32_t)(kf[j] >= key_lo && kf[j] <= key_hi) << j;
                if (RC && !CANON) vr |= (uint32_t)(kr[j] >= key_lo && kr[j] <= key_hi) << j;
            }
        }
        vf &= valid;
        vr &= valid;
        const uint32_t cnt = __popc(vf) + (RC && !CANON ? __popc(vr) : 0);
        uint32_t total;
        const uint32_t loff = block_exclusive_scan<ET>(cnt, SumU32(), 0u, lds_scan, &total);
#if defined(KMAN_ABL) && (KMAN_ABL & 32)
        // ablation build only: no look-back (wrong offsets, measures the rest)
        if (threadIdx.x == 0) {
            lds_base = tb;
            st_store(&status[tile], st_make(ST_INCL, epoch, tb + total));
        }
#else
        if (pmap) {
            // marked windows (a redo that sorts them next): places by one
            // atomic per tile that has any, no look-back chain through the
            // tiles that have none (`status` is the u64 cursor here)
            if (threadIdx.x == 0)
                lds_base = total ? (uint64_t)atomicAdd((unsigned long long *)status, (unsigned long long)total) : 0ull;
        } else if (threadIdx.x < 64) {
            const uint64_t b = wave_lookback<0>(status, tile, total, epoch, err);
            if (threadIdx.x == 0) lds_base = b;
        }
#endif
        // stage keys at compacted offsets
        {
            uint32_t o = loff;
#pragma unroll
            for (int j = 0; j < EI; j++) {
                if ((vf >> j) & 1u) skeys[o++] = kf[j];
                if (RC && !CANON && ((vr >> j) & 1u)) skeys[o++] = kr[j];
            }
        }
        __syncthreads();
        const uint64_t base = lds_base;
        for (uint32_t q = threadIdx.x; q < total; q += ET) {
            const uint64_t key = skeys[q];
            if (base + q < cap) keys[base + q] = key;  // (a key range past cap: counted, not written)
#if defined(KMAN_ABL) && (KMAN_ABL & 64)
            if (false) {
#else
            if (hist) {
#endif
                for (int p = 0; p < plan.npass; p++) {
                    const uint32_t d = (uint32_t)(key >> plan.shift[p]) & ((1u << plan.bits[p]) - 1);
                    atomicAdd(&lhist[p][d], 1u);
                }
            }
        }
        if constexpr (HAS_POS) {
            __syncthreads();
            P *spos = reinterpret_cast<P *>(skeys);
            uint32_t o = loff;
#pragma unroll
            for (int j = 0; j < EI; j++) {
                const P pv = (P)((p0 + j) << 1);
                if ((vf >> j) & 1u) spos[o++] = pv;
                if (RC && !CANON && ((vr >> j) & 1u)) spos[o++] = pv | 1;
            }
            __syncthreads();
            for (uint32_t q = threadIdx.x; q < total; q += ET)
                if (base + q < cap) pos[base + q] = spos[q];
        }
        __syncthreads();
    }
    if (hist) {
        __syncthreads();
        for (int p = 0; p < plan.npass; p++) {
            const uint32_t c = lhist[p][threadIdx.x];
            if (c) atomicAdd((unsigned long long *)&hist[p * 256 + threadIdx.x], (unsigned long long)c);
        }
    }
}

// kman_extract_marked's coarse bitmap: bit c (c < 2^cb, the top cb key bits)
// set when any map entry under prefix c holds val (map of mb key bits; for
// mb <= cb the entry above c); one thread per c, packed by ballots, every
// word written (bits past 2^cb zero)
__global__ __launch_bounds__(256) void map_coarse(const uint8_t *__restrict__ map, uint32_t mb, uint32_t val,
                                                  uint32_t cb, uint32_t *__restrict__ bits) {
    const uint32_t c = blockIdx.x * 256 + threadIdx.x;  // (65536 threads: 2^16 >= 2^cb)
    bool hit = false;
    if (c < (1u << cb)) {
        if (mb <= cb) {
            hit = map[c >> (cb - mb)] == val;
        } else {
            const uint32_t s = mb - cb;
            const uint8_t *e = map + ((uint64_t)c << s);
            for (uint32_t i = 0; i < (1u << s) && !hit; i++) hit = e[i] == val;
        }
    }
    const uint64_t m = __ballot(hit);
    const int lane = threadIdx.x & 63;
    if (lane < 2) bits[(c - lane) / 32 + lane] = (uint32_t)(m >> (32 * lane));
}

// valid-window count only (sizing)
template <int EI>
__global__ __launch_bounds__(ET) void count_kernel(const uint8_t *__restrict__ codes, uint64_t n_bases,
                                                   uint64_t n_tiles, int k, unsigned long long *__restrict__ out) {
    constexpr int TILE = ET * EI;
    __shared__ __attribute__((aligned(16))) uint8_t scodes[TILE + 64];
    __shared__ uint32_t lds_scan[ET / 64];
    const uint64_t mask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    uint64_t acc = 0;
    for (uint64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const uint64_t tb = tile * TILE;
        stage_codes<ET, EI>(codes, n_bases, tb, scodes);
        __syncthreads();
        uint64_t kf[EI], kr[EI];
        const uint64_t p0 = tb + (uint64_t)threadIdx.x * EI;
        acc += __popc(roll<EI, true>(scodes, threadIdx.x * EI, k, mask, p0, n_bases, kf, kr));
        __syncthreads();
    }
    uint32_t tot;
    block_exclusive_scan<ET>((uint32_t)acc, SumU32(), 0u, lds_scan, &tot);
    if (threadIdx.x == 0 && tot) atomicAdd(out, (unsigned long long)tot);
}

// valid-window count and the radix-digit histograms of every pass of `plan`,
// no keys written: the pre-pass of the fused extract + first sort pass
// (kman_extract_sorted needs the global digit-0 counts before any key moves)
#ifndef KMAN_KH_C
#define KMAN_KH_C 2
#endif
// Counters are spread over KH_C copies (lane & (KH_C - 1)) interleaved per bin,
// so same-digit lanes of one wave update different words.
constexpr int KH_C = KMAN_KH_C;

template <int EI, bool RC, int NP>
__global__ __launch_bounds__(ET) void kmer_hist_kernel(const uint8_t *__restrict__ codes, uint64_t n_bases,
                                                       uint64_t n_tiles, int k, unsigned long long *__restrict__ count,
                                                       unsigned long long *__restrict__ seg_hist, Plan plan,
                                                       uint32_t nseg, uint64_t seg_w) {
    constexpr int TILE = ET * EI;
    __shared__ __attribute__((aligned(16))) uint8_t scodes[TILE + 64];
    __shared__ uint32_t lds_scan[ET / 64];
    // counters [pass][seg][bin][copy]: pass p at plan.off[p]; segment of pass 0
    // = window range (seg_w windows), of pass p >= 1 = group of digit p - 1
    // ((d * nseg) >> bits): the input segments of the segmented passes
    extern __shared__ uint32_t lhist[];
    const uint32_t ncnt = plan.off[NP - 1] + ((nseg << plan.bits[NP - 1]) * KH_C);
    const uint64_t mask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    for (uint32_t i = threadIdx.x; i < ncnt; i += ET) lhist[i] = 0;
    const uint32_t copy = (uint32_t)lane_id() & (KH_C - 1);
    uint64_t acc = 0;
    // the next tile's codes are loaded into registers while this one counts
    CodeVecs<ET, EI> cv;
    if ((uint64_t)blockIdx.x < n_tiles) load_codes<ET, EI>(codes, n_bases, (uint64_t)blockIdx.x * TILE, cv);
    for (uint64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const uint64_t tb = tile * TILE;
        store_codes<ET, EI>(cv, codes, n_bases, tb, scodes);
        __syncthreads();
        if (tile + gridDim.x < n_tiles) load_codes<ET, EI>(codes, n_bases, (tile + gridDim.x) * TILE, cv);
        uint64_t kf[EI], kr[EI];
        const uint64_t p0 = tb + (uint64_t)threadIdx.x * EI;
        const uint32_t valid = roll<EI, false>(scodes, threadIdx.x * EI, k, mask, p0, n_bases, kf, kr);
        acc += __popc(valid) * (RC ? 2 : 1);
        // EI windows of a thread never straddle a window segment (seg_w % EI == 0)
        const uint32_t wseg = (uint32_t)(p0 / seg_w);
#if defined(KMAN_ABL) && (KMAN_ABL & 128)
        // ablation build only: no histogram atomics
        if (valid == 0x12345) acc += kf[3] ^ kr[5] ^ wseg;
        else continue;
#endif
#pragma unroll
        for (int j = 0; j < EI; j++) {
            if ((valid >> j) & 1u) {
                uint32_t sf = wseg, sr = wseg;
                // NP passes unrolled: the plan sits in scalar registers
#pragma unroll
                for (int p = 0; p < NP; p++) {
                    const uint32_t b = plan.bits[p], dm = (1u << b) - 1;
                    uint32_t *h = lhist + plan.off[p] + copy;
                    const uint32_t df = (uint32_t)(kf[j] >> plan.shift[p]) & dm;
                    atomicAdd(&h[((sf << b) | df) * KH_C], 1u);
                    sf = (df * nseg) >> b;
                    if (RC) {
                        const uint32_t dr = (uint32_t)(kr[j] >> plan.shift[p]) & dm;
                        atomicAdd(&h[((sr << b) | dr) * KH_C], 1u);
                        sr = (dr * nseg) >> b;
                    }
                }
            }
        }
        __syncthreads();
    }
    uint32_t tot;
    block_exclusive_scan<ET>((uint32_t)acc, SumU32(), 0u, lds_scan, &tot);
    if (threadIdx.x == 0 && tot) atomicAdd(count, (unsigned long long)tot);
    for (int p = 0; p < plan.npass; p++) {
        const uint32_t b = plan.bits[p];
        for (uint32_t i = threadIdx.x; i < (nseg << b); i += ET) {
            uint32_t c = 0;
#pragma unroll
            for (int cc = 0; cc < KH_C; cc++) c += lhist[plan.off[p] + i * KH_C + cc];
            // output [pass][seg][256]
            if (c) atomicAdd(&seg_hist[((uint64_t)p * nseg + (i >> b)) * 256 + (i & ((1u << b) - 1))],
                             (unsigned long long)c);
        }
    }
}

template <int EI, bool RC, int CANON, typename P>
int launch_extract(kman_ctx *ctx, const uint8_t *codes, uint64_t n_bases, int k, uint64_t *keys, P *pos,
                   uint64_t *hist, const Plan &plan, uint64_t klo, uint64_t khi, uint64_t cap, const uint8_t *pmap,
                   uint32_t pshift, uint32_t pval, uint32_t cshift, uint32_t cexact) {
    const uint64_t n_tiles = ceil_div(n_bases, (uint64_t)ET * EI);
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, n_tiles, &epoch, &counter));
    uint64_t *status = ctx->d_status;
    if (pmap) {  // (the marked windows' cursor: extract_filtered reads it back)
        void *scr;
        KMAN_TRY(kman_scratch(ctx, 256, &scr));
        HIP_TRY(ctx, hipMemsetAsync(scr, 0, 8, ctx->stream));
        status = (uint64_t *)scr;
    }
    auto fn = extract_kernel<EI, RC, CANON, P>;
    const int grid = kman_persistent_grid(ctx, (const void *)fn, ET, n_tiles);
    KTimer kt_(ctx, "extract");
    hipLaunchKernelGGL(fn, dim3(grid), dim3(ET), 0, ctx->stream, codes, n_bases, n_tiles, k, keys, pos, status,
                       counter, epoch, ctx->d_err, hist, plan, klo, khi, cap, pmap, pshift, pval, ctx->d_mapbits,
                       cshift, cexact);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}

template <typename P>
int dispatch_extract(kman_ctx *ctx, const uint8_t *codes, uint64_t n_bases, int k, uint32_t flags, uint64_t *keys,
                     P *pos, uint64_t *hist, const Plan &plan, uint64_t klo, uint64_t khi, uint64_t cap,
                     const uint8_t *pmap, uint32_t pshift, uint32_t pval, uint32_t cshift, uint32_t cexact) {
    if ((flags & KMAN_CANONICAL) && (flags & KMAN_MIXED))
        return launch_extract<16, false, 2, P>(ctx, codes, n_bases, k, keys, pos, hist, plan, klo, khi, cap, pmap,
                                               pshift, pval, cshift, cexact);
    if (flags & KMAN_CANONICAL)
        return launch_extract<16, false, 1, P>(ctx, codes, n_bases, k, keys, pos, hist, plan, klo, khi, cap, pmap,
                                               pshift, pval, cshift, cexact);
    if (flags & KMAN_RC)
        return launch_extract<8, true, 0, P>(ctx, codes, n_bases, k, keys, pos, hist, plan, klo, khi, cap, pmap,
                                                 pshift, pval, cshift, cexact);
    return launch_extract<16, false, 0, P>(ctx, codes, n_bases, k, keys, pos, hist, plan, klo, khi, cap, pmap,
                                               pshift, pval, cshift, cexact);
}

}  // namespace

extern "C" int kman_count_kmers(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                                uint64_t *n_kmers) {
    if (!ctx || !n_kmers) return KMAN_EINVAL;
    if (k < 2 || k > 32) return kman_fail(ctx, KMAN_EINVAL, "k must be in [2, 32] on the GPU path, got %u", k);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    *n_kmers = 0;
    if (n_bases == 0) return KMAN_OK;
    void *scr;
    KMAN_TRY(kman_scratch(ctx, 256, &scr));
    HIP_TRY(ctx, hipMemsetAsync(scr, 0, 8, ctx->stream));
    const uint64_t n_tiles = ceil_div(n_bases, (uint64_t)ET * 16);
    uint64_t grid = n_tiles < 4096 ? n_tiles : 4096;
    hipLaunchKernelGGL(count_kernel<16>, dim3((uint32_t)grid), dim3(ET), 0, ctx->stream, d_codes, n_bases, n_tiles,
                       (int)k, (unsigned long long *)scr);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_small, scr, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t w = ctx->h_small[0];
    *n_kmers = (flags & KMAN_RC) && !(flags & KMAN_CANONICAL) ? 2 * w : w;
    return KMAN_OK;
}

extern "C" int kman_extract(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                            uint64_t *d_keys, void *d_pos, uint32_t pos_bytes, uint64_t cap, uint64_t *d_hist,
                            uint64_t *n_kmers) {
    return kman_extract_range(ctx, d_codes, n_bases, k, flags, 0, ~0ull, d_keys, d_pos, pos_bytes, cap, d_hist,
                              n_kmers);
}

namespace {
int extract_filtered(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                     uint64_t key_lo, uint64_t key_hi, const uint8_t *pmap, uint32_t pshift, uint32_t pval,
                     uint64_t *d_keys, void *d_pos, uint32_t pos_bytes, uint64_t cap, uint64_t *d_hist,
                     uint64_t *n_kmers, uint32_t cshift = 0, uint32_t cexact = 0) {
    const bool ranged = key_lo != 0 || key_hi != ~0ull || pmap;
    if (!ctx || !n_kmers) return KMAN_EINVAL;
    if (k < 2 || k > 32) return kman_fail(ctx, KMAN_EINVAL, "k must be in [2, 32] on the GPU path, got %u", k);
    const bool want_pos = flags & KMAN_WANT_POS;
    if (want_pos && pos_bytes != 4 && pos_bytes != 8)
        return kman_fail(ctx, KMAN_EINVAL, "pos_bytes must be 4 or 8");
    if (want_pos && pos_bytes == 4 && (n_bases << 1) > 0xffffffffull)
        return kman_fail(ctx, KMAN_EINVAL, "u32 pos payload cannot address %llu bases", (unsigned long long)n_bases);
    if (((uintptr_t)d_codes & 15) != 0) return kman_fail(ctx, KMAN_EINVAL, "codes must be 16-byte aligned");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    *n_kmers = 0;
    if (n_bases == 0) return KMAN_OK;
    const uint64_t bound = (flags & KMAN_RC) && !(flags & KMAN_CANONICAL) ? 2 * n_bases : n_bases;
    if (cap < bound) {
        // only size exactly when the caller's buffer is below the trivial bound
        // (a key range is sized by the caller: kman_kmer_prefix_hist)
        uint64_t need;
        if (!ranged) {
            KMAN_TRY(kman_count_kmers(ctx, d_codes, n_bases, k, flags, &need));
            if (need > cap)
                return kman_fail(ctx, KMAN_ECAP, "key capacity %llu < %llu", (unsigned long long)cap,
                                 (unsigned long long)need);
        }
    }
    Plan plan{};
    uint32_t np, sh[MAXPASS], bi[MAXPASS];
    // histograms for the passes over bits [lo, 2k) (kman_split_bits), all
    // bits when the caller passes no KMAN_HIST_LO
    const uint32_t hist_lo = KMAN_HIST_LO_OF(flags);
    if (hist_lo > 2 * k) return kman_fail(ctx, KMAN_EINVAL, "histogram low bit %u > 2k", hist_lo);
    KMAN_TRY(kman_sort_plan_range(hist_lo, 2 * k, &np, sh, bi));
    plan.npass = (int)np;
    for (uint32_t i = 0; i < np; i++) {
        plan.shift[i] = (uint8_t)sh[i];
        plan.bits[i] = (uint8_t)bi[i];
    }
    if (!want_pos) {
        KMAN_TRY(dispatch_extract<NoPos>(ctx, d_codes, n_bases, (int)k, flags, d_keys, nullptr, d_hist, plan, key_lo,
                                         key_hi, cap, pmap, pshift, pval, cshift, cexact));
    } else if (pos_bytes == 4) {
        KMAN_TRY(dispatch_extract<uint32_t>(ctx, d_codes, n_bases, (int)k, flags, d_keys, (uint32_t *)d_pos, d_hist,
                                            plan, key_lo, key_hi, cap, pmap, pshift, pval, cshift, cexact));
    } else {
        KMAN_TRY(dispatch_extract<uint64_t>(ctx, d_codes, n_bases, (int)k, flags, d_keys, (uint64_t *)d_pos, d_hist,
                                            plan, key_lo, key_hi, cap, pmap, pshift, pval, cshift, cexact));
    }
    // the last tile's inclusive prefix is the number of k-mers written (a
    // marked extraction: its cursor)
    if (pmap) {
        void *scr;
        KMAN_TRY(kman_scratch(ctx, 256, &scr));
        HIP_TRY(ctx, hipMemcpyAsync(ctx->h_small, scr, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        *n_kmers = ctx->h_small[0];
    } else {
        const uint64_t n_tiles =
            ceil_div(n_bases, (uint64_t)ET * ((flags & KMAN_RC) && !(flags & KMAN_CANONICAL) ? 8 : 16));
        KMAN_TRY(kman_lookback_total(ctx, n_tiles, n_kmers));
    }
    if (*n_kmers > cap)
        return kman_fail(ctx, KMAN_ECAP, "key range holds %llu keys > capacity %llu", (unsigned long long)*n_kmers,
                         (unsigned long long)cap);
    return KMAN_OK;
}
}  // namespace

extern "C" int kman_extract_range(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                                  uint64_t key_lo, uint64_t key_hi, uint64_t *d_keys, void *d_pos, uint32_t pos_bytes,
                                  uint64_t cap, uint64_t *d_hist, uint64_t *n_kmers) {
    return extract_filtered(ctx, d_codes, n_bases, k, flags, key_lo, key_hi, nullptr, 0, 0, d_keys, d_pos, pos_bytes,
                            cap, d_hist, n_kmers);
}

extern "C" int kman_extract_marked(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k,
                                   uint32_t flags, const uint8_t *d_map, uint32_t map_bits, uint32_t map_val,
                                   uint64_t *d_keys, void *d_pos, uint32_t pos_bytes, uint64_t cap,
                                   uint64_t *n_kmers) {
    if (!ctx || !n_kmers) return KMAN_EINVAL;
    if (!d_map || map_bits == 0 || map_bits > 2 * k || map_bits > 30)
        return kman_fail(ctx, KMAN_EINVAL, "kman_extract_marked: map of %u key bits (k = %u)", map_bits, k);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->d_mapbits) HIP_TRY(ctx, hipMalloc(&ctx->d_mapbits, MAXPASS * 256 * sizeof(uint32_t)));
    // the coarse bitmap over the top CB key bits (exact when the map is no finer)
    const uint32_t cb = 2 * k < 16 ? 2 * k : 16;
    hipLaunchKernelGGL(map_coarse, dim3(256), dim3(256), 0, ctx->stream, d_map, map_bits, map_val, cb,
                       ctx->d_mapbits);
    HIP_TRY(ctx, hipGetLastError());
    return extract_filtered(ctx, d_codes, n_bases, k, flags, 0, ~0ull, d_map, 2 * k - map_bits, map_val, d_keys,
                            d_pos, pos_bytes, cap, nullptr, n_kmers, 2 * k - cb, map_bits <= cb ? 1u : 0u);
}

// top-8-bit histogram of the stream's keys (the k-mer count is its sum): the
// sizing of kman_extract_range's key ranges
extern "C" int kman_kmer_prefix_hist(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k,
                                     uint32_t flags, uint64_t *d_hist256, uint64_t *n_kmers) {
    if (!ctx || !n_kmers || !d_hist256) return KMAN_EINVAL;
    if (k < 2 || k > 32) return kman_fail(ctx, KMAN_EINVAL, "k must be in [2, 32] on the GPU path, got %u", k);
    if (flags & KMAN_CANONICAL) return kman_fail(ctx, KMAN_EINVAL, "prefix histogram of canonical keys: not built");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    *n_kmers = 0;
    if (n_bases == 0) {
        HIP_TRY(ctx, hipMemsetAsync(d_hist256, 0, 256 * 8, ctx->stream));
        return KMAN_OK;
    }
    const uint32_t lo = 2 * k > 8 ? 2 * k - 8 : 0;
    return kman_kmer_hist(ctx, d_codes, n_bases, k, flags & KMAN_RC, lo, 1, 1ull << 62, d_hist256, n_kmers);
}

// pre-pass of kman_extract_sorted: n_kmers and d_hist (zeroed here) for the
// passes over bits [lo_bit, 2k); flags: KMAN_RC only
int kman_kmer_hist(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                   uint32_t lo_bit, uint32_t nseg, uint64_t seg_w, uint64_t *d_seg, uint64_t *n_kmers) {
    Plan plan{};
    uint32_t np, sh[MAXPASS], bi[MAXPASS];
    KMAN_TRY(kman_sort_plan_range(lo_bit, 2 * k, &np, sh, bi));
    if (np == 0) return kman_fail(ctx, KMAN_EINVAL, "empty digit plan");
    if (nseg < 1 || seg_w == 0 || seg_w % 16) return kman_fail(ctx, KMAN_EINVAL, "bad segments %u / %llu", nseg,
                                                                (unsigned long long)seg_w);
    plan.npass = (int)np;
    uint32_t ncnt = 0;
    for (uint32_t i = 0; i < np; i++) {
        plan.shift[i] = (uint8_t)sh[i];
        plan.bits[i] = (uint8_t)bi[i];
        plan.off[i] = ncnt;
        ncnt += (nseg << bi[i]) * KH_C;
    }
    const size_t lds = (size_t)ncnt * 4;
    if (lds > 64 * 1024) return kman_fail(ctx, KMAN_EINVAL, "histogram tables need %zu B of LDS", lds);
    void *scr;
    KMAN_TRY(kman_scratch(ctx, 256, &scr));
    HIP_TRY(ctx, hipMemsetAsync(scr, 0, 8, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(d_seg, 0, (size_t)np * nseg * 256 * 8, ctx->stream));
    const bool rc = flags & KMAN_RC;
    const int EI = 16;
    const uint64_t n_tiles = ceil_div(n_bases, (uint64_t)ET * EI);
    if (np > 4) return kman_fail(ctx, KMAN_EINVAL, "histogram pre-pass plans at most 4 passes, got %u", np);
    using KFn = void (*)(const uint8_t *, uint64_t, uint64_t, int, unsigned long long *, unsigned long long *, Plan,
                         uint32_t, uint64_t);
    static const KFn fns[2][4] = {
        {kmer_hist_kernel<16, false, 1>, kmer_hist_kernel<16, false, 2>, kmer_hist_kernel<16, false, 3>,
         kmer_hist_kernel<16, false, 4>},
        {kmer_hist_kernel<16, true, 1>, kmer_hist_kernel<16, true, 2>, kmer_hist_kernel<16, true, 3>,
         kmer_hist_kernel<16, true, 4>}};
    const KFn fn = fns[rc ? 1 : 0][np - 1];
    const int grid = kman_persistent_grid(ctx, (const void *)fn, ET, n_tiles, lds);
    {
        KTimer kt_(ctx, "kmer_hist");
        hipLaunchKernelGGL(fn, dim3(grid), dim3(ET), lds, ctx->stream, d_codes, n_bases, n_tiles, (int)k,
                           (unsigned long long *)scr, (unsigned long long *)d_seg, plan, nseg, seg_w);
        HIP_TRY(ctx, hipGetLastError());
    }
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_small, scr, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *n_kmers = ctx->h_small[0];
    return KMAN_OK;
}

// diagnostic entry (not in kman.h): the histogram pre-pass alone, for timing
// (one segment; d_hist [pass][256])
extern "C" int kman_debug_kmer_hist(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k,
                                    uint32_t flags, uint32_t lo_bit, uint64_t *d_hist, uint64_t *n_kmers) {
    if (!ctx || !n_kmers) return KMAN_EINVAL;
    return kman_kmer_hist(ctx, d_codes, n_bases, k, flags, lo_bit, 1, 1ull << 62, d_hist, n_kmers);
}

// ===================================================================== k > 32
// Wide keys (k in 33..64; Sequence.yield_kmers has no k limit, seq.py:285-328):
// key = hi (the first k - 32 bases, 2(k-32) bits) : lo (the last 32 bases),
// MSB-first in each word, so (hi, lo) in lexicographic order == the
// reference's str order.  Tiles of ET x WEI windows rolled from LDS-staged
// codes (the 64-code halo covers k - 1 <= 63), compacted in stream order by a
// decoupled look-back; hi == nullptr counts only.
namespace {

constexpr int WEI = 8;

template <bool RC, bool CANON, typename P>
__global__ __launch_bounds__(ET) void extract_wide_kernel(const uint8_t *__restrict__ codes, uint64_t n_bases,
                                                          uint64_t n_tiles, int k, uint64_t *__restrict__ hi,
                                                          uint64_t *__restrict__ lo, P *__restrict__ pos,
                                                          uint64_t *__restrict__ status, uint32_t *__restrict__ counter,
                                                          uint32_t epoch, uint32_t *__restrict__ err, uint64_t cap) {
    constexpr int TILE = ET * WEI;
    constexpr bool HAS_POS = !std::is_same<P, NoPos>::value;
    __shared__ __attribute__((aligned(16))) uint8_t scodes[TILE + 64];
    __shared__ uint32_t lds_scan[ET / 64];
    __shared__ uint64_t lds_base;
    __shared__ uint32_t lds_tile;
    const int kh = k - 32;
    const uint64_t mh = kh >= 32 ? ~0ull : ((1ull << (2 * kh)) - 1);
    for (;;) {
        const int64_t tile = grab_tile(counter, &lds_tile);
        if ((uint64_t)tile >= n_tiles) break;
        const uint64_t tb = (uint64_t)tile * TILE;
        stage_codes<ET, WEI>(codes, n_bases, tb, scodes);
        __syncthreads();
        const int base = threadIdx.x * WEI;
        const uint64_t p0 = tb + (uint64_t)base;
        uint64_t fh = 0, fl = 0, rh = 0, rl = 0;
        uint32_t run = 0;
        auto push = [&](uint32_t c) {
            run = (c & 8) ? 0 : run;
            run = (c & 4) ? 0 : run + 1;
            fh = ((fh << 2) | (fl >> 62)) & mh;
            fl = (fl << 2) | (c & 3);
            rl = (rl >> 2) | (rh << 62);
            rh = (rh >> 2) | ((uint64_t)(3 - (c & 3)) << (2 * kh - 2));
        };
        for (int q = 0; q < k - 1; q++) push(scodes[base + q]);
        uint64_t oh[WEI][2], ol[WEI][2];
        uint32_t valid = 0;
#pragma unroll
        for (int j = 0; j < WEI; j++) {
            push(scodes[base + k - 1 + j]);
            const bool ok = run >= (uint32_t)k && p0 + j < n_bases;
            valid |= (uint32_t)ok << j;
            if (CANON) {
                const bool fwd = fh < rh || (fh == rh && fl <= rl);
                oh[j][0] = fwd ? fh : rh;
                ol[j][0] = fwd ? fl : rl;
            } else {
                oh[j][0] = fh;
                ol[j][0] = fl;
                oh[j][1] = rh;
                ol[j][1] = rl;
            }
        }
        constexpr uint32_t PER = RC && !CANON ? 2u : 1u;
        uint32_t total;
        const uint32_t off = block_exclusive_scan<ET>((uint32_t)__popc(valid) * PER, SumU32(), 0u, lds_scan, &total);
        if (threadIdx.x < 64) {
            const uint64_t b = wave_lookback<0>(status, tile, total, epoch, err);
            if (threadIdx.x == 0) lds_base = b;
        }
        __syncthreads();
        if (hi) {
            uint64_t o = lds_base + off;
#pragma unroll
            for (int j = 0; j < WEI; j++) {
                if (!((valid >> j) & 1u)) continue;
#pragma unroll
                for (uint32_t s = 0; s < PER; s++) {
                    if (o < cap) {
                        hi[o] = oh[j][s];
                        lo[o] = ol[j][s];
                        if constexpr (HAS_POS) pos[o] = (P)(((p0 + j) << 1) | s);
                    }
                    o++;
                }
            }
        }
        __syncthreads();
    }
}

template <bool RC, bool CANON, typename P>
int launch_wide(kman_ctx *ctx, const uint8_t *codes, uint64_t n_bases, int k, uint64_t *hi, uint64_t *lo, P *pos,
                uint64_t cap, uint64_t *n_out) {
    const uint64_t n_tiles = ceil_div(n_bases, (uint64_t)ET * WEI);
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, n_tiles, &epoch, &counter));
    auto fn = extract_wide_kernel<RC, CANON, P>;
    const int grid = kman_persistent_grid(ctx, (const void *)fn, ET, n_tiles);
    {
        KTimer kt_(ctx, "extract");
        hipLaunchKernelGGL(fn, dim3(grid), dim3(ET), 0, ctx->stream, codes, n_bases, n_tiles, k, hi, lo, pos,
                           ctx->d_status, counter, epoch, ctx->d_err, cap);
        HIP_TRY(ctx, hipGetLastError());
    }
    return kman_lookback_total(ctx, n_tiles, n_out);
}

template <typename P>
int dispatch_wide(kman_ctx *ctx, const uint8_t *codes, uint64_t n_bases, int k, uint32_t flags, uint64_t *hi,
                  uint64_t *lo, P *pos, uint64_t cap, uint64_t *n_out) {
    if (flags & KMAN_CANONICAL) return launch_wide<false, true, P>(ctx, codes, n_bases, k, hi, lo, pos, cap, n_out);
    if (flags & KMAN_RC) return launch_wide<true, false, P>(ctx, codes, n_bases, k, hi, lo, pos, cap, n_out);
    return launch_wide<false, false, P>(ctx, codes, n_bases, k, hi, lo, pos, cap, n_out);
}

}  // namespace

extern "C" int kman_extract_wide(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                                 uint64_t *d_hi, uint64_t *d_lo, void *d_pos, uint32_t pos_bytes, uint64_t cap,
                                 uint64_t *n_kmers) {
    if (!ctx || !n_kmers) return KMAN_EINVAL;
    if (k < 33 || k > 64) return kman_fail(ctx, KMAN_EINVAL, "kman_extract_wide: k must be in [33, 64], got %u", k);
    const bool want_pos = flags & KMAN_WANT_POS;
    if ((d_hi == nullptr) != (d_lo == nullptr)) return kman_fail(ctx, KMAN_EINVAL, "hi and lo go together");
    if (want_pos && d_hi && pos_bytes != 4 && pos_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "pos_bytes must be 4 or 8");
    if (want_pos && pos_bytes == 4 && (n_bases << 1) > 0xffffffffull)
        return kman_fail(ctx, KMAN_EINVAL, "u32 pos payload cannot address %llu bases", (unsigned long long)n_bases);
    if (((uintptr_t)d_codes & 15) != 0) return kman_fail(ctx, KMAN_EINVAL, "codes must be 16-byte aligned");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    *n_kmers = 0;
    if (n_bases == 0) return KMAN_OK;
    if (!want_pos || !d_hi)
        KMAN_TRY(dispatch_wide<NoPos>(ctx, d_codes, n_bases, (int)k, flags, d_hi, d_lo, nullptr, cap, n_kmers));
    else if (pos_bytes == 4)
        KMAN_TRY(dispatch_wide<uint32_t>(ctx, d_codes, n_bases, (int)k, flags, d_hi, d_lo, (uint32_t *)d_pos, cap,
                                         n_kmers));
    else
        KMAN_TRY(dispatch_wide<uint64_t>(ctx, d_codes, n_bases, (int)k, flags, d_hi, d_lo, (uint64_t *)d_pos, cap,
                                         n_kmers));
    if (d_hi && *n_kmers > cap)
        return kman_fail(ctx, KMAN_ECAP, "%llu k-mers > capacity %llu", (unsigned long long)*n_kmers,
                         (unsigned long long)cap);
    return KMAN_OK;
}
