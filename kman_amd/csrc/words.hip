// words.hip — k-mers of any length k >= 2 as W = ceil(k / 32) 64-bit words.
//
// The reference has no k limit (Sequence.yield_kmers, kmermaid/seq.py:285-328;
// FastaBatcher.do only asserts k > 1, batcher.py:477-478) and compares k-mers
// as Python strings (Batch.sorted, batch.py:156-168; Crawler's heap merge,
// join.py:63-93).  A k-mer is stored MSB-first over W words: word 0 holds the
// first h = k - 32 (W - 1) bases in its low 2h bits, words 1 .. W-1 hold 32
// bases each, so the lexicographic order of (w_0, .., w_{W-1}) is the string
// order (A < C < G < T).  Word-major planes: word j of item i at
// words[j * stride + i].  For W = 2 this is the (hi, lo) pair of
// kman_extract_wide.
//
//   kman_extract_words   valid windows in stream order (records in file
//                        order, positions ascending, + then - with -r; one
//                        canonical key per window with KMAN_CANONICAL) ->
//                        words + pos ((global base << 1) | strand); two
//                        launches: per-tile counts, then (host scan of the
//                        tile counts) the writes at their offsets
//   kman_rle_words       run-length of sorted word keys: (key, group size) or
//                        the keys of groups of one with their payload
//                        (Crawler.do_batch + join_sequence_count /
//                        join_unique, join.py:95-130, 244-285)
//   kman_batch_tags      batch index of every item of a permutation (the
//                        per-batch sort of `kmer batch` / Batch.sorted)
//
// The sort itself is LSD over the planes by stable kman_sort passes with an
// index payload (kman_amd/engine.py sort_words).  Not the hot path: the
// region kernels serve k <= 32; this serves every k the reference accepts.
#include "common.h"

#include <vector>

namespace {

constexpr int XT = 256;  // threads per tile
constexpr int XE = 8;    // window starts per thread
constexpr uint64_t XTILE = (uint64_t)XT * XE;

// the windows of [s0, s0 + XE) that are valid: every code ACGT (bit 2 clear),
// no record start (bit 3) after the window's first base, inside the codes.
// A window is scanned from its end; a breaker found at q rules out every
// window of the run that holds it, and after a valid window only the one new
// base of the next needs a look, so a thread reads about k + XE codes.
KMAN_DEV uint32_t valid_windows(const uint8_t *__restrict__ codes, uint64_t n_bases, uint64_t s0, uint32_t k) {
    uint32_t ok = 0;
    uint32_t j = 0;
    bool prev = false;  // window s0 + j - 1 was valid
    while (j < (uint32_t)XE) {
        const uint64_t s = s0 + j;
        if (s + k > n_bases) break;  // (and every later window)
        uint64_t q = s + k;
        bool broke = false;
        if (prev) {
            // [s, s + k - 1) was inside the previous window: clean, and no
            // record start after s; only the new base s + k - 1 is unseen
            q = s + k - 1;
            const uint32_t c = codes[q];
            broke = (c & 4) || (c & 8);
        } else {
            while (q > s) {
                --q;
                const uint32_t c = codes[q];
                if ((c & 4) || (q > s && (c & 8))) {
                    broke = true;
                    break;
                }
            }
        }
        if (!broke) {
            ok |= 1u << j;
            j++;
            prev = true;
        } else {
            // a code that is not ACGT at q breaks the windows that start at
            // or before q; a record start at q breaks those before q
            const uint32_t c = codes[q];
            const uint64_t next = (c & 4) ? q + 1 : q;
            j = (uint32_t)(next - s0 < (uint64_t)XE ? next - s0 : (uint64_t)XE);
            prev = false;
        }
    }
    return ok;
}

// forward word j of the window at s (MSB-first)
KMAN_DEV uint64_t fwd_word(const uint8_t *__restrict__ codes, uint64_t s, uint32_t k, uint32_t W, uint32_t j) {
    const uint32_t h = k - 32 * (W - 1);
    const uint64_t a = j == 0 ? s : s + h + 32ull * (j - 1);
    const uint32_t len = j == 0 ? h : 32;
    uint64_t w = 0;
    for (uint32_t t = 0; t < len; t++) w = (w << 2) | (codes[a + t] & 3u);
    return w;
}

// word j of the reverse complement R of the window at s: R[a:b] is the
// reverse complement of the forward bases [k - b, k - a)
KMAN_DEV uint64_t rc_word(const uint8_t *__restrict__ codes, uint64_t s, uint32_t k, uint32_t W, uint32_t j) {
    const uint32_t h = k - 32 * (W - 1);
    const uint32_t ra = j == 0 ? 0 : h + 32 * (j - 1);
    const uint32_t len = j == 0 ? h : 32;
    const uint64_t fb = s + k - ra;  // one past the forward segment's last base
    uint64_t w = 0;
    for (uint32_t t = 1; t <= len; t++) w = (w << 2) | (3u - (codes[fb - t] & 3u));
    return w;
}

// -1 / 0 / 1: forward vs reverse complement, lexicographic over the words
KMAN_DEV int cmp_fwd_rc(const uint8_t *__restrict__ codes, uint64_t s, uint32_t k, uint32_t W) {
    for (uint32_t j = 0; j < W; j++) {
        const uint64_t f = fwd_word(codes, s, k, W, j), r = rc_word(codes, s, k, W, j);
        if (f != r) return f < r ? -1 : 1;
    }
    return 0;
}

// items per window: 1, 2 with -r (not canonical)
template <bool WRITE>
__global__ __launch_bounds__(XT) void words_kernel(const uint8_t *__restrict__ codes, uint64_t n_bases, uint32_t k,
                                                   uint32_t W, uint32_t flags, const uint64_t *__restrict__ tile_off,
                                                   uint32_t *__restrict__ tile_cnt, uint64_t *__restrict__ words,
                                                   uint64_t stride, void *__restrict__ pos, uint32_t pos_bytes,
                                                   uint64_t cap) {
    __shared__ uint32_t lds_scan[XT / 64];
    const uint64_t tile = blockIdx.x;
    const uint64_t s0 = tile * XTILE + (uint64_t)threadIdx.x * XE;
    const bool canon = flags & KMAN_CANONICAL;
    const bool rc = (flags & KMAN_RC) && !canon;
    const uint32_t ok = s0 < n_bases ? valid_windows(codes, n_bases, s0, k) : 0u;
    const uint32_t mine = (uint32_t)__popc(ok) * (rc ? 2u : 1u);
    uint32_t total;
    const uint32_t off = block_exclusive_scan<XT>(mine, SumU32(), 0u, lds_scan, &total);
    if (!WRITE) {
        if (threadIdx.x == 0) tile_cnt[tile] = total;
        return;
    }
    uint64_t o = tile_off[tile] + off;
    for (uint32_t j = 0; j < (uint32_t)XE; j++) {
        if (!((ok >> j) & 1u)) continue;
        const uint64_t s = s0 + j;
        for (uint32_t strand = 0; strand < (rc ? 2u : 1u); strand++, o++) {
            if (o >= cap) continue;
            bool minus = strand == 1;
            if (canon) minus = cmp_fwd_rc(codes, s, k, W) > 0;
            if (words)
                for (uint32_t w = 0; w < W; w++)
                    words[w * stride + o] = minus ? rc_word(codes, s, k, W, w) : fwd_word(codes, s, k, W, w);
            if (pos) {
                // (canonical keys carry the + pos: one key per window, as count -r's x <= rc(x) rows)
                const uint64_t v = (s << 1) | (uint64_t)(strand == 1);
                if (pos_bytes == 4) ((uint32_t *)pos)[o] = (uint32_t)v;
                else ((uint64_t *)pos)[o] = v;
            }
        }
    }
}

// ---------------------------------------------------------------- run-length
constexpr int RT_ = 256;
constexpr int RE = 8;  // items per thread
constexpr uint64_t RTILE = (uint64_t)RT_ * RE;

KMAN_DEV bool same_key(const uint64_t *__restrict__ w, uint64_t stride, uint32_t W, uint64_t a, uint64_t b) {
    for (uint32_t j = 0; j < W; j++)
        if (w[j * stride + a] != w[j * stride + b]) return false;
    return true;
}

// mode 1 (count): emit every group head; mode 2 (uniq): groups of one.
// WRITE: the emitted keys (+ the uniq payload, or the head index for the
// count pass that follows)
template <bool WRITE>
__global__ __launch_bounds__(RT_) void rle_words_kernel(const uint64_t *__restrict__ w, uint32_t W, uint64_t stride,
                                                        uint64_t n, int mode, const uint64_t *__restrict__ tile_off,
                                                        uint32_t *__restrict__ tile_cnt, uint64_t *__restrict__ ow,
                                                        uint64_t ostride, const void *__restrict__ vals, uint32_t vb,
                                                        void *__restrict__ ovals, uint32_t ovb,
                                                        uint64_t *__restrict__ heads) {
    __shared__ uint32_t lds_scan[RT_ / 64];
    const uint64_t tile = blockIdx.x;
    const uint64_t i0 = tile * RTILE + (uint64_t)threadIdx.x * RE;
    uint32_t emit = 0;
    for (uint32_t j = 0; j < (uint32_t)RE; j++) {
        const uint64_t i = i0 + j;
        if (i >= n) break;
        const bool h = i == 0 || !same_key(w, stride, W, i, i - 1);
        bool e = h;
        if (mode == KMAN_FINISH_UNIQ) e = h && (i + 1 == n || !same_key(w, stride, W, i, i + 1));
        emit |= (uint32_t)e << j;
    }
    uint32_t total;
    const uint32_t off = block_exclusive_scan<RT_>((uint32_t)__popc(emit), SumU32(), 0u, lds_scan, &total);
    if (!WRITE) {
        if (threadIdx.x == 0) tile_cnt[tile] = total;
        return;
    }
    uint64_t o = tile_off[tile] + off;
    for (uint32_t j = 0; j < (uint32_t)RE; j++) {
        if (!((emit >> j) & 1u)) continue;
        const uint64_t i = i0 + j;
        for (uint32_t q = 0; q < W; q++) ow[q * ostride + o] = w[q * stride + i];
        if (mode == KMAN_FINISH_UNIQ) {
            const uint64_t v = vb == 4 ? ((const uint32_t *)vals)[i] : ((const uint64_t *)vals)[i];
            if (ovb == 4) ((uint32_t *)ovals)[o] = (uint32_t)v;
            else ((uint64_t *)ovals)[o] = v;
        } else {
            heads[o] = i;
        }
        o++;
    }
}

// count rows: group size = next head - this head
__global__ __launch_bounds__(256) void group_sizes_kernel(const uint64_t *__restrict__ heads, uint64_t m, uint64_t n,
                                                          void *__restrict__ ovals, uint32_t ovb) {
    const uint64_t o = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= m) return;
    const uint64_t c = (o + 1 < m ? heads[o + 1] : n) - heads[o];
    if (ovb == 4) ((uint32_t *)ovals)[o] = (uint32_t)c;
    else ((uint64_t *)ovals)[o] = c;
}

__global__ __launch_bounds__(256) void batch_tags_kernel(const uint64_t *__restrict__ perm, uint64_t n, uint64_t start,
                                                         uint64_t per_batch, uint64_t *__restrict__ tags) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) tags[i] = (start + perm[i]) / per_batch;
}

// tile counts -> exclusive offsets (host scan: one u32 per 2048 items), total
int scan_tiles(kman_ctx *ctx, const uint32_t *d_cnt, uint64_t tiles, uint64_t *d_off, uint64_t *total) {
    std::vector<uint32_t> c(tiles);
    std::vector<uint64_t> o(tiles);
    HIP_TRY(ctx, hipMemcpyAsync(c.data(), d_cnt, tiles * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t at = 0;
    for (uint64_t t = 0; t < tiles; t++) {
        o[t] = at;
        at += c[t];
    }
    HIP_TRY(ctx, hipMemcpyAsync(d_off, o.data(), tiles * 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // (o leaves scope)
    *total = at;
    return KMAN_OK;
}

}  // namespace

extern "C" int kman_extract_words(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                                  uint64_t *d_words, uint64_t stride, void *d_pos, uint32_t pos_bytes, uint64_t cap,
                                  uint64_t *n_out) {
    if (!ctx || !n_out) return KMAN_EINVAL;
    *n_out = 0;
    if (k < 2) return kman_fail(ctx, KMAN_EINVAL, "k must be >= 2, got %u", k);
    if (d_pos && pos_bytes != 4 && pos_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "pos_bytes must be 4 or 8");
    if (d_words && stride < cap) return kman_fail(ctx, KMAN_EINVAL, "word stride %llu < capacity %llu",
                                                  (unsigned long long)stride, (unsigned long long)cap);
    if (n_bases == 0) return KMAN_OK;
    if (!d_codes) return kman_fail(ctx, KMAN_EINVAL, "null buffer");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint32_t W = (k + 31) / 32;
    const uint64_t tiles = ceil_div(n_bases, XTILE);
    if (tiles > 0x7fffffffull) return kman_fail(ctx, KMAN_EINVAL, "input too large");
    void *scr;
    KMAN_TRY(kman_scratch(ctx, tiles * 12, &scr));
    uint32_t *d_cnt = (uint32_t *)scr;
    uint64_t *d_off = (uint64_t *)((char *)scr + ceil_div(tiles * 4, 8) * 8);
    KTimer kt_(ctx, "extract_words");
    hipLaunchKernelGGL(words_kernel<false>, dim3((uint32_t)tiles), dim3(XT), 0, ctx->stream, d_codes, n_bases, k, W,
                       flags, nullptr, d_cnt, nullptr, 0, nullptr, 0, 0);
    HIP_TRY(ctx, hipGetLastError());
    uint64_t total = 0;
    KMAN_TRY(scan_tiles(ctx, d_cnt, tiles, d_off, &total));
    *n_out = total;
    if (!d_words && !d_pos) return KMAN_OK;  // count only
    if (total > cap) return KMAN_ECAP;
    hipLaunchKernelGGL(words_kernel<true>, dim3((uint32_t)tiles), dim3(XT), 0, ctx->stream, d_codes, n_bases, k, W,
                       flags, d_off, nullptr, d_words, stride, d_pos, pos_bytes, cap);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}

extern "C" int kman_rle_words(kman_ctx *ctx, int mode, const uint64_t *d_words, uint32_t W, uint64_t stride,
                              const void *d_vals, uint32_t val_bytes, uint64_t n, uint64_t *d_owords, uint64_t ostride,
                              void *d_ovals, uint32_t oval_bytes, uint64_t *n_out) {
    if (!ctx || !n_out) return KMAN_EINVAL;
    *n_out = 0;
    if (mode != KMAN_FINISH_COUNT && mode != KMAN_FINISH_UNIQ) return kman_fail(ctx, KMAN_EINVAL, "bad mode");
    if (W < 1) return kman_fail(ctx, KMAN_EINVAL, "W must be >= 1");
    if (oval_bytes != 4 && oval_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "oval_bytes must be 4 or 8");
    if (mode == KMAN_FINISH_UNIQ && val_bytes != 4 && val_bytes != 8)
        return kman_fail(ctx, KMAN_EINVAL, "val_bytes must be 4 or 8");
    if (n == 0) return KMAN_OK;
    if (!d_words || !d_owords || !d_ovals || (mode == KMAN_FINISH_UNIQ && !d_vals))
        return kman_fail(ctx, KMAN_EINVAL, "null buffer");
    if (stride < n || ostride < n) return kman_fail(ctx, KMAN_EINVAL, "stride below n");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t tiles = ceil_div(n, RTILE);
    if (tiles > 0x7fffffffull) return kman_fail(ctx, KMAN_EINVAL, "input too large");
    // scratch: tile counts, tile offsets, then (count mode) the head indices
    const uint64_t a = ceil_div(tiles * 4, 8) * 8, b = a + tiles * 8;
    void *scr;
    KMAN_TRY(kman_scratch(ctx, b + (mode == KMAN_FINISH_COUNT ? n * 8 : 0), &scr));
    uint32_t *d_cnt = (uint32_t *)scr;
    uint64_t *d_off = (uint64_t *)((char *)scr + a);
    uint64_t *d_heads = (uint64_t *)((char *)scr + b);
    KTimer kt_(ctx, mode == KMAN_FINISH_UNIQ ? "rle_uniq" : "rle_count");
    hipLaunchKernelGGL(rle_words_kernel<false>, dim3((uint32_t)tiles), dim3(RT_), 0, ctx->stream, d_words, W, stride,
                       n, mode, nullptr, d_cnt, nullptr, 0, nullptr, 0, nullptr, 0, nullptr);
    HIP_TRY(ctx, hipGetLastError());
    uint64_t total = 0;
    KMAN_TRY(scan_tiles(ctx, d_cnt, tiles, d_off, &total));
    hipLaunchKernelGGL(rle_words_kernel<true>, dim3((uint32_t)tiles), dim3(RT_), 0, ctx->stream, d_words, W, stride,
                       n, mode, d_off, nullptr, d_owords, ostride, d_vals, val_bytes, d_ovals, oval_bytes, d_heads);
    HIP_TRY(ctx, hipGetLastError());
    if (mode == KMAN_FINISH_COUNT && total) {
        if (oval_bytes == 4 && n > 0xffffffffull)
            return kman_fail(ctx, KMAN_EINVAL, "u32 counts cannot hold a group of up to %llu", (unsigned long long)n);
        hipLaunchKernelGGL(group_sizes_kernel, dim3((uint32_t)ceil_div(total, 256)), dim3(256), 0, ctx->stream,
                           d_heads, total, n, d_ovals, oval_bytes);
        HIP_TRY(ctx, hipGetLastError());
    }
    *n_out = total;
    return KMAN_OK;
}

extern "C" int kman_batch_tags(kman_ctx *ctx, const uint64_t *d_perm, uint64_t n, uint64_t start, uint64_t per_batch,
                               uint64_t *d_tags) {
    if (!ctx) return KMAN_EINVAL;
    if (per_batch == 0) return kman_fail(ctx, KMAN_EINVAL, "per_batch must be >= 1");
    if (n == 0) return KMAN_OK;
    if (!d_perm || !d_tags) return kman_fail(ctx, KMAN_EINVAL, "null buffer");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(batch_tags_kernel, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, ctx->stream, d_perm, n, start,
                       per_batch, d_tags);
    HIP_TRY(ctx, hipGetLastError());
    return KMAN_OK;
}
