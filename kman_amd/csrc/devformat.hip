// devformat.hip — device-side output writers: the reference's
// output lines built in HBM, byte-identical to format.cpp / the reference:
//
//   count  "%s\t%d\n" % (seq, len(headers))       kmermaid/join.py:283-284
//   uniq   ">%s\n%s\n" % (header, seq)            kmermaid/join.py:261-262
//   header "%s:%d-%d:%s" % (ref, start, end, +/-)  kmermaid/seq.py:103-104
//
// One kernel per format.  A tile of FT x FI rows: every thread sizes its FI
// consecutive rows, a block scan gives the thread offsets, a decoupled
// look-back over the tiles gives the tile's output offset.  The tile's lines
// are built in an LDS byte buffer (ds byte writes are cheap) and copied out
// as 16-byte-aligned global stores, funnel-shifted from the LDS words, so HBM
// sees full-line writes; only the two partial words at the tile's ends take
// byte stores.  A tile whose text exceeds the LDS buffer (uniq rows with very
// long record names) writes its lines straight to HBM instead.  Rows past
// `cap` are not written: the total is still computed (KMAN_ECAP + size).
#include "common.h"

namespace {

constexpr int FT = 256;
constexpr int FI = 2;
constexpr int FTILE = FT * FI;
constexpr uint32_t FB = 32768;  // LDS text bytes per tile

KMAN_DEV uint32_t ndig(uint64_t v) {
    uint32_t n = 1;
    if (v < 0x100000000ull) {
        uint32_t x = (uint32_t)v;
        while (x >= 10) {
            x /= 10;
            n++;
        }
        return n;
    }
    while (v >= 10) {
        v /= 10;
        n++;
    }
    return n;
}

// byte sinks: LDS buffer or global memory
struct LdsSink {
    uint8_t *b;
    KMAN_DEV void put(uint32_t at, uint8_t c) const { b[at] = c; }
};
struct GlobalSink {
    uint8_t *b;  // out + tile base
    KMAN_DEV void put(uint32_t at, uint8_t c) const { b[at] = c; }
};

template <typename S>
KMAN_DEV uint32_t put_dec(const S &s, uint32_t at, uint64_t v, uint32_t nd) {
    uint32_t e = at + nd;
    if (v < 0x100000000ull) {
        uint32_t x = (uint32_t)v;
        do {
            s.put(--e, (uint8_t)('0' + x % 10));
            x /= 10;
        } while (x);
    } else {
        do {
            s.put(--e, (uint8_t)('0' + v % 10));
            v /= 10;
        } while (v);
    }
    return at + nd;
}

template <typename S>
KMAN_DEV uint32_t put_seq(const S &s, uint32_t at, uint64_t key, uint32_t k) {
    for (int j = (int)k - 1; j >= 0; j--) s.put(at++, (uint8_t)"ACGT"[(key >> (2 * j)) & 3]);
    return at;
}

// k > 32: the key is (hi, lo), the first k - 32 bases in hi
template <typename S>
KMAN_DEV uint32_t put_key(const S &s, uint32_t at, const uint64_t *hi, uint64_t khi, uint64_t key, uint32_t k) {
    if (!hi) return put_seq(s, at, key, k);
    at = put_seq(s, at, khi, k - 32);
    return put_seq(s, at, key, 32);
}

// any k: W word planes (words.hip layout: word 0 the first k - 32 (W - 1)
// bases, then 32 per word), row i's word j at words[j * stride + i]
struct WordKeys {
    const uint64_t *words = nullptr;
    uint64_t stride = 0;
    uint32_t W = 0;
    template <typename S>
    KMAN_DEV uint32_t put(const S &s, uint32_t at, uint64_t i, uint32_t k) const {
        const uint32_t h = k - 32 * (W - 1);
        for (uint32_t j = 0; j < W; j++) at = put_seq(s, at, words[j * stride + i], j ? 32u : h);
        return at;
    }
};

struct CountRows {
    const uint64_t *keys;
    const void *vals;
    uint32_t vb, k;
    const uint64_t *hi = nullptr;  // word-pair keys (k > 32)
    WordKeys wk = {};              // or W word planes (keys unused)
    KMAN_DEV uint64_t val(uint64_t i) const {
        return vb == 4 ? ((const uint32_t *)vals)[i] : ((const uint64_t *)vals)[i];
    }
    struct Row {
        uint64_t key, khi, c, idx;
        uint32_t nd;
    };
    KMAN_DEV Row load(uint64_t i) const {
        Row r;
        r.idx = i;
        r.key = wk.words ? 0 : keys[i];
        r.khi = hi ? hi[i] : 0;
        r.c = val(i);
        r.nd = ndig(r.c);
        return r;
    }
    KMAN_DEV uint32_t len(const Row &r) const { return k + 2 + r.nd; }
    template <typename S>
    KMAN_DEV uint32_t write(const S &s, uint32_t at, const Row &r) const {
        at = wk.words ? wk.put(s, at, r.idx, k) : put_key(s, at, hi, r.khi, r.key, k);
        s.put(at++, '\t');
        at = put_dec(s, at, r.c, r.nd);
        s.put(at++, '\n');
        return at;
    }
};

struct UniqRows {
    const uint64_t *keys;
    const void *vals;
    uint32_t vb, k;
    const uint8_t *names;
    const uint64_t *name_off, *rec_seq;
    uint64_t R;
    const uint64_t *hi = nullptr;  // word-pair keys (k > 32)
    WordKeys wk = {};              // or W word planes (keys unused)
    struct Row {
        uint64_t key, khi, st, noff, idx;
        uint32_t nlen, nd0, nd1;
        bool minus;
    };
    KMAN_DEV Row load(uint64_t i) const {
        Row r;
        r.idx = i;
        r.key = wk.words ? 0 : keys[i];
        r.khi = hi ? hi[i] : 0;
        const uint64_t v = vb == 4 ? ((const uint32_t *)vals)[i] : ((const uint64_t *)vals)[i];
        const uint64_t g = v >> 1;
        r.minus = v & 1;
        // record owning base g: the last record whose first base is <= g
        // (std::upper_bound - 1, format.cpp Names::find)
        uint64_t lo = 0, hi = R;  // first index with rec_seq > g in [lo, hi]
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (rec_seq[mid] <= g) lo = mid + 1;
            else hi = mid;
        }
        const uint64_t rec = lo - 1;
        r.st = g - rec_seq[rec];
        r.noff = name_off[rec];
        r.nlen = (uint32_t)(name_off[rec + 1] - r.noff);
        r.nd0 = ndig(r.st);
        r.nd1 = ndig(r.st + k);
        return r;
    }
    // ">" name ":" start "-" end ":" s "\n" seq "\n"
    KMAN_DEV uint32_t len(const Row &r) const { return 1 + r.nlen + 1 + r.nd0 + 1 + r.nd1 + 3 + k + 1; }
    template <typename S>
    KMAN_DEV uint32_t write(const S &s, uint32_t at, const Row &r) const {
        s.put(at++, '>');
        for (uint32_t j = 0; j < r.nlen; j++) s.put(at++, names[r.noff + j]);
        s.put(at++, ':');
        at = put_dec(s, at, r.st, r.nd0);
        s.put(at++, '-');
        at = put_dec(s, at, r.st + k, r.nd1);
        s.put(at++, ':');
        s.put(at++, r.minus ? '-' : '+');
        s.put(at++, '\n');
        at = wk.words ? wk.put(s, at, r.idx, k) : put_key(s, at, hi, r.khi, r.key, k);
        s.put(at++, '\n');
        return at;
    }
};

template <typename Rows>
__global__ __launch_bounds__(FT) void format_kernel(Rows rows, uint64_t n, uint8_t *__restrict__ out, uint64_t cap,
                                                    uint64_t *__restrict__ status, uint32_t *__restrict__ counter,
                                                    uint32_t epoch, uint32_t *__restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint32_t text[FB / 4 + 8];
    __shared__ uint32_t lds_scan[FT / 64];
    __shared__ uint64_t lds_base;
    __shared__ uint32_t lds_tile;
    const int64_t tile = grab_tile(counter, &lds_tile);
    const uint64_t i0 = (uint64_t)tile * FTILE + (uint64_t)threadIdx.x * FI;
    typename Rows::Row r[FI];
    uint32_t len = 0;
#pragma unroll
    for (int j = 0; j < FI; j++) {
        if (i0 + j < n) {
            r[j] = rows.load(i0 + j);
            len += rows.len(r[j]);
        }
    }
    uint32_t total;
    const uint32_t off = block_exclusive_scan<FT>(len, SumU32(), 0u, lds_scan, &total);
    if (threadIdx.x < 64) {
        const uint64_t b = wave_lookback<0>(status, tile, total, epoch, err);
        if (threadIdx.x == 0) lds_base = b;
    }
    __syncthreads();
    const uint64_t base = lds_base;
    if (!out || base + total > cap) return;  // sizing only / past the capacity
    if (total > FB) {
        const GlobalSink s{out + base};
        uint32_t at = off;
#pragma unroll
        for (int j = 0; j < FI; j++)
            if (i0 + j < n) at = rows.write(s, at, r[j]);
        return;
    }
    {
        const LdsSink s{reinterpret_cast<uint8_t *>(text)};
        uint32_t at = off;
#pragma unroll
        for (int j = 0; j < FI; j++)
            if (i0 + j < n) at = rows.write(s, at, r[j]);
    }
    __syncthreads();
    // out[base, base + total) <- text[0, total): 16-byte global words; the
    // word w covers text bytes [16w - base, 16w - base + 16)
    const uint8_t *tb = reinterpret_cast<const uint8_t *>(text);
    const uint64_t end = base + total;
    const uint64_t w0 = base >> 4, w1 = (end + 15) >> 4;
    for (uint64_t w = w0 + threadIdx.x; w < w1; w += FT) {
        const uint64_t a = w << 4;
        if (a >= base && a + 16 <= end) {
            const uint32_t q = (uint32_t)(a - base), m = q >> 2, rs = (q & 3) * 8;
            uint32_t v[5];
#pragma unroll
            for (int t = 0; t < 5; t++) v[t] = text[m + t];
            uint4 o;
            if (rs) {
                o.x = (v[0] >> rs) | (v[1] << (32 - rs));
                o.y = (v[1] >> rs) | (v[2] << (32 - rs));
                o.z = (v[2] >> rs) | (v[3] << (32 - rs));
                o.w = (v[3] >> rs) | (v[4] << (32 - rs));
            } else {
                o = make_uint4(v[0], v[1], v[2], v[3]);
            }
            *reinterpret_cast<uint4 *>(out + a) = o;
        } else {
            for (uint64_t b = a < base ? base : a; b < a + 16 && b < end; b++) out[b] = tb[b - base];
        }
    }
}

template <typename Rows>
int run_format(kman_ctx *ctx, const Rows &rows, uint64_t n, char *d_out, size_t cap, size_t *used) {
    *used = 0;
    if (n == 0) return KMAN_OK;
    if (d_out && ((uintptr_t)d_out & 15)) return kman_fail(ctx, KMAN_EINVAL, "output must be 16-byte aligned");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t T = ceil_div(n, (uint64_t)FTILE);
    if (T > 0xffffffffull) return kman_fail(ctx, KMAN_EINVAL, "too many rows");
    uint32_t epoch, *counter;
    KMAN_TRY(kman_lookback_begin(ctx, T, &epoch, &counter));
    {
        KTimer kt_(ctx, "format");
        hipLaunchKernelGGL(format_kernel<Rows>, dim3((uint32_t)T), dim3(FT), 0, ctx->stream, rows, n,
                           reinterpret_cast<uint8_t *>(d_out), (uint64_t)(d_out ? cap : 0), ctx->d_status, counter,
                           epoch, ctx->d_err);
        HIP_TRY(ctx, hipGetLastError());
    }
    uint64_t tot = 0;
    KMAN_TRY(kman_lookback_total(ctx, T, &tot));
    *used = (size_t)tot;
    return tot > (d_out ? cap : 0) ? KMAN_ECAP : KMAN_OK;
}

}  // namespace

extern "C" int kman_format_count_dev(kman_ctx *ctx, const uint64_t *d_ukeys, const void *d_counts,
                                     uint32_t count_bytes, uint64_t n, uint32_t k, char *d_out, size_t cap,
                                     size_t *used) {
    if (!ctx || !used || (n && (!d_ukeys || !d_counts))) return KMAN_EINVAL;
    if (k < 1 || k > 32) return kman_fail(ctx, KMAN_EINVAL, "k must be in [1, 32], got %u", k);
    if (count_bytes != 4 && count_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "count_bytes must be 4 or 8");
    return run_format(ctx, CountRows{d_ukeys, d_counts, count_bytes, k}, n, d_out, cap, used);
}

extern "C" int kman_format_uniq_dev(kman_ctx *ctx, const uint64_t *d_keys, const void *d_pos, uint32_t pos_bytes,
                                    uint64_t n, uint32_t k, const char *d_names, const uint64_t *d_name_off,
                                    const uint64_t *d_rec_seq, uint64_t n_records, char *d_out, size_t cap,
                                    size_t *used) {
    if (!ctx || !used || (n && (!d_keys || !d_pos || !d_name_off || !d_rec_seq || !n_records))) return KMAN_EINVAL;
    if (k < 1 || k > 32) return kman_fail(ctx, KMAN_EINVAL, "k must be in [1, 32], got %u", k);
    if (pos_bytes != 4 && pos_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "pos_bytes must be 4 or 8");
    return run_format(ctx,
                      UniqRows{d_keys, d_pos, pos_bytes, k, reinterpret_cast<const uint8_t *>(d_names), d_name_off,
                               d_rec_seq, n_records},
                      n, d_out, cap, used);
}

extern "C" int kman_format_count_wide_dev(kman_ctx *ctx, const uint64_t *d_hi, const uint64_t *d_lo,
                                          const void *d_counts, uint32_t count_bytes, uint64_t n, uint32_t k,
                                          char *d_out, size_t cap, size_t *used) {
    if (!ctx || !used || (n && (!d_hi || !d_lo || !d_counts))) return KMAN_EINVAL;
    if (k < 33 || k > 64) return kman_fail(ctx, KMAN_EINVAL, "k must be in [33, 64], got %u", k);
    if (count_bytes != 4 && count_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "count_bytes must be 4 or 8");
    return run_format(ctx, CountRows{d_lo, d_counts, count_bytes, k, d_hi}, n, d_out, cap, used);
}

extern "C" int kman_format_uniq_wide_dev(kman_ctx *ctx, const uint64_t *d_hi, const uint64_t *d_lo, const void *d_pos,
                                         uint32_t pos_bytes, uint64_t n, uint32_t k, const char *d_names,
                                         const uint64_t *d_name_off, const uint64_t *d_rec_seq, uint64_t n_records,
                                         char *d_out, size_t cap, size_t *used) {
    if (!ctx || !used || (n && (!d_hi || !d_lo || !d_pos || !d_name_off || !d_rec_seq || !n_records)))
        return KMAN_EINVAL;
    if (k < 33 || k > 64) return kman_fail(ctx, KMAN_EINVAL, "k must be in [33, 64], got %u", k);
    if (pos_bytes != 4 && pos_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "pos_bytes must be 4 or 8");
    return run_format(ctx,
                      UniqRows{d_lo, d_pos, pos_bytes, k, reinterpret_cast<const uint8_t *>(d_names), d_name_off,
                               d_rec_seq, n_records, d_hi},
                      n, d_out, cap, used);
}

// any k >= 2 as W = ceil(k / 32) word planes (words.hip)
extern "C" int kman_format_count_words_dev(kman_ctx *ctx, const uint64_t *d_words, uint64_t stride,
                                           const void *d_counts, uint32_t count_bytes, uint64_t n, uint32_t k,
                                           char *d_out, size_t cap, size_t *used) {
    if (!ctx || !used || (n && (!d_words || !d_counts))) return KMAN_EINVAL;
    if (k < 2) return kman_fail(ctx, KMAN_EINVAL, "k must be >= 2, got %u", k);
    if (count_bytes != 4 && count_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "count_bytes must be 4 or 8");
    if (stride < n) return kman_fail(ctx, KMAN_EINVAL, "stride below n");
    CountRows rows{nullptr, d_counts, count_bytes, k};
    rows.wk = WordKeys{d_words, stride, (k + 31) / 32};
    return run_format(ctx, rows, n, d_out, cap, used);
}

extern "C" int kman_format_uniq_words_dev(kman_ctx *ctx, const uint64_t *d_words, uint64_t stride, const void *d_pos,
                                          uint32_t pos_bytes, uint64_t n, uint32_t k, const char *d_names,
                                          const uint64_t *d_name_off, const uint64_t *d_rec_seq, uint64_t n_records,
                                          char *d_out, size_t cap, size_t *used) {
    if (!ctx || !used || (n && (!d_words || !d_pos || !d_name_off || !d_rec_seq || !n_records))) return KMAN_EINVAL;
    if (k < 2) return kman_fail(ctx, KMAN_EINVAL, "k must be >= 2, got %u", k);
    if (pos_bytes != 4 && pos_bytes != 8) return kman_fail(ctx, KMAN_EINVAL, "pos_bytes must be 4 or 8");
    if (stride < n) return kman_fail(ctx, KMAN_EINVAL, "stride below n");
    UniqRows rows{nullptr, d_pos, pos_bytes, k, reinterpret_cast<const uint8_t *>(d_names), d_name_off, d_rec_seq,
                  n_records};
    rows.wk = WordKeys{d_words, stride, (k + 31) / 32};
    return run_format(ctx, rows, n, d_out, cap, used);
}
