// format.cpp — byte-exact output writers (host side).
//
//   count  "%s\t%d\n" % (seq, len(headers))       kmermaid/join.py:283-284
//   uniq   ">%s\n%s\n" % (header, seq)            kmermaid/join.py:261-262
//   batch  KMer.as_fasta ">%s\n%s\n"               kmermaid/seq.py:489-495
//   header "%s:%d-%d:%s" % (ref, start, end, +/-)  kmermaid/seq.py:103-104
//
// The formatting runs on host threads over host copies of the device results:
// each thread sizes its slice, an exclusive scan gives the slice offsets, then
// every thread writes its slice in place.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/kman.h"

namespace {

inline int ndigits(uint64_t v) {
    int n = 1;
    while (v >= 10) {
        v /= 10;
        n++;
    }
    return n;
}

inline char *put_u64(char *p, uint64_t v) {
    char t[24];
    int n = 0;
    do {
        t[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    while (n) *p++ = t[--n];
    return p;
}

inline char *put_seq(char *p, uint64_t key, uint32_t k) {
    static const char B[4] = {'A', 'C', 'G', 'T'};
    for (int j = (int)k - 1; j >= 0; j--) *p++ = B[(key >> (2 * j)) & 3];
    return p;
}

// k > 32: the first k - 32 bases in hi, the last 32 in lo
inline char *put_seq_wide(char *p, uint64_t hi, uint64_t lo, uint32_t k) {
    p = put_seq(p, hi, k - 32);
    return put_seq(p, lo, 32);
}

// any k: W word planes (words.hip layout), row i's word j at w[j * stride + i]
struct Words {
    const uint64_t *w;
    uint64_t stride;
    uint32_t W;
    char *put(char *p, uint64_t i, uint32_t k) const {
        const uint32_t h = k - 32 * (W - 1);
        for (uint32_t j = 0; j < W; j++) p = put_seq(p, w[j * stride + i], j ? 32u : h);
        return p;
    }
};

inline uint64_t get_val(const void *a, uint32_t bytes, uint64_t i) {
    return bytes == 4 ? ((const uint32_t *)a)[i] : ((const uint64_t *)a)[i];
}

template <typename SizeF, typename WriteF>
int run_sliced(uint64_t n, char *out, size_t cap, size_t *used, int threads, SizeF size_of, WriteF write_at) {
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n / 4096 + 1) threads = (int)(n / 4096 + 1);
    std::vector<size_t> sz(threads + 1, 0);
    auto slice = [&](int t, uint64_t *b, uint64_t *e) {
        *b = n * t / threads;
        *e = n * (t + 1) / threads;
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++)
            th.emplace_back([&, t] {
                uint64_t b, e;
                slice(t, &b, &e);
                size_t s = 0;
                for (uint64_t i = b; i < e; i++) s += size_of(i);
                sz[t + 1] = s;
            });
        for (auto &x : th) x.join();
    }
    for (int t = 0; t < threads; t++) sz[t + 1] += sz[t];
    *used = sz[threads];
    if (sz[threads] > cap || !out) return KMAN_ECAP;
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++)
            th.emplace_back([&, t] {
                uint64_t b, e;
                slice(t, &b, &e);
                char *p = out + sz[t];
                for (uint64_t i = b; i < e; i++) p = write_at(i, p);
            });
        for (auto &x : th) x.join();
    }
    return KMAN_OK;
}

struct Names {
    const char *names;
    const uint64_t *off;
    const uint64_t *rec_seq;
    uint64_t R;
    // record owning global base p: the last record whose first base is <= p
    uint64_t find(uint64_t p) const {
        const uint64_t *it = std::upper_bound(rec_seq, rec_seq + R, p);
        return (uint64_t)(it - rec_seq) - 1;
    }
};

int format_fasta_impl(const uint64_t *keys, const void *pos, uint32_t pos_bytes, uint64_t n, uint32_t k,
                      const Names &nm, char *out, size_t cap, size_t *used, int threads,
                      const uint64_t *hi = nullptr, const Words *wd = nullptr) {
    auto size_of = [&](uint64_t i) -> size_t {
        const uint64_t v = get_val(pos, pos_bytes, i);
        const uint64_t p = v >> 1;
        const uint64_t r = nm.find(p);
        const uint64_t st = p - nm.rec_seq[r];
        // ">" name ":" start "-" end ":" s "\n" seq "\n"
        return 1 + (nm.off[r + 1] - nm.off[r]) + 1 + ndigits(st) + 1 + ndigits(st + k) + 2 + 1 + k + 1;
    };
    auto write_at = [&](uint64_t i, char *p) -> char * {
        const uint64_t v = get_val(pos, pos_bytes, i);
        const uint64_t g = v >> 1;
        const uint64_t r = nm.find(g);
        const uint64_t st = g - nm.rec_seq[r];
        *p++ = '>';
        const uint64_t L = nm.off[r + 1] - nm.off[r];
        memcpy(p, nm.names + nm.off[r], L);
        p += L;
        *p++ = ':';
        p = put_u64(p, st);
        *p++ = '-';
        p = put_u64(p, st + k);
        *p++ = ':';
        *p++ = (v & 1) ? '-' : '+';
        *p++ = '\n';
        p = wd ? wd->put(p, i, k) : hi ? put_seq_wide(p, hi[i], keys[i], k) : put_seq(p, keys[i], k);
        *p++ = '\n';
        return p;
    };
    return run_sliced(n, out, cap, used, threads, size_of, write_at);
}

}  // namespace

extern "C" int kman_format_count(const uint64_t *ukeys, const void *counts, uint32_t count_bytes, uint64_t n,
                                 uint32_t k, char *out, size_t cap, size_t *used, int threads) {
    if (!used || (n && (!ukeys || !counts)) || k < 1 || k > 32) return KMAN_EINVAL;
    if (count_bytes != 4 && count_bytes != 8) return KMAN_EINVAL;
    auto size_of = [&](uint64_t i) -> size_t { return k + 2 + ndigits(get_val(counts, count_bytes, i)); };
    auto write_at = [&](uint64_t i, char *p) -> char * {
        p = put_seq(p, ukeys[i], k);
        *p++ = '\t';
        p = put_u64(p, get_val(counts, count_bytes, i));
        *p++ = '\n';
        return p;
    };
    return run_sliced(n, out, cap, used, threads, size_of, write_at);
}

// one abundance vector as text, "%d\n" per entry (AbundanceVector.write_to,
// abundance.py:151-168, after its "# k=%d" line): entries v[0], v[stride], ..
extern "C" int kman_format_vector(const uint32_t *v, uint64_t n, uint64_t stride, char *out, size_t cap,
                                  size_t *used, int threads) {
    if (!used || (n && !v) || stride == 0) return KMAN_EINVAL;
    auto size_of = [&](uint64_t i) -> size_t { return ndigits(v[i * stride]) + 1; };
    auto write_at = [&](uint64_t i, char *p) -> char * {
        p = put_u64(p, v[i * stride]);
        *p++ = '\n';
        return p;
    };
    return run_sliced(n, out, cap, used, threads, size_of, write_at);
}

extern "C" int kman_format_uniq(const uint64_t *keys, const void *pos, uint32_t pos_bytes, uint64_t n, uint32_t k,
                                const char *names, const uint64_t *name_off, const uint64_t *rec_seq,
                                uint64_t n_records, char *out, size_t cap, size_t *used, int threads) {
    if (!used || (n && (!keys || !pos || !name_off || !rec_seq || !n_records)) || k < 1 || k > 32) return KMAN_EINVAL;
    if (pos_bytes != 4 && pos_bytes != 8) return KMAN_EINVAL;
    Names nm{names, name_off, rec_seq, n_records};
    return format_fasta_impl(keys, pos, pos_bytes, n, k, nm, out, cap, used, threads);
}

// uniq rows over several sources (a multi-source join: FASTA inputs and
// reloaded batch files): one merged record table in global base indices;
// rec_kind[r] = 0: a FASTA record (header name:start-end:strand), 1: a batch
// file record whose title is the header as written (the k-mer's own
// "ref:start-end:strand").
namespace {
int uniq_mixed_impl(const uint64_t *keys, const Words *wd, const uint64_t *pos, uint64_t n, uint32_t k,
                    const char *names, const uint64_t *name_off, const uint64_t *rec_seq, const uint8_t *rec_kind,
                    uint64_t n_records, char *out, size_t cap, size_t *used, int threads) {
    Names nm{names, name_off, rec_seq, n_records};
    auto size_of = [&](uint64_t i) -> size_t {
        const uint64_t g = pos[i] >> 1;
        const uint64_t r = nm.find(g);
        const size_t L = nm.off[r + 1] - nm.off[r];
        if (rec_kind[r]) return 1 + L + 1 + k + 1;
        const uint64_t st = g - nm.rec_seq[r];
        return 1 + L + 1 + ndigits(st) + 1 + ndigits(st + k) + 2 + 1 + k + 1;
    };
    auto write_at = [&](uint64_t i, char *p) -> char * {
        const uint64_t v = pos[i], g = v >> 1;
        const uint64_t r = nm.find(g);
        const uint64_t L = nm.off[r + 1] - nm.off[r];
        *p++ = '>';
        memcpy(p, nm.names + nm.off[r], L);
        p += L;
        if (!rec_kind[r]) {
            const uint64_t st = g - nm.rec_seq[r];
            *p++ = ':';
            p = put_u64(p, st);
            *p++ = '-';
            p = put_u64(p, st + k);
            *p++ = ':';
            *p++ = (v & 1) ? '-' : '+';
        }
        *p++ = '\n';
        p = wd ? wd->put(p, i, k) : put_seq(p, keys[i], k);
        *p++ = '\n';
        return p;
    };
    return run_sliced(n, out, cap, used, threads, size_of, write_at);
}
}  // namespace

extern "C" int kman_format_uniq_mixed(const uint64_t *keys, const uint64_t *pos, uint64_t n, uint32_t k,
                                      const char *names, const uint64_t *name_off, const uint64_t *rec_seq,
                                      const uint8_t *rec_kind, uint64_t n_records, char *out, size_t cap,
                                      size_t *used, int threads) {
    if (!used || (n && (!keys || !pos || !name_off || !rec_seq || !rec_kind || !n_records)) || k < 1 || k > 32)
        return KMAN_EINVAL;
    return uniq_mixed_impl(keys, nullptr, pos, n, k, names, name_off, rec_seq, rec_kind, n_records, out, cap, used,
                           threads);
}

// the same over W word planes (any k >= 2; words.hip layout)
extern "C" int kman_format_uniq_mixed_words(const uint64_t *words, uint64_t stride, const uint64_t *pos, uint64_t n,
                                            uint32_t k, const char *names, const uint64_t *name_off,
                                            const uint64_t *rec_seq, const uint8_t *rec_kind, uint64_t n_records,
                                            char *out, size_t cap, size_t *used, int threads) {
    if (!used || (n && (!words || !pos || !name_off || !rec_seq || !rec_kind || !n_records)) || k < 2 || stride < n)
        return KMAN_EINVAL;
    const Words wd{words, stride, (k + 31) / 32};
    return uniq_mixed_impl(nullptr, &wd, pos, n, k, names, name_off, rec_seq, rec_kind, n_records, out, cap, used,
                           threads);
}

// any k >= 2 over W word planes: the count table and the uniq / batch FASTA
extern "C" int kman_format_count_words(const uint64_t *words, uint64_t stride, const void *counts,
                                       uint32_t count_bytes, uint64_t n, uint32_t k, char *out, size_t cap,
                                       size_t *used, int threads) {
    if (!used || (n && (!words || !counts)) || k < 2 || stride < n) return KMAN_EINVAL;
    if (count_bytes != 4 && count_bytes != 8) return KMAN_EINVAL;
    const Words wd{words, stride, (k + 31) / 32};
    auto size_of = [&](uint64_t i) -> size_t { return k + 2 + ndigits(get_val(counts, count_bytes, i)); };
    auto write_at = [&](uint64_t i, char *p) -> char * {
        p = wd.put(p, i, k);
        *p++ = '\t';
        p = put_u64(p, get_val(counts, count_bytes, i));
        *p++ = '\n';
        return p;
    };
    return run_sliced(n, out, cap, used, threads, size_of, write_at);
}

extern "C" int kman_format_uniq_words(const uint64_t *words, uint64_t stride, const void *pos, uint32_t pos_bytes,
                                      uint64_t n, uint32_t k, const char *names, const uint64_t *name_off,
                                      const uint64_t *rec_seq, uint64_t n_records, char *out, size_t cap,
                                      size_t *used, int threads) {
    if (!used || (n && (!words || !pos || !name_off || !rec_seq || !n_records)) || k < 2 || stride < n)
        return KMAN_EINVAL;
    if (pos_bytes != 4 && pos_bytes != 8) return KMAN_EINVAL;
    Names nm{names, name_off, rec_seq, n_records};
    const Words wd{words, stride, (k + 31) / 32};
    return format_fasta_impl(nullptr, pos, pos_bytes, n, k, nm, out, cap, used, threads, nullptr, &wd);
}

// k in 33..64: keys as (hi, lo) word pairs (kman_extract_wide)
extern "C" int kman_format_count_wide(const uint64_t *hi, const uint64_t *lo, const void *counts, uint32_t count_bytes,
                                      uint64_t n, uint32_t k, char *out, size_t cap, size_t *used, int threads) {
    if (!used || (n && (!hi || !lo || !counts)) || k < 33 || k > 64) return KMAN_EINVAL;
    if (count_bytes != 4 && count_bytes != 8) return KMAN_EINVAL;
    auto size_of = [&](uint64_t i) -> size_t { return k + 2 + ndigits(get_val(counts, count_bytes, i)); };
    auto write_at = [&](uint64_t i, char *p) -> char * {
        p = put_seq_wide(p, hi[i], lo[i], k);
        *p++ = '\t';
        p = put_u64(p, get_val(counts, count_bytes, i));
        *p++ = '\n';
        return p;
    };
    return run_sliced(n, out, cap, used, threads, size_of, write_at);
}

extern "C" int kman_format_uniq_wide(const uint64_t *hi, const uint64_t *lo, const void *pos, uint32_t pos_bytes,
                                     uint64_t n, uint32_t k, const char *names, const uint64_t *name_off,
                                     const uint64_t *rec_seq, uint64_t n_records, char *out, size_t cap, size_t *used,
                                     int threads) {
    if (!used || (n && (!hi || !lo || !pos || !name_off || !rec_seq || !n_records)) || k < 33 || k > 64)
        return KMAN_EINVAL;
    if (pos_bytes != 4 && pos_bytes != 8) return KMAN_EINVAL;
    Names nm{names, name_off, rec_seq, n_records};
    return format_fasta_impl(lo, pos, pos_bytes, n, k, nm, out, cap, used, threads, hi);
}
