// kmer.h — sliding-window k-mer helpers shared by extract.hip and the fused
// extract + first-pass kernel in sort.hip (Sequence.yield_kmers,
// kmermaid/seq.py:285-328; codes from kman_parse_fasta: bits 0-1 base, bit 2
// not ACGT, bit 3 record start).
#pragma once
#include "common.h"
#include "rollfast.h"

namespace {

// The codes of windows [tb, tb + NT*EI) plus a 64-byte halo, in 16-byte
// vectors (past the padded end, code 4 = not ACGT).  load_codes issues every
// load of a thread (no wait); store_codes puts them into LDS.
template <int NT, int EI>
struct CodeVecs {
    static constexpr int NV = (NT * EI + 64) / 16;  // 16-byte vectors
    static constexpr int R = (NV + NT - 1) / NT;    // per thread
    uint4 v[R];
    bool full[R];
};

template <int NT, int EI>
KMAN_DEV void load_codes(const uint8_t *__restrict__ codes, uint64_t n_bases, uint64_t tb, CodeVecs<NT, EI> &cv) {
    using C = CodeVecs<NT, EI>;
    const uint64_t limit = n_bases + 64;  // padded region is valid memory, value 4
#pragma unroll
    for (int i = 0; i < C::R; i++) {
        const int vi = threadIdx.x + i * NT;
        const uint64_t off = tb + (uint64_t)vi * 16;
        cv.full[i] = vi < C::NV && off + 16 <= limit;
        // unconditional (a safe address when not full); volatile keeps the
        // compiler from sinking a load into its store's branch
        const volatile uint4 *src = reinterpret_cast<const volatile uint4 *>(codes + (cv.full[i] ? off : 0));
        cv.v[i].x = src->x;
        cv.v[i].y = src->y;
        cv.v[i].z = src->z;
        cv.v[i].w = src->w;
    }
}

template <int NT, int EI>
KMAN_DEV void store_codes(const CodeVecs<NT, EI> &cv, const uint8_t *__restrict__ codes, uint64_t n_bases,
                          uint64_t tb, uint8_t *s) {
    using C = CodeVecs<NT, EI>;
    const uint64_t limit = n_bases + 64;
#pragma unroll
    for (int i = 0; i < C::R; i++) {
        const int vi = threadIdx.x + i * NT;
        if (vi < C::NV) *reinterpret_cast<uint4 *>(s + vi * 16) = cv.v[i];
    }
    // the vectors that cross the padded end, byte by byte (last tile only)
#pragma unroll
    for (int i = 0; i < C::R; i++) {
        const int vi = threadIdx.x + i * NT;
        const uint64_t off = tb + (uint64_t)vi * 16;
        if (vi < C::NV && !cv.full[i])
            for (int b = 0; b < 16; b++) s[vi * 16 + b] = (off + b < limit) ? codes[off + b] : 4;
    }
}

template <int NT, int EI>
KMAN_DEV void stage_codes(const uint8_t *__restrict__ codes, uint64_t n_bases, uint64_t tb, uint8_t *s) {
    CodeVecs<NT, EI> cv;
    load_codes<NT, EI>(codes, n_bases, tb, cv);
    store_codes<NT, EI>(cv, codes, n_bases, tb, s);
}

// Roll the EI windows starting at s[base .. base+EI) (k from LDS bytes), one
// base at a time (kept for A/B timing: make EXTRA=-DKMAN_ROLL_SEQ).
template <int EI, int CANON>
KMAN_DEV uint32_t roll_seq(const uint8_t *s, int base, int k, uint64_t mask, uint64_t p0, uint64_t n_bases,
                       uint64_t (&kf)[EI], uint64_t (&kr)[EI]) {
    uint64_t f = 0, r = 0;
    uint32_t run = 0;
    const int rsh = 2 * k - 2;
    for (int q = 0; q < k - 1; q++) {
        const uint32_t c = s[base + q];
        run = (c & 8) ? 0 : run;
        run = (c & 4) ? 0 : run + 1;
        f = (f << 2) | (c & 3);
        r = (r >> 2) | ((uint64_t)(3 - (c & 3)) << rsh);
    }
    uint32_t valid = 0;
#pragma unroll
    for (int j = 0; j < EI; j++) {
        const uint32_t c = s[base + k - 1 + j];
        run = (c & 8) ? 0 : run;
        run = (c & 4) ? 0 : run + 1;
        f = (f << 2) | (c & 3);
        r = (r >> 2) | ((uint64_t)(3 - (c & 3)) << rsh);
        const uint64_t fm = f & mask;
        if (CANON) {
            kf[j] = fm < r ? fm : r;
            if (CANON == 2) kf[j] = mix_key(kf[j], k);
        } else {
            kf[j] = fm;
            kr[j] = r;
        }
        valid |= (uint32_t)(run >= (uint32_t)k && p0 + j < n_bases) << j;
    }
    return valid;
}

// The same windows bit-parallel (rollfast.h): aligned LDS word reads packed
// four codes per multiply, each window a funnel shift of the packed stream.
// base = threadIdx.x * EI at every call site and s is 16-byte aligned, so the
// words are read as 16- or 8-byte vectors when EI is a multiple of 16 / 8.
template <int EI, int CANON>
KMAN_DEV uint32_t roll(const uint8_t *s, int base, int k, uint64_t mask, uint64_t p0, uint64_t n_bases,
                       uint64_t (&kf)[EI], uint64_t (&kr)[EI]) {
#ifdef KMAN_ROLL_SEQ
    return roll_seq<EI, CANON>(s, base, k, mask, p0, n_bases, kf, kr);
#else
#ifdef KMAN_ROLL_A4
    constexpr int A = 4;  // (A/B: 4-byte word reads)
#else
    constexpr int A = EI % 16 == 0 ? 16 : (EI % 8 == 0 ? 8 : 4);
#endif
    return roll_fast<EI, CANON, A>(s, base, k, mask, p0, n_bases, kf, kr);
#endif
}

}  // namespace
