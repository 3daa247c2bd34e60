// rollfast.h — the windows of kmer.h's roll() computed bit-parallel: the
// thread's code bytes are read as aligned 32-bit words and packed four at a
// time (one multiply each) into 2-bit streams, so a window's key is a funnel
// shift of the packed stream instead of k - 1 + EI dependent steps.
//
// Semantics (Sequence.yield_kmers, kmermaid/seq.py:285-328, on the codes of
// kman_parse_fasta: bits 0-1 base, bit 2 not ACGT, bit 3 record start):
// window j covers codes [base + j, base + j + k); it is valid when none of its
// k codes is not-ACGT, no code after its first starts a record, and its start
// p0 + j < n_bases.  kf = forward key (first base most significant), kr =
// reverse complement; CANON: kf = min(forward, reverse complement) (CANON == 2:
// through mix_key).
//
// Host-compilable (tests/test_rollfast.py checks it against a per-base roll).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define KMAN_RF_HD __host__ __device__ __forceinline__
#else
#define KMAN_RF_HD static inline
#endif

// bytes b0..b3 of x (b0 least significant), low 2 bits each, first byte in
// the top pair (BE) or bottom pair (LE); bit `bit` of each byte (4 bits, b0 at
// bit 0).  The multiplies place each field at its target bits with no carry
// into them from the cross terms below (every cross term sits >= 2 bits lower).
KMAN_RF_HD uint32_t rf_be8(uint32_t x) { return ((x & 0x03030303u) * 0x40100401u) >> 24; }
KMAN_RF_HD uint32_t rf_le8(uint32_t x) { return (((x & 0x03030303u) * 0x00041041u) >> 18) & 0xffu; }
KMAN_RF_HD uint32_t rf_bit4(uint32_t x, int bit) {
    return ((((x >> bit) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu;
}

// A bijection of the 2k-bit keys (odd multiply, xorshift, odd multiply, all
// mod 2^2k): canonical keys mixed by it keep their multiset of counts, so an
// abundance spectrum is unchanged, while the top key bits -- the buckets of
// the region passes -- become uniform (min(fwd, rc) alone puts about twice
// the average into the low buckets).  CANON == 2 selects it.
KMAN_RF_HD uint64_t mix_key(uint64_t x, int k) {
    const int kb = 2 * k;
    const uint64_t m = kb >= 64 ? ~0ull : ((1ull << kb) - 1);
    x = (x * 0x9E3779B97F4A7C15ull) & m;
    x ^= x >> (kb / 2);
    return (x * 0xBF58476D1CE4E5B9ull) & m;
}

// Validity of windows 0 .. EI-1 starting at codes 0 .. EI-1 (EI <= 16): with
// inv = not-ACGT flags and y = inv | record-start flags (one bit per code),
// window j is bad when code j is not ACGT or any of codes j+1 .. j+k-1 is
// flagged -- an OR over a (k-1)-wide window of y, built by doubling (widths
// 2, 4, 8, 16, then two overlapping ones); past n_bases nothing is valid.
// 2 <= k <= 32.
template <int EI>
KMAN_RF_HD uint32_t rf_valid_bits(uint64_t inv, uint64_t y, int k, uint64_t p0, uint64_t n_bases) {
    static_assert(EI <= 16, "windows within the first 64 flag bits");
    const int wd = k - 1;  // 1 .. 31
    const uint64_t y2 = y | (y >> 1), y4 = y2 | (y2 >> 2), y8 = y4 | (y4 >> 4), y16 = y8 | (y8 >> 8);
    const int m = wd >= 16 ? 16 : wd >= 8 ? 8 : wd >= 4 ? 4 : wd >= 2 ? 2 : 1;
    const uint64_t ym = m == 16 ? y16 : m == 8 ? y8 : m == 4 ? y4 : m == 2 ? y2 : y;
    const uint64_t yw = ym | (ym >> (wd - m));
    uint32_t valid = ~(uint32_t)(inv | (yw >> 1)) & (uint32_t)((1ull << EI) - 1);
    if (p0 + EI > n_bases) valid &= p0 >= n_bases ? 0u : (uint32_t)((1ull << (n_bases - p0)) - 1);
    return valid;
}

// ALIGN (16 or 8): s + base is that aligned (base = thread * EI with EI a
// multiple of it), so the words are read as 16- / 8-byte LDS vectors --
// with consecutive threads EI bytes apart, ds_read_b128 / ds_read_b64 hit
// every bank once per lane group, where ds_read_b32 at a 16-byte stride is
// 4-way conflicted
template <int EI, int CANON, int ALIGN = 4>
KMAN_RF_HD uint32_t roll_fast(const uint8_t *s, int base, int k, uint64_t mask, uint64_t p0, uint64_t n_bases,
                              uint64_t (&kf)[EI], uint64_t (&kr)[EI]) {
    // words covering (base & 3) + k - 1 + EI codes for any k <= 32
    constexpr int NW = (3 + 31 + EI + 3) / 4;
    static_assert(NW <= 16, "at most 64 codes");
    static_assert(ALIGN == 4 || ALIGN == 8 || ALIGN == 16, "4-, 8- or 16-byte word reads");
    const int b4 = base & ~3, dl = ALIGN > 4 ? 0 : base & 3;
    uint32_t w[NW];
    if constexpr (ALIGN == 16) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(s + base);
#pragma unroll
        for (int q = 0; q < (NW + 3) / 4; q++) {
            uint32_t v[4];
            __builtin_memcpy(v, __builtin_assume_aligned(p + 4 * q, 16), 16);
#pragma unroll
            for (int e = 0; e < 4; e++)
                if (4 * q + e < NW) w[4 * q + e] = v[e];
        }
    } else if constexpr (ALIGN == 8) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(s + base);
#pragma unroll
        for (int q = 0; q < (NW + 1) / 2; q++) {
            uint32_t v[2];
            __builtin_memcpy(v, __builtin_assume_aligned(p + 2 * q, 8), 8);
#pragma unroll
            for (int e = 0; e < 2; e++)
                if (2 * q + e < NW) w[2 * q + e] = v[e];
        }
    } else {
#pragma unroll
        for (int i = 0; i < NW; i++) w[i] = *reinterpret_cast<const uint32_t *>(s + b4 + 4 * i);
    }
    // code c (0 .. 4 * NW) of the thread's words: BE stream be0:be1 (code 0 at
    // the top of be0), LE stream le0:le1 (code 0 at the bottom of le0); the
    // not-ACGT and record-start flags, one bit per code
    uint32_t be[2 * ((NW + 3) / 4)], le[2 * ((NW + 3) / 4)];
#pragma unroll
    for (int i = 0; i < 2 * ((NW + 3) / 4); i++) be[i] = le[i] = 0;
    uint64_t inv = 0, rst = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        be[i / 4] |= rf_be8(w[i]) << (24 - 8 * (i % 4));
        le[i / 4] |= rf_le8(w[i]) << (8 * (i % 4));
        inv |= (uint64_t)rf_bit4(w[i], 2) << (4 * i);
        rst |= (uint64_t)rf_bit4(w[i], 3) << (4 * i);
    }
    const uint64_t be0 = ((uint64_t)be[0] << 32) | be[1];
    const uint64_t be1 = NW > 8 ? ((uint64_t)be[2] << 32) | be[3] : 0ull;
    const uint64_t le0 = ((uint64_t)le[1] << 32) | le[0];
    const uint64_t le1 = NW > 8 ? ((uint64_t)le[3] << 32) | le[2] : 0ull;
    const uint64_t km = (k >= 64) ? ~0ull : ((1ull << k) - 1);
    const int ksh = 64 - 2 * k;
    uint32_t valid = 0;
#pragma unroll
    for (int j = 0; j < EI; j++) {
        const int o = dl + j;  // < 32
        const uint64_t t = o ? (be0 << (2 * o)) | (be1 >> (64 - 2 * o)) : be0;
        const uint64_t fwd = t >> ksh;
        const uint64_t u = o ? (le0 >> (2 * o)) | (le1 << (64 - 2 * o)) : le0;
        const uint64_t rc = (u & mask) ^ mask;
        if (CANON) {
            kf[j] = fwd < rc ? fwd : rc;
            if (CANON == 2) kf[j] = mix_key(kf[j], k);
        } else {
            kf[j] = fwd;
            kr[j] = rc;
        }
        if constexpr (ALIGN == 4 || EI > 16) {
            const bool ok = !((inv >> o) & km) && !((rst >> (o + 1)) & (km >> 1)) && p0 + j < n_bases;
            valid |= (uint32_t)ok << j;
        }
    }
    if constexpr (ALIGN > 4 && EI <= 16) {
        // (window j at code j: the validity of all EI windows bit-parallel,
        // as roll_top below -- an OR over a (k-1)-wide window of flags)
        valid = rf_valid_bits<EI>(inv, inv | rst, k, p0, n_bases);
    }
    return valid;
}

// Only the top 8 key bits (the region passes' bucket) of each window, and
// its validity -- what the shard histogram counts: bf[j] = the window's first
// four codes (the forward key's top byte), br[j] (RC) = the reverse
// complement's top byte (the complements of its last four codes, the last
// one highest); validity by rf_valid_bits.  base is a multiple of 4 and of
// ALIGN (window j starts at code j of the thread's words); k >= 4 (a key of
// 8 bits or more).
template <int EI, bool RC, int ALIGN>
KMAN_RF_HD uint32_t roll_top(const uint8_t *s, int base, int k, uint64_t p0, uint64_t n_bases,
                             uint32_t (&bf)[EI], uint32_t (&br)[EI]) {
    static_assert(ALIGN == 4 || ALIGN == 8 || ALIGN == 16, "4-, 8- or 16-byte word reads");
    static_assert(EI % 4 == 0 && EI <= 16, "windows start at word boundaries, within 64 flag bits");
    constexpr int NW = (31 + EI + 3) / 4;  // codes 0 .. EI + 30
    constexpr int AW = ALIGN / 4;
    uint32_t w[(NW + AW - 1) / AW * AW];
    const uint32_t *p = reinterpret_cast<const uint32_t *>(s + base);
#pragma unroll
    for (int q = 0; q < (NW + AW - 1) / AW; q++) {
        uint32_t v[AW];
        __builtin_memcpy(v, __builtin_assume_aligned(p + AW * q, ALIGN), ALIGN);
#pragma unroll
        for (int e = 0; e < AW; e++) w[AW * q + e] = v[e];
    }
    uint64_t inv = 0, y = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        inv |= (uint64_t)rf_bit4(w[i], 2) << (4 * i);
        y |= (uint64_t)rf_bit4(w[i] | (w[i] >> 1), 2) << (4 * i);
    }
    // forward: codes 0 .. EI + 2 as a big-endian 2-bit stream
    constexpr int NF = (EI + 3 + 3) / 4;
    uint64_t be = 0;
#pragma unroll
    for (int i = 0; i < NF; i++) be |= (uint64_t)rf_be8(w[i]) << (56 - 8 * i);
#pragma unroll
    for (int j = 0; j < EI; j++) bf[j] = (uint32_t)(be >> (56 - 2 * j)) & 0xffu;
    if constexpr (RC) {
        // codes 0 .. 63 as a little-endian 2-bit stream le0:le1; window j's
        // last four codes start at code j + k - 4
        uint64_t le0 = 0, le1 = 0;
#pragma unroll
        for (int i = 0; i < NW; i++) {
            if (i < 8) le0 |= (uint64_t)rf_le8(w[i]) << (8 * i);
            else le1 |= (uint64_t)rf_le8(w[i]) << (8 * (i - 8));
        }
#pragma unroll
        for (int j = 0; j < EI; j++) {
            const int sh = 2 * (j + k - 4);  // 0 .. 86
            const uint64_t u = sh >= 64 ? le1 >> (sh - 64) : sh ? (le0 >> sh) | (le1 << (64 - sh)) : le0;
            br[j] = ~(uint32_t)u & 0xffu;
        }
    }
    return rf_valid_bits<EI>(inv, y, k, p0, n_bases);
}
