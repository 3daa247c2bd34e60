// kmer.h — sliding-window k-mer helpers shared by extract.hip and the fused
// extract + first-pass kernel in sort.hip (Sequence.yield_kmers,
// kmermaid/seq.py:285-328; codes from kman_parse_fasta: bits 0-1 base, bit 2
// not ACGT, bit 3 record start).
#pragma once
#include "common.h"

namespace {

// the codes of windows [tb, tb + NT*EI) plus a 64-byte halo into LDS (16-byte
// loads; past the padded end, code 4 = not ACGT)
template <int NT, int EI>
KMAN_DEV void stage_codes(const uint8_t *__restrict__ codes, uint64_t n_bases, uint64_t tb, uint8_t *s) {
    constexpr int BYTES = NT * EI + 64;
    const uint64_t limit = n_bases + 64;  // padded region is valid memory, value 4
    for (int v = threadIdx.x; v < BYTES / 16; v += NT) {
        const uint64_t off = tb + (uint64_t)v * 16;
        if (off + 16 <= limit) {
            *reinterpret_cast<uint4 *>(s + v * 16) = *reinterpret_cast<const uint4 *>(codes + off);
        } else {
#pragma unroll
            for (int b = 0; b < 16; b++) s[v * 16 + b] = (off + b < limit) ? codes[off + b] : 4;
        }
    }
}

// Roll the EI windows starting at s[base .. base+EI) (k from LDS bytes).
template <int EI, bool CANON>
KMAN_DEV uint32_t roll(const uint8_t *s, int base, int k, uint64_t mask, uint64_t p0, uint64_t n_bases,
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
        } else {
            kf[j] = fm;
            kr[j] = r;
        }
        valid |= (uint32_t)(run >= (uint32_t)k && p0 + j < n_bases) << j;
    }
    return valid;
}

}  // namespace
