// Host check of kman_amd/csrc/rollfast.h against a per-base roll (the
// semantics of kmer.h's roll(): Sequence.yield_kmers, kmermaid/seq.py:285-328).
// Built and run by tests/test_rollfast.py; prints "ok N" or the first mismatch.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../kman_amd/csrc/rollfast.h"

template <int EI, bool CANON>
static uint32_t roll_ref(const uint8_t *s, int base, int k, uint64_t mask, uint64_t p0, uint64_t n_bases,
                         uint64_t (&kf)[EI], uint64_t (&kr)[EI]) {
    uint32_t valid = 0;
    for (int j = 0; j < EI; j++) {
        uint64_t f = 0, r = 0;
        bool ok = p0 + j < n_bases;
        for (int q = 0; q < k; q++) {
            const uint32_t c = s[base + j + q];
            if (c & 4) ok = false;
            if (q > 0 && (c & 8)) ok = false;
            f = (f << 2) | (c & 3);
            r |= (uint64_t)(3 - (c & 3)) << (2 * q);
        }
        f &= mask;
        if (CANON) {
            kf[j] = f < r ? f : r;
        } else {
            kf[j] = f;
            kr[j] = r;
        }
        valid |= (uint32_t)ok << j;
    }
    return valid;
}

// A: the word-read width roll() picks for base = thread * EI (16- / 8-byte
// vectors when EI is a multiple of 16 / 8), or 4 (any base)
template <int EI, bool CANON, int A = 4>
static int check(std::mt19937_64 &g, long &n) {
    alignas(16) uint8_t s[4096 + 128];
    for (int trial = 0; trial < 300; trial++) {
        const int mode = trial % 3;
        for (auto &c : s) {
            const uint32_t x = (uint32_t)g();
            c = (uint8_t)(x & 3);
            if (mode && (x >> 8) % (mode == 1 ? 50 : 7) == 0) c |= 4;
            if (mode && (x >> 16) % (mode == 1 ? 60 : 9) == 0) c |= 8;
        }
        for (int k = 2; k <= 32; k++) {
            const uint64_t mask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1);
            for (int t = 0; t < 64; t++) {
                const int base = t * EI;
                const uint64_t p0 = 1000 + base, nb = (trial % 5 == 0) ? p0 + (t % (EI + 1)) : ~0ull;
                uint64_t a[EI], b[EI], c[EI], d[EI];
                memset(b, 0, sizeof b);
                memset(d, 0, sizeof d);
                const uint32_t va = roll_fast<EI, CANON, A>(s, base, k, mask, p0, nb, a, b);
                const uint32_t vb = roll_ref<EI, CANON>(s, base, k, mask, p0, nb, c, d);
                if (va != vb) {
                    printf("valid mismatch EI=%d canon=%d A=%d k=%d base=%d: %x vs %x\n", EI, CANON, A, k, base, va, vb);
                    return 1;
                }
                for (int j = 0; j < EI; j++) {
                    if (!((va >> j) & 1)) continue;
                    if (a[j] != c[j] || (!CANON && b[j] != d[j])) {
                        printf("key mismatch EI=%d canon=%d k=%d base=%d j=%d: %llx/%llx vs %llx/%llx\n", EI, CANON,
                               k, base, j, (unsigned long long)a[j], (unsigned long long)b[j],
                               (unsigned long long)c[j], (unsigned long long)d[j]);
                        return 1;
                    }
                    n++;
                }
            }
        }
    }
    return 0;
}

// roll_top (the shard histogram's top bytes): valid bits and the top 8 bits
// of both keys against the per-base roll, k = 4 .. 32
template <int EI, bool RC, int A>
static int check_top(std::mt19937_64 &g, long &n) {
    alignas(16) uint8_t s[4096 + 128];
    for (int trial = 0; trial < 300; trial++) {
        const int mode = trial % 3;
        for (auto &c : s) {
            const uint32_t x = (uint32_t)g();
            c = (uint8_t)(x & 3);
            if (mode && (x >> 8) % (mode == 1 ? 50 : 7) == 0) c |= 4;
            if (mode && (x >> 16) % (mode == 1 ? 60 : 9) == 0) c |= 8;
        }
        for (int k = 4; k <= 32; k++) {
            const uint64_t mask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1);
            for (int t = 0; t < 64; t++) {
                const int base = t * EI;
                const uint64_t p0 = 1000 + base, nb = (trial % 5 == 0) ? p0 + (t % (EI + 1)) : ~0ull;
                uint32_t a[EI], b[EI];
                uint64_t c[EI], d[EI];
                memset(b, 0, sizeof b);
                const uint32_t va = roll_top<EI, RC, A>(s, base, k, p0, nb, a, b);
                const uint32_t vb = roll_ref<EI, false>(s, base, k, mask, p0, nb, c, d);
                if (va != vb) {
                    printf("top valid mismatch EI=%d rc=%d A=%d k=%d base=%d: %x vs %x\n", EI, RC, A, k, base, va, vb);
                    return 1;
                }
                for (int j = 0; j < EI; j++) {
                    if (!((va >> j) & 1)) continue;
                    const uint32_t tf = (uint32_t)(c[j] >> (2 * k - 8)), tr = (uint32_t)(d[j] >> (2 * k - 8));
                    if (a[j] != tf || (RC && b[j] != tr)) {
                        printf("top mismatch EI=%d rc=%d k=%d base=%d j=%d: %x/%x vs %x/%x\n", EI, RC, k, base, j,
                               a[j], b[j], tf, tr);
                        return 1;
                    }
                    n++;
                }
            }
        }
    }
    return 0;
}

int main() {
    std::mt19937_64 g(7);
    long n = 0;
    if (check<4, false>(g, n) || check<6, false>(g, n) || check<8, false>(g, n) || check<12, false>(g, n) ||
        check<16, false>(g, n) || check<8, true>(g, n) || check<12, true>(g, n) || check<16, true>(g, n) ||
        check<8, false, 8>(g, n) || check<16, false, 16>(g, n) || check<16, false, 8>(g, n) ||
        check<16, true, 16>(g, n) || check<8, true, 8>(g, n) || check_top<16, false, 16>(g, n) ||
        check_top<16, true, 16>(g, n) || check_top<8, true, 8>(g, n) || check_top<8, false, 8>(g, n) ||
        check_top<12, false, 4>(g, n) || check_top<12, true, 4>(g, n) || check_top<4, false, 4>(g, n))
        return 1;
    printf("ok %ld\n", n);
    return 0;
}
