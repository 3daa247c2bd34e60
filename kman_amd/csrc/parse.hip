// parse.hip — FASTA text -> cleaned base codes + record table, on the GPU.
//
// Restates SmartFastaParser.parse (kmermaid/parsers.py:86-128) byte-parallel:
//   * the file is read in text mode, so "\n", "\r\n" and a lone "\r" end a line
//     (universal newlines);
//   * lines before the first line that starts with '>' are skipped
//     (__skip_blank_and_comments, parsers.py:43-56); no such line at all ->
//     AssertionError("premature end of file or empty file") (parsers.py:105-107);
//   * a line starting with '>' opens a record; every other line is a sequence
//     line whose content is line.rstrip() (parsers.py:72), joined, with " " and
//     "\r" removed (parsers.py:114).
//
// Per byte the only non-local facts are (a) which kind of line it sits in,
// which depends on bytes to its left, and (b) for the rare non-space
// whitespace chars (\t \v \f \x1c-\x1f), whether a non-whitespace char follows
// later in the same line (rstrip).  (a) is a scan over a 3-state machine
//   PRE (no header seen yet) / HDR (inside a header line) / SEQ (sequence line)
// whose per-chunk summary is a transformer "incoming state -> (outgoing state,
// kept chars)"; transformers compose associatively, so the whole file is
// parsed with a reduce -> two-level scan -> downsweep over 16 KiB tiles.  (b) is resolved
// right-to-left inside each thread's 64-byte chunk plus, only when a chunk
// ends inside a whitespace run, a forward probe past the chunk.
//
// Memory traffic: the text is read twice (reduce + downsweep), codes written
// once: 3 B per input byte (algorithmic bytes in DESIGN.md).
#include "common.h"

namespace {

constexpr int PT = 256;           // threads per tile
constexpr int PB = 64;            // bytes per thread
constexpr int PTILE = PT * PB;    // 16 KiB per tile
constexpr int SCAN_T = 1024;      // tiles per block of the two-level tile scan
constexpr uint32_t XF_ID_OUTS = 0u | (1u << 2) | (2u << 4);

enum : uint32_t { S_PRE = 0, S_HDR = 1, S_SEQ = 2 };

struct Xf {  // 3-state transformer over a thread chunk (counts fit 32 bits)
    uint32_t outs;
    uint32_t kept[3];
    uint32_t nhdr;
};
struct Xf64 {  // the same over tiles / tile ranges
    uint32_t outs;
    uint32_t pad;
    uint64_t kept[3];
    uint64_t nhdr;
};
struct TileIn {  // concrete state entering a tile
    uint64_t kept;
    uint64_t nhdr;
    uint32_t state;
};

KMAN_DEV uint32_t xf_out(uint32_t outs, uint32_t s) { return (outs >> (2 * s)) & 3u; }
// select without runtime array indexing (which would go to scratch)
template <typename T>
KMAN_DEV T sel3(const T (&a)[3], uint32_t s) { return s == 0 ? a[0] : (s == 1 ? a[1] : a[2]); }

struct ComposeXf {
    KMAN_DEV Xf operator()(const Xf &a, const Xf &b) const {
        Xf r;
        r.outs = 0;
#pragma unroll
        for (uint32_t s = 0; s < 3; s++) {
            const uint32_t m = xf_out(a.outs, s);
            r.outs |= xf_out(b.outs, m) << (2 * s);
            r.kept[s] = a.kept[s] + sel3(b.kept, m);
        }
        r.nhdr = a.nhdr + b.nhdr;
        return r;
    }
};
struct ComposeXf64 {
    KMAN_DEV Xf64 operator()(const Xf64 &a, const Xf64 &b) const {
        Xf64 r;
        r.outs = 0;
        r.pad = 0;
#pragma unroll
        for (uint32_t s = 0; s < 3; s++) {
            const uint32_t m = xf_out(a.outs, s);
            r.outs |= xf_out(b.outs, m) << (2 * s);
            r.kept[s] = a.kept[s] + sel3(b.kept, m);
        }
        r.nhdr = a.nhdr + b.nhdr;
        return r;
    }
};

KMAN_DEV bool is_term(uint32_t c) { return c == '\n' || c == '\r'; }
// Python str.isspace() over ASCII: what str.rstrip() strips.
KMAN_DEV bool py_space(uint32_t c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }
// whitespace that is kept unless it is trailing (terminators and ' ' never kept)
KMAN_DEV bool exotic_ws(uint32_t c) { return c == 9 || c == 11 || c == 12 || (c >= 0x1c && c <= 0x1f); }

// A thread's 64-byte chunk of the text, reduced to bit masks (bit i = byte i).
// Bytes are kept in 16 registers and only ever indexed at compile time.
struct Chunk {
    uint32_t w[PB / 4];
    int cnt;
    uint64_t ls;     // byte starts a line (universal newlines)
    uint64_t hls;    // byte starts a header line ('>' at a line start)
    uint64_t keep;   // content byte (not a terminator, not ' ', not trailing ws)
    uint64_t hdr;    // byte lies in a header line
};

KMAN_DEV uint32_t byte_at(const uint32_t (&w)[PB / 4], int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xffu; }

// SWAR byte tests on 4 packed bytes: 0x80 in every byte equal to zero
KMAN_DEV uint32_t zero_bytes(uint32_t t) { return ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t | 0x7f7f7f7fu); }
KMAN_DEV uint32_t eq_bytes(uint32_t w, uint32_t c) { return zero_bytes(w ^ (c * 0x01010101u)); }
// the 0x80 bits of four bytes -> a 4-bit mask
KMAN_DEV uint32_t hibits4(uint32_t m) {
    m >>= 7;
    return (m | (m >> 7) | (m >> 14) | (m >> 21)) & 0xfu;
}
// base codes of four bytes (A/a 0, C/c 1, G/g 2, T/t 3, else 4): (c >> 1) & 3
// maps A C T G to 0 1 2 3, x ^ (x >> 1) swaps the last two
KMAN_DEV uint32_t codes4(uint32_t w) {
    const uint32_t x = (w >> 1) & 0x03030303u;
    const uint32_t code = x ^ ((x >> 1) & 0x01010101u);
    const uint32_t y = w | 0x20202020u;
    const uint32_t ok = eq_bytes(y, 'a') | eq_bytes(y, 'c') | eq_bytes(y, 'g') | eq_bytes(y, 't');
    return (code & ((ok >> 7) * 3u)) | ((~ok & 0x80808080u) >> 5);
}
KMAN_DEV uint64_t bits_from(int i) { return i >= 64 ? 0ull : (~0ull << i); }
KMAN_DEV uint64_t bits_below(int i) { return i >= 64 ? ~0ull : ((1ull << i) - 1); }

KMAN_DEV void load_chunk(const uint8_t *text, uint64_t n, uint64_t pos, Chunk &ch) {
    ch.cnt = pos < n ? (int)((n - pos) < (uint64_t)PB ? (n - pos) : (uint64_t)PB) : 0;
    if (ch.cnt == PB) {
        const uint4 *p = reinterpret_cast<const uint4 *>(text + pos);
#pragma unroll
        for (int v = 0; v < PB / 16; v++) {
            const uint4 x = p[v];
            ch.w[4 * v + 0] = x.x;
            ch.w[4 * v + 1] = x.y;
            ch.w[4 * v + 2] = x.z;
            ch.w[4 * v + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < PB / 4; q++) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int i = 4 * q + b;
                v |= (i < ch.cnt ? (uint32_t)text[pos + i] : 0u) << (8 * b);
            }
            ch.w[q] = v;
        }
    }
    // position 0 starts a line; a chunk wholly past the end reads nothing (its
    // byte before may lie past the allocation)
    const uint32_t prev = pos == 0 ? '\n' : (pos <= n ? text[pos - 1] : 0u);
    if (ch.cnt == PB) {
        // fast path (plain sequence text): no byte below 0x21 except '\n' and
        // no '>'; then only newlines matter and every other byte is content
        uint32_t spec = 0;
        uint64_t nl = 0;
#pragma unroll
        for (int v = 0; v < PB / 4; v++) {
            const uint32_t w = ch.w[v];
            const uint32_t znl = eq_bytes(w, '\n');
            const uint32_t lt21 = ~((w & 0x7f7f7f7fu) + 0x5f5f5f5fu) & ~w & 0x80808080u;
            spec |= (lt21 & ~znl) | eq_bytes(w, '>');
            nl |= (uint64_t)hibits4(znl) << (4 * v);
        }
        if (!spec) {
            const uint64_t ls0 = (prev == '\n' || (prev == '\r' && !(nl & 1ull))) ? 1ull : 0ull;
            ch.ls = (nl << 1) | ls0;
            ch.hls = 0;
            ch.keep = ~nl;
            ch.hdr = 0;
            return;
        }
    }
    uint64_t keep = 0, ls = 0, gt = 0, exo = 0, term = 0, nonws = 0;
    uint32_t pc = prev;
#pragma unroll
    for (int i = 0; i < PB; i++) {
        const uint32_t c = byte_at(ch.w, i);
        const uint64_t in = i < ch.cnt;
        ls |= (in & (uint64_t)(pc == '\n' || (pc == '\r' && c != '\n'))) << i;
        keep |= (in & (uint64_t)!(c == '\n' || c == '\r' || c == ' ')) << i;
        gt |= (uint64_t)(c == '>') << i;
        exo |= (in & (uint64_t)exotic_ws(c)) << i;
        term |= (uint64_t)is_term(c) << i;
        nonws |= (uint64_t)!py_space(c) << i;
        pc = c;
    }
    if (exo) {
        // rstrip: an exotic whitespace byte survives only if a non-whitespace
        // byte follows it in the same line (possibly beyond this chunk).
        bool later = false;
        for (uint64_t j = pos + ch.cnt; j < n; j++) {
            const uint32_t c = text[j];
            if (is_term(c)) break;
            if (!py_space(c)) {
                later = true;
                break;
            }
        }
#pragma unroll
        for (int i = PB - 1; i >= 0; i--) {
            if (i < ch.cnt) {
                if (((exo >> i) & 1ull) && !later) keep &= ~(1ull << i);
                if ((term >> i) & 1ull) later = false;
                else if ((nonws >> i) & 1ull) later = true;
            }
        }
    }
    // bytes of header lines: from each header line start to the next line start
    const uint64_t hls = ls & gt;
    uint64_t hdr = 0;
    for (uint64_t m = hls; m; m &= m - 1) {
        const int h = __ffsll((unsigned long long)m) - 1;
        const uint64_t after = ls & bits_from(h + 1);
        const int nx = after ? __ffsll((unsigned long long)after) - 1 : 64;
        hdr |= bits_from(h) & bits_below(nx);
    }
    ch.ls = ls;
    ch.hls = hls;
    ch.keep = keep;
    ch.hdr = hdr;
}

// The fast path alone (plain sequence text, a full chunk): false when the
// chunk needs load_chunk (then its whole tile goes to the SLOW kernels).
// Kept apart so the common kernels carry none of the general path's registers.
KMAN_DEV bool load_chunk_fast(const uint8_t *text, uint64_t n, uint64_t pos, Chunk &ch) {
    ch.cnt = pos < n ? (int)((n - pos) < (uint64_t)PB ? (n - pos) : (uint64_t)PB) : 0;
    if (ch.cnt != PB) return false;
    const uint4 *p = reinterpret_cast<const uint4 *>(text + pos);
#pragma unroll
    for (int v = 0; v < PB / 16; v++) {
        const uint4 x = p[v];
        ch.w[4 * v + 0] = x.x;
        ch.w[4 * v + 1] = x.y;
        ch.w[4 * v + 2] = x.z;
        ch.w[4 * v + 3] = x.w;
    }
    const uint32_t prev = pos == 0 ? '\n' : text[pos - 1];
    uint32_t spec = 0;
    uint64_t nl = 0;
#pragma unroll
    for (int v = 0; v < PB / 4; v++) {
        const uint32_t w = ch.w[v];
        const uint32_t znl = eq_bytes(w, '\n');
        const uint32_t lt21 = ~((w & 0x7f7f7f7fu) + 0x5f5f5f5fu) & ~w & 0x80808080u;
        spec |= (lt21 & ~znl) | eq_bytes(w, '>');
        nl |= (uint64_t)hibits4(znl) << (4 * v);
    }
    if (spec) return false;
    const uint64_t ls0 = (prev == '\n' || (prev == '\r' && !(nl & 1ull))) ? 1ull : 0ull;
    ch.ls = (nl << 1) | ls0;
    ch.hls = 0;
    ch.keep = ~nl;
    ch.hdr = 0;
    return true;
}

// content bytes that land in the cleaned sequence, per incoming state
struct Emit {
    uint64_t lead;  // bytes before the first line start (kept iff incoming SEQ)
    uint64_t mid;   // non-header lines before the first header (kept iff incoming != PRE)
    uint64_t all;   // non-header lines after a header (always kept)
};

KMAN_DEV Emit chunk_emit(const Chunk &ch) {
    const int F = ch.ls ? __ffsll((unsigned long long)ch.ls) - 1 : 64;
    const int H = ch.hls ? __ffsll((unsigned long long)ch.hls) - 1 : 64;
    const uint64_t body = ch.keep & ~ch.hdr;
    Emit e;
    e.lead = ch.keep & bits_below(F);
    e.mid = body & bits_from(F) & bits_below(H);
    e.all = body & bits_from(H);
    return e;
}

KMAN_DEV uint64_t emit_mask(const Emit &e, uint32_t s) {
    return e.all | (s != S_PRE ? e.mid : 0ull) | (s == S_SEQ ? e.lead : 0ull);
}

KMAN_DEV Xf chunk_xf(const Chunk &ch) {
    const Emit e = chunk_emit(ch);
    Xf x;
    x.kept[S_PRE] = __popcll(e.all);
    x.kept[S_HDR] = __popcll(e.all | e.mid);
    x.kept[S_SEQ] = __popcll(e.all | e.mid | e.lead);
    x.nhdr = __popcll(ch.hls);
    if (!ch.ls) {
        x.outs = XF_ID_OUTS;
    } else {
        const int L = 63 - __clzll((unsigned long long)ch.ls);
        if ((ch.hls >> L) & 1ull) {
            x.outs = S_HDR | (S_HDR << 2) | (S_HDR << 4);
        } else if (ch.hls) {
            x.outs = S_SEQ | (S_SEQ << 2) | (S_SEQ << 4);
        } else {
            x.outs = S_PRE | (S_SEQ << 2) | (S_SEQ << 4);
        }
    }
    return x;
}

// Two variants: !SLOW, one block per tile, handles the tiles of plain
// sequence text (every chunk on the fast path) and lists the others (pad = 1,
// slow[1 + i]; slow[0] = how many); SLOW walks only that list with the general
// per-byte path ((PT, 3): three waves per SIMD, 168 VGPRs, a few spilled).
template <bool SLOW>
__global__ __launch_bounds__(PT, 3) void parse_reduce(const uint8_t *__restrict__ text, uint64_t n,
                                                   Xf64 *__restrict__ tiles, uint32_t *__restrict__ slow) {
    __shared__ Xf lds[PT / 64];
    const uint32_t nit = SLOW ? slow[0] : 1u;
    for (uint32_t it = SLOW ? blockIdx.x : 0u; it < nit; it += SLOW ? gridDim.x : 1u) {
    const uint32_t tb = SLOW ? slow[1 + it] : blockIdx.x;
    const uint64_t pos = (uint64_t)tb * PTILE + (uint64_t)threadIdx.x * PB;
    Chunk ch;
    if (SLOW) {
        load_chunk(text, n, pos, ch);
    } else {
        const bool fast = load_chunk_fast(text, n, pos, ch);
        if (__syncthreads_or(!fast)) {  // (block-uniform) a tile for the SLOW variant
            if (threadIdx.x == 0) {
                tiles[tb].pad = 1;
                slow[1 + atomicAdd(&slow[0], 1u)] = tb;
            }
            return;
        }
    }
    Xf x = chunk_xf(ch);
    Xf id;
    id.outs = XF_ID_OUTS;
    id.kept[0] = id.kept[1] = id.kept[2] = 0;
    id.nhdr = 0;
    Xf tot;
    block_exclusive_scan<PT>(x, ComposeXf(), id, lds, &tot);
    if (threadIdx.x == 0) {
        Xf64 t;
        t.outs = tot.outs;
        t.pad = SLOW ? 1u : 0u;  // (keeps the flag for parse_emit)
        for (int s = 0; s < 3; s++) t.kept[s] = tot.kept[s];
        t.nhdr = tot.nhdr;
        tiles[tb] = t;
    }
    __syncthreads();  // (lds is the next listed tile's)
    }
}

KMAN_DEV Xf64 xf64_id() {
    Xf64 id;
    id.outs = XF_ID_OUTS;
    id.pad = 0;
    id.kept[0] = id.kept[1] = id.kept[2] = 0;
    id.nhdr = 0;
    return id;
}

// Tile scan, level 1: SCAN_T tiles per block -> each tile's exclusive prefix
// inside its block, and the block's total.
__global__ __launch_bounds__(SCAN_T) void parse_scan_blocks(const Xf64 *__restrict__ tiles, uint64_t T,
                                                            Xf64 *__restrict__ local, Xf64 *__restrict__ btot) {
    __shared__ Xf64 lds[SCAN_T / 64];
    const uint64_t t = (uint64_t)blockIdx.x * SCAN_T + threadIdx.x;
    const Xf64 id = xf64_id();
    const Xf64 x = t < T ? tiles[t] : id;
    Xf64 tot;
    const Xf64 ex = block_exclusive_scan<SCAN_T>(x, ComposeXf64(), id, lds, &tot);
    if (t < T) local[t] = ex;
    if (threadIdx.x == 0) btot[blockIdx.x] = tot;
}

// Level 2 (one block): exclusive prefixes of the block totals, and the file
// totals (n_bases, n_records).
__global__ __launch_bounds__(SCAN_T) void parse_scan_top(const Xf64 *__restrict__ btot, uint64_t NB,
                                                         Xf64 *__restrict__ bpre, uint64_t *__restrict__ info,
                                                         uint32_t s0) {
    __shared__ Xf64 lds[SCAN_T / 64];
    const Xf64 id = xf64_id();
    ComposeXf64 op;
    Xf64 carry = id;
    for (uint64_t b0 = 0; b0 < NB; b0 += SCAN_T) {
        const uint64_t b = b0 + threadIdx.x;
        const Xf64 x = b < NB ? btot[b] : id;
        Xf64 tot;
        const Xf64 ex = block_exclusive_scan<SCAN_T>(x, op, id, lds, &tot);
        if (b < NB) bpre[b] = op(carry, ex);
        carry = op(carry, tot);
    }
    if (threadIdx.x == 0) {
        info[0] = s0 == S_PRE ? carry.kept[S_PRE] : carry.kept[S_SEQ];  // n_bases
        info[1] = carry.nhdr;         // n_records
    }
}

// the same split: the tiles parse_reduce<false> listed take SLOW
template <bool SLOW>
__global__ __launch_bounds__(PT, 3) void parse_emit(const uint8_t *__restrict__ text, uint64_t n,
                                                 const Xf64 *__restrict__ tiles, const uint32_t *__restrict__ slow,
                                                 const Xf64 *__restrict__ local, const Xf64 *__restrict__ bpre,
                                                 uint8_t *__restrict__ codes, uint64_t code_off, uint32_t s0,
                                                 uint64_t *__restrict__ rec_hdr, uint64_t *__restrict__ rec_seq) {
    __shared__ Xf lds[PT / 64];
    __shared__ __attribute__((aligned(16))) uint8_t stage[PTILE + 32];
    const uint32_t nit = SLOW ? slow[0] : 1u;
    for (uint32_t it = SLOW ? blockIdx.x : 0u; it < nit; it += SLOW ? gridDim.x : 1u) {
    const uint32_t tb = SLOW ? slow[1 + it] : blockIdx.x;
    if (!SLOW && tiles[tb].pad != 0) return;  // (block-uniform) a listed tile
    const uint64_t pos = (uint64_t)tb * PTILE + (uint64_t)threadIdx.x * PB;
    Chunk ch;
    if (SLOW) load_chunk(text, n, pos, ch);
    else (void)load_chunk_fast(text, n, pos, ch);
    const Xf x = chunk_xf(ch);
    Xf id;
    id.outs = XF_ID_OUTS;
    id.kept[0] = id.kept[1] = id.kept[2] = 0;
    id.nhdr = 0;
    Xf tot;
    const Xf pre = block_exclusive_scan<PT>(x, ComposeXf(), id, lds, &tot);
    // the concrete state entering this tile: the file prefix applied to PRE
    TileIn ti;
    {
        const Xf64 p = ComposeXf64()(bpre[tb / SCAN_T], local[tb]);
        ti.state = xf_out(p.outs, s0);
        ti.kept = s0 == S_PRE ? p.kept[S_PRE] : p.kept[S_SEQ];
        ti.nhdr = p.nhdr;
    }
    const uint32_t s = xf_out(pre.outs, ti.state);  // state entering this thread's chunk
    const uint32_t lk0 = ti.state == 0 ? pre.kept[0] : (ti.state == 1 ? pre.kept[1] : pre.kept[2]);        // tile-local kept offset of this thread
    const uint64_t nh0 = ti.nhdr + pre.nhdr;
    const uint32_t tile_kept = ti.state == 0 ? tot.kept[0] : (ti.state == 1 ? tot.kept[1] : tot.kept[2]);
    const uint64_t em = emit_mask(chunk_emit(ch), s);
    // records opened in this chunk: '>' offset and the global index of the next kept char
    {
        uint64_t nh = nh0;
        for (uint64_t m = ch.hls; m; m &= m - 1) {
            const int h = __ffsll((unsigned long long)m) - 1;
            rec_hdr[nh] = pos + h;
            rec_seq[nh] = code_off + ti.kept + lk0 + __popcll(em & bits_below(h));
            nh++;
        }
    }
    // codes staged at the tile's output alignment, so LDS and HBM agree mod 16
    // (codes holds 16-byte aligned memory; this call writes from code_off on)
    const uint32_t al = (uint32_t)((code_off + ti.kept) & 15u);
    uint32_t cw[PB / 4];
#pragma unroll
    for (int v = 0; v < PB / 4; v++) cw[v] = codes4(ch.w[v]);
    uint32_t lk = al + lk0;
    if (!SLOW && __popcll(~em) <= 8) {
        // the chunk's kept codes compacted in registers (each dropped byte --
        // a newline, mostly -- shifts the bytes above it down), then written
        // as whole LDS words, bytewise only where a word is shared with the
        // neighbouring chunks: 17 word stores instead of 64 byte stores
        // whose lanes, 64 bytes apart, all hit a few banks
        uint64_t rmv = ~em;
        while (rmv) {
            const int p = 63 - __clzll((unsigned long long)rmv);
            rmv &= ~(1ull << p);
            const int q = p >> 2;
            const uint32_t lowm = (1u << (8 * (p & 3))) - 1u;
#pragma unroll
            for (int i = 0; i < PB / 4; i++) {
                const uint32_t nxt = i + 1 < PB / 4 ? cw[i + 1] : 0u;
                const uint32_t sh = (cw[i] >> 8) | (nxt << 24);
                cw[i] = i < q ? cw[i] : (i == q ? ((cw[i] & lowm) | (sh & ~lowm)) : sh);
            }
        }
        const uint32_t e = lk + (uint32_t)__popcll(em), sa = lk & 3u, a0 = lk >> 2;
        uint32_t *st32 = reinterpret_cast<uint32_t *>(stage);
#pragma unroll
        for (int j = 0; j <= PB / 4; j++) {
            const uint32_t lo = j ? cw[j - 1] : 0u, hi = j < PB / 4 ? cw[j] : 0u;
            const uint32_t word = sa ? ((hi << (8 * sa)) | (lo >> (32 - 8 * sa))) : hi;
            const uint32_t wb = 4 * (a0 + (uint32_t)j);
            const uint32_t b0 = wb > lk ? wb : lk, b1 = wb + 4 < e ? wb + 4 : e;
            if (b0 >= b1) continue;
            if (b0 == wb && b1 == wb + 4) {
                st32[a0 + j] = word;
            } else {
                for (uint32_t b = b0; b < b1; b++) stage[b] = (uint8_t)(word >> (8 * (b - wb)));
            }
        }
    } else if (em == ~0ull) {
#pragma unroll
        for (int i = 0; i < PB; i++) stage[lk + i] = (uint8_t)byte_at(cw, i);
    } else {
#pragma unroll
        for (int i = 0; i < PB; i++) {
            if ((em >> i) & 1ull) stage[lk++] = (uint8_t)byte_at(cw, i);
        }
    }
    __syncthreads();
    // [al, al + tile_kept) of stage -> codes + ti.kept: whole 16-byte words as
    // vectors, the two partial end words (shared with the neighbour tiles) bytewise
    uint8_t *dst = codes + (code_off + ti.kept - al);
    const uint32_t end = al + tile_kept;
    const uint32_t nwords = (end + 15) / 16;
    for (uint32_t q = threadIdx.x; q < nwords; q += PT) {
        const uint32_t b0 = q * 16;
        if (b0 >= al && b0 + 16 <= end) {
            *reinterpret_cast<uint4 *>(dst + b0) = *reinterpret_cast<const uint4 *>(stage + b0);
        } else {
            for (uint32_t b = b0; b < b0 + 16; b++)
                if (b >= al && b < end) dst[b] = stage[b];
        }
    }
    __syncthreads();  // (lds and stage are the next listed tile's)
    }
}

// bit 3 on the first code of every non-empty record
__global__ void mark_records(uint8_t *__restrict__ codes, const uint64_t *__restrict__ rec_seq, uint64_t R,
                             uint64_t n_bases) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < R) {
        const uint64_t p = rec_seq[r];
        if (p < n_bases) codes[p] |= 8;
    }
}

}  // namespace

extern "C" int kman_parse_fasta(kman_ctx *ctx, const uint8_t *d_text, uint64_t n_bytes, uint8_t *d_codes,
                                uint64_t *d_rec_hdr, uint64_t *d_rec_seq, uint64_t rec_cap,
                                kman_parse_info *info) {
    return kman_parse_fasta_at(ctx, d_text, n_bytes, 0, d_codes, 0, d_rec_hdr, d_rec_seq, rec_cap, info);
}

extern "C" int kman_parse_fasta_at(kman_ctx *ctx, const uint8_t *d_text, uint64_t n_bytes, uint32_t flags,
                                   uint8_t *d_codes, uint64_t code_off, uint64_t *d_rec_hdr, uint64_t *d_rec_seq,
                                   uint64_t rec_cap, kman_parse_info *info) {
    if (!ctx || !info) return KMAN_EINVAL;
    info->n_bases = info->n_records = 0;
    const bool cont = flags & KMAN_PARSE_IN_RECORD;
    // a continuation chunk (inside a record) may be empty or hold no header
    if (cont && n_bytes == 0) return KMAN_OK;
    if (n_bytes && (!d_text || !d_codes)) return kman_fail(ctx, KMAN_EINVAL, "null buffer");
    if (((uintptr_t)d_text & 15) != 0) return kman_fail(ctx, KMAN_EINVAL, "text must be 16-byte aligned");
    if (((uintptr_t)d_codes & 15) != 0) return kman_fail(ctx, KMAN_EINVAL, "codes must be 16-byte aligned");
    const uint32_t s0 = cont ? S_SEQ : S_PRE;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t T = n_bytes ? ceil_div(n_bytes, PTILE) : 0;
    if (T == 0) return kman_fail(ctx, KMAN_EFORMAT, "premature end of file or empty file");
    // scratch: tile transformers, their in-block prefixes, block totals and
    // prefixes (Xf64 each), info
    const uint64_t NB = ceil_div(T, (uint64_t)SCAN_T);
    const size_t xf_bytes = ((T * sizeof(Xf64)) + 255) & ~size_t(255);
    const size_t nb_bytes = ((NB * sizeof(Xf64)) + 255) & ~size_t(255);
    void *scr;
    const size_t sl_bytes = ((4 * (T + 1)) + 255) & ~size_t(255);
    KMAN_TRY(kman_scratch(ctx, 2 * xf_bytes + 2 * nb_bytes + 256 + sl_bytes, &scr));
    Xf64 *d_xf = (Xf64 *)scr;
    Xf64 *d_local = (Xf64 *)((char *)scr + xf_bytes);
    Xf64 *d_btot = (Xf64 *)((char *)scr + 2 * xf_bytes);
    Xf64 *d_bpre = (Xf64 *)((char *)scr + 2 * xf_bytes + nb_bytes);
    uint64_t *d_info = (uint64_t *)((char *)scr + 2 * xf_bytes + 2 * nb_bytes);
    uint32_t *d_slow = (uint32_t *)((char *)scr + 2 * xf_bytes + 2 * nb_bytes + 256);  // [count, tiles...]
    const uint32_t gslow = (uint32_t)(T < 2048 ? T : 2048);  // (blocks walking the listed tiles)
    { KTimer kt_(ctx, "parse");
    HIP_TRY(ctx, hipMemsetAsync(d_xf, 0, T * sizeof(Xf64), ctx->stream));  // (pad = 0: not listed)
    HIP_TRY(ctx, hipMemsetAsync(d_slow, 0, 4, ctx->stream));
    hipLaunchKernelGGL(parse_reduce<false>, dim3((uint32_t)T), dim3(PT), 0, ctx->stream, d_text, n_bytes, d_xf, d_slow);
    hipLaunchKernelGGL(parse_reduce<true>, dim3(gslow), dim3(PT), 0, ctx->stream, d_text, n_bytes, d_xf, d_slow);
    hipLaunchKernelGGL(parse_scan_blocks, dim3((uint32_t)NB), dim3(SCAN_T), 0, ctx->stream, d_xf, T, d_local, d_btot);
    hipLaunchKernelGGL(parse_scan_top, dim3(1), dim3(SCAN_T), 0, ctx->stream, d_btot, NB, d_bpre, d_info, s0); }
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_small, d_info, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    info->n_bases = ctx->h_small[0];
    info->n_records = ctx->h_small[1];
    if (info->n_records == 0 && !cont) return kman_fail(ctx, KMAN_EFORMAT, "premature end of file or empty file");
    if (info->n_records > rec_cap)
        return kman_fail(ctx, KMAN_ECAP, "record capacity %llu < %llu", (unsigned long long)rec_cap,
                         (unsigned long long)info->n_records);
    { KTimer kt_(ctx, "parse");
    hipLaunchKernelGGL(parse_emit<false>, dim3((uint32_t)T), dim3(PT), 0, ctx->stream, d_text, n_bytes, d_xf, d_slow,
                       d_local, d_bpre, d_codes, code_off, s0, d_rec_hdr, d_rec_seq);
    hipLaunchKernelGGL(parse_emit<true>, dim3(gslow), dim3(PT), 0, ctx->stream, d_text, n_bytes, d_xf, d_slow,
                       d_local, d_bpre, d_codes, code_off, s0, d_rec_hdr, d_rec_seq);
    const uint64_t R = info->n_records;
    if (R)
        hipLaunchKernelGGL(mark_records, dim3((uint32_t)ceil_div(R, 256)), dim3(256), 0, ctx->stream, d_codes,
                           d_rec_seq, R, code_off + info->n_bases); }
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemsetAsync(d_codes + code_off + info->n_bases, 4, 64, ctx->stream));
    return KMAN_OK;
}
