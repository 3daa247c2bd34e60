"""Deterministic FASTA inputs shared by the golden generator, the tests and bench.py.

Every input is rebuilt from a seed, so only small files and the expected outputs
need to live in git.  The shapes follow SURVEY.md §8c ("golden vectors to
generate here") and §8d (synthetic generator: i.i.d. uniform ACGT, 80 columns,
records named ``syn<i>``).
"""

from __future__ import annotations

import gzip
import os
import random

import numpy as np


def wrap(seq: str, width: int = 80) -> str:
    return "".join(seq[i : i + width] + "\n" for i in range(0, len(seq), width))


def syn_python(n: int, seed: int, name: str = "syn0") -> bytes:
    """Config-1 input: ``random.seed(seed); random.choices('ACGT', k=n)``.

    This is the exact recipe BASELINE.md used for the reference CPU timings
    (1 MB, seed 42).
    """
    rng = random.Random(seed)
    seq = "".join(rng.choices("ACGT", k=n))
    return (">%s\n" % name + wrap(seq)).encode()


def syn_numpy(n_bases: int, seed: int, record_len: int = 256 << 20, width: int = 80) -> bytes:
    """SURVEY §8d generator: numpy PCG64(seed), i.i.d. uniform ACGT, 80 columns.

    Records of at most ``record_len`` bases named ``syn<i>``.  Built with numpy
    so a 1 GB input takes seconds, not minutes.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    alphabet = np.frombuffer(b"ACGT", dtype=np.uint8)
    out = []
    left = n_bases
    rec = 0
    while left > 0:
        L = min(left, record_len)
        codes = rng.integers(0, 4, size=L, dtype=np.uint8)
        bases = alphabet[codes]
        full = L // width
        tail = L - full * width
        body = np.empty(full * (width + 1) + (tail + 1 if tail else 0), dtype=np.uint8)
        if full:
            grid = body[: full * (width + 1)].reshape(full, width + 1)
            grid[:, :width] = bases[: full * width].reshape(full, width)
            grid[:, width] = ord("\n")
        if tail:
            body[full * (width + 1) : -1] = bases[full * width :]
            body[-1] = ord("\n")
        out.append((">syn%d\n" % rec).encode())
        out.append(body.tobytes())
        left -= L
        rec += 1
    return b"".join(out)


class SynthLayout:
    """The ONE global synthetic FASTA of the multi-GPU benchmark (SURVEY §8d
    config 4: byte-range sharded across ranks): records ``syn<i>`` of at most
    record_len bases in lines of ``width`` bases; base j of the file is
    "ACGT"[splitmix64(seed * 0xD1B54A32D192ED03 + j) >> 62], so any byte range
    can be generated on its own -- here (synth_np) or on the device
    (kman_synth_fasta, byte-identical)."""

    def __init__(self, n_bases: int, seed: int, record_len: int = 256 << 20, width: int = 80):
        self.n_bases, self.seed, self.width = int(n_bases), int(seed), int(width)
        lens, hb, bb = [], [], []
        at = bat = 0
        left, r = self.n_bases, 0
        while left > 0:
            L = min(left, record_len)
            hb.append(at)
            bb.append(bat)
            lens.append(L)
            at += 5 + len(str(r)) + L + (L + width - 1) // width
            bat += L
            left -= L
            r += 1
        self.size = at
        self.tab = np.array([v for t in zip(hb, bb, lens) for v in t], dtype=np.uint64)
        self.n_records = len(lens)

    def read(self, lo: int, hi: int) -> bytes:
        return synth_np(self, lo, hi)


_M64 = (1 << 64) - 1


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def synth_np(lay: "SynthLayout", lo: int, hi: int) -> bytes:
    """Bytes [lo, hi) of the global synthetic FASTA (numpy restatement of
    kman_synth_fasta)."""
    lo, hi = max(0, int(lo)), min(int(hi), lay.size)
    if hi <= lo:
        return b""
    g = np.arange(lo, hi, dtype=np.uint64)
    tab = lay.tab.reshape(-1, 3)
    r = np.searchsorted(tab[:, 0], g, side="right").astype(np.int64) - 1
    hb, bb, L = tab[r, 0], tab[r, 1], tab[r, 2]
    rel = g - hb
    nd = np.array([len(str(x)) for x in range(lay.n_records)], dtype=np.uint64)[r]
    hl = np.uint64(5) + nd
    out = np.empty(len(g), dtype=np.uint8)
    inh = rel < hl
    w = np.uint64(lay.width)
    rel2 = np.where(inh, np.uint64(0), rel - hl)
    ln, col = rel2 // (w + np.uint64(1)), rel2 % (w + np.uint64(1))
    bi = ln * w + col
    nl = (col == w) | (bi >= L)
    with np.errstate(over="ignore"):
        h = _splitmix64(np.uint64(lay.seed) * np.uint64(0xD1B54A32D192ED03) + bb + bi)
    out[:] = np.frombuffer(b"ACGT", dtype=np.uint8)[(h >> np.uint64(62)).astype(np.int64)]
    out[nl] = ord("\n")
    for j in np.nonzero(inh)[0].tolist():  # header bytes (few)
        hdr = (">syn%d\n" % int(r[j])).encode()
        out[j] = hdr[int(rel[j])]
    return out.tobytes()


def grch38_like(seed: int, n_bases: int = 1_000_000, n_records: int = 5, width: int = 60) -> bytes:
    """A GRCh38-shaped synthetic FASTA (BASELINE config 5 stand-in: GRCh38 is
    not in this container): records ``chr<i> AC:... description``, 60-column
    lines, soft-masked (lower-case) stretches, N runs (telomere / gap blocks),
    interspersed copies of a few repeat elements (~300 bp, a few % mutated)
    and tandem satellite arrays, so k-mer counts are skewed like a genome's."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    elems = [rng.integers(0, 4, size=int(rng.integers(200, 400)), dtype=np.uint8) for _ in range(4)]
    sat = rng.integers(0, 4, size=171, dtype=np.uint8)
    out = []
    per = n_bases // n_records
    for r in range(n_records):
        L = per if r + 1 < n_records else n_bases - per * (n_records - 1)
        seq = rng.integers(0, 4, size=L, dtype=np.uint8)
        # repeat copies
        for _ in range(L // 2500):
            e = elems[int(rng.integers(0, len(elems)))].copy()
            mut = rng.random(len(e)) < 0.03
            e[mut] = rng.integers(0, 4, size=int(mut.sum()), dtype=np.uint8)
            at = int(rng.integers(0, max(1, L - len(e))))
            seq[at:at + len(e)] = e[:L - at]
        # one satellite array
        n_sat = min(L // 10, 40 * len(sat))
        at = int(rng.integers(0, max(1, L - n_sat)))
        seq[at:at + n_sat] = np.tile(sat, n_sat // len(sat) + 1)[:n_sat]
        chars = acgt[seq].copy()
        # soft-masking: ~half the repeats' bases lower-case, in runs
        for _ in range(L // 5000):
            a = int(rng.integers(0, L))
            chars[a:a + int(rng.integers(50, 1500))] += 32
        # N runs: the record ends and a few gaps
        nN = min(L // 20, 1000)
        chars[:nN] = ord("N")
        chars[L - nN:] = ord("N")
        for _ in range(3):
            a = int(rng.integers(0, L))
            chars[a:a + int(rng.integers(10, 500))] = ord("N")
        out.append(b">chr%d AC:CM0006%02d.2 gi:5688%02d LN:%d rl:Chromosome M5:x AS:GRCh38\n" % (r + 1, r, r, L))
        full = L // width
        grid = np.empty((full, width + 1), dtype=np.uint8)
        grid[:, :width] = chars[:full * width].reshape(full, width)
        grid[:, width] = ord("\n")
        out.append(grid.tobytes())
        if L > full * width:
            out.append(bytes(chars[full * width:]) + b"\n")
    return b"".join(out)


def grch38_skewed(seed: int, n_bases: int = 1_000_000, n_records: int = 5, width: int = 60) -> bytes:
    """A GRCh38-shaped synthetic FASTA with a genome's repeat skew (BASELINE
    config 5 stand-in; GRCh38 itself is not in this container): besides
    grch38_like's records, soft-masking and N blocks,
      * an Alu-like family: one 300-bp consensus, a copy every ~3.1 kb (about
        a million copies over 3.1 Gbp, ~10 % of the sequence), each ~10 %
        diverged (independent substitutions), on either strand;
      * per record a tandem satellite array of min(L / 40, 3 Mbp): a 171-bp
        monomer, ~2 % diverged copy to copy (the alpha-satellite arrays of
        the centromeres);
      * long poly-A / poly-T runs (1-20 kb) and poly-N gaps (10 kb - 1 Mb).
    Vectorised (numpy), ~10 s per Gbp."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    alu = rng.integers(0, 4, size=300, dtype=np.uint8)
    mono = rng.integers(0, 4, size=171, dtype=np.uint8)
    out = []
    per = n_bases // n_records
    for r in range(n_records):
        L = per if r + 1 < n_records else n_bases - per * (n_records - 1)
        seq = rng.integers(0, 4, size=L, dtype=np.uint8)
        # Alu-like copies, 10 % diverged, half reverse-complemented
        n_alu = L // 3100
        if n_alu and L > 300:
            for c0 in range(0, n_alu, 1 << 16):
                m = min(1 << 16, n_alu - c0)
                cp = np.broadcast_to(alu, (m, 300)).copy()
                mut = rng.random((m, 300)) < 0.10
                cp[mut] = rng.integers(0, 4, size=int(mut.sum()), dtype=np.uint8)
                flip = rng.random(m) < 0.5
                cp[flip] = 3 - cp[flip, ::-1]
                at = rng.integers(0, L - 300, size=m)
                idx = at[:, None] + np.arange(300)[None, :]
                seq[idx.reshape(-1)] = cp.reshape(-1)
        # a tandem satellite array, ~2 % diverged monomers
        n_sat = min(L // 40, 3_000_000) // 171
        if n_sat:
            arr = np.broadcast_to(mono, (n_sat, 171)).copy()
            mut = rng.random((n_sat, 171)) < 0.02
            arr[mut] = rng.integers(0, 4, size=int(mut.sum()), dtype=np.uint8)
            at = int(rng.integers(0, max(1, L - n_sat * 171)))
            seq[at:at + n_sat * 171] = arr.reshape(-1)[:L - at]
        # poly-A / poly-T runs
        for _ in range(max(1, L // 2_000_000)):
            a = int(rng.integers(0, L))
            seq[a:a + int(rng.integers(1_000, 20_000))] = 0 if rng.random() < 0.5 else 3
        chars = acgt[seq].copy()
        # soft-masking in runs
        for _ in range(L // 50_000):
            a = int(rng.integers(0, L))
            chars[a:a + int(rng.integers(500, 15_000))] += 32
        # N: the record ends (telomeres) and gaps of 10 kb - 1 Mb
        nN = min(L // 20, 10_000)
        chars[:nN] = ord("N")
        chars[L - nN:] = ord("N")
        for _ in range(max(1, L // 20_000_000)):
            a = int(rng.integers(0, L))
            chars[a:a + int(rng.integers(10_000, min(1_000_000, max(10_001, L // 10))))] = ord("N")
        out.append(b">chr%d AC:CM0006%02d.2 gi:5688%02d LN:%d rl:Chromosome M5:x AS:GRCh38\n" % (r + 1, r, r, L))
        full = L // width
        grid = np.empty((full, width + 1), dtype=np.uint8)
        grid[:, :width] = chars[:full * width].reshape(full, width)
        grid[:, width] = ord("\n")
        out.append(grid.tobytes())
        if L > full * width:
            out.append(bytes(chars[full * width:]) + b"\n")
    return b"".join(out)


def messy_records(seed: int, n_records: int = 24, max_len: int = 3000) -> bytes:
    """Multi-record FASTA exercising the parser/extractor edge cases of §8c/§A:
    descriptions after the name, a tab inside the title, lowercase runs, N and
    IUPAC runs, internal spaces, trailing tabs/spaces, CRLF and lone-CR line
    ends, blank lines, records shorter than k and an empty record."""
    rng = random.Random(seed)
    parts = ["; a comment line before the first record\n", "\n"]
    for r in range(n_records):
        L = rng.choice([0, 1, 3, 7, 20, 21, 22, 40, 150, 500, max_len, rng.randrange(max_len)])
        chars = []
        i = 0
        while i < L:
            roll = rng.random()
            run = rng.randrange(1, 40)
            if roll < 0.75:
                chars.extend(rng.choices("ACGT", k=run))
            elif roll < 0.87:
                chars.extend(rng.choices("acgt", k=run))
            elif roll < 0.93:
                chars.extend("N" * run)
            elif roll < 0.96:
                chars.extend(rng.choices("RYKMSWn", k=run))
            else:
                chars.extend(rng.choices("ACGT", k=run))
            i += run
        seq = "".join(chars[:L])
        kind = r % 6
        if kind == 0:
            title = "rec%d description words here" % r
        elif kind == 1:
            title = "rec%d\tx y" % r
        elif kind == 2:
            title = "chr%d" % r
        elif kind == 3:
            title = "rec%d:1-5:+  " % r
        elif kind == 4:
            title = "r%d" % r
        else:
            title = "seq_%d|tag=%d" % (r, rng.randrange(1000))
        parts.append(">" + title + "\n")
        if not seq:
            # a non-first record with NO sequence line makes the reference's
            # SmartFastaParser re-yield it forever (parsers.py:646 never advances
            # __pos); a blank line keeps the case parseable.
            parts.append("\n")
        width = rng.choice([60, 70, 80, 13])
        pos = 0
        while pos < len(seq):
            line = seq[pos : pos + width]
            pos += width
            deco = rng.random()
            if deco < 0.05:
                line = line[: len(line) // 2] + " " + line[len(line) // 2 :]
            elif deco < 0.08:
                line = line + " \t "
            elif deco < 0.10:
                line = line[: len(line) // 2] + "\t" + line[len(line) // 2 :]
            end = "\n"
            e = rng.random()
            if e < 0.08:
                end = "\r\n"
            elif e < 0.10:
                end = "\r"
            parts.append(line + end)
            if rng.random() < 0.03:
                parts.append("\n")
    return "".join(parts).encode()


EDGE_FA = (
    b"\n"
    b">r\n"
    b">short x\n"
    b"ACG\n"
    b">chr0\tx y\n"
    b"ACGATCGATCGAacgatcgatNNACGTACGTAC\n"
    b"GGGGGGGGGG  \t\n"
    b"\n"
    b"TTTTacgtRYACGT\r\n"
    b">dup1 desc\n"
    b"ACGTACGTACGTACGT\n"
    b">dup2\n"
    b"acgtacgtacgtacgt\n"
    b">pal\n"
    b"GATCGATC\n"
)


def vec_shared() -> bytes:
    """Records a, b, c: b holds 60 bases of a (positions 20-79), c is its
    own; lowercase in b (the reference upper-cases before the check)."""
    rng = random.Random(77)
    a = "".join(rng.choice("ACGT") for _ in range(120))
    b = "".join(rng.choice("ACGT") for _ in range(30)) + a[20:80].lower() + "".join(rng.choice("ACGT") for _ in range(25))
    c = "".join(rng.choice("ACGT") for _ in range(90))
    return (">a one\n" + wrap(a) + ">b\ttwo\n" + wrap(b) + ">c\n" + wrap(c)).encode()


def build_inputs(root: str) -> dict:
    files = {
        "edge": EDGE_FA,
        "messy1": messy_records(1),
        "messy2": messy_records(2, n_records=40, max_len=5000),
        "syn64k_a": syn_python(64000, 7),
        "syn64k_b": syn_numpy(64000, 11, record_len=9000, width=70),
        "empty": b"",
        "noheader": b"ACGTACGT\nACGT\n",
        "emptyname": b">chr1\nACGTAC\n> desc only\nACGTAC\n",
        "emptyname_short": b">chr1\nACGTAC\n> desc only\nACG\n",
        "syn1m": syn_python(10**6, 42),
        # VEC_COUNT_MASKED (round 4): a 60-base segment of record a copied
        # into record b (k-mers shared by two names), and one sequence under
        # one name twice (shared by one name only)
        "vecshare": vec_shared(),
        "vecsame": (">same first\n" + wrap("".join(random.Random(5).choices("ACGT", k=90))) + ">same second\n"
                    + wrap("".join(random.Random(5).choices("ACGT", k=90)))).encode(),
    }
    paths = {}
    for name, data in files.items():
        p = os.path.join(root, name + ".fa")
        with open(p, "wb") as fh:
            fh.write(data)
        paths[name] = p
    gz = os.path.join(root, "messy1.fa.gz")
    with gzip.open(gz, "wb") as fh:
        fh.write(files["messy1"])
    paths["messy1.gz"] = gz
    return paths
