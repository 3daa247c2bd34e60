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
