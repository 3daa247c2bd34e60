"""Kernel-level CPU restatement (numpy) of the reference's k-mer path.

TEST INFRASTRUCTURE ONLY — the checker for the individual HIP stages, never
imported by the product (kman_amd) or timed as the product.  Whole-command
parity (count / uniq / batch output bytes) is checked with the C restatement
kman_oracle.c, itself pinned to the reference's outputs in tests/golden/.

Functions and the reference lines they restate:
  parse_fasta    kmermaid/parsers.py:86-128 (+ text-mode universal newlines)
  record_name    kmermaid/batcher.py:551
  stream_kmers   kmermaid/seq.py:285-328 (upper, ACGT check, rc with same coords)
  stable_sort    kmermaid/batch.py:156-168 (stable by sequence)
  rle_count      kmermaid/join.py:95-130 + 266-285
  rle_uniq       kmermaid/join.py:95-130 + 244-263
"""

from __future__ import annotations

import re

import numpy as np

_WS = b" \t\n\x0b\x0c\r\x1c\x1d\x1e\x1f"  # str.isspace() over ASCII


def _lines(text: bytes):
    """Universal-newline line split: yields line contents without terminators."""
    for m in re.finditer(rb"([^\r\n]*)(\r\n|\r|\n|$)", text):
        if m.start() == len(text) and not m.group(1):
            break
        yield m.group(1)
        if m.group(2) == b"":
            break


def parse_fasta(text: bytes):
    """-> (list of (title_bytes, cleaned_seq_bytes)).  Raises AssertionError on
    a file without any '>' line (parsers.py:105-107)."""
    recs = []
    cur = None
    for line in _lines(text):
        if line[:1] == b">":
            if cur is not None:
                recs.append(cur)
            cur = [line[1:].rstrip(_WS), []]
        elif cur is not None:
            cur[1].append(line.rstrip(_WS))
    if cur is None:
        raise AssertionError("premature end of file or empty file")
    recs.append(cur)
    return [(t, b"".join(s).replace(b" ", b"").replace(b"\r", b"")) for t, s in recs]


def record_name(title: bytes) -> bytes:
    return title.decode("utf-8", "surrogateescape").split(" ")[0].encode("utf-8", "surrogateescape")


_CODE = np.full(256, 4, dtype=np.uint8)
for _i, _c in enumerate(b"ACGT"):
    _CODE[_c] = _i
    _CODE[_c | 0x20] = _i


def codes_of(records) -> tuple:
    """Device code layout of kman_parse_fasta: (codes u8, rec_seq u64)."""
    seqs = [s for _, s in records]
    rec_seq = np.zeros(len(seqs), dtype=np.uint64)
    acc = 0
    for i, s in enumerate(seqs):
        rec_seq[i] = acc
        acc += len(s)
    joined = np.frombuffer(b"".join(seqs), dtype=np.uint8)
    codes = _CODE[joined].copy()
    for i, s in enumerate(seqs):
        if len(s):
            codes[int(rec_seq[i])] |= 8
    return codes, rec_seq


def stream_kmers(records, k: int, rc: bool = False, canonical: bool = False):
    """Keys (2-bit MSB-first) and pos payloads ((global base << 1) | strand)
    in the reference's emission order."""
    keys, pos = [], []
    base = 0
    mask = (1 << (2 * k)) - 1
    for _, s in records:
        c = _CODE[np.frombuffer(s, dtype=np.uint8)] if s else np.zeros(0, np.uint8)
        L = len(c)
        if L >= k:
            bad = (c > 3).astype(np.int64)
            cs = np.concatenate([[0], np.cumsum(bad)])
            starts = np.nonzero(cs[k:] - cs[: L - k + 1] == 0)[0]
            if len(starts):
                cc = c.astype(np.uint64)
                f = np.zeros(len(starts), dtype=np.uint64)
                r = np.zeros(len(starts), dtype=np.uint64)
                for j in range(k):
                    f = (f << np.uint64(2)) | cc[starts + j]
                    r = r | ((np.uint64(3) - cc[starts + j]) << np.uint64(2 * j))
                f &= np.uint64(mask)
                gp = (starts.astype(np.uint64) + np.uint64(base)) << np.uint64(1)
                if canonical:
                    keys.append(np.minimum(f, r))
                    pos.append(gp)
                elif rc:
                    kk = np.empty(2 * len(starts), dtype=np.uint64)
                    kk[0::2] = f
                    kk[1::2] = r
                    pp = np.empty(2 * len(starts), dtype=np.uint64)
                    pp[0::2] = gp
                    pp[1::2] = gp | np.uint64(1)
                    keys.append(kk)
                    pos.append(pp)
                else:
                    keys.append(f)
                    pos.append(gp)
        base += L
    if not keys:
        return np.zeros(0, np.uint64), np.zeros(0, np.uint64)
    return np.concatenate(keys), np.concatenate(pos)


def stable_sort(keys: np.ndarray, vals: np.ndarray | None = None):
    order = np.argsort(keys, kind="stable")
    return keys[order], (vals[order] if vals is not None else None)


def rle_count(sorted_keys: np.ndarray):
    if len(sorted_keys) == 0:
        return sorted_keys, np.zeros(0, np.uint64)
    u, c = np.unique(sorted_keys, return_counts=True)
    return u, c.astype(np.uint64)


def rle_uniq(sorted_keys: np.ndarray, vals: np.ndarray):
    n = len(sorted_keys)
    if n == 0:
        return sorted_keys, vals
    head = np.ones(n, bool)
    head[1:] = sorted_keys[1:] != sorted_keys[:-1]
    tail = np.ones(n, bool)
    tail[:-1] = sorted_keys[1:] != sorted_keys[:-1]
    m = head & tail
    return sorted_keys[m], vals[m]


def decode(key: int, k: int) -> bytes:
    return bytes(b"ACGT"[(int(key) >> (2 * (k - 1 - j))) & 3] for j in range(k))


def mix_keys(x, k: int):
    """KMAN_MIXED's bijection of the 2k-bit keys (kman_amd/csrc/rollfast.h
    mix_key: odd multiply, xorshift by k, odd multiply, mod 2^2k) -- the
    engine's own key transform for abundance spectra, not the reference's."""
    x = np.asarray(x, dtype=np.uint64)
    kb = 2 * k
    m = np.uint64((1 << kb) - 1) if kb < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        x = (x * np.uint64(0x9E3779B97F4A7C15)) & m
        x = x ^ (x >> np.uint64(kb // 2))
        return (x * np.uint64(0xBF58476D1CE4E5B9)) & m
