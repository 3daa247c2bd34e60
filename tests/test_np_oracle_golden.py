"""Pin the kernel-level numpy oracle (oracle/np_oracle.py) to the reference
directly: for every golden count / uniq case with k <= 32 (and the config-1
1 MB input), np_oracle's rows -- parse_fasta -> stream_kmers -> stable_sort ->
rle_count / rle_uniq -- are formatted into the reference's bytes
(join.py:284 "%s\\t%d\\n"; join.py:262 ">%s\\n%s\\n" with the KMer header
"%s:%d-%d:%s" of seq.py:104, record-relative 0-based coordinates, the +
strand's coordinates on the - record, seq.py:274-282) and their sha256 is
compared with tests/golden/manifest.json, the reference's own outputs.
Every GPU kernel test compares against np_oracle, so this closes the chain
kernel -> np_oracle -> reference without going through the C oracle.  CPU
only."""

from __future__ import annotations

import gzip
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _cases():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        m = json.load(fh)
    out = [c for c in m["cases"] if c["k"] <= 32 and c["cmd"] in ("count", "uniq") and c["result"]["ok"]]
    out += [dict(c, flags=[]) for c in m["config1"]]
    return out


def _seqs(keys: np.ndarray, k: int) -> np.ndarray:
    """(n, k) ASCII bytes of 2-bit MSB-first keys."""
    sh = (np.uint64(2) * (np.uint64(k - 1) - np.arange(k, dtype=np.uint64)))
    d = ((keys[:, None] >> sh[None, :]) & np.uint64(3)).astype(np.uint8)
    return np.frombuffer(b"ACGT", np.uint8)[d]


def format_count(keys: np.ndarray, counts: np.ndarray, k: int) -> bytes:
    s = _seqs(keys, k)
    return b"".join(bytes(s[i]) + b"\t%d\n" % int(counts[i]) for i in range(len(keys)))


def format_uniq(keys: np.ndarray, pos: np.ndarray, k: int, records) -> bytes:
    import np_oracle

    names = [np_oracle.record_name(t) for t, _ in records]
    starts = np.cumsum([0] + [len(s) for _, s in records])[:-1].astype(np.int64)
    base = (pos >> np.uint64(1)).astype(np.int64)
    rec = np.searchsorted(starts, base, side="right") - 1
    s = _seqs(keys, k)
    out = []
    for i in range(len(keys)):
        r = int(rec[i])
        a = int(base[i] - starts[r])
        out.append(b">%s:%d-%d:%s\n%s\n" % (names[r], a, a + k, b"-" if int(pos[i]) & 1 else b"+", bytes(s[i])))
    return b"".join(out)


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_np_oracle_matches_reference_bytes(case, golden_inputs):
    import np_oracle

    path = golden_inputs[case["input"]]
    if path.endswith(".gz"):
        with gzip.open(path, "rb") as fh:
            text = fh.read()
    else:
        with open(path, "rb") as fh:
            text = fh.read()
    k = case["k"]
    rc = "-r" in case["flags"]
    records = np_oracle.parse_fasta(text)
    keys, pos = np_oracle.stream_kmers(records, k, rc=rc)
    sk, sp = np_oracle.stable_sort(keys, pos)
    if case["cmd"] == "count":
        uk, uc = np_oracle.rle_count(sk)
        data = format_count(uk, uc, k)
    else:
        uk, up = np_oracle.rle_uniq(sk, sp)
        data = format_uniq(uk, up, k, records)
    assert hashlib.sha256(data).hexdigest() == case["sha256"]
