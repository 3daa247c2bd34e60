"""GPU parity of the multi-batch device join (BASELINE config 3):
engine.ranged_groups cuts the stream into key ranges (kman_kmer_prefix_hist
-> key_ranges), extracts each range from the resident codes
(kman_extract_range), prefix-sorts and finishes it, and appends its output.

Bar: byte-identical command output to the reference's own `kmer count` /
`kmer uniq` outputs (tests/golden manifest sha256) with the input forced into
several key ranges, and bit-exact against np_oracle (stream_kmers -> stable
sort -> RLE: seq.py:285-328, batch.py:156-168, join.py:95-130,244-285) on
larger synthetic inputs."""

from __future__ import annotations

from ctypes import byref, c_uint64, c_void_p

import numpy as np
import pytest

from conftest import sha256_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from kman_amd import engine

    return engine.default_device()


def _small_batches(dev, text, k, rc):
    """max_keys for about 4 ranges (at least the largest prefix bin).  k > 32
    (word-pair keys) has no key-range batching: those inputs run whole
    through engine.wide_groups whatever max_keys says."""
    from kman_amd import engine

    p = engine.parse(dev, text)
    try:
        if k > engine.MAX_K:
            n = engine.count_kmers(p, k, rc)
            return n // 4 + 1, n
        h, n = engine.prefix_hist(p, k, rc)
    finally:
        p.free()
    return max(int(h.max()) if len(h) else 1, n // 4 + 1, 1), n


def _golden_cases():
    import json
    import os

    from conftest import GOLDEN

    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        cases = json.load(fh)["cases"]
    return [c for c in cases if c["cmd"] in ("count", "uniq") and c["result"]["ok"] and 2 <= c["k"] <= 64
            and all(f == "-r" for f in c["flags"])]


@pytest.mark.parametrize("case", _golden_cases(), ids=lambda c: c["name"])
def test_ranged_matches_reference_outputs(dev, golden_inputs, case):
    from kman_amd import engine

    text = engine.read_input(golden_inputs[case["input"]])
    rc = "-r" in case["flags"]
    mk, n = _small_batches(dev, text, case["k"], rc)
    fn = engine.count_text if case["cmd"] == "count" else engine.uniq_text
    assert sha256_bytes(fn(text, case["k"], rc=rc, dev=dev, max_keys=mk)) == case["sha256"]


def _oracle(text, k, rc, mode):
    import np_oracle

    recs = np_oracle.parse_fasta(text)
    keys, pos = np_oracle.stream_kmers(recs, k, rc=rc)
    sk, sp = np_oracle.stable_sort(keys, pos)
    return np_oracle.rle_count(sk) if mode == "count" else np_oracle.rle_uniq(sk, sp)


@pytest.mark.parametrize("k", [3, 13, 21, 31, 32])
@pytest.mark.parametrize("rc", [False, True])
@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("parts", [1, 3, 17])
def test_ranged_matches_oracle(dev, k, rc, mode, parts):
    import inputs
    from kman_amd import engine

    text = inputs.messy_records(5 + k, n_records=40, max_len=30000) + inputs.syn_numpy(400_000, k)
    p = engine.parse(dev, text)
    try:
        h, n = engine.prefix_hist(p, k, rc)
        mk = max(int(h.max()), n // parts + 1)
        ranges = engine.key_ranges(h, k, mk)
        assert sum(r[2] for r in ranges) == n
        if parts > 1 and k >= 4:
            assert len(ranges) > 1
        r = engine.ranged_groups(p, k, rc, mode, max_keys=mk)
        try:
            got = engine.download_count(dev, r) if mode == "count" else engine.download_uniq(dev, r)
        finally:
            for b in ((r.ukeys, r.counts) if mode == "count" else (r.keys, r.pos)):
                b.free()
    finally:
        p.free()
    want = _oracle(text, k, rc, mode)
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1].astype(np.uint64), want[1])


@pytest.mark.parametrize("k", [2, 3, 4, 21, 31])
@pytest.mark.parametrize("rc", [False, True])
def test_prefix_hist_matches_oracle(dev, k, rc):
    import inputs
    import np_oracle
    from kman_amd import engine

    text = inputs.messy_records(k, n_records=30, max_len=20000)
    p = engine.parse(dev, text)
    try:
        h, n = engine.prefix_hist(p, k, rc)
    finally:
        p.free()
    keys, _ = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k, rc=rc)
    assert n == len(keys)
    sh = max(0, 2 * k - 8)
    want = np.bincount((keys >> np.uint64(sh)).astype(np.int64), minlength=len(h))
    np.testing.assert_array_equal(h, want.astype(np.uint64))


def test_extract_range_capacity(dev):
    """A key range holding more keys than cap: counted, nothing written past
    cap, KMAN_ECAP."""
    import inputs
    from kman_amd import _native as N
    from kman_amd import engine

    text = inputs.syn_numpy(200_000, 4)
    p = engine.parse(dev, text)
    keys = dev.alloc(8 * 1024 + 8 * 64)
    try:
        dev.memset(keys, 0xAB, 8 * 1024 + 8 * 64)
        got = c_uint64(0)
        L = N.lib()
        rc = L.kman_extract_range(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, 21, 0, 0, (1 << 42) - 1,
                                  c_void_p(keys.ptr), None, 0, 1024, None, byref(got))
        assert rc == N.KMAN_ECAP
        assert got.value == p.n_bases - 20
        tail = dev.download(keys, 64, np.uint64, offset=8 * 1024)
        assert (tail == np.uint64(0xABABABABABABABAB)).all()
        # the same range with room: every key, in stream order
        full = dev.alloc(8 * p.n_bases)
        try:
            lo, hi = 5 << 34, (9 << 34) - 1
            assert L.kman_extract_range(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, 21, 0, lo, hi,
                                        c_void_p(full.ptr), None, 0, p.n_bases, None, byref(got)) == N.KMAN_OK
            import np_oracle

            ks, _ = np_oracle.stream_kmers(np_oracle.parse_fasta(text), 21, rc=False)
            want = ks[(ks >= lo) & (ks <= hi)]
            np.testing.assert_array_equal(dev.download(full, got.value, np.uint64), want)
        finally:
            full.free()
    finally:
        keys.free()
        p.free()


def test_ranged_single_prefix_too_big(dev):
    """One 8-bit prefix with more k-mers than a batch: MemoryError, not a
    silent truncation."""
    from kman_amd import engine

    text = b">a\n" + b"A" * 5000 + b"\n"
    p = engine.parse(dev, text)
    try:
        with pytest.raises(MemoryError):
            engine.ranged_groups(p, 21, False, "count", max_keys=1000)
    finally:
        p.free()


@pytest.mark.parametrize("mode", ["count", "uniq"])
def test_ranged_heavy_prefix_is_bisected(dev, mode):
    """A prefix bin larger than a batch (a poly-A run + a repeat) is cut by
    key (kman_extract_range counts) instead of raising MemoryError."""
    import inputs

    from kman_amd import engine

    text = inputs.syn_numpy(60_000, 5, record_len=20_000) + b">polyA\n" + b"A" * 5_000 + b"\n>rep\n" + \
        b"AAAACAGGTAACCAGGTTTGA" * 400 + b"\n"
    fn = engine.count_text if mode == "count" else engine.uniq_text
    for k in (13, 21):
        p = engine.parse(dev, text)
        try:
            h, _ = engine.prefix_hist(p, k, False)
        finally:
            p.free()
        assert int(h.max()) > 5_000  # the AAAA.. bin is larger than a batch
        got = fn(text, k, dev=dev, max_keys=5_000)
        assert got == fn(text, k, dev=dev)  # the one-batch paths
