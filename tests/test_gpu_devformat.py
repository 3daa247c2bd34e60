"""GPU parity of the device-side writers (kman_format_count_dev /
kman_format_uniq_dev, devformat.hip): byte-identical to the
host writers (format.cpp, themselves pinned by the reference outputs) and to
the reference's own `kmer count` / `kmer uniq` outputs (golden sha256), over
LDS-staged tiles, tiles too long for LDS (long record names), row slices,
u64 counts and positions past 2^32."""

from __future__ import annotations

import types
from ctypes import byref, c_size_t, c_void_p

import numpy as np
import pytest

from conftest import sha256_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from kman_amd import engine

    return engine.default_device()


def _cases():
    import json
    import os

    from conftest import GOLDEN

    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        cases = json.load(fh)["cases"]
    return [c for c in cases if c["cmd"] in ("count", "uniq") and c["result"]["ok"] and 2 <= c["k"]]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_device_format_matches_reference(dev, golden_inputs, case, monkeypatch):
    from kman_amd import engine

    monkeypatch.delenv("KMAN_HOST_FORMAT", raising=False)
    text = engine.read_input(golden_inputs[case["input"]])
    rc = "-r" in case["flags"]
    fn = engine.count_text if case["cmd"] == "count" else engine.uniq_text
    assert sha256_bytes(fn(text, case["k"], rc=rc, dev=dev)) == case["sha256"]


def _upload(dev, a):
    b = dev.alloc(max(16, a.nbytes))
    if a.nbytes:
        dev.upload(b, a)
    return b


@pytest.mark.parametrize("cb", [4, 8])
@pytest.mark.parametrize("k", [1, 2, 21, 32])
@pytest.mark.parametrize("chunk", [None, 4096])
def test_count_rows_device_equals_host(dev, cb, k, chunk, monkeypatch):
    from kman_amd import engine

    if chunk:
        monkeypatch.setattr(engine, "_FMT_CHUNK", chunk)
    rng = np.random.default_rng(k * 10 + cb)
    n = 20011
    keys = rng.integers(0, 1 << min(63, 2 * k), n, dtype=np.uint64)
    hi = (1 << 32) - 1 if cb == 4 else (1 << 63)
    counts = rng.integers(1, hi, n, dtype=np.uint64)
    counts[::7] = rng.integers(1, 12, len(counts[::7]))
    counts = counts.astype(np.uint32 if cb == 4 else np.uint64)
    want = engine.format_count(keys, counts, k)
    dk, dc = _upload(dev, keys), _upload(dev, counts)
    try:
        r = engine.CountResult(dk, dc, cb, n, k)
        assert engine.format_count_dev(dev, r) == want
    finally:
        dk.free()
        dc.free()


@pytest.mark.parametrize("pb", [4, 8])
@pytest.mark.parametrize("name_len", [0, 3, 1500])
def test_uniq_rows_device_equals_host(dev, pb, name_len):
    """Records with long names push a tile's text past the LDS buffer (the
    straight-to-HBM path); u64 positions put starts past 2^32."""
    from kman_amd import engine

    rng = np.random.default_rng(pb + name_len)
    R, k = 37, 21
    span = (1 << 34) if pb == 8 else (1 << 30)
    rec_seq = np.sort(rng.choice(span // 2, R - 1, replace=False).astype(np.uint64))
    rec_seq = np.concatenate([[np.uint64(0)], rec_seq]).astype(np.uint64)
    names = [("r%d" % i + "\tx" * (name_len // 2)).encode()[:name_len] if name_len else b"" for i in range(R)]
    name_off = np.zeros(R + 1, np.uint64)
    name_off[1:] = np.cumsum([len(x) for x in names])
    p = types.SimpleNamespace(dev=dev, names_blob=b"".join(names), name_off=name_off, rec_seq=rec_seq, n_records=R,
                              n_bases=int(span // 2 + 1000))
    n = 9000
    g = rng.integers(0, span // 2, n, dtype=np.uint64)
    pos = ((g << np.uint64(1)) | rng.integers(0, 2, n, dtype=np.uint64)).astype(np.uint32 if pb == 4 else np.uint64)
    keys = rng.integers(0, 1 << 42, n, dtype=np.uint64)
    want = engine.format_fasta(keys, pos, k, p)
    dk, dp = _upload(dev, keys), _upload(dev, pos)
    try:
        assert engine.format_uniq_dev(p, engine.UniqResult(dk, dp, pb, n, k)) == want
    finally:
        dk.free()
        dp.free()


def test_format_capacity(dev):
    """cap below the text: KMAN_ECAP with the size, nothing written past cap;
    NULL output sizes only."""
    from kman_amd import _native as N

    keys = np.arange(5000, dtype=np.uint64)
    counts = np.full(5000, 123, np.uint32)
    dk, dc = _upload(dev, keys), _upload(dev, counts)
    out = dev.alloc(4096 + 256)
    try:
        dev.memset(out, 0x5A, 4096 + 256)
        used = c_size_t(0)
        L = N.lib()
        assert L.kman_format_count_dev(dev.ctx, c_void_p(dk.ptr), c_void_p(dc.ptr), 4, 5000, 21, None, 0,
                                       byref(used)) == N.KMAN_ECAP
        assert used.value == 5000 * (21 + 2 + 3)
        assert L.kman_format_count_dev(dev.ctx, c_void_p(dk.ptr), c_void_p(dc.ptr), 4, 5000, 21,
                                       c_void_p(out.ptr), 4096, byref(used)) == N.KMAN_ECAP
        tail = dev.download(out, 256, np.uint8, offset=4096)
        assert (tail == 0x5A).all()
    finally:
        for b in (dk, dc, out):
            b.free()
