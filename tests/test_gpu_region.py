"""GPU parity of the region path (kman_groups, kman_amd/csrc/region.hip):
count / uniq of a whole stream straight from the codes.

Bar: bit-exact against the numpy restatement of the reference's path
(np_oracle: stream_kmers -> stable sort -> run-length count / uniq, which
restates seq.py:285-328, batch.py:156-168 and join.py:95-130,244-285), and
identical to the general (prefix-split) GPU path on the same input.  Full
size (BASELINE config 2: 1 GB FASTA, k=21) is checked through
size-independent properties and against the general path's count output."""

from __future__ import annotations

import os
import ctypes
from ctypes import byref, c_uint64

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from kman_amd import engine

    return engine.default_device()


def _texts(golden_inputs):
    import inputs

    from kman_amd.engine import read_input

    return [
        read_input(golden_inputs["messy1"]),
        inputs.messy_records(11, n_records=60, max_len=20000),
        inputs.syn_numpy(100_000, 5),
        inputs.syn_numpy(3_000_000, 6, record_len=1 << 20),
    ]


def _oracle(text, k, rc, mode):
    import np_oracle

    recs = np_oracle.parse_fasta(text)
    keys, pos = np_oracle.stream_kmers(recs, k, rc=rc)
    sk, sp = np_oracle.stable_sort(keys, pos)
    if mode == "count":
        return np_oracle.rle_count(sk)
    return np_oracle.rle_uniq(sk, sp)


def _groups(dev, text, k, rc, mode):
    from kman_amd import engine

    p = engine.parse(dev, text)
    try:
        r = engine.groups(p, k, rc, mode)
        if r is None:
            return None
        try:
            if mode == "count":
                return engine.download_count(dev, r)
            return engine.download_uniq(dev, r)
        finally:
            for b in ((r.ukeys, r.counts) if mode == "count" else (r.keys, r.pos)):
                b.free()
    finally:
        p.free()


@pytest.mark.parametrize("k", [5, 9, 13, 21, 25])
@pytest.mark.parametrize("rc", [False, True])
@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("check", ["0", "1"])
def test_groups_matches_oracle(dev, golden_inputs, monkeypatch, k, rc, mode, check):
    """(check: the uniq finish without / with the early-count device check,
    the product default and the GPU test session's setting)"""
    from kman_amd import _native as N

    monkeypatch.setenv("KMAN_RG_CHECK", check)

    for text in _texts(golden_inputs):
        n_bases = sum(len(s) for _, s in __import__("np_oracle").parse_fasta(text))
        m = N.KMAN_FINISH_UNIQ if mode == "uniq" else N.KMAN_FINISH_COUNT
        flags = (N.KMAN_RC if rc else 0) | (N.KMAN_WANT_POS if mode == "uniq" else 0)
        wb = c_uint64(0)
        inside = N.lib().kman_groups_plan(n_bases, k, flags, m, byref(wb)) == N.KMAN_OK
        # outside: 2k - 8 key bits + the pos bits exceed one u64 item, or no
        # key bits left below the 8 + b2 region bits (b2 as region.hip picks it)
        W = n_bases * (2 if rc else 1)
        q = max(1, int(W - 1).bit_length()) if mode == "uniq" else 0
        b2 = 1
        while b2 < 9 and (W >> (8 + b2)) > 6144:
            b2 += 1
        assert inside == (2 * k - 8 + q <= 64 and 2 * k >= 8 + b2 + 1 and (W >> (8 + b2)) <= 7800)
        got = _groups(dev, text, k, rc, mode)
        if not inside:
            assert got is None
            continue
        assert got is not None, "input inside the region path fell back"
        want = _oracle(text, k, rc, mode)
        np.testing.assert_array_equal(got[0], want[0])
        np.testing.assert_array_equal(got[1].astype(np.uint64), want[1])


@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("copies", [3, 100, 1000])
def test_groups_repeats(dev, mode, copies):
    """Repeated segments: runs of equal keys inside a finish region (and, at
    1000 copies, a region past its capacity: the general path)."""
    import inputs

    rng = np.random.default_rng(copies)
    seg = "".join(rng.choice(list("ACGT"), 300))
    body = inputs.syn_numpy(200_000, 3).split(b"\n", 1)[1].replace(b"\n", b"")
    text = b">r\n" + body + b"\n>s\n" + (seg * copies).encode() + b"\n"
    got = _groups(dev, text, 21, False, mode)
    want = _oracle(text, 21, False, mode)
    if got is None:
        # 1000 copies overflow a region: the engine's general path instead
        assert copies >= 1000
        from kman_amd import engine

        out = (engine.count_text if mode == "count" else engine.uniq_text)(text, 21, dev=dev)
        assert out.count(b"\n") == len(want[0]) * (1 if mode == "count" else 2)
        return
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1].astype(np.uint64), want[1])


def test_groups_plan_domain():
    """kman_groups_plan: KMAN_EFALLBACK outside the path, a size inside it."""
    from kman_amd import _native as N

    L = N.lib()
    wb = c_uint64(0)
    U, C = N.KMAN_FINISH_UNIQ, N.KMAN_FINISH_COUNT
    assert L.kman_groups_plan(1_000_000_000, 21, N.KMAN_WANT_POS, U, byref(wb)) == N.KMAN_OK and wb.value > 0
    assert L.kman_groups_plan(1_000_000_000, 21, 0, C, byref(wb)) == N.KMAN_OK
    assert L.kman_groups_plan(1000, 31, 0, C, byref(wb)) == N.KMAN_OK  # count items: k <= 32
    assert L.kman_groups_plan(1000, 26, N.KMAN_WANT_POS, U, byref(wb)) == N.KMAN_EFALLBACK  # uniq: k <= 25
    assert L.kman_groups_plan(1000, 21, N.KMAN_CANONICAL, C, byref(wb)) == N.KMAN_OK  # canonical keys: in
    assert L.kman_groups_plan(1000, 4, 0, C, byref(wb)) == N.KMAN_EFALLBACK  # too few key bits
    assert L.kman_groups_plan(4_000_000_000, 21, 0, C, byref(wb)) == N.KMAN_EFALLBACK  # regions too full
    assert L.kman_groups_plan(1000, 21, 0, 0, byref(wb)) == N.KMAN_EINVAL  # SORT is not a groups mode


@pytest.mark.parametrize("mode", ["count", "uniq"])
def test_groups_overflow_falls_back(dev, mode):
    """A skewed stream (one k-mer repeated) overflows a region: kman_groups
    says KMAN_EFALLBACK and the command output still matches the oracle
    through the general path."""
    from kman_amd import engine

    text = b">a\n" + b"A" * 300_000 + b"\n>b\n" + b"ACGT" * 1000 + b"\n"
    assert _groups(dev, text, 21, False, mode) is None
    fn = engine.count_text if mode == "count" else engine.uniq_text
    got = fn(text, 21, dev=dev)
    want = _oracle(text, 21, False, mode)
    if mode == "count":
        lines = got.decode().splitlines()
        assert len(lines) == len(want[0])
        assert [int(x.split("\t")[1]) for x in lines] == want[1].tolist()
    else:
        assert got.count(b">") == len(want[0])


@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("rc", [False, True])
def test_pipeline_region_equals_split(dev, mode, rc):
    """ResidentPipeline: region path == prefix-split path, 60 Mbase input."""
    import inputs
    from kman_amd import engine

    text = inputs.syn_numpy(60_000_000, 9)
    outs = []
    for path in ("region", "split"):
        pipe = engine.ResidentPipeline(dev, text, 21, mode=mode, rc=rc, path=path)
        try:
            assert pipe.path == path
            n = pipe.step()
            n2 = pipe.step()  # a second step over the same resident input
            assert n == n2
            vt = np.uint32 if (pipe.count_bytes if mode == "count" else pipe.pos_bytes) == 4 else np.uint64
            outs.append((n, pipe.n_out, dev.download(pipe.out_keys, pipe.n_out, np.uint64),
                         dev.download(pipe.out_vals, pipe.n_out, vt)))
        finally:
            pipe.free()
    assert outs[0][0] == outs[1][0] and outs[0][1] == outs[1][1]
    np.testing.assert_array_equal(outs[0][2], outs[1][2])
    np.testing.assert_array_equal(outs[0][3], outs[1][3])


@pytest.mark.parametrize("check", ["0", "1"])
def test_full_size_region(dev, monkeypatch, check):
    """BASELINE config 2 (1 GB synthetic FASTA, k=21) on the region path:
    uniq keys are exactly the count-1 keys of the count run, counts sum to
    the k-mer count, keys strictly increase, the key checksum of the stream
    is preserved, and every uniq pos decodes (from the codes) to its key.
    check 0: the uniq finish the bench times (no device check of its early
    row count); 1: the checked one."""
    import inputs
    from kman_amd import engine

    monkeypatch.setenv("KMAN_RG_CHECK", check)

    text = inputs.syn_numpy(1_000_000_000, 1)
    pu = engine.ResidentPipeline(dev, text, 21, mode="uniq")
    assert pu.path == "region"
    n = pu.step()
    assert n == 1_000_000_000 - 4 * 20
    assert pu.path == "region"
    uk = dev.download(pu.out_keys, pu.n_out, np.uint64)
    up = dev.download(pu.out_vals, pu.n_out, np.uint32)
    codes = dev.download(pu.codes, pu.n_bases, np.uint8)
    pu.free()
    assert (uk[1:] > uk[:-1]).all()
    rng = np.random.default_rng(0)
    for j in rng.integers(0, len(uk), 2000):
        b = int(up[j]) >> 1
        w = codes[b : b + 21] & 3
        key = 0
        for c in w.tolist():
            key = (key << 2) | c
        assert key == int(uk[j])
    del codes
    pc = engine.ResidentPipeline(dev, text, 21, mode="count")
    del text
    assert pc.step() == n and pc.path == "region"
    ck = dev.download(pc.out_keys, pc.n_out, np.uint64)
    cc = dev.download(pc.out_vals, pc.n_out, np.uint32)
    pc.extract_only()
    keys = dev.download(pc.keys, n, np.uint64)
    pc.free()
    assert int(cc.sum()) == n
    assert (ck[1:] > ck[:-1]).all()
    assert int(np.sum(ck * cc.astype(np.uint64), dtype=np.uint64)) == int(np.sum(keys, dtype=np.uint64))
    del keys
    np.testing.assert_array_equal(ck[cc == 1], uk)


@pytest.mark.parametrize("k", [26, 31, 32])
@pytest.mark.parametrize("rc", [False, True])
def test_groups_count_long_k(dev, golden_inputs, k, rc):
    """Count items carry no window index, so the region path takes k up to
    32 (config 3's k = 31) -- bit-exact vs np_oracle."""
    for text in _texts(golden_inputs):
        got = _groups(dev, text, k, rc, "count")
        assert got is not None
        want = _oracle(text, k, rc, "count")
        np.testing.assert_array_equal(got[0], want[0])
        np.testing.assert_array_equal(got[1].astype(np.uint64), want[1])


@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("k,rc,canonical", [(21, False, False), (21, True, False), (31, False, False),
                                            (21, False, True)])
def test_local_rounds_match_oracle(dev, mode, k, rc, canonical):
    """dist.local_groups: the key rounds of the multi-GPU path on one GPU
    (the inputs kman_groups does not take), forced into >= 3 rounds."""
    import inputs
    import np_oracle
    from kman_amd import dist, engine

    if canonical and mode == "uniq":
        pytest.skip("canonical keys are counted")
    if mode == "uniq" and k > 25:
        pytest.skip("uniq items hold the window index: k <= 25")
    text = inputs.grch38_like(3, n_bases=250_000)
    p = engine.parse(dev, text)
    try:
        r = dist.local_groups(p, k, rc, mode, canonical, max_round_items=60_000)
        try:
            keys = dev.download(r.ukeys if mode == "count" else r.keys, r.n, np.uint64)
            vals = dev.download(r.counts if mode == "count" else r.pos, r.n,
                                np.uint32 if (r.count_bytes if mode == "count" else r.pos_bytes) == 4 else np.uint64)
        finally:
            engine.free_result(r)
    finally:
        p.free()
    kk, pp = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k, rc=rc, canonical=canonical)
    sk, sp = np_oracle.stable_sort(kk, pp)
    wk, wv = np_oracle.rle_count(sk) if mode == "count" else np_oracle.rle_uniq(sk, sp)
    np.testing.assert_array_equal(keys, wk)
    np.testing.assert_array_equal(vals.astype(np.uint64), wv)


def test_skewed_input_takes_the_rounds(dev):
    """A repeat that overflows kman_groups' regions: count_text / uniq_text go
    through the local key rounds (only the overflowing round redone by key
    range) and stay byte-exact vs the C oracle."""
    import subprocess
    import tempfile

    import inputs
    from conftest import ROOT
    from kman_amd import engine

    rep = b"ACGTTGCAAGGCTTACGATCGATCGGATCC"
    text = inputs.SynthLayout(150_000, 8, record_len=40_000).read(0, 10**9) + b">rep\n" + \
        b"\n".join([rep * 2] * 20_000) + b"\n"
    exe = os.path.join(ROOT, "oracle", "kman_oracle")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "in.fa")
        open(src, "wb").write(text)
        for cmd, fn in (("count", engine.count_text), ("uniq", engine.uniq_text)):
            subprocess.run([exe, cmd, src, os.path.join(d, "w"), "21"], check=True)
            assert fn(text, 21, dev=dev) == open(os.path.join(d, "w"), "rb").read()


@pytest.mark.parametrize("k,rc", [(21, False), (13, True), (25, False), (9, False)])
def test_groups_early_count_checked(dev, golden_inputs, monkeypatch, k, rc):
    """The uniq finish under its early-count check (KMAN_RG_CHECK=1: every
    thread compares the singleton marks of the early count with the rows its
    sorted keys give) returns the oracle's rows and raises nothing."""
    monkeypatch.setenv("KMAN_RG_CHECK", "1")
    for text in _texts(golden_inputs):
        got = _groups(dev, text, k, rc, "uniq")
        if got is None:
            continue
        want = _oracle(text, k, rc, "uniq")
        np.testing.assert_array_equal(got[0], want[0])
        np.testing.assert_array_equal(got[1].astype(np.uint64), want[1])


def test_groups_early_count_check_catches_a_wrong_mark(dev, monkeypatch):
    """One wrong singleton mark (KMAN_RG_CHECK=hook=<region>: the test hook
    flips the early count's mark of one item in that region) fails the call
    with the early-count error, not a look-back timeout; the next call on the
    same context is correct again."""
    import inputs

    text = inputs.syn_numpy(3_000_000, 6, record_len=1 << 20)
    monkeypatch.setenv("KMAN_RG_CHECK", "hook=3")
    with pytest.raises(RuntimeError, match="early row count"):
        _groups(dev, text, 21, False, "uniq")
    monkeypatch.setenv("KMAN_RG_CHECK", "0")
    got = _groups(dev, text, 21, False, "uniq")
    want = _oracle(text, 21, False, "uniq")
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1].astype(np.uint64), want[1])
