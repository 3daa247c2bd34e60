"""GPU parity: every HIP stage against the oracle, and whole commands against
the reference's golden outputs.  Run on an MI355X with ``pytest -m gpu``.

Bar: bit-exact (integer / byte work).  Stage checks compare with the numpy
restatement (oracle/np_oracle.py); command checks compare output bytes with
the sha256 the reference itself produced (tests/golden/manifest.json)."""

from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from kman_amd import engine

    return engine.default_device()


def _read(path):
    from kman_amd.engine import read_input

    return read_input(path)


WEIRD = [
    b">a\nACGT\n",
    b">a",
    b">a\n",
    b"\n\n>x y\nAC\nGT\n>y\r\nAAAA\rCCCC\r\n>z\rGG\tTT \t \nTT\n",
    b";c\n>\tname\tx\nacgtn\x0bACGT\x0b \n\x0c\n>q\n" + b"A" * 200 + b"\n",
    b">r1\n" + b"ACGT" * 1000 + b"\n>r2\n\n>r3\n" + b"GATTACA\t\t\t\n" * 50,
    b">a\n" + b" \t" * 3000 + b"A\n",  # whitespace run across thread chunks
    b">L\n" + b"ACGTTGCA" * 5000,  # one long line, no final newline
]


def _messy(seed):
    import inputs

    return inputs.messy_records(seed, n_records=60, max_len=20000)


@pytest.mark.parametrize("width", [1, 3, 4, 7, 8, 13, 31, 60, 63, 64, 65, 80, 127, 1000])
def test_parse_fast_tiles_match_oracle(dev, width):
    """Plain sequence text (the fast parse kernels: newline bytes dropped by
    in-register compaction, whole-word LDS staging) at every line width
    around the 4-byte words and 64-byte chunks, upper / lower case and N runs,
    records long enough that most 16 KiB tiles hold no header."""
    import np_oracle
    from kman_amd import engine

    rng = np.random.default_rng(width)
    parts = []
    for r in range(5):
        n = int(rng.integers(20_000, 90_000))
        seq = rng.choice(np.frombuffer(b"ACGTacgtN", np.uint8), n, p=[.24, .24, .24, .24, .01, .01, .01, .005, .005])
        body = seq.tobytes()
        lines = [body[i:i + width] for i in range(0, n, width)]
        parts.append(b">rec%d some description\n" % r + b"\n".join(lines) + b"\n")
    text = b"".join(parts)
    recs = np_oracle.parse_fasta(text)
    codes_ref, rec_seq_ref = np_oracle.codes_of(recs)
    p = engine.parse(dev, text)
    try:
        assert p.n_records == len(recs) and p.n_bases == len(codes_ref)
        got = dev.download(p.codes, p.n_bases + 64, np.uint8)
        np.testing.assert_array_equal(got[: p.n_bases], codes_ref)
        np.testing.assert_array_equal(p.rec_seq, rec_seq_ref)
    finally:
        p.free()


@pytest.mark.parametrize("idx", range(len(WEIRD) + 3))
def test_parse_matches_oracle(dev, golden_inputs, idx):
    import np_oracle
    from kman_amd import engine

    if idx < len(WEIRD):
        text = WEIRD[idx]
    elif idx == len(WEIRD):
        text = _read(golden_inputs["messy2"])
    else:
        text = _messy(idx)
    recs = np_oracle.parse_fasta(text)
    codes_ref, rec_seq_ref = np_oracle.codes_of(recs)
    p = engine.parse(dev, text)
    try:
        assert p.n_records == len(recs)
        assert p.n_bases == len(codes_ref)
        got = dev.download(p.codes, p.n_bases + 64, np.uint8)
        np.testing.assert_array_equal(got[: p.n_bases], codes_ref)
        assert (got[p.n_bases:] == 4).all()
        np.testing.assert_array_equal(p.rec_seq, rec_seq_ref)
        assert p.names == [np_oracle.record_name(t) for t, _ in recs]
        for h, (t, _) in zip(p.rec_hdr, recs):
            assert text[int(h)] == ord(">")
    finally:
        p.free()


@pytest.mark.parametrize("k", [2, 3, 5, 13, 21, 31, 32])
@pytest.mark.parametrize("mode", ["fwd", "rc", "canon"])
def test_extract_matches_oracle(dev, golden_inputs, k, mode):
    import np_oracle
    from kman_amd import engine

    for text in (_read(golden_inputs["messy1"]), _messy(99), WEIRD[5]):
        recs = np_oracle.parse_fasta(text)
        kref, pref = np_oracle.stream_kmers(recs, k, rc=mode == "rc", canonical=mode == "canon")
        p = engine.parse(dev, text)
        try:
            km = engine.extract(p, k, rc=mode == "rc", want_pos=True, canonical=mode == "canon")
            try:
                assert km.n == len(kref)
                keys = dev.download(km.keys, km.n, np.uint64)
                pos = dev.download(km.pos, km.n, np.uint32 if km.pos_bytes == 4 else np.uint64)
                np.testing.assert_array_equal(keys, kref)
                np.testing.assert_array_equal(pos.astype(np.uint64), pref)
                # fused radix histograms == histograms of the keys
                hist = dev.download(km.hist, 8 * 256, np.uint64).reshape(8, 256)
                from kman_amd import _native as N
                import ctypes

                npass, sh, bi = ctypes.c_uint32(), (ctypes.c_uint32 * 8)(), (ctypes.c_uint32 * 8)()
                N.lib().kman_sort_plan_range(km.lo_bit, 2 * k, ctypes.byref(npass), sh, bi)
                for q in range(npass.value):
                    d = (kref >> np.uint64(sh[q])) & np.uint64((1 << bi[q]) - 1)
                    want = np.bincount(d.astype(np.int64), minlength=256)
                    np.testing.assert_array_equal(hist[q], want)
            finally:
                km.free()
        finally:
            p.free()


@pytest.mark.parametrize("k", [2, 5, 13, 21, 25, 31])
@pytest.mark.parametrize("rc", [False, True])
@pytest.mark.parametrize("want_pos", [True, False])
def test_extract_sorted_matches_oracle(dev, golden_inputs, k, rc, want_pos):
    """kman_extract_sorted (histogram pre-pass + fused extract/first pass +
    remaining prefix passes; k > 25 runs extract + sort_range) == the stream
    k-mers stably sorted by their top bits [lo, 2k)."""
    import ctypes
    from ctypes import byref, c_void_p
    import np_oracle
    from kman_amd import _native as N, engine

    L = N.lib()
    for text in (_read(golden_inputs["messy1"]), _messy(7), WEIRD[5], b">x\n" + b"ACGT" * 40000 + b"\n"):
        recs = np_oracle.parse_fasta(text)
        kref, pref = np_oracle.stream_kmers(recs, k, rc=rc)
        p = engine.parse(dev, text)
        try:
            nb = max(p.n_bases * (2 if rc else 1), 1)
            for lo in sorted({engine.split_bits(nb, 2 * k), max(0, 2 * k - 7), 0}):
                bufs = [dev.alloc(8 * nb) for _ in range(2)]
                pbufs = [dev.alloc(4 * nb) for _ in range(2)] if want_pos else [None, None]
                try:
                    n, res = ctypes.c_uint64(0), ctypes.c_int(0)
                    P = lambda b: c_void_p(b.ptr if b is not None else None)  # noqa: E731
                    flags = (N.KMAN_RC if rc else 0) | (N.KMAN_WANT_POS if want_pos else 0)
                    N.check(dev.ctx, L.kman_extract_sorted(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k, flags, lo,
                                                           P(bufs[0]), P(bufs[1]), P(pbufs[0]), P(pbufs[1]), 4, nb,
                                                           byref(n), byref(res)), "extract_sorted")
                    assert n.value == len(kref)
                    c = res.value
                    order = np.argsort(kref >> np.uint64(lo) if lo < 64 else np.zeros(len(kref), np.uint64),
                                       kind="stable")
                    got = dev.download(bufs[c], n.value, np.uint64)
                    np.testing.assert_array_equal(got, kref[order])
                    if want_pos:
                        gp = dev.download(pbufs[c], n.value, np.uint32).astype(np.uint64)
                        np.testing.assert_array_equal(gp, pref[order])
                finally:
                    for b in bufs + pbufs:
                        if b is not None:
                            b.free()
        finally:
            p.free()


def _sort_case(dev, keys, vals, key_bits):
    from kman_amd import engine

    n = len(keys)
    km = engine.Kmers(dev.alloc(8 * max(n, 1)), dev.alloc(8 * max(n, 1)), None, None, 0, n, key_bits // 2,
                      dev.alloc(8 * 256 * 8))
    if vals is not None:
        vb = vals.dtype.itemsize
        km.pos, km.pos_alt, km.pos_bytes = dev.alloc(vb * max(n, 1)), dev.alloc(vb * max(n, 1)), vb
        dev.upload(km.pos, vals)
    dev.upload(km.keys, keys)
    # no precomputed histogram: exercise kman_sort's own histogram pass
    import ctypes
    from kman_amd import _native as N

    res = ctypes.c_int(0)
    rc = N.lib().kman_sort(dev.ctx, ctypes.c_void_p(km.keys.ptr), ctypes.c_void_p(km.alt.ptr),
                           ctypes.c_void_p(km.pos.ptr if km.pos else None),
                           ctypes.c_void_p(km.pos_alt.ptr if km.pos_alt else None), km.pos_bytes, n, key_bits,
                           None, ctypes.byref(res))
    N.check(dev.ctx, rc, "kman_sort")
    kb = km.alt if res.value else km.keys
    got_k = dev.download(kb, n, np.uint64)
    got_v = None
    if vals is not None:
        vbuf = km.pos_alt if res.value else km.pos
        got_v = dev.download(vbuf, n, vals.dtype)
    km.free()
    return got_k, got_v


@pytest.mark.parametrize("n", [0, 1, 2, 63, 4095, 4096, 4097, 100_003, 3_000_001])
@pytest.mark.parametrize("key_bits", [8, 14, 42, 64])
def test_sort_stable(dev, n, key_bits):
    import np_oracle

    rng = np.random.default_rng(n * 131 + key_bits)
    if key_bits == 64:
        keys = rng.integers(0, 2**63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n).astype(np.uint64)
    else:
        # few distinct values too, so ties exercise stability
        hi = min(2**key_bits, 1000 if n > 1000 and key_bits < 20 else 2**key_bits)
        keys = rng.integers(0, hi, size=n, dtype=np.uint64)
        keys = keys << np.uint64(max(0, key_bits - int(np.ceil(np.log2(max(hi, 2))))))
    vals = np.arange(n, dtype=np.uint32)
    want_k, want_v = np_oracle.stable_sort(keys, vals)
    got_k, got_v = _sort_case(dev, keys, vals, key_bits)
    np.testing.assert_array_equal(got_k, want_k)
    np.testing.assert_array_equal(got_v, want_v)
    if n and key_bits == 42:
        got_k2, _ = _sort_case(dev, keys, None, key_bits)
        np.testing.assert_array_equal(got_k2, want_k)
        v64 = np.arange(n, dtype=np.uint64) * np.uint64(3)
        got_k3, got_v3 = _sort_case(dev, keys, v64, key_bits)
        np.testing.assert_array_equal(got_k3, want_k)
        np.testing.assert_array_equal(got_v3, np_oracle.stable_sort(keys, v64)[1])


@pytest.mark.parametrize("n", [1, 2, 4096, 4097, 50_000, 2_000_000])
@pytest.mark.parametrize("distinct", [1, 7, 1000, 10**9])
def test_rle_count_and_uniq(dev, n, distinct):
    import np_oracle
    from kman_amd import engine

    rng = np.random.default_rng(n + distinct)
    keys = np.sort(rng.integers(0, distinct, size=n, dtype=np.uint64))
    vals = rng.integers(0, 2**31, size=n, dtype=np.uint32)
    km = engine.Kmers(dev.alloc(8 * n), dev.alloc(8), dev.alloc(4 * n), None, 4, n, 31, dev.alloc(8))
    dev.upload(km.keys, keys)
    dev.upload(km.pos, vals)
    km.sorted = True
    r = engine.rle_count(km, dev)
    uk, uc = engine.download_count(dev, r)
    wk, wc = np_oracle.rle_count(keys)
    np.testing.assert_array_equal(uk, wk)
    np.testing.assert_array_equal(uc.astype(np.uint64), wc)
    q = engine.rle_uniq(km, dev)
    sk, sv = engine.download_uniq(dev, q)
    wk2, wv2 = np_oracle.rle_uniq(keys, vals)
    np.testing.assert_array_equal(sk, wk2)
    np.testing.assert_array_equal(sv, wv2)
    km.free()


def _keys_of(dist, n, key_bits, rng):
    top = 2**key_bits if key_bits < 64 else 2**64
    if dist == "uniform":
        return rng.integers(0, top, size=n, dtype=np.uint64) if key_bits < 64 else \
            rng.integers(0, 2**63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n).astype(np.uint64)
    if dist == "ties":  # few distinct values spread over the whole key range
        pool = rng.integers(0, min(top, 2**63), size=37, dtype=np.uint64)
        return pool[rng.integers(0, len(pool), size=n)]
    # skew: half the keys are one value, a quarter share one prefix, rest uniform
    keys = rng.integers(0, min(top, 2**63), size=n, dtype=np.uint64)
    hot = np.uint64(rng.integers(0, min(top, 2**63)))
    keys[rng.random(n) < 0.5] = hot
    sel = rng.random(n) < 0.25
    low = np.uint64((1 << max(1, key_bits // 3)) - 1)
    keys[sel] = (hot & ~low) | (keys[sel] & low)
    return keys


def _finish_case(dev, keys, vals, key_bits, lo_bit, mode, ob):
    """kman_sort_range over [lo_bit, key_bits) + kman_finish on the device."""
    import ctypes
    from ctypes import byref, c_void_p
    from kman_amd import _native as N

    L = N.lib()
    n = len(keys)
    vb = vals.dtype.itemsize if vals is not None else 0
    bufs = [dev.alloc(8 * max(n, 1)), dev.alloc(8 * max(n, 1))]
    vbufs = [dev.alloc(vb * max(n, 1)), dev.alloc(vb * max(n, 1))] if vb else [None, None]
    okeys, ovals = dev.alloc(8 * max(n, 1)), dev.alloc(8 * max(n, 1))
    try:
        dev.upload(bufs[0], keys)
        if vb:
            dev.upload(vbufs[0], vals)
        res = ctypes.c_int(0)
        p = lambda b: c_void_p(b.ptr if b is not None else None)  # noqa: E731
        N.check(dev.ctx, L.kman_sort_range(dev.ctx, p(bufs[0]), p(bufs[1]), p(vbufs[0]), p(vbufs[1]), vb, n, lo_bit,
                                           key_bits, None, byref(res)), "sort_range")
        c = res.value
        if os.environ.get("KMAN_TEST_VERIFY"):
            got = dev.download(bufs[c], n, np.uint64)
            order = np.argsort(keys >> np.uint64(lo_bit) if lo_bit < 64 else np.zeros(n, np.uint64), kind="stable")
            assert np.array_equal(got, keys[order]), "prefix sort wrong: %d mismatches" % int((got != keys[order]).sum())
        out = ctypes.c_uint64(0)
        N.check(dev.ctx, L.kman_finish(dev.ctx, p(bufs[c]), p(bufs[c ^ 1]), p(vbufs[c]), p(vbufs[c ^ 1]), vb, n,
                                       key_bits, lo_bit, mode, p(okeys), p(ovals), ob, byref(out)), "finish")
        m = int(out.value)
        dev.sync()
        if mode == N.KMAN_FINISH_SORT:
            assert m == n
            return dev.download(bufs[c], n, np.uint64), (dev.download(vbufs[c], n, vals.dtype) if vb else None)
        return dev.download(okeys, m, np.uint64), dev.download(ovals, m, np.uint32 if ob == 4 else np.uint64)
    finally:
        for b in bufs + vbufs + [okeys, ovals]:
            if b is not None:
                b.free()


@pytest.mark.parametrize("n", [1, 2, 1000, 4096, 4097, 100_003, 2_000_001])
@pytest.mark.parametrize("key_bits", [14, 42, 64])
@pytest.mark.parametrize("dist", ["uniform", "ties", "skew"])
@pytest.mark.parametrize("split", ["auto", "coarse"])
def test_finish_modes(dev, n, key_bits, dist, split):
    """prefix sort + kman_finish == stable sort / RLE count / uniq of the
    oracle; 'coarse' prefixes (3 bits) force big segments through the
    presorted-slice fallback, 'skew' makes groups span many chunks."""
    import np_oracle
    from kman_amd import _native as N, engine

    rng = np.random.default_rng(n * 7 + key_bits * 3 + len(dist) + len(split))
    keys = _keys_of(dist, n, key_bits, rng)
    lo = engine.split_bits(n, key_bits) if split == "auto" else key_bits - 3
    vals = np.arange(n, dtype=np.uint32)
    gk, gv = _finish_case(dev, keys, vals, key_bits, lo, N.KMAN_FINISH_SORT, 0)
    wk, wv = np_oracle.stable_sort(keys, vals)
    np.testing.assert_array_equal(gk, wk)
    np.testing.assert_array_equal(gv, wv)
    ck, cc = _finish_case(dev, keys, None, key_bits, lo, N.KMAN_FINISH_COUNT, 4 if n % 2 else 8)
    rk, rcnt = np_oracle.rle_count(wk)
    np.testing.assert_array_equal(ck, rk)
    np.testing.assert_array_equal(cc.astype(np.uint64), rcnt)
    v = rng.integers(0, 2**40, size=n, dtype=np.uint64) if n % 2 else rng.integers(0, 2**31, size=n, dtype=np.uint32)
    uk, uv = _finish_case(dev, keys, v, key_bits, lo, N.KMAN_FINISH_UNIQ, v.dtype.itemsize)
    sk, sv = np_oracle.stable_sort(keys, v)
    qk, qv = np_oracle.rle_uniq(sk, sv)
    np.testing.assert_array_equal(uk, qk)
    np.testing.assert_array_equal(uv, qv)


def test_finish_single_value(dev):
    """every key equal: one segment of n keys, one group spanning every chunk."""
    from kman_amd import _native as N

    n = 300_000
    keys = np.full(n, 12345, dtype=np.uint64)
    vals = np.arange(n, dtype=np.uint32)
    gk, gv = _finish_case(dev, keys, vals, 42, 21, N.KMAN_FINISH_SORT, 0)
    np.testing.assert_array_equal(gk, keys)
    np.testing.assert_array_equal(gv, vals)
    ck, cc = _finish_case(dev, keys, None, 42, 21, N.KMAN_FINISH_COUNT, 4)
    assert ck.tolist() == [12345] and cc.tolist() == [n]
    uk, uv = _finish_case(dev, keys, vals, 42, 21, N.KMAN_FINISH_UNIQ, 4)
    assert len(uk) == 0 and len(uv) == 0


def _golden_cases(key):
    import json

    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return [c for c in json.load(fh)[key] if c["k"] <= 64]


@pytest.mark.parametrize("case", _golden_cases("cases") + _golden_cases("config1"), ids=lambda c: c["name"])
def test_command_matches_reference(dev, golden_inputs, case):
    from kman_amd import engine

    text = _read(golden_inputs[case["input"]])
    rc = "-r" in case.get("flags", [])
    fn = engine.count_text if case["cmd"] == "count" else engine.uniq_text
    out = fn(text, case["k"], rc=rc, dev=dev)
    assert hashlib.sha256(out).hexdigest() == case["sha256"]


def test_error_cases(dev, golden_inputs):
    from kman_amd import engine

    with pytest.raises(AssertionError, match="premature end of file or empty file"):
        engine.count_text(b"", 3, dev=dev)
    with pytest.raises(AssertionError, match="premature end of file or empty file"):
        engine.count_text(b"ACGT\nACGT\n", 3, dev=dev)
    with pytest.raises(AssertionError, match="k must be >= 1, got 1 instead."):
        engine.count_text(b">a\nACGT\n", 1, dev=dev)
    with pytest.raises(AssertionError, match="incompatible string: :0-3:\\+"):
        engine.count_text(_read(golden_inputs["emptyname"]), 3, dev=dev)
    assert engine.count_text(_read(golden_inputs["emptyname_short"]), 5, dev=dev) == b"ACGTA\t1\nCGTAC\t1\n"


def test_full_size_properties(dev):
    """BASELINE config 2 shape (1 GB synthetic FASTA, k=21) through
    size-independent properties: counts sum to the k-mer count, keys strictly
    increase, and the key checksum is preserved by sort + RLE."""
    import inputs
    from kman_amd import engine

    text = inputs.syn_numpy(1_000_000_000, 1)
    p = engine.parse(dev, text)
    del text
    km = engine.extract(p, 21, rc=False, want_pos=False)
    n = km.n
    assert p.n_records == 4 and n == 1_000_000_000 - 4 * 20  # records of <= 256 Mi bases
    unsorted = dev.download(km.keys, n, np.uint64)
    checksum = int(np.sum(unsorted, dtype=np.uint64))
    xor = int(np.bitwise_xor.reduce(unsorted))
    del unsorted
    engine.sort(km, dev)
    r = engine.rle_count(km, dev)
    uk, uc = engine.download_count(dev, r)
    assert int(uc.sum()) == n
    assert (uk[1:] > uk[:-1]).all()
    # u ~ 1 at k=21 over 1e9 uniform k-mers (4^21 = 4.4e12): expected dups ~ n^2 / 2 / 4^21
    assert abs((n - len(uk)) - n * n / 2 / 4**21) < 5 * np.sqrt(n * n / 2 / 4**21) + 10
    sorted_keys = dev.download(km.keys, n, np.uint64)
    assert (sorted_keys[1:] >= sorted_keys[:-1]).all()
    assert int(np.sum(sorted_keys, dtype=np.uint64)) == checksum
    assert int(np.bitwise_xor.reduce(sorted_keys)) == xor
    assert int(np.sum(uk * uc.astype(np.uint64), dtype=np.uint64)) == checksum
    km.free()
    r.ukeys.free()
    r.counts.free()
    p.free()


@pytest.mark.parametrize("k", [33, 40, 57, 64, 65, 96, 127, 200])
@pytest.mark.parametrize("rc,canonical", [(False, False), (True, False), (False, True)])
def test_wide_keys_match_oracle(dev, k, rc, canonical):
    """k > 32 (word keys: two rolled words up to k = 64, kman_extract_words
    beyond): count and uniq rows bit-exact against a restatement over byte
    strings (seq.py:285-328, batch.py:156-168, join.py:95-130,244-285),
    including -r and canonical keys."""
    import inputs
    import np_oracle
    from kman_amd import engine

    text = inputs.messy_records(k, n_records=20, max_len=5000) + inputs.syn_numpy(30_000, k, record_len=9000)
    recs = np_oracle.parse_fasta(text)
    keys, pos = [], []
    base = 0
    comp = bytes.maketrans(b"ACGT", b"TGCA")
    for _, s in recs:
        u = s.upper()
        for i in range(len(u) - k + 1):
            w = u[i:i + k]
            if w.strip(b"ACGT"):
                continue
            r = w.translate(comp)[::-1]
            if canonical:
                keys.append(min(w, r))
                pos.append((base + i) << 1)
            else:
                keys.append(w)
                pos.append((base + i) << 1)
                if rc:
                    keys.append(r)
                    pos.append(((base + i) << 1) | 1)
        base += len(s)
    order = sorted(range(len(keys)), key=lambda j: keys[j])
    sk = [keys[j] for j in order]
    sp = [pos[j] for j in order]
    p = engine.parse(dev, text)
    try:
        for mode in ("count", "uniq"):
            r = engine.words_groups(p, k, rc, mode, canonical)
            try:
                rows = engine.download_words(dev, r.words, r.n, k)
                vals = dev.download(r.vals, r.n, np.uint32 if r.val_bytes == 4 else np.uint64)
            finally:
                engine.free_result(r)
            got = [engine.decode_words(row, k).encode() for row in rows]
            if mode == "count":
                want_k, want_v = [], []
                for j, x in enumerate(sk):
                    if j and x == sk[j - 1]:
                        want_v[-1] += 1
                    else:
                        want_k.append(x)
                        want_v.append(1)
            else:
                want_k, want_v = [], []
                for j, x in enumerate(sk):
                    if (j == 0 or sk[j - 1] != x) and (j + 1 == len(sk) or sk[j + 1] != x):
                        want_k.append(x)
                        want_v.append(sp[j])
            assert got == want_k
            assert vals.tolist() == want_v
    finally:
        p.free()


@pytest.mark.parametrize("nruns", [1, 2, 3, 7, 16])
@pytest.mark.parametrize("vb", [0, 4, 8])
def test_merge_runs_is_a_stable_merge(dev, nruns, vb):
    """kman_merge_runs == heapq.merge over the sorted runs in run order
    (join.py:63-93): equal keys keep run order, then in-run order."""
    import ctypes
    from ctypes import c_void_p

    from kman_amd import _native as N

    rng = np.random.default_rng(nruns * 10 + vb)
    runs = [np.sort(rng.integers(0, 300, size=int(rng.integers(0, 5000)), dtype=np.uint64)) for _ in range(nruns)]
    vals = [np.arange(len(r), dtype=np.uint64) + np.uint64(i << 40) for i, r in enumerate(runs)]
    keys = np.concatenate(runs)
    allv = np.concatenate(vals)
    n = len(keys)
    dt = np.uint32 if vb == 4 else np.uint64
    dk, dv = dev.alloc(8 * max(n, 1)), dev.alloc(8 * max(n, 1))
    ok, ov, tk, tv = (dev.alloc(8 * max(n, 1)) for _ in range(4))
    try:
        if n:
            dev.upload(dk, keys)
            dev.upload(dv, allv.astype(dt) if vb else allv)
        rr, at = [], 0
        for r in runs:
            rr.append(N.Run(dk.ptr + 8 * at, (dv.ptr + vb * at) if vb else None, len(r)))
            at += len(r)
        arr = (N.Run * nruns)(*rr)
        N.check(dev.ctx, N.lib().kman_merge_runs(dev.ctx, arr, nruns, vb, c_void_p(ok.ptr),
                                                 c_void_p(ov.ptr) if vb else None, c_void_p(tk.ptr),
                                                 c_void_p(tv.ptr) if vb else None), "merge")
        # heapq.merge over (key, run, index) == a stable sort of the concatenation
        order = np.argsort(keys, kind="stable")
        np.testing.assert_array_equal(dev.download(ok, n, np.uint64), keys[order])
        if vb:
            np.testing.assert_array_equal(dev.download(ov, n, dt), allv.astype(dt)[order])
        d = ctypes.c_uint64(0)
        N.check(dev.ctx, N.lib().kman_count_descents(dev.ctx, c_void_p(dk.ptr), n, ctypes.byref(d)), "descents")
        assert d.value == (0 if nruns == 1 else int((keys[1:] < keys[:-1]).sum()))
    finally:
        for b in (dk, dv, ok, ov, tk, tv):
            b.free()
