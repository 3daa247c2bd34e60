"""The multi-GPU data path and config 5 at their own sizes (VERDICT r05 items
1-2), checked through size-independent properties and by comparing whole
outputs with kman_row_digest (a position-keyed checksum of every row, run on
the device: no oracle finishes giga-k-mer inputs in a test).

  * kman_row_digest itself against a numpy restatement;
  * G = 8 simulated ranks (dist.SimGroup: 8 contexts on one GPU, the
    all-to-all as device copies) over a 4 GB synthetic FASTA in R >= 3 key
    rounds: every rank's exchange is a real destination-major send arena and
    the concatenated rows must equal, bit for bit, one rank's rows over the
    whole file (join.py:63-93: one globally ordered output);
  * config 5 (GRCh38, k = 21, canonical abundance spectrum) on the 3.1 Gbp
    GRCh38-shaped and GRCh38-skewed stand-ins (GRCh38 itself is not in the
    container): the counts sum to the valid windows counted on the host, the
    unordered (KMAN_MIXED) spectrum equals the key-ordered rows' spectrum,
    and the rows of one canonical key range equal the general path's count
    of the same range (canonical counts = the `count -r` rows with key <=
    rc(key) for odd k, seq.py:274-282, pinned at small sizes by
    test_gpu_canonical.py)."""

from __future__ import annotations

from ctypes import byref, c_int, c_uint64, c_void_p

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K = 21


def _digest(dev, keys, vals, vb, n, first=0):
    from kman_amd import _native as N

    out = (c_uint64 * 4)()
    N.check(dev.ctx, N.lib().kman_row_digest(dev.ctx, c_void_p(keys.ptr), c_void_p(vals.ptr) if vals else None, vb, n,
                                             first, out), "kman_row_digest")
    return [int(x) for x in out]


def _mix(x):
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xFF51AFD7ED558CCD)
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xC4CEB9FE1A85EC53)
    return x ^ (x >> np.uint64(33))


def digest_np(keys, vals, first=0):
    """numpy restatement of kman_row_digest (include/kman.h)."""
    with np.errstate(over="ignore"):
        i = np.arange(first, first + len(keys), dtype=np.uint64)
        v = np.zeros(len(keys), np.uint64) if vals is None else vals.astype(np.uint64)
        h = _mix(keys ^ _mix(v + i * np.uint64(0x9E3779B97F4A7C15)))
        hs = int(h.sum(dtype=np.uint64))
        vs = int(v.sum(dtype=np.uint64))
    return [hs, int(np.bitwise_xor.reduce(h)) if len(h) else 0, vs, int(np.count_nonzero(keys[1:] <= keys[:-1]))]


def _combine(parts):
    out = [0, 0, 0, 0]
    for d in parts:
        out[0] = (out[0] + d[0]) & ((1 << 64) - 1)
        out[1] ^= d[1]
        out[2] = (out[2] + d[2]) & ((1 << 64) - 1)
        out[3] += d[3]
    return out


@pytest.mark.parametrize("vb", [0, 4, 8])
def test_row_digest_matches_numpy(vb):
    from kman_amd import engine

    dev = engine.default_device()
    rng = np.random.default_rng(vb)
    n = 3_000_017
    keys = np.sort(rng.integers(0, 1 << 42, n, dtype=np.uint64))
    keys[1000] = keys[999]  # one non-increase
    vdt = {4: np.uint32, 8: np.uint64}.get(vb)
    vals = rng.integers(0, 1 << 31, n).astype(vdt) if vb else None
    dk = dev.alloc(8 * n)
    dv = dev.alloc(max(vb, 1) * n)
    try:
        dev.upload(dk, keys)
        if vb:
            dev.upload(dv, vals)
        got = _digest(dev, dk, dv if vb else None, vb, n)
        assert got == digest_np(keys, vals)
        assert got[3] >= 1  # (the forced one; random 42-bit keys may repeat too)
        # slices combine (first = the slice's start)
        a = 1_234_567
        from kman_amd import _native as N

        parts = []
        for lo, hi in ((0, a), (a, n)):
            o = (c_uint64 * 4)()
            N.check(dev.ctx, N.lib().kman_row_digest(dev.ctx, c_void_p(dk.ptr + 8 * lo),
                                                     c_void_p(dv.ptr + vb * lo) if vb else None, vb, hi - lo, lo, o),
                    "digest")
            parts.append([int(x) for x in o])
        c = _combine(parts)
        assert c == got  # (the non-increase at 1000 lies inside the first slice)
    finally:
        dk.free()
        dv.free()


def _sim_rows_digest(pipes):
    """Digest of the G ranks' rows concatenated in rank order (uniq pos
    rebased to global base indices on the device first)."""
    from kman_amd import _native as N

    parts, at, n = [], 0, 0
    for p in pipes:
        ok_, ov_, vb = p._out
        if p.mode == "uniq" and p.n_out:
            offs = np.ascontiguousarray(np.asarray(p.base_off, np.uint64))
            N.check(p.dev.ctx, N.lib().kman_rebase_pos(p.dev.ctx, c_void_p(ov_.ptr), p.n_out,
                                                       offs.ctypes.data_as(c_void_p), len(offs)), "rebase")
        d = _digest(p.dev, ok_, ov_, vb, p.n_out, at)
        parts.append(d)
        at += p.n_out
        n += p.n_out
    c = _combine(parts)
    # rows strictly increase across the rank boundaries too
    last = None
    for p in pipes:
        if not p.n_out:
            continue
        ok_ = p._out[0]
        first = int(p.dev.download(ok_, 1, np.uint64)[0])
        if last is not None:
            assert first > last
        last = int(p.dev.download(ok_, 1, np.uint64, offset=8 * (p.n_out - 1))[0])
    return n, c


@pytest.mark.parametrize("mode,gb,max_round", [("count", 4.0, 200_000_000), ("uniq", 1.0, 50_000_000)])
def test_dist_g8_multi_gb_matches_one_rank(mode, gb, max_round):
    """8 simulated ranks over one multi-GB FASTA, R >= 3 key rounds, each
    round's exchange through the destination-major send arena: the rows
    concatenated in rank order equal one rank's rows over the whole file."""
    import inputs
    from kman_amd import dist, engine, shard

    lay = inputs.SynthLayout(int(gb * 1e9), 7)
    rd = shard.SynthReader(lay)
    lens = lay.tab.reshape(-1, 3)[:, 2].astype(np.int64)
    windows = int(np.maximum(lens - K + 1, 0).sum())
    G = 8
    devs = [engine.Device(0) for _ in range(G)]
    pipes = []
    try:
        for r in range(G):
            pipes.append(dist.DistPipeline(devs[r], rd, K, mode, G, r, None, chunk_bytes=1 << 28,
                                           max_round_items=max_round))
        dist.SimGroup(pipes).step()
        assert all(p.path == "region" and p.fallback_rounds == 0 for p in pipes)
        assert len({p.rounds for p in pipes}) == 1 and pipes[0].rounds >= 3
        assert sum(p.exchanged_items for p in pipes) == windows
        assert sum(p.n_local for p in pipes) == windows
        n8, d8 = _sim_rows_digest(pipes)
    finally:
        for p in pipes:
            p.free()
        for d in devs:
            d.close()
    dev = engine.Device(0)
    one = dist.DistPipeline(dev, rd, K, mode, 1, 0, None, chunk_bytes=1 << 28)
    try:
        dist.SimGroup([one]).step()
        assert one.path == "region" and one.fallback_rounds == 0
        n1, d1 = _sim_rows_digest([one])
    finally:
        one.free()
        dev.close()
    assert d1[3] == 0 and d8[3] == 0  # strictly increasing keys
    if mode == "count":
        assert d1[2] == windows
    else:
        assert n1 > 0.999 * windows  # (k = 21 over random bases: almost every key once)
    assert (n8, d8) == (n1, d1)


# ----------------------------------------------------------------- config 5


def valid_windows(text: bytes, k: int) -> int:
    """Windows of k ACGT / acgt bases within one record (seq.py:313-327: the
    record upper-cased, a window skipped if any base is outside the DNA
    alphabet; N and every other letter skip), counted from the text itself
    per record (header line dropped, line ends removed) by runs of valid
    bases.  The GRCh38-shaped inputs have no CR, spaces or empty records."""
    a = np.frombuffer(text, np.uint8)
    lut = np.zeros(256, np.uint8)
    for c in b"ACGTacgt":
        lut[c] = 1
    lut[ord("\n")] = 2
    hdr = np.flatnonzero(a == ord(">"))
    total = 0
    for j, h in enumerate(hdr.tolist()):
        e = int(hdr[j + 1]) if j + 1 < len(hdr) else len(a)
        s = text.index(b"\n", h) + 1
        m = lut[a[s:e]]
        v = m[m != 2]
        c = np.concatenate([[0], np.cumsum(v, dtype=np.int64)])
        total += int(np.count_nonzero(c[k:] - c[:-k] == k))
    return total


@pytest.mark.parametrize("shape", ["like", "skewed"])
def test_config5_full_size(shape):
    """BASELINE config 5's workload at its size: 3.1 Gbp, k = 21, canonical
    counts + abundance spectrum, one GPU through the key rounds."""
    import inputs
    from kman_amd import _native as N
    from kman_amd import dist, engine

    gen = inputs.grch38_like if shape == "like" else inputs.grch38_skewed
    text = gen(38, n_bases=3_100_000_000, n_records=25)
    windows = valid_windows(text, K)
    dev = engine.default_device()
    p = engine.parse(dev, text)
    del text
    L = N.lib()
    NB = 16384
    d_h = dev.alloc(8 * NB)
    try:
        spectra = {}
        for ordered in (True, False):
            r = dist.local_groups(p, K, False, "count", True, ordered=ordered)
            assert r is not None
            try:
                d = _digest(dev, r.ukeys, r.counts, r.count_bytes, r.n)
                # 1. the canonical counts sum to the valid windows (one per window)
                assert d[2] == windows
                if ordered:
                    assert d[3] == 0  # key order
                N.check(dev.ctx, L.kman_count_hist(dev.ctx, c_void_p(r.counts.ptr), r.count_bytes, r.n,
                                                   c_void_p(d_h.ptr), NB), "hist")
                h = dev.download(d_h, NB, np.uint64)
                assert int(h.sum()) == r.n
                spectra[ordered] = (r.n, h)
                if ordered:
                    _canonical_range_matches_general(dev, p, r)
            finally:
                r.ukeys.free()
                r.counts.free()
        # 2. the unordered (mixed-key) spectrum is the ordered rows' spectrum
        assert spectra[True][0] == spectra[False][0]
        np.testing.assert_array_equal(spectra[True][1], spectra[False][1])
        # Σ c h[c] = the windows (exact while no count reaches the last bin,
        # which collects every count >= NB - 1)
        h = spectra[True][1]
        below = int((np.arange(NB - 1, dtype=np.uint64) * h[:-1]).sum())
        assert below == windows if h[-1] == 0 else below + (NB - 1) * int(h[-1]) <= windows
    finally:
        d_h.free()
        p.free()


def _lower_bound(dev, buf, n, key):
    lo, hi = 0, n
    while lo < hi:
        mid = (lo + hi) // 2
        if int(dev.download(buf, 1, np.uint64, offset=8 * mid)[0]) < key:
            lo = mid + 1
        else:
            hi = mid
    return lo


def _canonical_range_matches_general(dev, p, r):
    """3. the rows of canonical keys with top 14 bits 0x0a5c (a range of
    the satellite- and repeat-rich low keys) equal the general path's
    (kman_extract_range with KMAN_CANONICAL + kman_sort + kman_rle_count)."""
    from kman_amd import _native as N

    L = N.lib()
    shift = 2 * K - 14
    klo, khi = 0x0A5C << shift, ((0x0A5C + 1) << shift) - 1
    got = c_uint64(0)
    rc = L.kman_extract_range(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, K, N.KMAN_CANONICAL, klo, khi, None, None, 4,
                              0, None, byref(got))
    assert rc in (N.KMAN_OK, N.KMAN_ECAP)
    m = int(got.value)
    assert m > 0
    ka, kb, uk, uc = dev.alloc(8 * m), dev.alloc(8 * m), dev.alloc(8 * m), dev.alloc(4 * m)
    try:
        N.check(dev.ctx, L.kman_extract_range(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, K, N.KMAN_CANONICAL, klo, khi,
                                              c_void_p(ka.ptr), None, 4, m, None, byref(got)), "extract_range")
        alt = c_int(0)
        N.check(dev.ctx, L.kman_sort(dev.ctx, c_void_p(ka.ptr), c_void_p(kb.ptr), None, None, 0, m, 2 * K, None,
                                     byref(alt)), "sort")
        keys = kb if alt.value else ka
        nu = c_uint64(0)
        N.check(dev.ctx, L.kman_rle_count(dev.ctx, c_void_p(keys.ptr), m, c_void_p(uk.ptr), c_void_p(uc.ptr), 4,
                                          byref(nu)), "rle")
        want_k = dev.download(uk, nu.value, np.uint64)
        want_c = dev.download(uc, nu.value, np.uint32)
    finally:
        for b in (ka, kb, uk, uc):
            b.free()
    i0, i1 = _lower_bound(dev, r.ukeys, r.n, klo), _lower_bound(dev, r.ukeys, r.n, khi + 1)
    cdt = np.uint32 if r.count_bytes == 4 else np.uint64
    np.testing.assert_array_equal(dev.download(r.ukeys, i1 - i0, np.uint64, offset=8 * i0), want_k)
    np.testing.assert_array_equal(dev.download(r.counts, i1 - i0, cdt, offset=r.count_bytes * i0).astype(np.uint64),
                                  want_c.astype(np.uint64))


@pytest.mark.parametrize("rccl_self", ["0", "1"])
def test_world1_exchange_chunked_messages(monkeypatch, rccl_self):
    """1 GB at world size 1 through a real RCCL communicator with the
    exchange on: the rank's own part as a device copy (the default), or
    (KMAN_RCCL_SELF=1) through RCCL send/recv to self in 512 MiB chunks -- an
    8 GB message, 16 chunks, the loop every peer pair of an N > 1 run takes.
    Rows equal the exchange-free run's (kman_row_digest)."""
    import inputs
    from kman_amd import dist, engine, shard

    monkeypatch.setenv("KMAN_RCCL_SELF", rccl_self)
    lay = inputs.SynthLayout(1_000_000_000, 1)
    rd = shard.SynthReader(lay)
    dev = engine.default_device()
    got = {}
    for xch in (False, True):
        p = dist.DistPipeline(dev, rd, K, "count", 1, 0, dist.unique_id(), chunk_bytes=1 << 30, exchange=xch)
        try:
            p.step()
            if xch:
                assert p.exchanged_items == p.n_local and p.max_message > 8 * (512 << 20)
            ok_, ov_, vb = p._out
            got[xch] = (p.n_out, _digest(dev, ok_, ov_, vb, p.n_out))
        finally:
            p.free()
    assert got[True] == got[False] and got[True][1][3] == 0
