"""BASELINE config 3 at its stated size (10 GB FASTA, k = 31,
`kmer count`) inside a test: the synthetic 10 GB file is generated on the
device (kman_synth_fasta, byte-identical to tests/golden/inputs.SynthLayout),
parsed in 1 GiB chunks and counted through the key rounds (dist.LocalRounds,
the path the engine takes past the single-call region limit).

No CPU oracle finishes 10 G k-mers in a test, so the bar is size-independent
properties plus an independent GPU path on a slice:
  * the counts sum to the analytic number of windows (uniform ACGT: every
    window of a record of L >= k bases is a k-mer, L - k + 1 of them);
  * the output keys are strictly increasing (sorted, no key split over two
    rows), checked slice by slice with kman_count_descents + kman_rle_count;
  * the rows of one key range equal the general path's (kman_extract_range
    + kman_sort + kman_rle_count over the whole file for that range)."""

from __future__ import annotations

from ctypes import byref, c_int, c_uint64, c_void_p

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K = 31
SIZE = 10_000_000_000


def _lower_bound(dev, buf, n, key):
    """First row index with keys[i] >= key (device array, O(log n) reads)."""
    lo, hi = 0, n
    while lo < hi:
        mid = (lo + hi) // 2
        if int(dev.download(buf, 1, np.uint64, offset=8 * mid)[0]) < key:
            lo = mid + 1
        else:
            hi = mid
    return lo


def test_config3_full_size_count():
    import inputs
    from kman_amd import _native as N
    from kman_amd import dist, engine, shard

    lay = inputs.SynthLayout(SIZE, 2)
    rd = shard.SynthReader(lay)
    dev = engine.default_device()
    L = N.lib()
    sp = shard.shard_specs(rd, 1, K)[0]
    ld = shard.ShardLoader(dev, rd, sp, K, chunk_bytes=1 << 30)
    sh = ld.load()
    lr = None
    try:
        names = sh.names
        off = np.concatenate([[0], np.cumsum([len(x) for x in names])]).astype(np.uint64)
        p = engine.Parsed(dev, sh.codes, sh.n_own, len(names), np.zeros(len(names), np.uint64), sh.rec_seq, names,
                          b"".join(names), off)
        lens = lay.tab.reshape(-1, 3)[:, 2].astype(np.int64)
        want_kmers = int(np.maximum(lens - K + 1, 0).sum())
        assert p.n_bases == SIZE

        lr = dist.LocalRounds(p, K, False, "count")
        lr.step()
        r = lr.result()
        n = r.n
        assert lr.pipe.fallback_rounds == 0
        cdt = np.uint32 if r.count_bytes == 4 else np.uint64

        # 1. counts sum to the windows, 2. strictly increasing keys, by slices
        total, step = 0, 1 << 28
        tmp_k, tmp_c = dev.alloc(8 * step), dev.alloc(4 * step)
        try:
            prev_last = -1
            for a in range(0, n, step):
                m = min(step, n - a)
                cnt = dev.download(r.counts, m, cdt, offset=r.count_bytes * a)
                total += int(cnt.sum(dtype=np.uint64))
                d = c_uint64(0)
                N.check(dev.ctx, L.kman_count_descents(dev.ctx, c_void_p(r.ukeys.ptr + 8 * a), m, byref(d)), "desc")
                assert d.value == 0
                u = c_uint64(0)
                N.check(dev.ctx, L.kman_rle_count(dev.ctx, c_void_p(r.ukeys.ptr + 8 * a), m, c_void_p(tmp_k.ptr),
                                                  c_void_p(tmp_c.ptr), 4, byref(u)), "rle")
                assert u.value == m  # no key twice inside the slice
                first = int(dev.download(r.ukeys, 1, np.uint64, offset=8 * a)[0])
                assert first > prev_last  # nor across slices
                prev_last = int(dev.download(r.ukeys, 1, np.uint64, offset=8 * (a + m - 1))[0])
        finally:
            tmp_k.free()
            tmp_c.free()
        assert total == want_kmers

        # 3. one key range (top 16 key bits = 0x9e37) against the general path
        shift = 2 * K - 16
        klo = 0x9E37 << shift
        khi = ((0x9E37 + 1) << shift) - 1
        got = c_uint64(0)
        rc = L.kman_extract_range(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, K, 0, klo, khi, None, None, 4, 0, None,
                                  byref(got))
        assert rc in (N.KMAN_OK, N.KMAN_ECAP)
        m = int(got.value)
        assert m > 0
        ka, kb = dev.alloc(8 * m), dev.alloc(8 * m)
        uk, uc = dev.alloc(8 * m), dev.alloc(4 * m)
        try:
            N.check(dev.ctx, L.kman_extract_range(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, K, 0, klo, khi,
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
        i0, i1 = _lower_bound(dev, r.ukeys, n, klo), _lower_bound(dev, r.ukeys, n, khi + 1)
        np.testing.assert_array_equal(dev.download(r.ukeys, i1 - i0, np.uint64, offset=8 * i0), want_k)
        np.testing.assert_array_equal(dev.download(r.counts, i1 - i0, cdt, offset=r.count_bytes * i0), want_c)
    finally:
        if lr is not None:
            lr.free()
        ld.free()
