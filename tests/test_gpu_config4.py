"""BASELINE config 4's per-rank shape at full size inside a test (SURVEY §8:
100 GB synthetic FASTA, k = 21, over 8 GPUs, i.e. 12.5 GB per rank): a 12.5 GB
synthetic FASTA generated on the device (kman_synth_fasta, byte-identical to
tests/golden/inputs.SynthLayout), parsed in 1 GiB chunks and counted by the
multi-GPU pipeline with a real RCCL communicator at world size 1
(dist.DistPipeline: shard histogram, R key rounds of pass 0 / pass 1 /
pass 1b / the round finish) -- the code bench.py's `--dist --shard-gb 12.5`
line times, and that each rank of the 8-GPU run executes on its range.

No CPU oracle finishes 12.5 G k-mers in a test, so the bar is the one of
test_gpu_config3.py -- size-independent properties plus an independent GPU
path on a slice (reference behaviour kept: join.py:63-93, globally ordered
rows, one per distinct key; join.py:266-285, the counts):
  * the counts sum to the analytic number of windows (uniform ACGT: a record
    of L >= k bases holds L - k + 1 windows);
  * the output keys are strictly increasing (kman_count_descents + a
    run-length pass per slice, and across slice edges);
  * the rows of one key range equal the general path's (kman_extract_range +
    kman_sort + kman_rle_count over the same codes)."""

from __future__ import annotations

from ctypes import byref, c_int, c_uint64, c_void_p

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K = 21
PER_RANK = 12_500_000_000


def _lower_bound(dev, buf, n, key):
    lo, hi = 0, n
    while lo < hi:
        mid = (lo + hi) // 2
        if int(dev.download(buf, 1, np.uint64, offset=8 * mid)[0]) < key:
            lo = mid + 1
        else:
            hi = mid
    return lo


def test_config4_rank_shape_full_size():
    import inputs
    from kman_amd import _native as N
    from kman_amd import dist, engine, shard

    lay = inputs.SynthLayout(PER_RANK, 1)
    rd = shard.SynthReader(lay)
    dev = engine.default_device()
    L = N.lib()
    # the pipeline of one rank, with a real RCCL communicator of one rank:
    # the exchange degenerates, the rest is each rank's work in the 8-GPU
    # run of config 4 (bench.py --dist --shard-gb 12.5)
    pipe = dist.DistPipeline(dev, rd, K, "count", 1, 0, dist.unique_id(), chunk_bytes=1 << 30, reparse=False)
    try:
        assert pipe.comm.count() == (1, 0)
        n_k = pipe.step()
        assert pipe.path == "region" and pipe.fallback_rounds == 0 and pipe.rounds >= 2
        ok_, ov_, vb = pipe._out
        n = pipe.n_out
        cdt = np.uint32 if vb == 4 else np.uint64
        lens = lay.tab.reshape(-1, 3)[:, 2].astype(np.int64)
        want = int(np.maximum(lens - K + 1, 0).sum())
        assert n_k == want

        # 1. counts sum to the windows, 2. strictly increasing keys, by slices
        total, step = 0, 1 << 28
        tmp_k, tmp_c = dev.alloc(8 * step), dev.alloc(4 * step)
        try:
            prev_last = -1
            for a in range(0, n, step):
                m = min(step, n - a)
                total += int(dev.download(ov_, m, cdt, offset=vb * a).sum(dtype=np.uint64))
                d = c_uint64(0)
                N.check(dev.ctx, L.kman_count_descents(dev.ctx, c_void_p(ok_.ptr + 8 * a), m, byref(d)), "desc")
                assert d.value == 0
                u = c_uint64(0)
                N.check(dev.ctx, L.kman_rle_count(dev.ctx, c_void_p(ok_.ptr + 8 * a), m, c_void_p(tmp_k.ptr),
                                                  c_void_p(tmp_c.ptr), 4, byref(u)), "rle")
                assert u.value == m
                first = int(dev.download(ok_, 1, np.uint64, offset=8 * a)[0])
                assert first > prev_last
                prev_last = int(dev.download(ok_, 1, np.uint64, offset=8 * (a + m - 1))[0])
        finally:
            tmp_k.free()
            tmp_c.free()
        assert total == want

        # 3. one key range (top 16 key bits = 0x9e37) against the general path
        sh = pipe.shard
        shift = 2 * K - 16
        klo = 0x9E37 << shift
        khi = ((0x9E37 + 1) << shift) - 1
        got = c_uint64(0)
        rc = L.kman_extract_range(dev.ctx, c_void_p(sh.codes.ptr), sh.n_eff, K, 0, klo, khi, None, None, 4, 0, None,
                                  byref(got))
        assert rc in (N.KMAN_OK, N.KMAN_ECAP)
        m = int(got.value)
        assert m > 0
        ka, kb = dev.alloc(8 * m), dev.alloc(8 * m)
        uk, uc = dev.alloc(8 * m), dev.alloc(4 * m)
        try:
            N.check(dev.ctx, L.kman_extract_range(dev.ctx, c_void_p(sh.codes.ptr), sh.n_eff, K, 0, klo, khi,
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
        i0, i1 = _lower_bound(dev, ok_, n, klo), _lower_bound(dev, ok_, n, khi + 1)
        np.testing.assert_array_equal(dev.download(ok_, i1 - i0, np.uint64, offset=8 * i0), want_k)
        np.testing.assert_array_equal(dev.download(ov_, i1 - i0, cdt, offset=vb * i0), want_c)
    finally:
        pipe.free()
