"""BASELINE config 4's per-rank shape at full size inside a test (SURVEY §8:
100 GB synthetic FASTA, k = 21, over 8 GPUs, i.e. 12.5 GB per rank): a 12.5 GB
synthetic FASTA generated on the device (kman_synth_fasta, byte-identical to
tests/golden/inputs.SynthLayout), parsed in 1 GiB chunks and counted by the
multi-GPU pipeline with a real RCCL communicator at world size 1
(dist.DistPipeline: shard histogram, R key rounds of pass 0 / pass 1 /
pass 1b / the round finish).

Two data paths, both at full size:
  * exchange=False: one rank without an exchange (the shard extracted ONCE
    for every key round, KMAN_ONCE) -- a one-GPU-only shortcut;
  * exchange=True: what every rank of the 8-GPU run executes -- per round,
    extraction into the destination-major send arena and ONE kman_alltoallv
    (RCCL send/recv, here to self) whose messages are many 512 MiB chunks
    (comm.hip alltoallv_on), then the passes and the finish on the received
    items.  Its rows must be bit-identical to the exchange=False rows
    (kman_row_digest over all ~12.5 G rows of each run).

No CPU oracle finishes 12.5 G k-mers in a test, so the bar is the one of
test_gpu_config3.py -- size-independent properties plus an independent GPU
path on a slice (reference behaviour kept: join.py:63-93, globally ordered
rows, one per distinct key; join.py:266-285, the counts):
  * the counts sum to the analytic number of windows (uniform ACGT: a record
    of L >= k bases holds L - k + 1 windows);
  * the output keys are strictly increasing (no i with keys[i] <= keys[i-1]);
  * the rows of one key range equal the general path's (kman_extract_range +
    kman_sort + kman_rle_count over the same codes)."""

from __future__ import annotations

from ctypes import byref, c_int, c_uint64, c_void_p

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K = 21
PER_RANK = 12_500_000_000
_DIGESTS = {}


def _lower_bound(dev, buf, n, key):
    lo, hi = 0, n
    while lo < hi:
        mid = (lo + hi) // 2
        if int(dev.download(buf, 1, np.uint64, offset=8 * mid)[0]) < key:
            lo = mid + 1
        else:
            hi = mid
    return lo


def row_digest(dev, keys, vals, vb, n, first=0):
    """kman_row_digest: (hash sum, hash xor, value sum, non-increases)."""
    from kman_amd import _native as N

    out = (c_uint64 * 4)()
    N.check(dev.ctx, N.lib().kman_row_digest(dev.ctx, c_void_p(keys.ptr), c_void_p(vals.ptr) if vals else None, vb, n,
                                             first, out), "kman_row_digest")
    return tuple(int(x) for x in out)


def _range_matches_general_path(dev, pipe, ok_, ov_, n, cdt, vb):
    """The rows of the key range with top 16 key bits 0x9e37 equal the general
    path's count of the same codes."""
    from kman_amd import _native as N

    L = N.lib()
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


def _run_rank(exchange: bool):
    import inputs
    from kman_amd import dist, engine, shard

    lay = inputs.SynthLayout(PER_RANK, 1)
    rd = shard.SynthReader(lay)
    dev = engine.default_device()
    pipe = dist.DistPipeline(dev, rd, K, "count", 1, 0, dist.unique_id(), chunk_bytes=1 << 30, reparse=False,
                             exchange=exchange)
    lens = lay.tab.reshape(-1, 3)[:, 2].astype(np.int64)
    return dev, pipe, int(np.maximum(lens - K + 1, 0).sum())


@pytest.mark.parametrize("exchange", [False, True], ids=["once", "exchange"])
def test_config4_rank_shape_full_size(exchange):
    dev, pipe, want = _run_rank(exchange)
    try:
        assert pipe.comm.count() == (1, 0)
        n_k = pipe.step()
        assert pipe.path == "region" and pipe.fallback_rounds == 0 and pipe.rounds >= 2
        assert n_k == want
        if exchange:
            # the N > 1 data path: every round extracted into the send arena
            # and exchanged, in messages of many 512 MiB chunks
            assert "exchange" in pipe.phase_ms and pipe.exchanged_items == want
            assert pipe.max_message > 4 * (512 << 20)
        else:
            assert "exchange" not in pipe.phase_ms and pipe.exchanged_items == 0
        ok_, ov_, vb = pipe._out
        n = pipe.n_out
        cdt = np.uint32 if vb == 4 else np.uint64
        d = row_digest(dev, ok_, ov_, vb, n)
        # 1. counts sum to the windows, 2. strictly increasing keys
        assert d[2] == want and d[3] == 0
        _DIGESTS[exchange] = (n, d)
        # 3. one key range against the general path
        _range_matches_general_path(dev, pipe, ok_, ov_, n, cdt, vb)
    finally:
        pipe.free()
    if exchange:
        # 4. the exchange path's rows are the one-rank shortcut's, bit for bit
        if False not in _DIGESTS:
            dev, pipe, _ = _run_rank(False)
            try:
                pipe.step()
                ok_, ov_, vb = pipe._out
                _DIGESTS[False] = (pipe.n_out, row_digest(dev, ok_, ov_, vb, pipe.n_out))
            finally:
                pipe.free()
        assert _DIGESTS[True] == _DIGESTS[False]
