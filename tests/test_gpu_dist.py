"""GPU pieces of the multi-GPU join that a 1-GPU box can check: the prefix
histogram, the LUT-digit stable partition kernel, and the whole RCCL
pipeline at world size 1 (N>1 runs on the driver's 8-GPU node; the exchange
logic is rehearsed on CPU in tests/test_dist_cpu.py)."""

from __future__ import annotations

import ctypes
from ctypes import c_void_p

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from kman_amd import engine

    return engine.default_device()


@pytest.mark.parametrize("n", [1, 5000, 1_000_003])
@pytest.mark.parametrize("buckets", [1, 3, 8])
def test_prefix_hist_and_partition(dev, n, buckets):
    from kman_amd import _native as N
    from kman_amd.dist import plan_lut

    L = N.lib()
    rng = np.random.default_rng(n + buckets)
    keys = rng.integers(0, 1 << 42, size=n, dtype=np.uint64)
    keys[: n // 3] &= np.uint64((1 << 30) - 1)  # skew
    vals = np.arange(n, dtype=np.uint64) * np.uint64(7)
    dk, dk2, dv, dv2 = dev.alloc(8 * n), dev.alloc(8 * n), dev.alloc(8 * n), dev.alloc(8 * n)
    dh = dev.alloc(8 << 14)
    dl = dev.alloc(1 << 14)
    dev.upload(dk, keys)
    dev.upload(dv, vals)
    dev.memset(dh, 0, 8 << 14)
    N.check(dev.ctx, L.kman_prefix_hist(dev.ctx, c_void_p(dk.ptr), n, 42 - 14, 14, c_void_p(dh.ptr)), "hist")
    h = dev.download(dh, 1 << 14, np.uint64)
    want_h = np.bincount((keys >> np.uint64(28)).astype(np.int64), minlength=1 << 14)
    np.testing.assert_array_equal(h, want_h)
    lut = plan_lut(h, buckets)
    dev.upload(dl, lut.astype(np.uint8))
    counts = np.bincount(lut, weights=h.astype(np.float64), minlength=buckets).astype(np.uint64)
    N.check(dev.ctx, L.kman_partition(dev.ctx, c_void_p(dk.ptr), c_void_p(dk2.ptr), c_void_p(dv.ptr),
                                      c_void_p(dv2.ptr), 8, n, c_void_p(dl.ptr), 28, buckets,
                                      counts.ctypes.data_as(c_void_p)), "partition")
    dest = lut[(keys >> np.uint64(28)).astype(np.int64)]
    order = np.argsort(dest, kind="stable")
    np.testing.assert_array_equal(dev.download(dk2, n, np.uint64), keys[order])
    np.testing.assert_array_equal(dev.download(dv2, n, np.uint64), vals[order])
    for b in (dk, dk2, dv, dv2, dh, dl):
        b.free()


@pytest.mark.parametrize("path", ["region", "general"])
@pytest.mark.parametrize("mode", ["count", "uniq"])
def test_dist_pipeline_world1_equals_single(dev, mode, path, tmp_path, oracle_bin):
    """The RCCL pipeline at world size 1 (RCCL self-exchange): rows and the
    emitted file equal the single-GPU path / the C oracle."""
    import sys, os, subprocess

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import inputs
    import np_oracle
    from kman_amd import dist, shard

    text = inputs.messy_records(7, n_records=40, max_len=20000)
    p = dist.DistPipeline(dev, shard.BytesReader(text), 13, mode, 1, 0, dist.unique_id(), path=path,
                          max_round_items=40_000)
    try:
        for _ in range(2):
            p.step()
            assert p.path == path and p.rounds >= 2
        keys, vals = p.results()
        out = tmp_path / "o.txt"
        p.comm.run(p.emit_gen(str(out)))
    finally:
        p.free()
    recs = np_oracle.parse_fasta(text)
    kk, pp = np_oracle.stream_kmers(recs, 13)
    sk, sp = np_oracle.stable_sort(kk, pp)
    if mode == "count":
        wk, wc = np_oracle.rle_count(sk)
        np.testing.assert_array_equal(keys, wk)
        np.testing.assert_array_equal(vals, wc)
    else:
        wk, wv = np_oracle.rle_uniq(sk, sp)
        np.testing.assert_array_equal(keys, wk)
        np.testing.assert_array_equal(vals, wv)
    src = tmp_path / "in.fa"
    src.write_bytes(text)
    subprocess.run([oracle_bin, mode, str(src), str(tmp_path / "w.txt"), "13"], check=True)
    assert out.read_bytes() == (tmp_path / "w.txt").read_bytes()


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("input_", ["messy", "repeats"])
def test_dist_region_rccl_exchange_world1(dev, mode, overlap, input_):
    """The region path's data path of an N > 1 run, driven through RCCL at
    world size 1: each round's packed items leave through kman_alltoallv (RCCL
    send/recv to self, exchange=True) -- or, overlap=True, through the pieces'
    kman_alltoallv_async on the communication stream (second communicator)
    with kman_comm_wait before each piece's finish -- and the redo of
    overflowing key ranges (input "repeats") exchanges through RCCL too.
    Rows bit-exact against np_oracle."""
    import sys, os

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import inputs
    import np_oracle
    from kman_amd import dist, shard

    if input_ == "messy":
        text = inputs.messy_records(11, n_records=30, max_len=30000)
    else:  # a segment repeated far past a region's share: the partial redo
        rng = np.random.default_rng(5)
        seg = "".join(rng.choice(list("ACGT"), 300))
        body = inputs.syn_numpy(300_000, 4).split(b"\n", 1)[1].replace(b"\n", b"")
        text = b">r\n" + body + b"\n>s\n" + (seg * 3000).encode() + b"\n"
    p = dist.DistPipeline(dev, shard.BytesReader(text), 21, mode, 1, 0, dist.unique_id(), overlap=overlap,
                          exchange=True, max_round_items=30_000 if input_ == "messy" else 300_000)
    try:
        p.step()
        assert p.path == "region" and p.rounds >= 3
        if overlap:  # (every round, R >= 3: config 4's shape of plan)
            assert p.overlapped_rounds == p.rounds, "the overlapped exchange did not run in every round"
        assert p.exchanged_items == p.n_local
        if input_ == "repeats":
            assert p.partial_rounds >= 1, "no region overflowed: the RCCL redo did not run"
        keys, vals = p.results()
    finally:
        p.free()
    recs = np_oracle.parse_fasta(text)
    kk, pp = np_oracle.stream_kmers(recs, 21)
    sk, sp = np_oracle.stable_sort(kk, pp)
    if mode == "count":
        wk, wc = np_oracle.rle_count(sk)
        np.testing.assert_array_equal(keys, wk)
        np.testing.assert_array_equal(vals, wc)
    else:
        wk, wv = np_oracle.rle_uniq(sk, sp)
        np.testing.assert_array_equal(keys, wk)
        np.testing.assert_array_equal(vals, wv)


def test_dist_canonical_hist_rccl_world1(dev):
    """Config 5's data path through RCCL at world 1: canonical keys, the
    exchange forced through kman_alltoallv, rows as a multiset
    (ordered=False), the spectrum all-reduced; equal to the bincount of the
    oracle's canonical counts."""
    import sys, os

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import inputs
    import np_oracle
    from kman_amd import dist, shard

    text = inputs.messy_records(13, n_records=30, max_len=30000)
    p = dist.DistPipeline(dev, shard.BytesReader(text), 21, "count", 1, 0, dist.unique_id(), canonical=True,
                          exchange=True, ordered=False)
    try:
        p.step()
        h = p.comm.run(p.hist_gen(1000))
    finally:
        p.free()
    recs = np_oracle.parse_fasta(text)
    canon, _ = np_oracle.stream_kmers(recs, 21, canonical=True)
    _, c = np.unique(canon, return_counts=True)
    want = np.bincount(np.minimum(c, 999), minlength=1000).astype(np.uint64)
    np.testing.assert_array_equal(h, want)
