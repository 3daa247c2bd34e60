"""Multi-GPU join logic rehearsed on CPU: 2 ranks over gloo run the same
prefix-histogram / balanced-splitter / stable-partition / all-to-all-v plan as
kman_amd.dist.DistPipeline (shared code: plan_lut, bucket_counts,
recv_layout), with numpy standing in for the per-rank device sort.  The
rank-ordered concatenation of per-rank count/uniq results must equal the
single-process result over all shards."""

from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class GlooComm:
    def __init__(self, dist, world):
        self.dist, self.world = dist, world

    def allreduce(self, a):
        import torch

        t = torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy())
        self.dist.all_reduce(t)
        return t.numpy().view(np.uint64)

    def allgather(self, a):
        import torch

        t = torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy())
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return np.concatenate([o.numpy().view(np.uint64) for o in out])

    def alltoallv(self, parts):
        import torch

        sizes = torch.tensor([len(p) for p in parts], dtype=torch.int64)
        rsizes = torch.empty_like(sizes)
        self.dist.all_to_all_single(rsizes, sizes)
        send = torch.from_numpy(np.concatenate(parts).view(np.int64).copy()) if parts else torch.empty(0, dtype=torch.int64)
        recv = torch.empty(int(rsizes.sum()), dtype=torch.int64)
        self.dist.all_to_all_single(recv, send, rsizes.tolist(), sizes.tolist())
        r = recv.numpy().view(np.uint64)
        out, at = [], 0
        for c in rsizes.tolist():
            out.append(r[at:at + c])
            at += c
        return out


def _shard_kmers(rank, k):
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import inputs
    import np_oracle

    text = inputs.messy_records(100 + rank, n_records=30, max_len=6000) if rank % 2 else inputs.syn_numpy(150_000, 7 + rank, record_len=40_000)
    keys, pos = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k)
    return keys, pos | (np.uint64(rank) << np.uint64(56))


def _worker(rank, world, port, k, q):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import np_oracle
        from kman_amd import dist as kd

        keys, pos = _shard_kmers(rank, k)
        rk, rv, lut = kd.rehearse(keys, pos, k, world, rank, GlooComm(dist, world))
        ck, cc = np_oracle.rle_count(rk)
        uk, uv = np_oracle.rle_uniq(rk, rv)
        q.put((rank, ck, cc, uk, uv, lut))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k", [5, 21])
def test_two_rank_join_equals_single_process(k):
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import np_oracle

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference over the union of shards
    allk, allp = zip(*[_shard_kmers(r, k) for r in range(world)])
    keys = np.concatenate(allk)
    vals = np.concatenate(allp)
    sk, sv = np_oracle.stable_sort(keys, vals)
    wk, wc = np_oracle.rle_count(sk)
    uk, uv = np_oracle.rle_uniq(sk, sv)
    got_k = np.concatenate([r[1] for r in res])
    got_c = np.concatenate([r[2] for r in res])
    np.testing.assert_array_equal(got_k, wk)
    np.testing.assert_array_equal(got_c, wc)
    np.testing.assert_array_equal(np.concatenate([r[3] for r in res]), uk)
    np.testing.assert_array_equal(np.concatenate([r[4] for r in res]), uv)
    # prefix ranges are contiguous and in rank order
    assert (np.diff(res[0][5].astype(np.int64)) >= 0).all()
    if len(res[0][1]) and len(res[1][1]):
        assert res[0][1].max() < res[1][1].min()


def test_plan_is_balanced():
    from kman_amd.dist import bucket_counts, plan_lut, recv_layout

    rng = np.random.default_rng(3)
    h = rng.integers(0, 1000, size=1 << 14).astype(np.uint64)
    for world in (1, 2, 4, 8):
        lut = plan_lut(h, world)
        assert (np.diff(lut.astype(np.int64)) >= 0).all()
        c = bucket_counts(h, lut, world)
        assert int(c.sum()) == int(h.sum())
        assert c.max() - c.min() <= 2 * h.max()
    C = np.array([[1, 2], [3, 4]], dtype=np.uint64)
    s, so, r, ro = recv_layout(C, 1)
    assert list(s) == [3, 4] and list(so) == [0, 3] and list(r) == [2, 4] and list(ro) == [0, 2]


def test_region_bucket_ranges():
    """bucket_ranges: contiguous ranges covering the 256 buckets, ~1/G of the
    k-mers each; within nb_max for uniform counts (skewed counts may exceed it:
    the ranks then fall back together)."""
    from kman_amd import dist

    rng = np.random.default_rng(0)
    for G in (1, 2, 3, 5, 8):
        g = rng.poisson(3_900_000, 256).astype(np.uint64)
        b_lo, nb = dist.bucket_ranges(g, G)
        assert nb.sum() == 256 and b_lo[0] == 0 and (b_lo[1:] == np.cumsum(nb)[:-1]).all()
        assert (nb <= dist.nb_max(G)).all()
        share = np.array([g[b_lo[q]:b_lo[q] + nb[q]].sum() for q in range(G)], np.float64) / g.sum()
        assert np.abs(share - 1 / G).max() < 1.5 / 256 * G / G + 1e-9
