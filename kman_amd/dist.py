"""Multi-GPU k-mer join: prefix-range partition + one all-to-all.

One process per GPU.  Every rank extracts the k-mers of its own FASTA shard,
then:

1. histograms the top ``hb`` key bits            (kman_prefix_hist)
2. all-reduces the histogram                      (kman_allreduce_u64, RCCL)
3. cuts the prefix space into ``world`` contiguous ranges of ~equal k-mer
   count                                          (``plan_lut``, host)
4. stably partitions its keys (+ pos) by destination rank
                                                  (kman_partition, 1 onesweep pass)
5. exchanges per-destination counts and then the keys (+ pos)
                                                  (kman_allgather_u64 + kman_alltoallv)
6. sorts what it received by prefix and finishes it in LDS with the count / uniq
   output (kman_sort_range + kman_finish).

Rank r then holds the complete count/uniq result for its prefix range; the
ranges are in rank order, so concatenating the ranks' outputs is the global
sorted output of the reference (join.py:95-130) over all shards.  uniq
payloads carry the source rank in bits 56-63 so headers resolve against the
right shard's record table.

The planning functions are pure numpy and shared with the CPU rehearsal in
tests/test_dist_cpu.py (gloo, world_size 2), which checks the partition +
exchange logic end to end without GPUs.
"""

from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_uint64, c_void_p
from typing import List, Optional, Tuple

import numpy as np

from . import _native as N
from . import engine

RANK_SHIFT = 56


def hist_bits(k: int) -> int:
    return min(14, 2 * k)


def plan_lut(global_hist: np.ndarray, world: int) -> np.ndarray:
    """Destination rank of every prefix bin: contiguous ranges, each holding
    ~total/world keys (a bin goes to the rank owning its midpoint)."""
    h = np.asarray(global_hist, dtype=np.float64)
    total = h.sum()
    if total == 0:
        return np.zeros(len(h), dtype=np.uint8)
    mid = np.cumsum(h) - h / 2
    dest = np.floor(mid * world / total).astype(np.int64)
    return np.clip(dest, 0, world - 1).astype(np.uint8)


def bucket_counts(local_hist: np.ndarray, lut: np.ndarray, world: int) -> np.ndarray:
    return np.bincount(lut.astype(np.int64), weights=np.asarray(local_hist, np.float64),
                       minlength=world).astype(np.uint64)


def recv_layout(count_matrix: np.ndarray, rank: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """(send_counts, send_offsets, recv_counts, recv_offsets) of ``rank`` from
    the world x world matrix C[src][dst] of partition sizes."""
    C = np.asarray(count_matrix, dtype=np.uint64)
    send = C[rank].copy()
    send_off = np.concatenate([[0], np.cumsum(send)[:-1]]).astype(np.uint64)
    recv = C[:, rank].copy()
    recv_off = np.concatenate([[0], np.cumsum(recv)[:-1]]).astype(np.uint64)
    return send, send_off, recv, recv_off


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(c_void_p)


class DistPipeline:
    """Resident multi-GPU pipeline for one FASTA shard per rank (bench.py).

    ``step()`` = parse -> extract -> prefix hist -> all-reduce -> partition ->
    all-to-all -> sort -> count|uniq, leaving rank-local results on device."""

    def __init__(self, dev: engine.Device, text: bytes, k: int, mode: str, world: int, rank: int,
                 uid: bytes, slack: float = 1.25):
        engine._check_k(k)
        self.dev, self.k, self.mode, self.world, self.rank = dev, k, mode, world, rank
        L = N.lib()
        idb = ctypes.create_string_buffer(bytes(uid), 128)
        N.check(dev.ctx, L.kman_comm_init(dev.ctx, idb, world, rank), "kman_comm_init")
        self.local = engine.ResidentPipeline(dev, text, k, mode=mode, rc=False, pos_bytes=8)
        self.hb = hist_bits(k)
        self.hshift = 2 * k - self.hb
        self.d_hist = dev.alloc(8 << self.hb)
        self.d_ghist = dev.alloc(8 << self.hb)
        self.d_lut = dev.alloc(1 << self.hb)
        self.d_cnt = dev.alloc(8 * world)
        self.d_cmat = dev.alloc(8 * world * world)
        cap = int(self.local.bound * slack) + (1 << 20)
        self.cap = cap
        self.recv_keys = dev.alloc(8 * cap)
        self.recv_alt = dev.alloc(8 * cap)
        want_pos = mode == "uniq"
        self.recv_pos = dev.alloc(8 * cap) if want_pos else None
        self.recv_pos_alt = dev.alloc(8 * cap) if want_pos else None
        self.out_keys = dev.alloc(8 * cap)
        self.out_vals = dev.alloc(8 * cap)
        self.n_local = 0
        self.n_recv = 0
        self.n_out = 0
        self.sorted_in_alt = False

    def step(self) -> int:
        L, ctx, dev = N.lib(), self.dev.ctx, self.dev
        lp = self.local
        n = lp.extract_only()
        self.n_local = n
        if self.mode == "uniq":  # tag payloads with the source rank
            N.check(ctx, L.kman_or_u64(ctx, c_void_p(lp.pos.ptr), n, self.rank << RANK_SHIFT), "tag")
        # 1-2. prefix histogram, all-reduced
        dev.memset(self.d_hist, 0, 8 << self.hb)
        N.check(ctx, L.kman_prefix_hist(ctx, c_void_p(lp.keys.ptr), n, self.hshift, self.hb,
                                         c_void_p(self.d_hist.ptr)), "prefix_hist")
        N.check(ctx, L.kman_memcpy_d2d(ctx, c_void_p(self.d_ghist.ptr), c_void_p(self.d_hist.ptr), 8 << self.hb),
                "d2d")
        N.check(ctx, L.kman_allreduce_u64(ctx, c_void_p(self.d_ghist.ptr), 1 << self.hb), "allreduce")
        ghist = dev.download(self.d_ghist, 1 << self.hb, np.uint64)
        lhist = dev.download(self.d_hist, 1 << self.hb, np.uint64)
        # 3. plan
        lut = plan_lut(ghist, self.world)
        dev.upload(self.d_lut, lut)
        counts = bucket_counts(lhist, lut, self.world)
        # 4. stable partition by destination
        vb = 8 if self.mode == "uniq" else 0
        N.check(ctx, L.kman_partition(ctx, c_void_p(lp.keys.ptr), c_void_p(lp.alt.ptr),
                                       c_void_p(lp.pos.ptr if vb else None), c_void_p(lp.pos_alt.ptr if vb else None),
                                       vb, n, c_void_p(self.d_lut.ptr), self.hshift, self.world, _u64p(counts)),
                "partition")
        # 5. counts exchange, then the data
        dev.upload(self.d_cnt, counts)
        N.check(ctx, L.kman_allgather_u64(ctx, c_void_p(self.d_cnt.ptr), c_void_p(self.d_cmat.ptr), self.world),
                "allgather")
        C = dev.download(self.d_cmat, self.world * self.world, np.uint64).reshape(self.world, self.world)
        send, send_off, recv, recv_off = recv_layout(C, self.rank)
        nrecv = int(recv.sum())
        if nrecv > self.cap:
            raise RuntimeError("rank %d receives %d keys > capacity %d (prefix skew)" % (self.rank, nrecv, self.cap))
        N.check(ctx, L.kman_alltoallv(ctx, c_void_p(lp.alt.ptr), _u64p(send), _u64p(send_off),
                                       c_void_p(self.recv_keys.ptr), _u64p(recv), _u64p(recv_off), 8), "alltoallv")
        if vb:
            N.check(ctx, L.kman_alltoallv(ctx, c_void_p(lp.pos_alt.ptr), _u64p(send), _u64p(send_off),
                                           c_void_p(self.recv_pos.ptr), _u64p(recv), _u64p(recv_off), 8),
                    "alltoallv")
        self.n_recv = nrecv
        # 6. local prefix sort + finish (segments sorted in LDS, count | uniq)
        res = c_int(0)
        lo = engine.split_bits(nrecv, 2 * self.k)
        rp = c_void_p(self.recv_pos.ptr if vb else None)
        rpa = c_void_p(self.recv_pos_alt.ptr if vb else None)
        N.check(ctx, L.kman_sort_range(ctx, c_void_p(self.recv_keys.ptr), c_void_p(self.recv_alt.ptr), rp, rpa, vb,
                                       nrecv, lo, 2 * self.k, None, byref(res)), "kman_sort_range")
        self.sorted_in_alt = bool(res.value)
        skeys, okeys = (self.recv_alt, self.recv_keys) if res.value else (self.recv_keys, self.recv_alt)
        spos, opos = (rpa, rp) if res.value else (rp, rpa)
        out = c_uint64(0)
        mode = N.KMAN_FINISH_COUNT if self.mode == "count" else N.KMAN_FINISH_UNIQ
        N.check(ctx, L.kman_finish(ctx, c_void_p(skeys.ptr), c_void_p(okeys.ptr), spos, opos, vb, nrecv, 2 * self.k,
                                   lo, mode, c_void_p(self.out_keys.ptr), c_void_p(self.out_vals.ptr), 8, byref(out)),
                "kman_finish")
        self.n_out = int(out.value)
        return n

    # bench.py interface (same as engine.ResidentPipeline)
    @property
    def n_kmers(self) -> int:
        return self.n_local

    @property
    def n_sorted(self) -> int:
        return self.n_recv

    pos_bytes = 8

    def timing(self, enable: bool) -> None:
        self.local.timing(enable)

    def timed(self, tag: str):
        return self.local.timed(tag)

    def results(self):
        """Rank-local (keys, counts|pos) on the host (tests)."""
        keys = self.dev.download(self.out_keys, self.n_out, np.uint64)
        vals = self.dev.download(self.out_vals, self.n_out, np.uint64)
        return keys, vals

    def free(self) -> None:
        N.lib().kman_comm_destroy(self.dev.ctx)
        self.local.free()
        for b in (self.d_hist, self.d_ghist, self.d_lut, self.d_cnt, self.d_cmat, self.recv_keys, self.recv_alt,
                  self.recv_pos, self.recv_pos_alt, self.out_keys, self.out_vals):
            if b is not None:
                b.free()


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    rc = N.lib().kman_comm_unique_id(buf)
    if rc != N.KMAN_OK:
        raise RuntimeError("kman_comm_unique_id failed (%d)" % rc)
    return buf.raw


# ------------------------------------------------------------- CPU rehearsal


def rehearse(keys: np.ndarray, vals: Optional[np.ndarray], k: int, world: int, rank: int, comm) -> Tuple:
    """The same partition/exchange on host arrays with a ``comm`` object that
    provides ``allreduce(np.ndarray)``, ``allgather(np.ndarray)`` and
    ``alltoallv(list_of_arrays) -> list_of_arrays`` (gloo in the tests).
    Returns this rank's sorted (keys, vals) after the exchange."""
    hb = hist_bits(k)
    shift = 2 * k - hb
    lhist = np.bincount((keys >> np.uint64(shift)).astype(np.int64), minlength=1 << hb).astype(np.uint64)
    ghist = comm.allreduce(lhist)
    lut = plan_lut(ghist, world)
    dest = lut[(keys >> np.uint64(shift)).astype(np.int64)]
    order = np.argsort(dest, kind="stable")  # the stable partition kman_partition performs
    counts = bucket_counts(lhist, lut, world)
    assert (np.bincount(dest, minlength=world).astype(np.uint64) == counts).all()
    C = comm.allgather(counts).reshape(world, world)
    send, send_off, recv, recv_off = recv_layout(C, rank)
    pk = keys[order]
    parts = [pk[int(o):int(o + c)] for o, c in zip(send_off, send)]
    got = comm.alltoallv(parts)
    rk = np.concatenate(got) if got else np.zeros(0, np.uint64)
    rv = None
    if vals is not None:
        pv = vals[order]
        gv = comm.alltoallv([pv[int(o):int(o + c)] for o, c in zip(send_off, send)])
        rv = np.concatenate(gv)
    o2 = np.argsort(rk, kind="stable")
    return rk[o2], (rv[o2] if rv is not None else None), lut


__all__ = ["plan_lut", "bucket_counts", "recv_layout", "DistPipeline", "unique_id", "rehearse", "List"]
