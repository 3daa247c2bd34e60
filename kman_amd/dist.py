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

The default path is the region path across ranks (``_region_step``, C ABI
kman_dgroups_*): every rank runs the extraction pass of region.hip on its
shard (items grouped by their top 8 key bits), the 256 bucket counts are
all-reduced, each rank gets a contiguous bucket range of ~1/G of the k-mers
(``plan_lut``), the packed 8-byte items move in ONE all-to-all (half the bytes
of the key + pos exchange above), and each rank finishes its buckets with the
per-bucket passes and the LDS finish.  Any region overflow (skewed input) is
agreed on collectively and the step falls back to the prefix-range path.
The step is a generator that yields its collectives, so a test can drive G
ranks in one process on one GPU (``SimGroup``) and the real run executes them
with RCCL (``RcclComm``).
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


def split_overflow(count_matrix: np.ndarray, cap: int) -> Optional[Tuple[int, int]]:
    """(rank, keys) of the first rank whose receive size exceeds cap, else
    None.  A function of the all-gathered matrix only, so every rank reaches
    the same verdict."""
    recv = np.asarray(count_matrix, dtype=np.uint64).sum(axis=0)
    bad = np.nonzero(recv > np.uint64(cap))[0]
    return (int(bad[0]), int(recv[bad[0]])) if len(bad) else None


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(c_void_p)


def nb_max(world: int) -> int:
    """Buckets one rank may own on the region path (region.hip make_dplan)."""
    per = (256 + world - 1) // world
    return min(256, per + per // 2 + 4)


def bucket_ranges(global_counts: np.ndarray, world: int) -> Tuple[np.ndarray, np.ndarray]:
    """(b_lo, nb) per rank: contiguous ranges of the 256 top-8-bit buckets with
    ~1/world of the k-mers each (plan_lut over the buckets)."""
    lut = plan_lut(np.asarray(global_counts, np.uint64), world).astype(np.int64)
    nb = np.bincount(lut, minlength=world).astype(np.int64)
    b_lo = np.concatenate([[0], np.cumsum(nb)[:-1]]).astype(np.int64)
    return b_lo, nb


class RcclComm:
    """Executes a region step's collectives with RCCL on the context's stream."""

    def __init__(self, dev: engine.Device, world: int):
        self.dev, self.world = dev, world
        self.d_vec = dev.alloc(8 * 512)
        self.d_mat = dev.alloc(8 * 256 * world)

    def allreduce(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.uint64)
        self.dev.upload(self.d_vec, x)
        N.check(self.dev.ctx, N.lib().kman_allreduce_u64(self.dev.ctx, c_void_p(self.d_vec.ptr), len(x)), "allreduce")
        return self.dev.download(self.d_vec, len(x), np.uint64)

    def allgather(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.uint64)
        self.dev.upload(self.d_vec, x)
        N.check(self.dev.ctx, N.lib().kman_allgather_u64(self.dev.ctx, c_void_p(self.d_vec.ptr),
                                                          c_void_p(self.d_mat.ptr), len(x)), "allgather")
        return self.dev.download(self.d_mat, len(x) * self.world, np.uint64).reshape(self.world, len(x))

    def alltoallv(self, send, sc, so, recv, rc, ro) -> None:
        N.check(self.dev.ctx, N.lib().kman_alltoallv(self.dev.ctx, c_void_p(send.ptr), _u64p(sc), _u64p(so),
                                                      c_void_p(recv.ptr), _u64p(rc), _u64p(ro), 8), "alltoallv")

    def run(self, gen):
        """Drive one rank's step generator to its result."""
        try:
            req = next(gen)
            while True:
                op, arg = req
                if op == "allreduce":
                    req = gen.send(self.allreduce(arg))
                elif op == "allgather":
                    req = gen.send(self.allgather(arg))
                else:
                    self.alltoallv(*arg)
                    req = gen.send(None)
        except StopIteration as e:
            return e.value

    def free(self) -> None:
        self.d_vec.free()
        self.d_mat.free()


class SimGroup:
    """G ranks of region steps in ONE process on one GPU (tests): collectives
    are computed on the host and the all-to-all is device-to-device copies."""

    def __init__(self, pipes):
        self.pipes = pipes

    def step(self):
        gens = [p._region_step() for p in self.pipes]
        reqs = [next(g) for g in gens]
        results = [None] * len(gens)
        live = list(range(len(gens)))
        while live:
            op = reqs[live[0]][0]
            assert all(reqs[i][0] == op for i in live), "ranks diverged"
            if op == "allreduce":
                tot = sum(np.asarray(reqs[i][1], np.uint64) for i in live)
                outs = [tot.copy() for _ in live]
            elif op == "allgather":
                mat = np.stack([np.asarray(reqs[i][1], np.uint64) for i in live])
                outs = [mat.copy() for _ in live]
            else:
                L = N.lib()
                for dst in live:
                    pd = self.pipes[dst]
                    _, _, _, recv, rcnt, roff = reqs[dst][1]
                    for src in live:
                        send, scnt, soff = reqs[src][1][:3]
                        c = int(scnt[dst])
                        if c:
                            N.check(pd.dev.ctx, L.kman_memcpy_d2d(pd.dev.ctx, c_void_p(recv.ptr + 8 * int(roff[src])),
                                                                   c_void_p(send.ptr + 8 * int(soff[dst])), 8 * c),
                                    "d2d")
                    pd.dev.sync()
                outs = [None for _ in live]
            nxt = []
            for i, o in zip(live, outs):
                try:
                    reqs[i] = gens[i].send(o)
                    nxt.append(i)
                except StopIteration as e:
                    results[i] = e.value
            live = nxt
        return results


class DistPipeline:
    """Resident multi-GPU pipeline for one FASTA shard per rank (bench.py).

    ``step()`` = the region path across ranks (``_region_step``), or with
    path="split" / after a collective fallback: parse -> extract -> prefix
    hist -> all-reduce -> partition -> all-to-all -> sort -> count|uniq,
    leaving rank-local results on device."""

    def __init__(self, dev: engine.Device, text: bytes, k: int, mode: str, world: int, rank: int,
                 uid: Optional[bytes], slack: float = 1.25, path: str = "region", n_bases_q: Optional[int] = None):
        engine._check_k(k)
        self.dev, self.k, self.mode, self.world, self.rank = dev, k, mode, world, rank
        L = N.lib()
        self.sim = uid is None  # SimGroup (tests): no RCCL, no split fallback
        if not self.sim:
            idb = ctypes.create_string_buffer(bytes(uid), 128)
            N.check(dev.ctx, L.kman_comm_init(dev.ctx, idb, world, rank), "kman_comm_init")
        self.comm = None if self.sim else RcclComm(dev, world)
        self.local = engine.ResidentPipeline(dev, text, k, mode=mode, rc=False, pos_bytes=8, path="split")
        self.path = path
        self.rwork = self.send = self.recv = None
        if path == "region":
            self._region_init(n_bases_q)
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

    # ------------------------------------------------------------ region path
    def _region_init(self, n_bases_q: Optional[int]) -> None:
        L, dev = N.lib(), self.dev
        lp = self.local
        lp._parse()
        self.n_bases = lp.n_bases
        if n_bases_q is None:  # every rank's n_bases, all-reduced (one-hot)
            v = np.zeros(self.world, np.uint64)
            v[self.rank] = self.n_bases
            n_bases_q = int(self.comm.allreduce(v).max())
        self.n_bases_q = n_bases_q
        self.rmode = N.KMAN_FINISH_UNIQ if self.mode == "uniq" else N.KMAN_FINISH_COUNT
        self.rflags = engine.flags_for(False, self.mode == "uniq")
        wb = c_uint64(0)
        ok = L.kman_dgroups_plan(self.n_bases, n_bases_q, self.k, self.rflags, self.rmode, self.world, byref(wb))
        if not self.sim:  # every rank must take the same path
            ok = int(self.comm.allreduce(np.array([0 if ok == N.KMAN_OK else 1], np.uint64))[0])
        if ok != N.KMAN_OK:
            self.path = "split"
            return
        self.rwork_bytes = int(wb.value)
        self.rwork = dev.alloc(self.rwork_bytes)
        self.send = dev.alloc(8 * max(self.n_bases, 1))
        self.recv_cap = int(1.3 * n_bases_q) + (1 << 20)  # ~1/G of the k-mers of G shards of <= n_bases_q
        self.recv = dev.alloc(8 * self.recv_cap)
        self.out_keys_r = dev.alloc(8 * self.recv_cap)
        self.out_vals_r = dev.alloc(8 * self.recv_cap)

    def _region_step(self):
        """One step as a generator of collectives: ("allreduce", host u64
        array) -> summed array; ("allgather", array) -> (world, len) matrix;
        ("alltoallv", args) -> None.  Returns n_kmers of the local shard, or
        None when the ranks agreed to fall back."""
        L, ctx, dev = N.lib(), self.dev.ctx, self.dev
        lp = self.local
        lp._parse()
        counts = np.zeros(256, np.uint64)
        ovf = ctypes.c_uint32(0)
        N.check(ctx, L.kman_dgroups_extract(ctx, c_void_p(lp.codes.ptr), lp.n_bases, self.n_bases_q, self.k,
                                             self.rflags, self.rmode, self.world, c_void_p(self.rwork.ptr),
                                             self.rwork_bytes, c_void_p(self.send.ptr), _u64p(counts), byref(ovf)),
                "kman_dgroups_extract")
        g = yield ("allreduce", np.concatenate([counts, [ovf.value]]).astype(np.uint64))
        if g[256]:
            return None
        b_lo, nb = bucket_ranges(g[:256], self.world)
        C = yield ("allgather", counts)  # C[src][bucket]
        # every rank checks every rank's receive size and bucket count: one decision
        per_rank = np.array([C[:, b_lo[q]:b_lo[q] + nb[q]].sum() for q in range(self.world)], np.uint64)
        if (per_rank > self.recv_cap).any() or (nb > nb_max(self.world)).any():
            return None
        sc = np.array([counts[b_lo[q]:b_lo[q] + nb[q]].sum() for q in range(self.world)], np.uint64)
        so = np.concatenate([[0], np.cumsum(sc)[:-1]]).astype(np.uint64)
        me_lo, me_nb = int(b_lo[self.rank]), int(nb[self.rank])
        mine = np.ascontiguousarray(C[:, me_lo:me_lo + me_nb], np.uint64)  # [src][j]
        rcnt = mine.sum(axis=1).astype(np.uint64)
        roff = np.concatenate([[0], np.cumsum(rcnt)[:-1]]).astype(np.uint64)
        yield ("alltoallv", (self.send, sc, so, self.recv, rcnt, roff))
        self.n_recv = int(rcnt.sum())
        out = c_uint64(0)
        r = L.kman_dgroups_finish(ctx, c_void_p(self.recv.ptr), lp.n_bases, self.n_bases_q, self.k, self.rflags,
                                  self.rmode, self.world, me_lo, me_nb, _u64p(mine.reshape(-1)),
                                  c_void_p(self.rwork.ptr), self.rwork_bytes, c_void_p(self.out_keys_r.ptr),
                                  c_void_p(self.out_vals_r.ptr), 8, byref(out))
        fb = 1 if r == N.KMAN_EFALLBACK else 0
        if not fb:
            N.check(ctx, r, "kman_dgroups_finish")
        f = yield ("allreduce", np.array([fb], np.uint64))
        if f[0]:
            return None
        self.n_out = int(out.value)
        self.n_local = int(sum(counts))
        self._out = (self.out_keys_r, self.out_vals_r)
        return self.n_local

    def step(self) -> int:
        if self.path == "region":
            n = self.comm.run(self._region_step())
            if n is not None:
                return n
            self.path = "split"  # agreed by every rank
        return self._step_split()

    def _step_split(self) -> int:
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
        # every rank holds C: all of them see the same overflow and raise
        # before the exchange (a lone raise would leave the peers hanging in it)
        over = split_overflow(C, self.cap)
        if over is not None:
            raise RuntimeError("rank %d would receive %d keys > capacity %d (prefix skew)" % (over[0], over[1], self.cap))
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
        self._out = (self.out_keys, self.out_vals)
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
        ok, ov = self._out
        keys = self.dev.download(ok, self.n_out, np.uint64)
        vals = self.dev.download(ov, self.n_out, np.uint64)
        return keys, vals

    def free(self) -> None:
        if not self.sim:
            N.lib().kman_comm_destroy(self.dev.ctx)
            self.comm.free()
        self.local.free()
        for b in (self.d_hist, self.d_ghist, self.d_lut, self.d_cnt, self.d_cmat, self.recv_keys, self.recv_alt,
                  self.recv_pos, self.recv_pos_alt, self.out_keys, self.out_vals, self.rwork, self.send, self.recv,
                  getattr(self, "out_keys_r", None), getattr(self, "out_vals_r", None)):
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


__all__ = ["plan_lut", "bucket_counts", "recv_layout", "bucket_ranges", "nb_max", "DistPipeline", "RcclComm",
           "SimGroup", "unique_id", "rehearse", "List"]
