"""Multi-GPU k-mer join over byte-range shards of ONE FASTA.

One process per GPU.  Rank q of G loads the bytes [start_q, start_{q+1}) of
the input plus a (k-1)-base halo (kman_amd/shard.py: cuts at line starts, a
window belongs to the shard holding its first base), so the union of the
shards' windows is the reference's one k-mer stream over all records
(kmermaid/batcher.py:386-392, seq.py:285-328).  Then, per step:

1. ``kman_dshard_hist``: exact item counts per (top-8-bit bucket, position
   segment) of the shard; the bucket totals are all-gathered (C[src][b]).
2. The 256 buckets are cut into G x R contiguous parts of ~equal k-mers
   (``part_cuts``): rank q owns parts q*R .. q*R+R-1 -- a contiguous key
   range -- and round r handles part q*R + r of every rank q.  R is the
   fewest rounds whose working set fits every rank's arenas (12.5 GB of FASTA
   per rank, BASELINE config 4, takes several).
3. Per round: ``kman_dshard_extract`` writes the items of the round's buckets
   straight into the send buffer, destination-major (exact offsets from the
   histogram: no gather pass); ONE all-to-all of the packed 8-byte items
   (RCCL over xGMI); ``kman_dround_finish`` runs the per-bucket passes and the
   LDS finish, appending the round's rows to the rank's output.
4. The abundance spectrum (BASELINE config 5) is the local ``kman_count_hist``
   of the rank's counts, all-reduced.

Rank q's output is the slice of the global sorted output for its key range
(join.py:95-130 over all batches); the ranks' outputs in rank order are the
global output, and ``emit`` writes each rank's text at its offset of one file.
Uniq pos carry the source rank in bits 56-63 and are rebased to global base
indices (``kman_rebase_pos``) before the headers are formatted against the
all-gathered record table.

A region overflow (a key repeated more often than a region holds) is agreed
on collectively and only that round is redone through the general path (key
ranges by ``kman_extract_range``, exchanged keys + pos, ``kman_sort_range`` +
``kman_finish``), which also serves k > 25 and uniq shards too large for the
packed items.

Every step is a generator that yields its collectives: ``RcclComm`` runs
them with RCCL for the one rank of this process, ``SimGroup`` runs G ranks in
one process on one GPU (tests: host-side reductions, device-to-device copies).
"""

from __future__ import annotations

import ctypes
import os
import time
from ctypes import byref, c_int, c_uint32, c_uint64, c_void_p
from typing import List, Optional, Tuple

import numpy as np

from . import _native as N
from . import engine
from . import shard as S

RANK_SHIFT = 56
NB = 256  # top-8-bit buckets
RS = 64   # position segments of the shard's pass 0


def plan_lut(global_hist: np.ndarray, world: int) -> np.ndarray:
    """Part of every bin: contiguous ranges, each holding ~total/world items
    (a bin goes to the part owning its midpoint)."""
    h = np.asarray(global_hist, dtype=np.float64)
    total = h.sum()
    if total == 0:
        return np.zeros(len(h), dtype=np.int64)
    mid = np.cumsum(h) - h / 2
    dest = np.floor(mid * world / total).astype(np.int64)
    return np.clip(dest, 0, world - 1)


def part_cuts(totals: np.ndarray, nparts: int) -> np.ndarray:
    """nparts + 1 bucket cuts: part p = buckets [cuts[p], cuts[p+1])."""
    lut = plan_lut(totals, nparts)
    return np.searchsorted(lut, np.arange(nparts + 1), side="left").astype(np.int64)


def part_of(cuts: np.ndarray, R: int, q: int, r: int) -> Tuple[int, int]:
    p = q * R + r
    return int(cuts[p]), int(cuts[p + 1])


def round_send(H: np.ndarray, cuts: np.ndarray, G: int, R: int, r: int):
    """Send layout of round r on a rank with (bucket, segment) counts H
    [256, 64]: region base table (u64 [256 * 64], ~0 = bucket not in this
    round), per-destination counts and offsets."""
    H = np.asarray(H, dtype=np.uint64).reshape(NB, RS)
    rtab = np.full(NB * RS, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    sc = np.zeros(G, dtype=np.uint64)
    off = 0
    for q in range(G):
        lo, hi = part_of(cuts, R, q, r)
        blk = H[lo:hi].reshape(-1)
        if len(blk):
            ex = np.concatenate([[0], np.cumsum(blk)[:-1]]).astype(np.uint64)
            rtab[lo * RS:hi * RS] = ex + np.uint64(off)
            sc[q] = int(blk.sum())
            off += int(sc[q])
    so = np.concatenate([[0], np.cumsum(sc)[:-1]]).astype(np.uint64)
    return rtab, sc, so


def round_recv(C: np.ndarray, cuts: np.ndarray, R: int, rank: int, r: int):
    """(b_lo, nb, counts [G, nb], recv counts, recv offsets) of round r on
    `rank` from the all-gathered bucket totals C [G, 256]."""
    lo, hi = part_of(cuts, R, rank, r)
    counts = np.ascontiguousarray(np.asarray(C, dtype=np.uint64)[:, lo:hi])
    rc = counts.sum(axis=1).astype(np.uint64)
    ro = np.concatenate([[0], np.cumsum(rc)[:-1]]).astype(np.uint64)
    return lo, hi - lo, counts, rc, ro


def round_pieces(C: np.ndarray, cuts: np.ndarray, G: int, R: int, r: int, S: int) -> List[List[int]]:
    """Each destination's part of round r cut into S pieces of about equal
    k-mers (every rank derives the same cuts from the all-gathered bucket
    totals C [G, 256]): bounds[q] = S + 1 bucket indices."""
    tot = np.asarray(C, dtype=np.uint64).reshape(G, NB).sum(axis=0).astype(np.float64)
    out = []
    for q in range(G):
        lo, hi = part_of(cuts, R, q, r)
        b = [lo]
        if hi > lo:
            cum = np.cumsum(tot[lo:hi])
            for s_ in range(1, S):
                j = lo + int(np.searchsorted(cum, cum[-1] * s_ / S, side="left")) + 1
                b.append(min(max(j, b[-1]), hi))
        else:
            b += [lo] * (S - 1)
        b.append(hi)
        out.append(b)
    return out


def round_sizes(C: np.ndarray, cuts: np.ndarray, G: int, R: int):
    """send[q, r] / recv[q, r] items of every rank and round."""
    C = np.asarray(C, dtype=np.uint64)
    send = np.zeros((G, R), dtype=np.uint64)
    recv = np.zeros((G, R), dtype=np.uint64)
    for r in range(R):
        for q in range(G):
            lo, hi = part_of(cuts, R, q, r)
            recv[q, r] = C[:, lo:hi].sum()
            send[:, r] += C[:, lo:hi].sum(axis=1)
    return send, recv


def gather_ranges(cnt: np.ndarray, allr: np.ndarray, G: int) -> List[np.ndarray]:
    """Each destination's left-out [lo, hi] key ranges from the all-gathered
    range counts (cnt[q]) and zero-padded range arrays (allr[q])."""
    cnt = np.asarray(cnt, np.uint64).reshape(G)
    allr = np.asarray(allr, np.uint64).reshape(G, -1)
    return [allr[q, :2 * int(cnt[q])].reshape(-1, 2) for q in range(G)]


def redo_map(ranges: List[np.ndarray], key_bits: int, max_bits: int = 24) -> Tuple[int, np.ndarray]:
    """(pbits, map): map[p] = q + 1 when the keys with top pbits bits p lie in
    one of destination q's left-out ranges (0 elsewhere); pbits is the
    coarsest prefix length at which every range is whole.  Vectorised: a
    skewed genome leaves out thousands of ranges per round."""
    K = key_bits
    lo = np.concatenate([np.asarray(r, np.uint64).reshape(-1, 2)[:, 0] for r in ranges] + [np.zeros(0, np.uint64)])
    hi = np.concatenate([np.asarray(r, np.uint64).reshape(-1, 2)[:, 1] for r in ranges] + [np.zeros(0, np.uint64)])
    dst = np.concatenate([np.full(len(np.asarray(r).reshape(-1, 2)), q + 1, np.int64) for q, r in enumerate(ranges)]
                         + [np.zeros(0, np.int64)])
    pbits = 1
    if len(lo):
        def tz(x, full):
            # trailing zero bits (full when x == 0): exact via the lowest set bit's power of two
            low = x & (~x + np.uint64(1))
            t = np.zeros(len(x), np.int64)
            nz = low != 0
            t[nz] = np.round(np.log2(low[nz].astype(np.float64))).astype(np.int64)
            t[~nz] = full
            return t

        top = np.uint64((1 << K) - 1) if K < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
        end = hi + np.uint64(1)  # (wraps to 0 for the last key: a whole-space end)
        a = tz(lo, K)
        b = np.where(hi >= top, K, tz(end, K))
        pbits = max(1, int((K - np.minimum(a, b)).max()))
    if pbits > max_bits:
        raise NotImplementedError("left-out key ranges finer than %d key bits" % max_bits)
    sh = np.uint64(K - pbits)
    marks = np.zeros((1 << pbits) + 1, np.int64)
    if len(lo):
        np.add.at(marks, (lo >> sh).astype(np.int64), dst)
        np.add.at(marks, (hi >> sh).astype(np.int64) + 1, -dst)
    pmap = np.cumsum(marks[:-1]).astype(np.uint8)  # (the ranges are disjoint)
    return pbits, pmap


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(c_void_p)


class RoundPlanner:
    """The rounds of one step, identical on every rank (a function of C, the
    common budget and the common flags only)."""

    def __init__(self, k: int, flags: int, mode: int, world: int, n_bases_q: int):
        self.k, self.flags, self.mode, self.G, self.nbq = k, flags, mode, world, n_bases_q

    def arenas(self, C, cuts, R, q: int, r: int) -> Optional[Tuple[int, int]]:
        """(a, b) bytes of round r on rank q, or None when the region finish
        cannot take it (then the round runs the general path)."""
        lo, nb, counts, rc, _ = round_recv(C, cuts, R, q, r)
        a, b = c_uint64(0), c_uint64(0)
        ret = N.lib().kman_dround_plan(self.k, self.flags, self.mode, self.G, self.nbq, nb,
                                       _u64p(np.ascontiguousarray(counts.reshape(-1))), byref(a), byref(b))
        if ret != N.KMAN_OK:
            return None
        return int(a.value), max(int(b.value), 8 * int(rc.sum()))

    def roomy(self, C, cuts, R: int, budget: int, a: int, b: int) -> Tuple[bool, int, int]:
        """(True, a, b) when the same rounds fit `budget` with KMAN_ROOMY
        (pass-1 sub-regions at twice their expected fill: a genome's repeat
        families fit them, so a left-out region is redone from pass 1's
        output), else (False, a, b) unchanged.  The caller then passes
        self.flags | KMAN_ROOMY to every kman_dround_* call of the step."""
        if os.environ.get("KMAN_ROOMY", "1") == "0":
            return False, a, b
        base, self.flags = self.flags, self.flags | N.KMAN_ROOMY
        try:
            a2 = b2 = 0
            for q in range(self.G):
                for r in range(R):
                    ab = self.arenas(C, cuts, R, q, r)
                    if ab is None:
                        return False, a, b
                    a2, b2 = max(a2, ab[0]), max(b2, ab[1])
            send, _ = round_sizes(C, cuts, self.G, R)
            a2 = max(a2, 8 * int(send.max()))
            if a2 + b2 > budget:
                return False, a, b
            return True, a2, b2
        finally:
            self.flags = base

    def plan(self, C, budget: int, max_round_items: Optional[int] = None, max_rounds: int = 64):
        """(R, cuts, a_bytes, b_bytes): the fewest rounds whose largest arenas
        (over ranks and rounds) fit `budget` bytes (and whose rounds receive
        at most max_round_items on any rank)."""
        G = self.G
        tot = np.asarray(C, dtype=np.uint64).sum(axis=0)
        for R in range(1, max_rounds + 1):
            if G * R > NB and R > 1:
                break
            cuts = part_cuts(tot, G * R)
            send, recv = round_sizes(C, cuts, G, R)
            if max_round_items is not None and int(recv.max()) > max_round_items and R < max_rounds:
                continue
            a = b = 0
            ok = True
            for q in range(G):
                for r in range(R):
                    ab = self.arenas(C, cuts, R, q, r)
                    if ab is None:
                        ok = False
                        continue
                    a, b = max(a, ab[0]), max(b, ab[1])
            a = max(a, 8 * int(send.max()))
            if a + b <= budget or R == max_rounds or not ok:
                return R, cuts, a, b
        cuts = part_cuts(tot, G * R)
        send, recv = round_sizes(C, cuts, G, R)
        return R, cuts, 8 * int(send.max()), 8 * int(recv.max())


# ------------------------------------------------------------------ comms


class RcclComm:
    """Executes one rank's collectives with RCCL on the context's stream."""

    def __init__(self, dev: engine.Device, world: int, rank: int, uid: bytes):
        self.dev, self.world, self.rank = dev, world, rank
        idb = ctypes.create_string_buffer(bytes(uid), 128)
        N.check(dev.ctx, N.lib().kman_comm_init(dev.ctx, idb, world, rank), "kman_comm_init")
        self.cap = 0
        self.d_vec = self.d_mat = None

    def _bufs(self, n: int) -> None:
        if n > self.cap:
            for b in (self.d_vec, self.d_mat):
                if b is not None:
                    b.free()
            self.cap = max(n, 1024)
            self.d_vec = self.dev.alloc(8 * self.cap)
            self.d_mat = self.dev.alloc(8 * self.cap * self.world)

    def count(self) -> Tuple[int, int]:
        """(ranks, this rank) as the RCCL communicator counts them."""
        n, r = ctypes.c_int(0), ctypes.c_int(0)
        N.check(self.dev.ctx, N.lib().kman_comm_count(self.dev.ctx, ctypes.byref(n), ctypes.byref(r)),
                "kman_comm_count")
        return int(n.value), int(r.value)

    def allreduce(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.uint64)
        self._bufs(len(x))
        self.dev.upload(self.d_vec, x)
        N.check(self.dev.ctx, N.lib().kman_allreduce_u64(self.dev.ctx, c_void_p(self.d_vec.ptr), len(x)), "allreduce")
        return self.dev.download(self.d_vec, len(x), np.uint64)

    def allgather(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.uint64)
        self._bufs(len(x))
        self.dev.upload(self.d_vec, x)
        N.check(self.dev.ctx, N.lib().kman_allgather_u64(self.dev.ctx, c_void_p(self.d_vec.ptr),
                                                          c_void_p(self.d_mat.ptr), len(x)), "allgather")
        return self.dev.download(self.d_mat, len(x) * self.world, np.uint64).reshape(self.world, len(x))

    def alltoallv(self, send, sc, so, recv, rc, ro, eb=8) -> None:
        N.check(self.dev.ctx, N.lib().kman_alltoallv(self.dev.ctx, c_void_p(send), _u64p(sc), _u64p(so),
                                                      c_void_p(recv), _u64p(rc), _u64p(ro), eb), "alltoallv")

    def alltoallv_async(self, send, sc, so, recv, rc, ro, eb, slot) -> None:
        sc, so, rc, ro = (np.ascontiguousarray(x, np.uint64) for x in (sc, so, rc, ro))
        N.check(self.dev.ctx, N.lib().kman_alltoallv_async(self.dev.ctx, c_void_p(send), _u64p(sc), _u64p(so),
                                                            c_void_p(recv), _u64p(rc), _u64p(ro), eb, slot),
                "alltoallv_async")

    def run(self, gen):
        """Drive this rank's generator to its result."""
        try:
            req = next(gen)
            while True:
                op, arg = req
                if op == "allreduce":
                    req = gen.send(self.allreduce(arg))
                elif op == "allgather":
                    req = gen.send(self.allgather(arg))
                elif op == "alltoallv_async":
                    self.alltoallv_async(*arg)
                    req = gen.send(None)
                elif op == "comm_wait":
                    N.check(self.dev.ctx, N.lib().kman_comm_wait(self.dev.ctx, int(arg)), "kman_comm_wait")
                    req = gen.send(None)
                else:
                    self.alltoallv(*arg)
                    req = gen.send(None)
        except StopIteration as e:
            return e.value

    def free(self) -> None:
        N.lib().kman_comm_destroy(self.dev.ctx)
        for b in (self.d_vec, self.d_mat):
            if b is not None:
                b.free()


class LocalComm:
    """One rank on its own (no RCCL): the collectives of a step generator are
    identities and a general round's exchange is a device copy.  Serves the
    single-GPU inputs outside kman_groups (local_groups)."""

    def __init__(self, dev: engine.Device):
        self.dev = dev

    def count(self) -> Tuple[int, int]:
        return 1, 0

    def run(self, gen):
        try:
            req = next(gen)
            while True:
                op, arg = req
                if op == "allreduce":
                    req = gen.send(np.asarray(arg, np.uint64).copy())
                elif op == "allgather":
                    req = gen.send(np.asarray(arg, np.uint64).reshape(1, -1).copy())
                elif op == "comm_wait":
                    req = gen.send(None)
                else:  # alltoallv (async: the same copy, in stream order)
                    send, sc, so, recv, rc, ro, eb = arg[:7]
                    if int(sc[0]):
                        N.check(self.dev.ctx, N.lib().kman_memcpy_d2d(self.dev.ctx, c_void_p(recv), c_void_p(send),
                                                                       eb * int(sc[0])), "d2d")
                    req = gen.send(None)
        except StopIteration as e:
            return e.value

    def free(self) -> None:
        pass


class SimGroup:
    """G ranks in ONE process on one GPU (tests): collectives computed on the
    host, the all-to-all as device-to-device copies."""

    def __init__(self, pipes):
        self.pipes = pipes

    def run(self, make_gen):
        gens = [make_gen(p) for p in self.pipes]
        results = [None] * len(gens)
        reqs = [None] * len(gens)
        live = []
        for i, g in enumerate(gens):
            try:
                reqs[i] = next(g)
                live.append(i)
            except StopIteration as e:
                results[i] = e.value
        while live:
            op = reqs[live[0]][0]
            assert all(reqs[i][0] == op for i in live), "ranks diverged"
            assert len(live) == len(gens), "a rank finished early"
            if op == "allreduce":
                tot = sum(np.asarray(reqs[i][1], np.uint64) for i in live)
                outs = [tot.copy() for _ in live]
            elif op == "allgather":
                mat = np.stack([np.asarray(reqs[i][1], np.uint64) for i in live])
                outs = [mat.copy() for _ in live]
            elif op == "comm_wait":
                outs = [None for _ in live]
            else:  # alltoallv (async: done right away, which any later wait allows)
                L = N.lib()
                for src in live:  # (every send buffer complete on its own rank's stream)
                    self.pipes[src].dev.sync()
                for dst in live:
                    pd = self.pipes[dst]
                    _, _, _, recv, rcnt, roff, eb = reqs[dst][1][:7]
                    for src in live:
                        send, scnt, soff = reqs[src][1][:3]
                        c = int(scnt[dst])
                        if c:
                            N.check(pd.dev.ctx, L.kman_memcpy_d2d(pd.dev.ctx, c_void_p(recv + eb * int(roff[src])),
                                                                   c_void_p(send + eb * int(soff[dst])), eb * c), "d2d")
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

    def step(self):
        return self.run(lambda p: p.step_gen())


# --------------------------------------------------------------- pipeline


class _Grow:
    """A device buffer that grows (never shrinks) to the largest request."""

    def __init__(self, dev: engine.Device):
        self.dev, self.buf = dev, None

    def get(self, nbytes: int) -> engine.DeviceBuffer:
        if self.buf is None or self.buf.nbytes < nbytes:
            if self.buf is not None:
                self.buf.free()
                self.buf = None
            self.buf = self.dev.alloc(max(nbytes, 64))
        return self.buf

    def free(self) -> None:
        if self.buf is not None:
            self.buf.free()
            self.buf = None


class _View:
    """A window [ptr, ptr + nbytes) of a buffer owned elsewhere."""

    def __init__(self, ptr: int, nbytes: int):
        self.ptr, self.nbytes = ptr, nbytes


class DistPipeline:
    """One rank of the multi-GPU join (bench.py, CLI, tests).

    reader: the whole FASTA (shard.BytesReader / PinnedReader / SynthReader);
    every rank cuts the same shards and loads its own.  uid: the RCCL id
    (None: the caller drives the generators, SimGroup).  canonical: keys
    min(fwd, rc) (config 5).  path: "region" (default; per-round fallback to
    the general path) or "general".  max_round_items: force more rounds
    (tests).  reload: re-upload + re-parse the shard in every step (the
    pinned-host benchmark line); reparse: keep the shard's text in HBM and
    parse it in every step (a shard of one chunk: the benchmark's step then
    covers parse + histogram + rounds, as the single-GPU step covers parse +
    join).  ordered=False: the rows are wanted only as a multiset (the
    abundance spectrum, config 5), so a partial redo appends the redone key
    ranges' rows after the region rows instead of merging them into key
    order (no copy, no merge pass)."""

    def __init__(self, dev: engine.Device, reader, k: int, mode: str, world: int, rank: int,
                 uid: Optional[bytes] = None, canonical: bool = False, rc: bool = False, path: str = "region",
                 max_round_items: Optional[int] = None, chunk_bytes: int = 256 << 20, reload: bool = False,
                 mem_frac: float = 0.85, shard: Optional[S.ShardCodes] = None, local: bool = False,
                 reparse: bool = False, overlap: Optional[bool] = None, ordered: bool = True,
                 exchange: bool = False):
        engine._check_k(k)
        if mode not in ("count", "uniq"):
            raise ValueError(mode)
        if canonical and mode != "count":
            raise ValueError("canonical k-mers are counted (config 5), not uniq'd")
        self.dev, self.k, self.mode, self.world, self.rank = dev, k, mode, world, rank
        self.canonical, self.rc = canonical, rc and not canonical
        self.path, self.max_round_items, self.reload, self.mem_frac = path, max_round_items, reload, mem_frac
        self.reparse, self.ordered = reparse, ordered
        # overlapped rounds (round_pieces): opt-in (overlap=True or
        # KMAN_DIST_OVERLAP=1) until a run on two or more GPUs has passed the
        # dist region tests with it; their all-to-alls run on a second
        # communicator (comm.hip), so the two streams never share one
        env = os.environ.get("KMAN_DIST_OVERLAP")
        self.overlap = (env == "1") if env is not None else bool(overlap)
        # exchange: run the round's all-to-all even on one rank (RCCL's
        # send/recv to self), so the 8-GPU data path runs at world 1 (tests:
        # exchange=True or KMAN_DIST_EXCHANGE=1); off, one rank extracts
        # straight into its receive buffer
        envx = os.environ.get("KMAN_DIST_EXCHANGE")
        self.exchange = world > 1 or (envx == "1" if envx is not None else bool(exchange))
        self.pieces = 4
        self.overlapped_rounds = 0
        self.fmode = N.KMAN_FINISH_UNIQ if mode == "uniq" else N.KMAN_FINISH_COUNT
        # rows wanted as a multiset only (the spectrum): canonical keys are
        # mixed (KMAN_MIXED) so the key rounds see uniform buckets
        self.mixed = canonical and not ordered
        self.flags = engine.flags_for(self.rc, mode == "uniq", canonical, self.mixed)
        self.reader = reader
        if shard is None:
            self.spec = S.shard_specs(reader, world, k)[rank]
            self.loader = S.ShardLoader(dev, reader, self.spec, k, chunk_bytes, resident=reparse)
            self.shard = self.loader.load()
        else:  # an input already on the device (one rank: local_groups)
            self.spec, self.loader, self.shard = shard.spec, None, shard
        if uid is not None:
            self.comm = RcclComm(dev, world, rank, uid)
        else:
            self.comm = LocalComm(dev) if local else None
        self.d_hist = dev.alloc(4 * NB * RS)
        self.d_rtab = dev.alloc(8 * NB * RS)
        self.d_small = dev.alloc(8 * 16384)  # prefix / abundance histograms
        self.arena_a, self.arena_b = _Grow(dev), _Grow(dev)
        self.out_keys, self.out_vals = _Grow(dev), _Grow(dev)
        self.gen_bufs = [_Grow(dev) for _ in range(6)]  # general path: send/recv keys, pos, alt keys, alt pos
        self.part_bufs = [_Grow(dev), _Grow(dev), _Grow(dev)]  # the redone key ranges' rows (keys, values), map
        self.n_local = self.n_out = self.n_recv = 0
        self.rounds = 0
        self.fallback_rounds = 0
        self.partial_rounds = 0
        self.redone_kmers = 0
        self.exchanged_items = self.max_message = 0
        self.phase_ms = {}
        self.ready = False
        if self.comm is not None:
            self.comm.run(self.setup_gen())

    def take_result(self):
        """The output rows as an engine CountResult / UniqResult (uniq pos are
        u64, source rank 0 on one rank); the buffers pass to the caller."""
        ok_, ov_, vb = self._out
        if self.mode == "uniq":
            r = engine.UniqResult(ok_, ov_, 8, self.n_out, self.k)
        else:
            r = engine.CountResult(ok_, ov_, vb, self.n_out, self.k)
        self.out_keys.buf = self.out_vals.buf = None
        return r

    # ---------------------------------------------------------------- setup
    def setup_gen(self):
        """Collectives of the first step: global record table, common pos
        bound, path agreement, common memory budget."""
        sh, G = self.shard, self.world
        R = len(sh.names)
        nlen = sum(len(x) for x in sh.names)
        ok = 1 if self.path == "region" else 0
        M = yield ("allgather", np.array([sh.n_own, sh.n_eff, R, nlen], np.uint64))
        self.n_own_all = M[:, 0].astype(np.int64)
        self.n_bases_q = max(1, int(M[:, 1].max()))
        self.base_off = np.concatenate([[0], np.cumsum(self.n_own_all)[:-1]]).astype(np.uint64)
        if ok and N.lib().kman_dshard_plan(sh.n_eff, self.n_bases_q, self.k, self.flags, self.fmode) != N.KMAN_OK:
            ok = 0
        # record table: every rank's record first bases and names
        rmax, lmax = int(M[:, 2].max()), int(M[:, 3].max())
        seqs = np.zeros(rmax + 1, np.uint64)
        seqs[:R] = sh.rec_seq
        seqs_all = yield ("allgather", seqs)
        lens = np.zeros(rmax + 1, np.uint64)
        lens[:R] = [len(x) for x in sh.names]
        lens_all = yield ("allgather", lens)
        blob = np.zeros((lmax + 7) // 8 + 1, np.uint64)
        bb = b"".join(sh.names)
        blob.view(np.uint8)[:len(bb)] = np.frombuffer(bb, np.uint8)
        blobs = yield ("allgather", blob)
        names, rec_seq = [], []
        for q in range(G):
            raw = blobs[q].view(np.uint8).tobytes()
            at = 0
            for j in range(int(M[q, 2])):
                ln = int(lens_all[q, j])
                names.append(raw[at:at + ln])
                at += ln
                rec_seq.append(int(seqs_all[q, j]) + int(self.base_off[q]))
        self.names, self.g_rec_seq = names, np.asarray(rec_seq, dtype=np.uint64)
        self.n_bases_total = int(self.n_own_all.sum())
        # empty record names with a k-mer raise before any output (seq.py:106-127)
        flag = np.array([0 if ok else 1, self._empty_name_kmer()], np.uint64)
        f = yield ("allreduce", flag)
        if int(f[1]):
            raise AssertionError("incompatible string: a record with an empty name yields k-mers")
        self.path = "region" if int(f[0]) == 0 else "general"
        free, _ = engine.mem_info(self.dev)
        bud = yield ("allgather", np.array([int(free * self.mem_frac)], np.uint64))
        self.budget = int(bud.min())
        self.ready = True

    def _empty_name_kmer(self) -> int:
        """1 when a record that starts in this shard has an empty name and
        yields a window (checked on this shard's own codes; a record that
        continues past the shard is checked on its first shard's part)."""
        sh = self.shard
        for j, nm in enumerate(sh.names):
            if nm:
                continue
            b = int(sh.rec_seq[j])
            e = int(sh.rec_seq[j + 1]) if j + 1 < len(sh.names) else sh.n_eff
            if e - b >= self.k:
                codes = self.dev.download(sh.codes, e - b, np.uint8, offset=b)
                if engine.first_window(codes, self.k) >= 0:
                    return 1
        return 0

    # ----------------------------------------------------------------- step
    def step(self) -> int:
        if self.comm is None:
            raise RuntimeError("a simulated rank is stepped by SimGroup")
        return self.comm.run(self.step_gen())

    def step_gen(self):
        if not self.ready:
            yield from self.setup_gen()
        L, ctx, dev, sh = N.lib(), self.dev.ctx, self.dev, self.shard
        if (self.reload or self.reparse) and self.loader is not None:
            self.shard = sh = self.loader.load()
        G, me = self.world, self.rank
        self.phase_ms = {}
        tick = [time.perf_counter()]

        def lap(tag):  # host-side phase times (KMAN_DIST_TIMES=1 synchronises after each phase)
            if os.environ.get("KMAN_DIST_TIMES"):
                dev.sync()
            t = time.perf_counter()
            self.phase_ms[tag] = self.phase_ms.get(tag, 0.0) + (t - tick[0]) * 1e3
            tick[0] = t

        # once: no exchange (one rank), so the shard is extracted ONCE for all
        # key rounds, round-major into the output-key buffer, instead of
        # re-rolled every round (KMAN_ONCE: the same tiles for the histogram)
        xch = self.exchange and not isinstance(self.comm, LocalComm)
        once = self.path == "region" and not xch and not self.overlap and os.environ.get("KMAN_DIST_ONCE", "1") != "0"
        fl = self.flags | (N.KMAN_ONCE if once else 0)
        # 1. (bucket, segment) counts of the shard, bucket totals all-gathered
        H = np.zeros(NB * RS, np.uint32)
        if self.path == "region":
            N.check(ctx, L.kman_dshard_hist(ctx, c_void_p(sh.codes.ptr), sh.n_eff, self.n_bases_q, self.k, fl,
                                            self.fmode, c_void_p(self.d_hist.ptr), H.ctypes.data_as(c_void_p)),
                    "kman_dshard_hist")
            c_local = H.reshape(NB, RS).sum(axis=1).astype(np.uint64)
        else:
            c_local = self._prefix_hist()
        lap("hist")
        C = yield ("allgather", c_local)
        self.n_local = int(c_local.sum())
        # 2. rounds
        pl = RoundPlanner(self.k, self.flags, self.fmode, G, self.n_bases_q)
        tot = int(np.asarray(C, np.uint64).sum())
        out_bytes = (8 + self._vb(C)) * (tot if G == 1 else int(tot * 1.1 / G) + (1 << 20))
        S_ = self.pieces
        # overlapped rounds hold a piece's two scratch arenas beside A and B
        # (about 2 / S of them): their plan leaves room for those
        # (a piece holds about 1 / S of a round's items: its two scratch
        # arenas about (a + b) / S, planned here with a margin; each round
        # checks the pieces' real plans against the budget before it runs
        # overlapped, _overlapped_round)
        ov_scale = 1.0 + 1.25 / S_ if (self.overlap and self.path == "region") else 1.0
        room = max(1, int((self.budget - out_bytes) / ov_scale))
        R, cuts, a_need, b_need = pl.plan(C, room, self.max_round_items)
        roomy = False
        if self.path == "region":
            roomy, a_need, b_need = pl.roomy(C, cuts, R, room, a_need, b_need)
        # the flags of this step's kman_dround_* calls
        self.rflags = self.flags | (N.KMAN_ROOMY if roomy else 0)
        self.rounds = R
        self.plan_info = {"budget_gb": self.budget / 1e9, "out_gb": out_bytes / 1e9, "arena_a_gb": a_need / 1e9,
                          "arena_b_gb": b_need / 1e9, "rounds": R, "roomy": roomy}
        _, recv = round_sizes(C, cuts, G, R)
        cap = int(recv[me].sum())
        vb = self._vb(C)
        ok_, ov_ = self.out_keys.get(8 * max(cap, 1)), self.out_vals.get(vb * max(cap, 1))
        n_out = 0
        lap("plan+alloc")
        self.fallback_rounds = 0
        self.partial_rounds = 0
        self.redone_kmers = 0
        self.overlapped_rounds = 0
        self.heavy_keys = 0  # keys its rounds' pass 1 counted apart (kman_dround_heavy, summed over rounds)
        self.local_redo_kmers = 0  # of redone_kmers, gathered from the finish's pass-1 output (kman_dround_left)
        self.exchanged_items = 0  # items this rank sent through kman_alltoallv (its rounds)
        self.max_message = 0  # bytes of its largest message to one peer
        # overlapped rounds (every round of the step, R >= 1): exchange piece
        # s + 1 crosses xGMI while piece s is sorted; they need two more
        # scratch arenas (a piece's a and b), which the plan above left room for
        use_ov = (self.path == "region" and self.overlap
                  and (a_need + b_need) * ov_scale + out_bytes <= self.budget * 1.0001)
        # once (R > 1): every round's items extracted by one pass into the
        # output-key buffer, round r's regions (b, s) at x_off[r] + their
        # round_send offsets.  Round r's rows are written from n_out on, and
        # n_out + rows <= x_off[r + 1] (a row is a distinct key of the round's
        # items), so they only ever overwrite rounds already consumed
        x_off = None
        if once and R > 1:
            rtab_all = np.full(NB * RS, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
            x_off, off = [], 0
            for r in range(R):
                rtab, sc, _ = round_send(H, cuts, G, R, r)
                m = rtab != np.uint64(0xFFFFFFFFFFFFFFFF)
                rtab_all[m] = rtab[m] + np.uint64(off)
                x_off.append(off)
                off += int(sc.sum())
            x_off.append(off)
            if 8 * off > ok_.nbytes:
                raise RuntimeError("rank %d: %d items exceed the output-key buffer" % (me, off))
            dev.upload(self.d_rtab, rtab_all)
            N.check(ctx, L.kman_dshard_extract(ctx, c_void_p(sh.codes.ptr), sh.n_eff, self.n_bases_q, self.k, fl,
                                               self.fmode, c_void_p(self.d_hist.ptr), c_void_p(self.d_rtab.ptr),
                                               c_void_p(ok_.ptr)), "kman_dshard_extract")
            lap("extract")
        for r in range(R):
            if use_ov:
                got_ = yield from self._overlapped_round(C, cuts, R, r, H, c_local, a_need, b_need, ok_, ov_, n_out, vb)
                if got_ is not None:
                    n_out = got_
                    lap("round")
                    continue
            if self.path == "region":
                A, B = self.arena_a.get(a_need), self.arena_b.get(b_need)
                if x_off is None:
                    rtab, sc, so = round_send(H, cuts, G, R, r)
                    dev.upload(self.d_rtab, rtab)
                    # the send buffer is arena A; one rank extracts straight
                    # into its receive buffer B (no exchange at all)
                    N.check(ctx, L.kman_dshard_extract(ctx, c_void_p(sh.codes.ptr), sh.n_eff, self.n_bases_q, self.k,
                                                       fl, self.fmode, c_void_p(self.d_hist.ptr),
                                                       c_void_p(self.d_rtab.ptr), c_void_p((A if xch else B).ptr)),
                            "kman_dshard_extract")
                    rin = B.ptr
                else:
                    rin = ok_.ptr + 8 * x_off[r]  # (extracted above, with every round)
                lo, nb, counts, rcnt, roff = round_recv(C, cuts, R, me, r)
                lap("extract")
                if xch:
                    yield ("alltoallv", (A.ptr, sc, so, B.ptr, rcnt, roff, 8))
                    self.exchanged_items += int(np.asarray(sc, np.uint64).sum())
                    self.max_message = max(self.max_message, 8 * int(np.asarray(sc, np.uint64).max()))
                    lap("exchange")
                got = c_uint64(0)
                ret = L.kman_dround_finish(ctx, c_void_p(rin), self.k, self.rflags, self.fmode, G, self.n_bases_q,
                                           lo, nb, _u64p(np.ascontiguousarray(counts.reshape(-1))),
                                           c_void_p(A.ptr), A.nbytes, c_void_p(B.ptr), B.nbytes,
                                           c_void_p(ok_.ptr + 8 * n_out), c_void_p(ov_.ptr + vb * n_out), vb,
                                           byref(got))
                fb = 1 if ret == N.KMAN_EFALLBACK else 0
                part = 1 if ret == N.KMAN_EPARTIAL else 0
                self._note_heavy()
                if not fb and not part:
                    N.check(ctx, ret, "kman_dround_finish")
                lap("finish")
                f = yield ("allreduce", np.array([fb, part], np.uint64))
                if int(f[0]) == 0 and int(f[1]) == 0:
                    n_out += int(got.value)
                    self._check_once_bound(x_off, r, n_out)
                    continue
                if int(f[0]) == 0:
                    # regions overflowed (a repeat far beyond its region's
                    # share): the other rows are in place, only the left-out
                    # key ranges go through the general path, merged in
                    self.partial_rounds += 1
                    mine = self._failed_ranges() if part else np.zeros((0, 2), np.uint64)
                    n_out += yield from self._redo_ranges(mine, int(got.value), A, B, ok_, ov_, n_out, vb)
                    self._check_once_bound(x_off, r, n_out)
                    lap("partial_redo")
                    continue
                self.fallback_rounds += 1
            # the general path for this round (every rank together)
            n_out += yield from self._general_round(C, cuts, R, r, ok_, ov_, n_out, vb)
            self._check_once_bound(x_off, r, n_out)
            lap("general_round")
        self.n_out = n_out
        self.n_recv = cap
        self._out = (ok_, ov_, vb)
        return self.n_local

    def _check_once_bound(self, x_off, r: int, n_out: int) -> None:
        """Extract-once rounds (x_off): round r's rows must end before the
        items of round r + 1 (a row is a distinct key of round r's items), or
        they have overwritten input of a later round -- fail loudly."""
        if x_off is not None and r + 1 < len(x_off) and n_out > x_off[r + 1]:
            raise RuntimeError("rank %d round %d: %d rows overran the next round's items at %d"
                               % (self.rank, r, n_out, x_off[r + 1]))

    def _overlapped_round(self, C, cuts, R, r, H, c_local, a_need, b_need, ok_, ov_, n_out, vb):
        """Round r with its exchange overlapped: one extraction (destination-
        major, as round_send lays it out), then each destination's part cut
        into S pieces (round_pieces); all S all-to-alls are queued on the
        communication stream at once, and piece s's passes + finish
        (kman_dround_finish over its buckets, into two scratch arenas of its
        own) wait only for exchange s -- so exchange s + 1 runs while piece s
        is sorted.  Regions that overflow are redone once every piece is in
        (_redo_ranges: the send and receive arenas are free then).
        Generator; returns the new n_out, or None when a piece's plan does
        not fit (every rank then runs the round the sequential way)."""
        L, ctx, sh = N.lib(), self.dev.ctx, self.shard
        G, me, S_ = self.world, self.rank, self.pieces
        C = np.asarray(C, np.uint64).reshape(G, NB)
        bounds = round_pieces(C, cuts, G, R, r, S_)
        my = bounds[me]
        plans, bad = [], 0
        a2 = b2 = 64
        for s_ in range(S_):
            b0, b1 = my[s_], my[s_ + 1]
            cnt = np.ascontiguousarray(C[:, b0:b1])
            a, b = c_uint64(0), c_uint64(0)
            if b1 > b0:
                ret = L.kman_dround_plan(self.k, self.rflags, self.fmode, G, self.n_bases_q, b1 - b0,
                                         _u64p(cnt.reshape(-1)), byref(a), byref(b))
                bad |= ret != N.KMAN_OK
            plans.append(cnt)
            a2, b2 = max(a2, int(a.value)), max(b2, int(b.value))
        # the round's arenas plus the pieces' must fit this rank's budget (the
        # plan's margin is an estimate): otherwise every rank runs this round
        # the sequential way
        rtab_, sc_, _ = round_send(H, cuts, G, R, r)
        _, _, _, rcnt_, _ = round_recv(C, cuts, R, me, r)
        need = (max(a_need, 8 * int(sc_.sum())) + max(b_need, 8 * int(rcnt_.sum())) + a2 + b2
                + self.out_keys.buf.nbytes + self.out_vals.buf.nbytes)
        bad |= need > self.budget
        f = yield ("allreduce", np.array([bad], np.uint64))
        if int(f[0]):
            return None
        self.overlapped_rounds += 1
        # arenas: A = the send buffer, B = the receive buffer (all pieces),
        # a2 / b2 = a piece's scratch (gen_bufs[1], [2]: free outside a general round)
        rtab, sc, so = round_send(H, cuts, G, R, r)
        _, _, _, rcnt, _ = round_recv(C, cuts, R, me, r)
        A = self.arena_a.get(max(a_need, 8 * int(sc.sum()), 64))
        B = self.arena_b.get(max(b_need, 8 * int(rcnt.sum()), 64))
        A2, B2 = self.gen_bufs[1].get(a2), self.gen_bufs[2].get(b2)
        self.dev.upload(self.d_rtab, rtab)
        N.check(ctx, L.kman_dshard_extract(ctx, c_void_p(sh.codes.ptr), sh.n_eff, self.n_bases_q, self.k, self.flags,
                                           self.fmode, c_void_p(self.d_hist.ptr), c_void_p(self.d_rtab.ptr),
                                           c_void_p(A.ptr)), "kman_dshard_extract")
        cl = np.asarray(c_local, np.uint64)
        at = 0
        recv_at = []
        for s_ in range(S_):
            ssc = np.zeros(G, np.uint64)
            sso = np.zeros(G, np.uint64)
            for q in range(G):
                lo_q = part_of(cuts, R, q, r)[0]
                b0, b1 = bounds[q][s_], bounds[q][s_ + 1]
                ssc[q] = cl[b0:b1].sum()
                sso[q] = so[q] + cl[lo_q:b0].sum()
            rc_s = plans[s_].sum(axis=1).astype(np.uint64)
            ro_s = (np.concatenate([[0], np.cumsum(rc_s)[:-1]]) + at).astype(np.uint64)
            recv_at.append(at)
            at += int(rc_s.sum())
            yield ("alltoallv_async", (A.ptr, ssc, sso, B.ptr, rc_s, ro_s, 8, s_))
            self.exchanged_items += int(ssc.sum())
            self.max_message = max(self.max_message, 8 * int(ssc.max()))
        start, mine = n_out, []
        for s_ in range(S_):
            yield ("comm_wait", s_)
            b0, b1 = my[s_], my[s_ + 1]
            if b1 <= b0:
                continue
            got = c_uint64(0)
            ret = L.kman_dround_finish(ctx, c_void_p(B.ptr + 8 * recv_at[s_]), self.k, self.rflags, self.fmode, G,
                                       self.n_bases_q, b0, b1 - b0, _u64p(plans[s_].reshape(-1)),
                                       c_void_p(A2.ptr), A2.nbytes, c_void_p(B2.ptr), B2.nbytes,
                                       c_void_p(ok_.ptr + 8 * n_out), c_void_p(ov_.ptr + vb * n_out), vb, byref(got))
            if ret == N.KMAN_EPARTIAL:
                mine.append(self._failed_ranges())
            elif ret != N.KMAN_OK:
                N.check(ctx, ret, "kman_dround_finish")
            self._note_heavy()
            n_out += int(got.value)
        f = yield ("allreduce", np.array([0, len(mine)], np.uint64))
        if int(f[1]):
            self.partial_rounds += 1
            mine = np.concatenate(mine) if mine else np.zeros((0, 2), np.uint64)
            rows = yield from self._redo_ranges(mine, n_out - start, A, B, ok_, ov_, start, vb, local=False)
            n_out = start + rows
        return n_out

    def _note_heavy(self) -> None:
        """Adds the heavy keys of the last kman_dround_finish (counted apart
        in its pass 1) to the step's total."""
        n = c_uint32(0)
        N.check(self.dev.ctx, N.lib().kman_dround_heavy(self.dev.ctx, byref(n)), "kman_dround_heavy")
        self.heavy_keys += int(n.value)

    def _failed_ranges(self) -> np.ndarray:
        """[lo, hi] key ranges the last kman_dround_finish left out."""
        L, ctx = N.lib(), self.dev.ctx
        n = c_uint64(0)
        N.check(ctx, L.kman_dround_failed(ctx, None, 0, byref(n)), "kman_dround_failed")
        out = np.zeros((int(n.value), 2), np.uint64)
        if n.value:
            N.check(ctx, L.kman_dround_failed(ctx, out.ctypes.data_as(c_void_p), n.value, byref(n)),
                    "kman_dround_failed")
        return out

    def _redo_ranges(self, mine: np.ndarray, n_region: int, A, B, ok_, ov_, n_out: int, vb: int,
                     local: bool = True):
        """The key ranges each rank's round finish left out (mine: this
        rank's), through the general path: every rank extracts the k-mers of
        each destination's ranges (kman_extract_marked), one exchange, then the
        destination sorts (kman_sort_range, every key bit) and groups them
        (kman_rle_count / kman_rle_uniq) and
        merges the rows with its n_region region rows at ok_/ov_[n_out]
        (kman_merge_runs: the ranges are disjoint).  Generator; returns the
        rows now at n_out."""
        L, ctx, dev, sh = N.lib(), self.dev.ctx, self.dev, self.shard
        G, me, k = self.world, self.rank, self.k
        uniq = self.mode == "uniq"
        tick = [time.perf_counter()]

        def lap(tag):  # (KMAN_DIST_TIMES=1: host-side phase times of the redo, synchronised)
            if os.environ.get("KMAN_DIST_TIMES"):
                dev.sync()
                t = time.perf_counter()
                self.phase_ms["redo_" + tag] = self.phase_ms.get("redo_" + tag, 0.0) + (t - tick[0]) * 1e3
                tick[0] = t

        # local: each rank's left-out items are still in its last finish's
        # pass-1 output (kman_dround_left; not after overlapped pieces, whose
        # scratch the later pieces reused) -- no re-extraction, no exchange.
        # Every rank or none (a rank whose pass 1 itself overflowed needs the
        # others' marked extraction)
        n_left = c_uint64(0)
        local = local and os.environ.get("KMAN_LOCAL_REDO", "1") != "0"
        rc_ = L.kman_dround_left(ctx, None, None, 0, byref(n_left)) if local else N.KMAN_EFALLBACK
        if rc_ not in (N.KMAN_OK, N.KMAN_EFALLBACK):
            N.check(ctx, rc_, "kman_dround_left")
        f = yield ("allreduce", np.array([0 if rc_ == N.KMAN_OK else 1], np.uint64))
        if int(f[0]) == 0:
            nr = int(n_left.value)
            if vb == 4 and nr > 0xFFFFFFFF:
                raise NotImplementedError("a redone key range of more than 2^32 k-mers would need u64 counts")
            rk, ak = (self.gen_bufs[i].get(8 * max(1, nr)) for i in (1, 2))
            rp = ap = None
            if uniq:
                rp, ap = (self.gen_bufs[i].get(8 * max(1, nr)) for i in (4, 5))
            got = c_uint64(0)
            N.check(ctx, L.kman_dround_left(ctx, c_void_p(rk.ptr), c_void_p(rp.ptr) if uniq else None, nr,
                                            byref(got)), "kman_dround_left")
            self.redone_kmers += nr
            self.local_redo_kmers += nr
            lap("gather")
            return (yield from self._redo_rows(rk, ak, rp, ap, nr, n_region, A, B, ok_, ov_, n_out, vb, lap, True))
        cnt = yield ("allgather", np.array([len(mine)], np.uint64))
        cnt = np.asarray(cnt, np.uint64).reshape(G)
        m = max(1, int(cnt.max()))
        pad = np.zeros(2 * m, np.uint64)
        pad[:2 * len(mine)] = np.asarray(mine, np.uint64).reshape(-1)
        allr = yield ("allgather", pad)
        ranges = gather_ranges(cnt, allr, G)
        # destination map over key prefixes, so each destination's k-mers
        # come out in one pass (kman_extract_marked) however many ranges it has
        pbits, pmap = redo_map(ranges, 2 * k)
        d_map = self.part_bufs[2].get(len(pmap))
        dev.upload(d_map, pmap)
        flags = engine.flags_for(self.rc, uniq, self.canonical, self.mixed)

        def marked(q, keys_ptr, pos_ptr, cap):
            got = c_uint64(0)
            rc_ = L.kman_extract_marked(ctx, c_void_p(sh.codes.ptr), sh.n_eff, k, flags, c_void_p(d_map.ptr), pbits,
                                        q + 1, c_void_p(keys_ptr) if keys_ptr else None,
                                        c_void_p(pos_ptr) if pos_ptr else None, 8, cap, byref(got))
            if rc_ not in (N.KMAN_OK, N.KMAN_ECAP) or (cap and rc_ != N.KMAN_OK):
                N.check(ctx, rc_, "kman_extract_marked")
            return int(got.value)

        lap("map")
        # the send buffers are the round's arenas (free once its finish is
        # done): each destination's k-mers extracted straight in, the count
        # coming back with them; only if they do not fit, counted first
        ecap = min(A.nbytes, B.nbytes if uniq else A.nbytes) // 8
        sc = np.zeros(G, np.uint64)
        at = 0
        sk, sp = A, (B if uniq else None)
        fits = True
        for q in range(G):
            if not len(ranges[q]):
                continue
            got = c_uint64(0)
            rc_ = L.kman_extract_marked(ctx, c_void_p(sh.codes.ptr), sh.n_eff, k, flags, c_void_p(d_map.ptr), pbits,
                                        q + 1, c_void_p(A.ptr + 8 * at), c_void_p(B.ptr + 8 * at) if uniq else None,
                                        8, max(0, ecap - at), byref(got))
            if rc_ == N.KMAN_ECAP:
                fits = False
                break
            N.check(ctx, rc_, "kman_extract_marked")
            sc[q] = int(got.value)
            at += int(got.value)
        if not fits:  # (more than the arenas hold: counted, then extracted into grown buffers)
            sc = np.array([marked(q, 0, 0, 0) if len(ranges[q]) else 0 for q in range(G)], np.uint64)
            ns = int(sc.sum())
            sk = self.gen_bufs[0].get(8 * max(1, ns))
            sp = self.gen_bufs[3].get(8 * max(1, ns)) if uniq else None
            at = 0
            for q in range(G):
                want = int(sc[q])
                if want and marked(q, sk.ptr + 8 * at, sp.ptr + 8 * at if uniq else 0, want) != want:
                    raise RuntimeError("rank %d: rank %d's left-out k-mers changed between passes" % (me, q))
                at += want
        if uniq:
            at = 0
            for q in range(G):
                if sc[q]:
                    N.check(ctx, L.kman_or_u64(ctx, c_void_p(sp.ptr + 8 * at), int(sc[q]), me << RANK_SHIFT), "tag")
                at += int(sc[q])
        lap("extract")
        sent = np.asarray((yield ("allgather", sc)), np.uint64).reshape(G, G)  # sent[src, dst]
        rcnt = sent[:, me].copy()
        roff = np.concatenate([[0], np.cumsum(rcnt)[:-1]]).astype(np.uint64)
        so = np.concatenate([[0], np.cumsum(sc)[:-1]]).astype(np.uint64)
        nr = int(rcnt.sum())
        self.redone_kmers += nr
        if vb == 4 and nr > 0xFFFFFFFF:
            raise NotImplementedError("a redone key range of more than 2^32 k-mers would need u64 counts")
        rk, ak = (self.gen_bufs[i].get(8 * max(1, nr)) for i in (1, 2))
        rp = ap = None
        if uniq:
            rp, ap = (self.gen_bufs[i].get(8 * max(1, nr)) for i in (4, 5))
        yield ("alltoallv", (sk.ptr, sc, so, rk.ptr, rcnt, roff, 8))
        if uniq:
            yield ("alltoallv", (sp.ptr, sc, so, rp.ptr, rcnt, roff, 8))
        lap("exchange")
        return (yield from self._redo_rows(rk, ak, rp, ap, nr, n_region, A, B, ok_, ov_, n_out, vb, lap, False))

    def _redo_rows(self, rk, ak, rp, ap, nr, n_region, A, B, ok_, ov_, n_out, vb, lap, heavy_fix):
        """The redone items rk (+ pos rp) -> rows: a full-key sort, run-length,
        and (ordered) a merge with the n_region region rows at ok_/ov_[n_out].
        heavy_fix: the items came from the finish's pass-1 output
        (kman_dround_left), so the heavy keys' dropped copies are added to
        their rows.  Generator (no collective); returns the rows at n_out."""
        L, ctx, k = N.lib(), self.dev.ctx, self.k
        uniq = self.mode == "uniq"
        me = self.rank
        n_gen = 0
        if self.ordered:
            gk, gv = self.part_bufs[0].get(8 * max(1, nr)), self.part_bufs[1].get(vb * max(1, nr))
        else:  # (rows as a multiset: straight after the region rows; they fit, rows <= received k-mers)
            if (n_out + n_region + nr) * 8 > ok_.nbytes or (n_out + n_region + nr) * vb > ov_.nbytes:
                # (the redone windows are a subset of the round's: the marked
                # extraction and the shard extraction disagree if this fires)
                raise RuntimeError("rank %d: %d region rows + %d redone k-mers past the output buffer (%d rows)"
                                   % (me, n_out + n_region, nr, ok_.nbytes // 8))
            gk, gv = (_View(ok_.ptr + 8 * (n_out + n_region), 8 * max(1, nr)),
                      _View(ov_.ptr + vb * (n_out + n_region), vb * max(1, nr)))
        if nr:
            # a full-key sort, then run-length: these ranges are where keys
            # repeat far beyond a region's share, so equal-prefix segments are
            # huge (kman_finish would re-sort them through its big-segment
            # path) while the sort's passes do not care
            res = c_int(0)
            vbytes = 8 if uniq else 0
            N.check(ctx, L.kman_sort_range(ctx, c_void_p(rk.ptr), c_void_p(ak.ptr), c_void_p(rp.ptr) if uniq else None,
                                           c_void_p(ap.ptr) if uniq else None, vbytes, nr, 0, 2 * k, None,
                                           byref(res)), "kman_sort_range")
            keys = ak if res.value else rk
            pos = (ap if res.value else rp) if uniq else None
            lap("sort")
            out = c_uint64(0)
            if uniq:
                N.check(ctx, L.kman_rle_uniq(ctx, c_void_p(keys.ptr), c_void_p(pos.ptr), 8, nr, c_void_p(gk.ptr),
                                             c_void_p(gv.ptr), byref(out)), "kman_rle_uniq")
            else:
                N.check(ctx, L.kman_rle_count(ctx, c_void_p(keys.ptr), nr, c_void_p(gk.ptr), c_void_p(gv.ptr), vb,
                                              byref(out)), "kman_rle_count")
            n_gen = int(out.value)
            if heavy_fix and not uniq:
                N.check(ctx, L.kman_dround_heavy_fix(ctx, c_void_p(gk.ptr), c_void_p(gv.ptr), vb, n_gen),
                        "kman_dround_heavy_fix")
            lap("finish")
        if n_gen and self.ordered:
            # the region rows move to the (now free) round arenas, then the two
            # sorted, key-disjoint runs merge back into place
            N.check(ctx, L.kman_memcpy_d2d(ctx, c_void_p(A.ptr), c_void_p(ok_.ptr + 8 * n_out), 8 * n_region), "copy")
            N.check(ctx, L.kman_memcpy_d2d(ctx, c_void_p(B.ptr), c_void_p(ov_.ptr + vb * n_out), vb * n_region),
                    "copy")
            lap("copy")
            runs = (N.Run * 2)(N.Run(c_void_p(A.ptr), c_void_p(B.ptr), n_region),
                               N.Run(c_void_p(gk.ptr), c_void_p(gv.ptr), n_gen))
            N.check(ctx, L.kman_merge_runs(ctx, runs, 2, vb, c_void_p(ok_.ptr + 8 * n_out),
                                           c_void_p(ov_.ptr + vb * n_out), None, None), "kman_merge_runs")
            lap("merge")
        return n_region + n_gen
        yield  # (a generator: the callers delegate with yield from)

    def _vb(self, C) -> int:
        """Output value bytes: uniq pos are u64 (source rank in bits 56-63);
        counts are u32 -- a region-path count is at most a region's size, and
        a general round checks its receive size (_general_round)."""
        return 8 if self.mode == "uniq" else 4

    def _prefix_hist(self) -> np.ndarray:
        """Top-8-bit bucket totals of the shard (general path)."""
        if self.canonical:
            raise NotImplementedError("canonical keys with k > 25 across ranks")
        sh = self.shard
        h = self.d_small
        n = c_uint64(0)
        N.check(self.dev.ctx, N.lib().kman_kmer_prefix_hist(self.dev.ctx, c_void_p(sh.codes.ptr), sh.n_eff, self.k,
                                                            N.KMAN_RC if self.rc else 0, c_void_p(h.ptr), byref(n)),
                "kman_kmer_prefix_hist")
        bins = NB if 2 * self.k >= 8 else 1 << (2 * self.k)
        out = np.zeros(NB, np.uint64)
        out[:bins] = self.dev.download(h, bins, np.uint64)
        return out

    def _general_round(self, C, cuts, R, r, ok_, ov_, n_out, vb):
        """Round r through key ranges: per destination q, kman_extract_range
        of part (q, r) into the send buffers; the keys (+ pos tagged with the
        source rank) exchanged; kman_sort_range + kman_finish appended to the
        output.  Generator; returns the rows written."""
        L, ctx, dev, sh = N.lib(), self.dev.ctx, self.dev, self.shard
        G, me, k = self.world, self.rank, self.k
        uniq = self.mode == "uniq"
        send, recv = round_sizes(C, cuts, G, R)
        ns, nr = int(send[me, r]), int(recv[me, r])
        if vb == 4 and int(recv[:, r].max()) > 0xFFFFFFFF:  # (every rank sees the same sizes)
            raise NotImplementedError("a general round of more than 2^32 k-mers would need u64 counts")
        sk, rk, ak = (self.gen_bufs[i].get(8 * max(1, n)) for i, n in ((0, ns), (1, nr), (2, nr)))
        sp = rp = ap = None
        if uniq:
            sp, rp, ap = (self.gen_bufs[i].get(8 * max(1, n)) for i, n in ((3, ns), (4, nr), (5, nr)))
        shift = max(0, 2 * k - 8)
        sc = np.zeros(G, np.uint64)
        at = 0
        flags = engine.flags_for(self.rc, uniq, self.canonical, self.mixed)
        for q in range(G):
            lo, hi = part_of(cuts, R, q, r)
            want = int(np.asarray(C, np.uint64)[me, lo:hi].sum())
            if want:
                got = c_uint64(0)
                key_hi = (hi << shift) - 1 if hi < NB else (1 << (2 * k)) - 1
                N.check(ctx, L.kman_extract_range(ctx, c_void_p(sh.codes.ptr), sh.n_eff, k, flags, lo << shift, key_hi,
                                                  c_void_p(sk.ptr + 8 * at), c_void_p(sp.ptr + 8 * at) if uniq else None,
                                                  8, want, None, byref(got)), "kman_extract_range")
                if int(got.value) != want:
                    raise RuntimeError("rank %d part (%d, %d): %d k-mers, histogram said %d"
                                       % (me, q, r, got.value, want))
                if uniq:
                    N.check(ctx, L.kman_or_u64(ctx, c_void_p(sp.ptr + 8 * at), want, me << RANK_SHIFT), "tag")
            sc[q] = want
            at += want
        so = np.concatenate([[0], np.cumsum(sc)[:-1]]).astype(np.uint64)
        _, _, _, rcnt, roff = round_recv(C, cuts, R, me, r)
        yield ("alltoallv", (sk.ptr, sc, so, rk.ptr, rcnt, roff, 8))
        if uniq:
            yield ("alltoallv", (sp.ptr, sc, so, rp.ptr, rcnt, roff, 8))
        if nr == 0:
            return 0
        res = c_int(0)
        lo_bit = engine.split_bits(nr, 2 * k)
        vbytes = 8 if uniq else 0
        N.check(ctx, L.kman_sort_range(ctx, c_void_p(rk.ptr), c_void_p(ak.ptr), c_void_p(rp.ptr) if uniq else None,
                                       c_void_p(ap.ptr) if uniq else None, vbytes, nr, lo_bit, 2 * k, None, byref(res)),
                "kman_sort_range")
        keys, alt = (ak, rk) if res.value else (rk, ak)
        pos, palt = ((ap, rp) if res.value else (rp, ap)) if uniq else (None, None)
        out = c_uint64(0)
        N.check(ctx, L.kman_finish(ctx, c_void_p(keys.ptr), c_void_p(alt.ptr), c_void_p(pos.ptr) if uniq else None,
                                   c_void_p(palt.ptr) if uniq else None, vbytes, nr, 2 * k, lo_bit, self.fmode,
                                   c_void_p(ok_.ptr + 8 * n_out), c_void_p(ov_.ptr + vb * n_out), vb, byref(out)),
                "kman_finish")
        return int(out.value)

    # -------------------------------------------------------------- results
    @property
    def n_kmers(self) -> int:
        return self.n_local

    @property
    def n_sorted(self) -> int:
        return self.n_recv

    def results(self):
        """Rank-local (keys, counts | pos) on the host; uniq pos keep the
        source rank in bits 56-63 (tests)."""
        ok_, ov_, vb = self._out
        keys = self.dev.download(ok_, self.n_out, np.uint64)
        vals = self.dev.download(ov_, self.n_out, np.uint32 if vb == 4 else np.uint64).astype(np.uint64)
        return keys, vals

    def hist_gen(self, nbins: int = 10001):
        """Abundance spectrum of the global counts: local kman_count_hist of
        this rank's rows, all-reduced (config 5).  Generator."""
        ok_, ov_, vb = self._out
        if nbins > 16384:
            raise ValueError("at most 16384 histogram bins")
        d_h = self.d_small
        N.check(self.dev.ctx, N.lib().kman_count_hist(self.dev.ctx, c_void_p(ov_.ptr), vb, self.n_out,
                                                      c_void_p(d_h.ptr), nbins), "kman_count_hist")
        h = self.dev.download(d_h, nbins, np.uint64)
        return (yield ("allreduce", h))

    def global_parsed(self) -> engine.Parsed:
        """The all-gathered record table as a Parsed (for the uniq formatter;
        no codes)."""
        names = self.names
        name_off = np.zeros(len(names) + 1, dtype=np.uint64)
        if names:
            name_off[1:] = np.cumsum([len(x) for x in names], dtype=np.uint64)
        return engine.Parsed(self.dev, None, self.n_bases_total, len(names), np.zeros(len(names), np.uint64),
                             self.g_rec_seq, names, b"".join(names), name_off)

    def text(self) -> bytes:
        """This rank's slice of the reference's output text (count rows, or
        uniq records with global headers), built on the device."""
        if not self.ordered:
            raise ValueError("ordered=False keeps the rows as a multiset (the spectrum): no output text")
        ok_, ov_, vb = self._out
        if self.mode == "count":
            r = engine.CountResult(ok_, ov_, vb, self.n_out, self.k)
            return bytes(engine.emit_count(self.dev, r) or b"")
        pos = self.dev.alloc(8 * max(1, self.n_out))
        try:
            N.check(self.dev.ctx, N.lib().kman_memcpy_d2d(self.dev.ctx, c_void_p(pos.ptr), c_void_p(ov_.ptr),
                                                          8 * self.n_out), "d2d")
            off = np.ascontiguousarray(self.base_off, dtype=np.uint64)
            N.check(self.dev.ctx, N.lib().kman_rebase_pos(self.dev.ctx, c_void_p(pos.ptr), self.n_out, _u64p(off),
                                                          self.world), "kman_rebase_pos")
            r = engine.UniqResult(ok_, pos, 8, self.n_out, self.k)
            return bytes(engine.emit_uniq(self.global_parsed(), r) or b"")
        finally:
            pos.free()

    def emit_gen(self, path: str):
        """Write the global output file: every rank formats its rows, the text
        sizes are all-gathered and each rank writes at its offset (the ranks'
        texts in rank order = the reference's output).  Generator."""
        t = self.text()
        sizes = yield ("allgather", np.array([len(t)], np.uint64))
        off = int(sizes[:self.rank, 0].sum())
        total = int(sizes[:, 0].sum())
        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            if self.rank == 0:
                os.ftruncate(fd, total)
            if t:
                os.pwrite(fd, t, off)
        finally:
            os.close(fd)
        yield ("allreduce", np.zeros(1, np.uint64))  # every slice written before anyone reads
        return total

    # bench.py interface
    pos_bytes = 8

    def timing(self, enable: bool) -> None:
        N.check(self.dev.ctx, N.lib().kman_timing_enable(self.dev.ctx, 1 if enable else 0), "timing")

    def timed(self, tag: str):
        n, ms = c_uint64(0), ctypes.c_double(0)
        N.check(self.dev.ctx, N.lib().kman_timing_query(self.dev.ctx, tag.encode(), byref(n), byref(ms)), "timing")
        return int(n.value), float(ms.value)

    def free(self) -> None:
        if self.comm is not None:
            self.comm.free()
            self.comm = None
        for b in ([self.d_hist, self.d_rtab, self.d_small, self.arena_a, self.arena_b, self.out_keys, self.out_vals]
                  + self.gen_bufs + self.part_bufs):
            b.free()
        if self.loader is not None:
            self.loader.free()


def local_groups(p: engine.Parsed, k: int, rc: bool, mode: str, canonical: bool = False,
                 max_round_items: Optional[int] = None, ordered: bool = True):
    """Count / uniq of one parsed input on one GPU through the key rounds of
    the multi-GPU path (shard histogram, exact extraction, per-bucket passes,
    LDS finish; a round whose regions overflow is redone by key range): the
    region-class kernels for the inputs kman_groups does not take -- more
    k-mers than its region capacities, `-r` on large inputs, skewed keys.
    None when the rounds do not take the input either (uniq with k > 25 or
    more pos bits than an item holds)."""
    flags = engine.flags_for(rc and not canonical, mode == "uniq", canonical, canonical and not ordered)
    fm = N.KMAN_FINISH_UNIQ if mode == "uniq" else N.KMAN_FINISH_COUNT
    if k > engine.MAX_K or N.lib().kman_dshard_plan(p.n_bases, p.n_bases, k, flags, fm) != N.KMAN_OK:
        return None
    sh = S.ShardCodes(p.dev, S.ShardSpec(0, 0, 0, 0, 0), k, codes=p.codes, n_own=p.n_bases, n_eff=p.n_bases,
                      names=list(p.names), rec_seq=np.asarray(p.rec_seq, dtype=np.uint64))
    t0 = time.perf_counter()
    pipe = DistPipeline(p.dev, None, k, mode, 1, 0, None, canonical=canonical, rc=rc, shard=sh, local=True,
                        max_round_items=max_round_items, ordered=ordered)
    try:
        t1 = time.perf_counter()
        pipe.step()
        p.dev.sync()
        t2 = time.perf_counter()
        LAST_LOCAL.clear()
        LAST_LOCAL.update(setup_ms=(t1 - t0) * 1e3, step_ms=(t2 - t1) * 1e3, rounds=pipe.rounds,
                          fallback_rounds=pipe.fallback_rounds, partial_rounds=pipe.partial_rounds,
                          redone_kmers=pipe.redone_kmers, heavy_keys=pipe.heavy_keys,
                          plan=getattr(pipe, "plan_info", None),
                          phases_ms=dict(pipe.phase_ms))
        return pipe.take_result()
    finally:
        pipe.free()


class LocalRounds:
    """local_groups with its buffers held across steps (tools/widebench.py
    times the compute the way bench.py times ResidentPipeline): step() runs
    the key rounds over the resident codes, result() views the rows."""

    def __init__(self, p: engine.Parsed, k: int, rc: bool, mode: str, canonical: bool = False,
                 max_round_items: Optional[int] = None, ordered: bool = True):
        sh = S.ShardCodes(p.dev, S.ShardSpec(0, 0, 0, 0, 0), k, codes=p.codes, n_own=p.n_bases, n_eff=p.n_bases,
                          names=list(p.names), rec_seq=np.asarray(p.rec_seq, dtype=np.uint64))
        self.pipe = DistPipeline(p.dev, None, k, mode, 1, 0, None, canonical=canonical, rc=rc, shard=sh, local=True,
                                 max_round_items=max_round_items, ordered=ordered)

    def step(self) -> int:
        return self.pipe.step()

    def result(self):
        ok_, ov_, vb = self.pipe._out
        if self.pipe.mode == "uniq":
            return engine.UniqResult(ok_, ov_, 8, self.pipe.n_out, self.pipe.k)
        return engine.CountResult(ok_, ov_, vb, self.pipe.n_out, self.pipe.k)

    def free(self) -> None:
        self.pipe.free()


LAST_LOCAL: dict = {}  # the last local_groups call: rounds, fallbacks, host-side phase times (tools/widebench.py)


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    rc = N.lib().kman_comm_unique_id(buf)
    if rc != N.KMAN_OK:
        raise RuntimeError("kman_comm_unique_id failed (%d)" % rc)
    return buf.raw


__all__ = ["plan_lut", "part_cuts", "part_of", "round_send", "round_recv", "round_sizes", "RoundPlanner",
           "DistPipeline", "RcclComm", "SimGroup", "unique_id", "rehearse", "List"]


# ------------------------------------------------------------- CPU rehearsal


def rehearse(keys: np.ndarray, k: int, world: int, rank: int, comm, n_bases_q: int, mode: str = "count",
             canonical: bool = False, max_round_items: Optional[int] = None, budget: int = 1 << 62, fail=()):
    """The planning and exchanges of DistPipeline.step_gen on host arrays
    (tests/test_dist_cpu.py over gloo): bucket totals all-gathered, the same
    RoundPlanner, per round the items of the round's buckets sent
    destination-major as round_send lays them out, one all-to-all, the finish
    by numpy; `fail` = {(rank, round)} raises a region overflow there, agreed
    by an all-reduce exactly like the device path: that rank's first bucket of
    the round is left out of its rows (as KMAN_EPARTIAL leaves overflowing
    regions out), the ranges all-gathered, every rank sends each destination
    its k-mers under redo_map, the destination merges them in (the device
    path's _redo_ranges).  comm: allgather(a) -> flat array, allreduce(a),
    alltoallv(list) -> list.  Returns (keys, counts, R, cuts, rounds_redone)."""
    shift = max(0, 2 * k - 8)
    keys = np.asarray(keys, dtype=np.uint64)
    b = (keys >> np.uint64(shift)).astype(np.int64)
    c_local = np.bincount(b, minlength=NB).astype(np.uint64)
    C = comm.allgather(c_local).reshape(world, NB)
    fm = N.KMAN_FINISH_UNIQ if mode == "uniq" else N.KMAN_FINISH_COUNT
    pl = RoundPlanner(k, engine.flags_for(False, mode == "uniq", canonical), fm, world, n_bases_q)
    R, cuts, _, _ = pl.plan(C, budget, max_round_items)
    outk, outc, redone = [], [], []
    for r in range(R):
        parts = []
        for q in range(world):
            lo, hi = part_of(cuts, R, q, r)
            parts.append(keys[(b >= lo) & (b < hi)])
        _, sc, _ = round_send(np.pad(c_local.reshape(NB, 1), ((0, 0), (0, RS - 1))), cuts, world, R, r)
        assert [len(p) for p in parts] == sc.tolist(), "send layout disagrees with the histogram"
        got = comm.alltoallv(parts)
        _, _, _, rc, _ = round_recv(C, cuts, R, rank, r)
        assert [len(g) for g in got] == rc.tolist(), "receive sizes disagree with the all-gathered counts"
        rk = np.sort(np.concatenate(got)) if got else np.zeros(0, np.uint64)
        mine = np.zeros((0, 2), np.uint64)
        if (rank, r) in fail:
            ql, qh = part_of(cuts, R, rank, r)
            if qh > ql:  # the part's first bucket overflowed
                mine = np.array([[ql << shift, ((ql + 1) << shift) - 1]], np.uint64)
        for lo, hi in mine:  # its rows are left out
            rk = rk[(rk < lo) | (rk > hi)]
        u, c = np.unique(rk, return_counts=True)
        f = comm.allreduce(np.array([0, len(mine)], np.uint64))
        if int(f[1]):
            redone.append(r)
            cnt = comm.allgather(np.array([len(mine)], np.uint64))
            m = max(1, int(np.asarray(cnt).max()))
            pad = np.zeros(2 * m, np.uint64)
            pad[:2 * len(mine)] = mine.reshape(-1)
            ranges = gather_ranges(cnt, comm.allgather(pad), world)
            pbits, pmap = redo_map(ranges, 2 * k)
            dest = pmap[(keys >> np.uint64(2 * k - pbits)).astype(np.int64)].astype(np.int64) - 1
            got = comm.alltoallv([keys[dest == q] for q in range(world)])
            gk, gc = np.unique(np.concatenate(got) if got else np.zeros(0, np.uint64), return_counts=True)
            o = np.argsort(np.concatenate([u, gk]), kind="stable")  # key-disjoint runs merged
            u, c = np.concatenate([u, gk])[o], np.concatenate([c, gc])[o]
        outk.append(u)
        outc.append(c.astype(np.uint64))
    return (np.concatenate(outk) if outk else np.zeros(0, np.uint64),
            np.concatenate(outc) if outc else np.zeros(0, np.uint64), R, cuts, redone)
