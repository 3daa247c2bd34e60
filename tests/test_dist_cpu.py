"""Multi-GPU join logic rehearsed on CPU (no GPU needed).

* Byte-range shards of ONE FASTA (kman_amd/shard.py): every shard's own
  windows, with the halo, concatenated in rank order are exactly the windows
  of the whole file (np_oracle over the file, seq.py:285-328).
* 2 ranks over gloo run the planning and exchanges of
  DistPipeline.step_gen (dist.rehearse: all-gathered bucket totals, the same
  RoundPlanner, round_send / round_recv layouts, one all-to-all per round, a
  region overflow agreed by all-reduce and the round redone by key range),
  with numpy standing in for the device passes.  The rank-ordered
  concatenation of the per-rank counts equals the single-process count.
* The round planner accepts BASELINE config 4 (100 GB over 8 ranks,
  12.5 G bases per rank) within one MI355X's HBM."""

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


def _shard_windows(text: bytes, world: int, k: int):
    """(keys, global pos) of every shard's own windows, in rank order, the
    way the device shard sees them: (a record opener if the shard starts in a
    record) + its bytes + halo; windows starting in its own bases only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import np_oracle
    from kman_amd import shard

    rd = shard.BytesReader(text)
    specs = shard.shard_specs(rd, world, k)
    keys, pos, base = [], [], 0
    for sp in specs:
        pre = b">\n" if sp.start > sp.h0 else b""
        if sp.own_end > sp.start and sp.own_end > sp.h0:
            own = sum(len(x) for _, x in np_oracle.parse_fasta(pre + text[sp.start:sp.own_end]))
        else:
            own = 0
        if own:
            kk, pp = np_oracle.stream_kmers(np_oracle.parse_fasta(pre + text[sp.start:sp.halo_end]), k)
            m = (pp >> np.uint64(1)) < np.uint64(own)
            keys.append(kk[m])
            pos.append(pp[m] + np.uint64(2 * base))
        base += own
    return specs, np.concatenate(keys) if keys else np.zeros(0, np.uint64), \
        np.concatenate(pos) if pos else np.zeros(0, np.uint64)


def _texts():
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import inputs

    lay = inputs.SynthLayout(60_000, 5, record_len=7_000, width=61)
    return [inputs.messy_records(11, n_records=30, max_len=3000), inputs.messy_records(12, n_records=8, max_len=9000),
            lay.read(0, lay.size), b"junk line\n\n>r1 x\nACGTACGTAC\r\nGGTT\n>r2\n\n>r3\nAC\nGT\nTTTTTTTT\n"]


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8, 17])
@pytest.mark.parametrize("k", [2, 5, 21])
def test_shards_cover_the_stream_exactly(world, k):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import np_oracle

    for text in _texts():
        specs, keys, pos = _shard_windows(text, world, k)
        wk, wp = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k)
        np.testing.assert_array_equal(keys, wk)
        np.testing.assert_array_equal(pos, wp)
        assert specs[0].start == 0 and specs[-1].own_end == len(text)
        for a, b in zip(specs, specs[1:]):
            assert a.own_end == b.start and a.start <= a.own_end <= a.halo_end
            c = b.start
            assert c == len(text) or text[c - 1:c] == b"\n" or (text[c - 1:c] == b"\r" and text[c:c + 1] != b"\n")


def test_synth_layout_reads_agree():
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import inputs
    import np_oracle

    lay = inputs.SynthLayout(10_000, 9, record_len=3_333, width=80)
    t = lay.read(0, lay.size)
    assert len(t) == lay.size
    assert t == b"".join(lay.read(a, min(a + 777, lay.size)) for a in range(0, lay.size, 777))
    recs = np_oracle.parse_fasta(t)
    assert [n for n, _ in recs] == [b"syn0", b"syn1", b"syn2", b"syn3"]
    assert sum(len(s) for _, s in recs) == 10_000 and all(len(s) <= 3_333 for _, s in recs)
    assert set(b"".join(s for _, s in recs)) == set(b"ACGT")


def _worker(rank, world, port, k, q, max_items, fail):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kman_amd import dist as kd

        text = _texts()[2]
        specs, keys, pos = _shard_windows(text, world, k)
        # this rank's windows: those whose global base lies in its own bases
        bases = np.cumsum([0] + [_own_bases(text, sp) for sp in specs])
        m = ((pos >> np.uint64(1)) >= np.uint64(bases[rank])) & ((pos >> np.uint64(1)) < np.uint64(bases[rank + 1]))
        ck, cc, R, cuts, redone = kd.rehearse(keys[m], k, world, rank, GlooComm(dist, world), int(bases[-1]),
                                              max_round_items=max_items, fail=fail)
        q.put((rank, ck, cc, R, list(cuts), redone))
    finally:
        dist.destroy_process_group()


def _own_bases(text, sp):
    import np_oracle

    pre = b">\n" if sp.start > sp.h0 else b""
    if sp.own_end <= sp.start or sp.own_end <= sp.h0:
        return 0
    return sum(len(x) for _, x in np_oracle.parse_fasta(pre + text[sp.start:sp.own_end]))


@pytest.mark.parametrize("k,max_items,fail", [(5, None, ()), (21, None, ()), (21, 9_000, ()),
                                              (21, 9_000, ((1, 1),)), (21, 9_000, ((0, 0), (0, 1), (1, 1))),
                                              (13, None, ((0, 0),))])
def test_two_rank_rounds_equal_single_process(k, max_items, fail):
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import np_oracle

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, q, max_items, fail)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    keys, _ = np_oracle.stream_kmers(np_oracle.parse_fasta(_texts()[2]), k)
    wk, wc = np_oracle.rle_count(np_oracle.stable_sort(keys)[0])
    np.testing.assert_array_equal(np.concatenate([r[1] for r in res]), wk)
    np.testing.assert_array_equal(np.concatenate([r[2] for r in res]), wc)
    R = res[0][3]
    assert all(r[3] == R and r[4] == res[0][4] for r in res), "ranks planned differently"
    if max_items:
        assert R >= 3
    # the left-out ranges are redone in the same rounds on both ranks
    assert res[0][5] == res[1][5] == sorted({r for (_, r) in fail})
    if len(res[0][1]) and len(res[1][1]):
        assert res[0][1].max() < res[1][1].min()  # rank order = key order


def test_part_cuts_are_contiguous_and_balanced():
    from kman_amd import dist

    rng = np.random.default_rng(0)
    for parts in (1, 2, 3, 5, 8, 24, 64):
        g = rng.poisson(3_900_000, 256).astype(np.uint64)
        cuts = dist.part_cuts(g, parts)
        assert cuts[0] == 0 and cuts[-1] == 256 and (np.diff(cuts) >= 0).all()
        share = np.array([g[cuts[p]:cuts[p + 1]].sum() for p in range(parts)], np.float64) / g.sum()
        assert np.abs(share - 1 / parts).max() <= 1.5 / 256 + 1e-9


def test_round_layouts_are_consistent():
    from kman_amd import dist

    rng = np.random.default_rng(1)
    G, R = 3, 4
    H = [rng.integers(0, 50, size=(256, 64)).astype(np.uint64) for _ in range(G)]
    C = np.stack([h.sum(axis=1) for h in H])
    cuts = dist.part_cuts(C.sum(axis=0), G * R)
    send, recv = dist.round_sizes(C, cuts, G, R)
    for r in range(R):
        for q in range(G):
            rtab, sc, so = dist.round_send(H[q], cuts, G, R, r)
            assert sc.sum() == send[q, r]
            kept = rtab != np.uint64(0xFFFFFFFFFFFFFFFF)
            # kept regions tile [0, send) exactly, destination-major
            base = rtab[kept].astype(np.int64)
            cnt = H[q].reshape(-1)[kept].astype(np.int64)
            assert (base[1:] == (base + cnt)[:-1]).all() and (len(base) == 0 or base[0] == 0)
            lo, nb, counts, rc, ro = dist.round_recv(C, cuts, R, q, r)
            assert rc.sum() == recv[q, r] and counts.shape == (G, nb)
            assert rc[q] == sum(H[q][b].sum() for b in range(lo, lo + nb))
    # every rank's rounds cover its buckets once; ranks in key order
    owned = [[dist.part_of(cuts, R, q, r) for r in range(R)] for q in range(G)]
    flat = [x for q in owned for x in q]
    assert flat[0][0] == 0 and flat[-1][1] == 256 and all(a[1] == b[0] for a, b in zip(flat, flat[1:]))


def test_config4_plan_fits_one_mi355x():
    """BASELINE config 4: 100 GB FASTA, k = 21, 8 ranks -> 12.5 G bases (k-mers)
    per rank.  The shard geometry is accepted and the rounds fit the HBM left
    after the codes (12.5 GB) and the count output (12 B per received k-mer)."""
    from kman_amd import _native as N
    from kman_amd import dist

    L = N.lib()
    nbase = 12_500_000_000
    assert L.kman_dshard_plan(nbase, nbase, 21, 0, N.KMAN_FINISH_COUNT) == N.KMAN_OK
    G = 8
    C = np.full((G, 256), nbase // 256, dtype=np.uint64)
    hbm = 288 * 10**9
    budget = int(0.85 * hbm) - nbase - 12 * (nbase + (1 << 20))
    pl = dist.RoundPlanner(21, 0, N.KMAN_FINISH_COUNT, G, nbase)
    R, cuts, a, b = pl.plan(C, budget)
    assert a + b <= budget and 1 < R <= 8
    for q in range(G):
        for r in range(R):
            assert pl.arenas(C, cuts, R, q, r) is not None


def test_roomy_plan_only_when_the_rounds_still_fit():
    """KMAN_ROOMY (pass-1 sub-regions at twice the expected fill, so that a
    left-out region can be redone from pass 1's output): kman_dround_plan's
    arena A grows by the pass-1 sub-regions' extra room, arena B does not;
    RoundPlanner.roomy takes it only when the same rounds fit the budget --
    so config 4's rank shape keeps its plain plan on one MI355X -- and
    KMAN_ROOMY=0 turns it off."""
    import os
    from ctypes import byref, c_uint64

    from kman_amd import _native as N
    from kman_amd import dist

    L = N.lib()
    counts = np.full(256, 12_000_000, dtype=np.uint64)
    ab = {}
    for fl in (0, N.KMAN_ROOMY):
        a, b = c_uint64(0), c_uint64(0)
        assert L.kman_dround_plan(21, fl, N.KMAN_FINISH_COUNT, 1, 3 * 10**9, 256, dist._u64p(counts), byref(a),
                                  byref(b)) == N.KMAN_OK
        ab[fl] = (a.value, b.value)
    extra = ab[N.KMAN_ROOMY][0] - ab[0][0]
    assert ab[N.KMAN_ROOMY][1] == ab[0][1]
    # the pass-1 items (8 bytes) of every sub-region once more, about
    assert 0.9 * 8 * counts.sum() < extra < 1.3 * 8 * counts.sum()
    C = counts.reshape(1, 256)
    pl = dist.RoundPlanner(21, 0, N.KMAN_FINISH_COUNT, 1, 3 * 10**9)
    R, cuts, a, b = pl.plan(C, 1 << 40)
    assert pl.roomy(C, cuts, R, 1 << 40, a, b) == (True, ab[N.KMAN_ROOMY][0], ab[0][1])
    assert pl.roomy(C, cuts, R, a + b, a, b) == (False, a, b)
    assert pl.flags == 0
    os.environ["KMAN_ROOMY"] = "0"
    try:
        assert pl.roomy(C, cuts, R, 1 << 40, a, b) == (False, a, b)
    finally:
        del os.environ["KMAN_ROOMY"]
    # config 4's rank shape on one MI355X: the plain plan
    nbase = 12_500_000_000
    G = 8
    C4 = np.full((G, 256), nbase // 256, dtype=np.uint64)
    budget = int(0.85 * 288 * 10**9) - nbase - 12 * (nbase + (1 << 20))
    pl4 = dist.RoundPlanner(21, 0, N.KMAN_FINISH_COUNT, G, nbase)
    R4, cuts4, a4, b4 = pl4.plan(C4, budget)
    assert pl4.roomy(C4, cuts4, R4, budget, a4, b4)[0] is False


@pytest.mark.parametrize("G,S", [(1, 4), (2, 4), (3, 2), (8, 4)])
def test_round_pieces_partition_each_part(G, S):
    """The overlapped rounds' pieces (dist.round_pieces): each destination's
    part cut into S contiguous, ordered bucket ranges that cover it exactly,
    the same on every rank, of about equal k-mers."""
    from kman_amd import dist

    rng = np.random.default_rng(G * 10 + S)
    C = rng.integers(0, 50_000, size=(G, 256)).astype(np.uint64)
    C[:, 17] += 2_000_000  # one heavy bucket
    pl = dist.RoundPlanner(21, 0, 1, G, 10**9)
    R, cuts, _, _ = pl.plan(C, 1 << 40)
    for r in range(R):
        bounds = dist.round_pieces(C, cuts, G, R, r, S)
        assert len(bounds) == G
        tot = C.sum(axis=0).astype(np.int64)
        for q in range(G):
            lo, hi = dist.part_of(cuts, R, q, r)
            b = bounds[q]
            assert len(b) == S + 1 and b[0] == lo and b[-1] == hi
            assert all(x <= y for x, y in zip(b, b[1:]))
            if hi - lo >= S and tot[lo:hi].sum():
                sizes = [tot[x:y].sum() for x, y in zip(b, b[1:])]
                # no piece above its share plus one bucket
                assert max(sizes) <= tot[lo:hi].sum() / S + tot[lo:hi].max()


def _redo_map_loops(ranges, K):
    """redo_map restated range by range (the vectorised version must agree)."""
    pbits = 1
    for rq in ranges:
        for lo, hi in rq:
            lo, end = int(lo), int(hi) + 1
            a = (lo & -lo).bit_length() - 1 if lo else K
            b = (end & -end).bit_length() - 1 if end < (1 << K) else K
            pbits = max(pbits, K - min(a, b))
    sh = K - pbits
    pmap = np.zeros(1 << pbits, np.uint8)
    for q, rq in enumerate(ranges):
        for lo, hi in rq:
            pmap[int(lo) >> sh:(int(hi) >> sh) + 1] = q + 1
    return pbits, pmap


@pytest.mark.parametrize("K", [16, 30, 42, 64])
def test_redo_map_matches_range_loops(K):
    from kman_amd import dist

    rng = np.random.default_rng(K)
    for _ in range(40):
        G = int(rng.integers(1, 6))
        pb = int(rng.integers(1, min(K, 20) + 1))
        cuts = np.sort(rng.choice(1 << pb, size=min(1 << pb, 2 * int(rng.integers(0, 60))), replace=False))
        ranges = [[] for _ in range(G)]
        for i in range(0, len(cuts) - 1, 2):
            a, b = int(cuts[i]), int(cuts[i + 1])
            ranges[int(rng.integers(0, G))].append([a << (K - pb), ((b + 1) << (K - pb)) - 1])
        ranges = [np.array(r, np.uint64).reshape(-1, 2) for r in ranges]
        got, want = dist.redo_map(ranges, K), _redo_map_loops(ranges, K)
        assert got[0] == want[0]
        np.testing.assert_array_equal(got[1], want[1])
