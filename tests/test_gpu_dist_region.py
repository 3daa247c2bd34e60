"""GPU parity of the multi-GPU path over byte-range shards of ONE FASTA
(kman_amd/shard.py, kman_amd/dist.py, kman_dshard_* / kman_dround_finish)
with G simulated ranks in ONE process on one GPU (dist.SimGroup: one engine
context per rank, host-side all-reduce / all-gather, device-to-device
all-to-all).  The real run executes the same step generators with RCCL.

Bar: the ranks' outputs concatenated in rank order are bit-exact against the
numpy restatement over the whole file (np_oracle: parse -> stream_kmers ->
stable sort -> run-length count / uniq, parsers.py:86-128, seq.py:285-328,
batch.py:156-168, join.py:95-130,244-285); the emitted output file is
byte-identical to the C oracle's `kmer count|uniq` output of the file."""

from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _texts():
    import inputs

    lay = inputs.SynthLayout(400_000, 21, record_len=90_000, width=70)
    return {"synth": lay.read(0, lay.size), "messy": inputs.messy_records(31, n_records=60, max_len=12_000)}


def _oracle(text, k, mode, canonical=False):
    import np_oracle

    keys, pos = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k, canonical=canonical)
    sk, sp = np_oracle.stable_sort(keys, pos)
    return np_oracle.rle_count(sk) if mode == "count" else np_oracle.rle_uniq(sk, sp)


def _run(text, k, mode, G, **kw):
    """G simulated ranks over one text, stepped twice (the resident buffers
    are reused); returns the rank-ordered outputs of both steps (uniq pos
    rebased to global base indices), the pipelines and the group."""
    from kman_amd import dist, engine, shard

    devs = [engine.Device(0) for _ in range(G)]
    pipes = []
    try:
        rd = shard.BytesReader(text)
        for r in range(G):
            pipes.append(dist.DistPipeline(devs[r], rd, k, mode, G, r, None, **kw))
            pipes[-1]._dev_owned = devs[r]
        grp = dist.SimGroup(pipes)
        outs = []
        for _ in range(2):
            grp.step()
            keys = np.concatenate([p.results()[0] for p in pipes])
            vals = np.concatenate([p.results()[1] for p in pipes])
            if mode == "uniq":  # source-tagged pos -> global pos
                src = (vals >> np.uint64(56)).astype(np.int64)
                vals = (vals & np.uint64((1 << 56) - 1)) + (pipes[0].base_off[src] << np.uint64(1))
            outs.append((keys, vals))
        return outs, pipes, grp
    except BaseException:
        for p in pipes:
            p.free()
        for d in devs:
            d.close()
        raise


def _close(pipes):
    for p in pipes:
        p.free()
        p._dev_owned.close()


@pytest.mark.parametrize("G", [1, 2, 3, 8])
@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("k", [15, 21])
@pytest.mark.parametrize("name", ["synth", "messy"])
def test_dist_shards_match_oracle(G, mode, k, name):
    text = _texts()[name]
    outs, pipes, _ = _run(text, k, mode, G)
    try:
        assert all(p.path == "region" for p in pipes)
        assert all(p.fallback_rounds == 0 for p in pipes)
        wk, wv = _oracle(text, k, mode)
        for keys, vals in outs:
            np.testing.assert_array_equal(keys, wk)
            np.testing.assert_array_equal(vals, wv)
    finally:
        _close(pipes)


# the finish kernels a round can run: the product uniq finish (early count
# unchecked, KMAN_RG_CHECK=0: what bench.py and the CLI run) and the checked
# one the GPU session defaults to
FINISH_VARIANTS = {"plain": {"KMAN_RG_CHECK": "0"}, "checked": {"KMAN_RG_CHECK": "1"}}


@pytest.mark.parametrize("variant", sorted(FINISH_VARIANTS))
@pytest.mark.parametrize("G", [1, 3])
@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("name", ["synth", "messy"])
def test_dist_finish_variants(monkeypatch, variant, G, mode, name):
    for k_, v_ in FINISH_VARIANTS[variant].items():
        monkeypatch.setenv(k_, v_)
    text = _texts()[name]
    outs, pipes, _ = _run(text, 21, mode, G)
    try:
        wk, wv = _oracle(text, 21, mode)
        for keys, vals in outs:
            np.testing.assert_array_equal(keys, wk)
            np.testing.assert_array_equal(vals, wv)
    finally:
        _close(pipes)


@pytest.mark.parametrize("variant", ["plain", "checked"])
@pytest.mark.parametrize("G,once", [(1, "1"), (1, "0"), (2, "1"), (8, "1")])
@pytest.mark.parametrize("mode", ["count", "uniq"])
def test_dist_streamed_rounds(monkeypatch, variant, G, once, mode):
    """R >= 3 key rounds forced by a small per-round budget: each rank's
    rounds append its key range in order.  One rank (no exchange) extracts
    the shard once for every round into its output-key buffer (KMAN_DIST_ONCE,
    the default), or round by round (0)."""
    for k_, v_ in FINISH_VARIANTS[variant].items():
        monkeypatch.setenv(k_, v_)
    monkeypatch.setenv("KMAN_DIST_ONCE", once)
    text = _texts()["synth"]
    outs, pipes, _ = _run(text, 21, mode, G, max_round_items=120_000 // G)
    try:
        assert all(p.rounds >= 3 for p in pipes) and len({p.rounds for p in pipes}) == 1
        wk, wv = _oracle(text, 21, mode)
        for keys, vals in outs:
            np.testing.assert_array_equal(keys, wk)
            np.testing.assert_array_equal(vals, wv)
    finally:
        _close(pipes)


@pytest.mark.parametrize("G", [2, 8])
@pytest.mark.parametrize("mode", ["count", "uniq"])
def test_dist_overlapped_streamed_rounds(G, mode):
    """Overlapped rounds at R >= 3 (config 4 plans R = 3 at 12.5 G k-mers per
    rank): every round's exchange in pieces, each piece's passes + finish
    after its own exchange; rows bit-exact against the oracle."""
    text = _texts()["synth"]
    outs, pipes, _ = _run(text, 21, mode, G, max_round_items=120_000 // G, overlap=True)
    try:
        assert all(p.rounds >= 3 and p.overlapped_rounds == p.rounds for p in pipes)
        wk, wv = _oracle(text, 21, mode)
        for keys, vals in outs:
            np.testing.assert_array_equal(keys, wk)
            np.testing.assert_array_equal(vals, wv)
    finally:
        _close(pipes)


def test_dist_wide_pass1b(monkeypatch):
    """Pass 1b with 7 bits (the width config 4's 390 M-item buckets take)."""
    monkeypatch.setenv("KMAN_DROUND_MIN_G", "7")
    text = _texts()["synth"]
    for mode in ("count", "uniq"):
        outs, pipes, _ = _run(text, 21, mode, 3)
        try:
            wk, wv = _oracle(text, 21, mode)
            np.testing.assert_array_equal(outs[0][0], wk)
            np.testing.assert_array_equal(outs[0][1], wv)
        finally:
            _close(pipes)


@pytest.mark.parametrize("G", [1, 8])
def test_dist_canonical_count_and_hist(G):
    """Config 5 across ranks: canonical counts + the all-reduced abundance
    spectrum equal the single-GPU path and the oracle (canonical counts =
    the `count -r` rows with key <= rc(key) for odd k, seq.py:274-282)."""
    import inputs
    from kman_amd import engine

    text = inputs.grch38_like(5, n_bases=300_000)
    outs, pipes, grp = _run(text, 21, "count", G, canonical=True)
    try:
        wk, wc = _oracle(text, 21, "count", canonical=True)
        np.testing.assert_array_equal(outs[-1][0], wk)
        np.testing.assert_array_equal(outs[-1][1], wc)
        hs = grp.run(lambda p: p.hist_gen(1001))
        want = np.bincount(np.minimum(wc.astype(np.int64), 1000), minlength=1001).astype(np.uint64)
        want[0] = 0
        for h in hs:
            np.testing.assert_array_equal(h, want)
        single = engine.abundance_hist(text, 21, canonical=True, nbins=1001, dev=pipes[0].dev)
        np.testing.assert_array_equal(hs[0], single)
    finally:
        _close(pipes)


@pytest.mark.parametrize("G", [1, 2, 3])
@pytest.mark.parametrize("heavy", ["0", "1"], ids=["table-off", "table-on"])
def test_dist_region_overflow_redoes_only_its_keys(G, heavy, monkeypatch):
    """A key repeated far more often than a region holds: its regions emit
    nothing (kman_dround_finish -> KMAN_EPARTIAL, kman_dround_failed) and only
    their key ranges go through the general path on every rank, merged into
    the region rows; results stay exact.  With the heavy-key table on
    (KMAN_HEAVY=1) the repeat's keys are counted apart in pass 1 instead and
    nothing overflows."""
    import inputs

    monkeypatch.setenv("KMAN_HEAVY", heavy)
    rep = b"ACGTTGCAAGGCTTACGATCGATCGGATCC"
    body = inputs.SynthLayout(200_000, 4, record_len=50_000).read(0, 10**9)
    text = body + b">rep\n" + b"\n".join([rep * 2] * 30_000) + b"\n"
    for mode in ("count", "uniq"):
        outs, pipes, _ = _run(text, 21, mode, G)
        try:
            assert all(p.fallback_rounds == 0 for p in pipes)
            redone, total = sum(p.redone_kmers for p in pipes), sum(p.n_kmers for p in pipes)
            if heavy == "1":
                assert sum(p.heavy_keys for p in pipes) > 0
                assert redone < total - 150_000
            else:
                assert sum(p.partial_rounds for p in pipes) >= 1
                # only the left-out ranges were redone: the repeat's 1.8 M
                # k-mers, not the 0.2 M of the random body
                assert 0 < redone < total - 150_000
            wk, wv = _oracle(text, 21, mode)
            for o in outs:
                np.testing.assert_array_equal(o[0], wk)
                np.testing.assert_array_equal(o[1], wv)
        finally:
            _close(pipes)


@pytest.mark.parametrize("G", [1, 3])
def test_dist_overflow_redo_canonical_and_rc(G, monkeypatch):
    """The partial redo with canonical keys (config 5's count) and with -r
    uniq: left-out ranges of min(fwd, rc) keys, and of both strands."""
    monkeypatch.setenv("KMAN_HEAVY", "0")  # (the partial redo itself; tables: test_dist_heavy_keys_counted_apart)
    import inputs

    rep = b"TTGACCATGACCGATTACAGATTGGC"
    body = inputs.SynthLayout(150_000, 6, record_len=40_000).read(0, 10**9)
    text = body + b">sat\n" + b"\n".join([rep * 3] * 20_000) + b"\n"
    outs, pipes, _ = _run(text, 21, "count", G, canonical=True)
    try:
        assert sum(p.partial_rounds for p in pipes) >= 1
        wk, wc = _oracle(text, 21, "count", canonical=True)
        for o in outs:
            np.testing.assert_array_equal(o[0], wk)
            np.testing.assert_array_equal(o[1], wc)
    finally:
        _close(pipes)


@pytest.mark.parametrize("G", [1, 3])
def test_dist_unordered_redo_spectrum(G, monkeypatch):
    """ordered=False (the abundance spectrum, config 5): a redone key range is
    appended after the region rows, not merged -- the rows are the oracle's
    as a multiset and the all-reduced spectrum is exact."""
    monkeypatch.setenv("KMAN_HEAVY", "0")  # (the partial redo itself; tables: test_dist_heavy_keys_counted_apart)
    import inputs
    from kman_amd import dist, engine

    rep = b"TTGACCATGACCGATTACAGATTGGC"
    body = inputs.SynthLayout(150_000, 6, record_len=40_000).read(0, 10**9)
    text = body + b">sat\n" + b"\n".join([rep * 3] * 20_000) + b"\n"
    import np_oracle

    outs, pipes, grp = _run(text, 21, "count", G, canonical=True, ordered=False)
    try:
        assert sum(p.partial_rounds for p in pipes) >= 1
        wk, wc = _oracle(text, 21, "count", canonical=True)
        # (rows as a multiset: canonical keys through KMAN_MIXED's bijection)
        mk = np.sort(np_oracle.mix_keys(wk, 21))
        mc = wc[np.argsort(np_oracle.mix_keys(wk, 21), kind="stable")]
        for keys, counts in outs:
            o = np.argsort(keys, kind="stable")
            np.testing.assert_array_equal(keys[o], mk)
            np.testing.assert_array_equal(counts[o], mc)
        hs = grp.run(lambda p: p.hist_gen(1001))
        want = np.bincount(np.minimum(wc.astype(np.int64), 1000), minlength=1001).astype(np.uint64)
        want[0] = 0
        for h in hs:
            np.testing.assert_array_equal(h, want)
    finally:
        _close(pipes)
    # one GPU through the key rounds (engine.abundance_hist's path for inputs
    # kman_groups does not take), ordered and not
    dev = engine.default_device()
    p = engine.parse(dev, text)
    try:
        for ordered in (True, False):
            r = dist.local_groups(p, 21, False, "count", True, max_round_items=200_000, ordered=ordered)
            try:
                keys = dev.download(r.ukeys, r.n, np.uint64)
                counts = dev.download(r.counts, r.n, np.uint32 if r.count_bytes == 4 else np.uint64)
            finally:
                r.ukeys.free()
                r.counts.free()
            if ordered:
                np.testing.assert_array_equal(keys, wk)
            o = np.argsort(keys, kind="stable")
            np.testing.assert_array_equal(keys[o], wk if ordered else mk)
            np.testing.assert_array_equal(counts[o].astype(np.uint64), (wc if ordered else mc).astype(np.uint64))
            assert dist.LAST_LOCAL["partial_rounds"] >= 1
    finally:
        p.free()


def test_dist_general_path_k27():
    """k = 27: count items still fit the region rounds; uniq (window index +
    key > 64 bits) and a forced path="general" take the general path (key
    ranges, exchanged keys + pos)."""
    text = _texts()["messy"]
    for mode, kw, want in (("count", {}, "region"), ("uniq", {}, "general"), ("count", {"path": "general"}, "general")):
        outs, pipes, _ = _run(text, 27, mode, 3, **kw)
        try:
            assert all(p.path == want for p in pipes)
            wk, wv = _oracle(text, 27, mode)
            np.testing.assert_array_equal(outs[0][0], wk)
            np.testing.assert_array_equal(outs[0][1], wv)
        finally:
            _close(pipes)


@pytest.mark.parametrize("mode", ["count", "uniq"])
def test_dist_emit_matches_reference_bytes(mode, tmp_path, oracle_bin):
    """The global output file written by the ranks at their offsets is the
    reference's `kmer count|uniq` output of the whole file (C oracle, pinned
    to the reference's own outputs in tests/golden)."""
    text = _texts()["messy"]
    src = tmp_path / "in.fa"
    src.write_bytes(text)
    want = tmp_path / "want.txt"
    subprocess.run([oracle_bin, mode, str(src), str(want), "13"], check=True)
    outs, pipes, grp = _run(text, 13, mode, 3)
    try:
        got = tmp_path / "got.txt"
        grp.run(lambda p: p.emit_gen(str(got)))
        assert got.read_bytes() == want.read_bytes()
    finally:
        _close(pipes)


@pytest.mark.parametrize("chunk", [1000, 4096, 1 << 20])
def test_chunked_loader_equals_parse(chunk):
    from kman_amd import engine, shard

    dev = engine.default_device()
    for text in _texts().values():
        a = engine.parse(dev, text)
        b = shard.load_text(dev, text, chunk)
        try:
            assert a.n_bases == b.n_bases and a.names == b.names
            np.testing.assert_array_equal(a.rec_seq, b.rec_seq)
            ca = dev.download(a.codes, a.n_bases + 64, np.uint8)
            cb = dev.download(b.codes, b.n_bases + 64, np.uint8)
            np.testing.assert_array_equal(ca, cb)
        finally:
            a.free()
            b.free()


def test_pinned_chunked_loader(tmp_path):
    """Async chunk copies from pinned memory (the pinned-host bench line)."""
    from kman_amd import engine, shard

    dev = engine.default_device()
    text = _texts()["synth"]
    rd = shard.PinnedReader(dev, text)
    try:
        sp = shard.shard_specs(rd, 1, 21)[0]
        ld = shard.ShardLoader(dev, rd, sp, 21, chunk_bytes=50_000)
        try:
            for _ in range(2):
                sh = ld.load()
                a = engine.parse(dev, text)
                try:
                    np.testing.assert_array_equal(dev.download(sh.codes, sh.n_own, np.uint8),
                                                  dev.download(a.codes, a.n_bases, np.uint8))
                finally:
                    a.free()
        finally:
            ld.free()
    finally:
        rd.free()


def test_synth_device_matches_numpy():
    import inputs
    from kman_amd import engine, shard

    dev = engine.default_device()
    lay = inputs.SynthLayout(300_000, 77, record_len=100_003, width=80)
    rd = shard.SynthReader(lay)
    buf = dev.alloc(lay.size + 64)
    try:
        for lo, hi in ((0, lay.size), (5, 1000), (100_000, 200_017), (lay.size - 33, lay.size)):
            rd.gen(dev, buf, lo, hi)
            assert dev.download(buf, hi - lo, np.uint8).tobytes() == lay.read(lo, hi)
    finally:
        buf.free()


@pytest.mark.parametrize("mode,k", [("count", 21), ("uniq", 13), ("count", 31)])
def test_streamed_overlap_matches_oracle(mode, k):
    """kman_groups_begin / _extract (one call per parsed chunk, behind the
    next chunk's copy) / _end give kman_groups' rows (StreamedPipeline with
    and without the overlap), bit-exact against np_oracle; stepped twice."""
    import inputs

    from kman_amd import engine, shard

    dev = engine.default_device()
    text = inputs.syn_numpy(3_000_000, 11, record_len=700_000, width=61) + _texts()["messy"]
    want = _oracle(text, k, mode)
    rd = shard.PinnedReader(dev, text)
    try:
        for ov in (True, False):
            sp = shard.StreamedPipeline(dev, rd, k, mode, chunk_bytes=333_333, overlap=ov)
            try:
                for _ in range(2):
                    sp.step()
                    keys = dev.download(sp.out_keys, sp.n_out, np.uint64)
                    vals = dev.download(sp.out_vals, sp.n_out, np.uint32).astype(np.uint64)
                    np.testing.assert_array_equal(keys, want[0])
                    np.testing.assert_array_equal(vals, want[1].astype(np.uint64))
            finally:
                sp.free()
    finally:
        rd.free()


def test_groups_extract_needs_begin():
    """kman_groups_extract without its kman_groups_begin (or after another
    look-back call) is refused, not run against stale status words."""
    from ctypes import byref, c_uint32, c_uint64, c_void_p

    from kman_amd import _native as N
    from kman_amd import engine

    dev = engine.default_device()
    L = N.lib()
    n, k, flags, m = 1 << 20, 21, 0, N.KMAN_FINISH_COUNT
    wb = c_uint64(0)
    N.check(dev.ctx, L.kman_groups_plan(n, k, flags, m, byref(wb)), "plan")
    work, codes = dev.alloc(int(wb.value)), dev.alloc(n + 128)
    ok, ov = dev.alloc(8 * n), dev.alloc(4 * n)
    try:
        rng = np.random.default_rng(5)
        dev.upload(codes, np.concatenate([rng.integers(0, 4, n, dtype=np.uint8), np.full(128, 4, np.uint8)]))
        args = (n, k, flags, m, c_void_p(work.ptr), wb.value)
        nt, tb = c_uint32(0), c_uint64(0)
        N.check(dev.ctx, L.kman_groups_begin(dev.ctx, *args, byref(nt), byref(tb)), "begin")
        assert nt.value > 1 and tb.value > 0
        N.check(dev.ctx, L.kman_groups_extract(dev.ctx, c_void_p(codes.ptr), *args, 1), "extract")
        nk, no = c_uint64(), c_uint64()
        N.check(dev.ctx, L.kman_groups_end(dev.ctx, c_void_p(codes.ptr), *args, c_void_p(ok.ptr), c_void_p(ov.ptr), 4,
                                           byref(nk), byref(no)), "end")
        assert nk.value == n - k + 1
        # the pass is closed: a further extract has no begin
        assert L.kman_groups_extract(dev.ctx, c_void_p(codes.ptr), *args, 2) == N.KMAN_EINVAL
    finally:
        for b in (work, codes, ok, ov):
            b.free()


@pytest.mark.parametrize("G", [1, 3, 8])
def test_dist_grch38_skewed_canonical(G):
    """Config 5 on a genome-skewed input (inputs.grch38_skewed: a ~10 %
    diverged Alu-like family every ~3 kb, a tandem satellite array, poly-A
    runs, N gaps, soft-masking): canonical counts across G ranks equal the
    oracle's, and the spectrum (rows as a multiset, mixed keys) is exact --
    the overflowing repeat regions go through the partial redo."""
    import inputs
    import np_oracle

    text = inputs.grch38_skewed(5, n_bases=3_000_000, n_records=3)
    wk, wc = _oracle(text, 21, "count", canonical=True)
    outs, pipes, _ = _run(text, 21, "count", G, canonical=True)
    try:
        for keys, counts in outs:
            np.testing.assert_array_equal(keys, wk)
            np.testing.assert_array_equal(counts, wc)
    finally:
        _close(pipes)
    outs, pipes, grp = _run(text, 21, "count", G, canonical=True, ordered=False)
    try:
        mk = np_oracle.mix_keys(wk, 21)
        o = np.argsort(mk, kind="stable")
        for keys, counts in outs:
            q = np.argsort(keys, kind="stable")
            np.testing.assert_array_equal(keys[q], mk[o])
            np.testing.assert_array_equal(counts[q], wc[o])
        hs = grp.run(lambda p: p.hist_gen(10001))
        want = np.bincount(np.minimum(wc.astype(np.int64), 10000), minlength=10001).astype(np.uint64)
        want[0] = 0
        for h in hs:
            np.testing.assert_array_equal(h, want)
    finally:
        _close(pipes)


@pytest.mark.parametrize("G", [1, 2, 3])
@pytest.mark.parametrize("mode,canonical", [("count", False), ("uniq", False), ("count", True)],
                         ids=["count", "uniq", "canon"])
def test_dist_heavy_keys_counted_apart(G, mode, canonical, monkeypatch):
    """Heavy keys (kman_dround_heavy): a round's sampled-twice keys are
    counted apart in pass 1 -- count mode keeps one copy per chain and adds
    the dropped ones to the row after the finish, uniq mode drops them all.
    On a repeat-rich input (inputs.grch38_like: a few 300-bp elements copied
    every 2.5 kb, a satellite array) with the table forced on (KMAN_HEAVY=1,
    any round size) and also split into 3 rounds, the rows equal the oracle's
    and equal the rows with the table off (KMAN_HEAVY=0); with it on, fewer
    k-mers go through the partial redo."""
    import inputs

    text = inputs.grch38_like(11, n_bases=2_000_000, n_records=2)
    wk, wv = _oracle(text, 21, mode, canonical=canonical)
    redone = {}
    for hv in ("1", "0"):
        monkeypatch.setenv("KMAN_HEAVY", hv)
        for mri in (None, 250_000):
            kw = {"canonical": canonical} if canonical else {}
            if mri:
                kw["max_round_items"] = mri
            outs, pipes, _ = _run(text, 21, mode, G, **kw)
            try:
                for keys, vals in outs:
                    np.testing.assert_array_equal(keys, wk)
                    np.testing.assert_array_equal(vals, wv)
                heavy = sum(p.heavy_keys for p in pipes)
                if hv == "1":
                    assert heavy > 0, "no heavy key sampled on a repeat-rich input"
                else:
                    assert heavy == 0
                if mri:
                    assert max(p.rounds for p in pipes) >= 2
                redone[hv, mri] = sum(p.redone_kmers for p in pipes)
            finally:
                _close(pipes)
    assert redone["1", None] <= redone["0", None]


@pytest.mark.parametrize("k,mode,rc", [(15, "count", False), (27, "count", False), (31, "count", False),
                                        (21, "count", True), (21, "uniq", True), (25, "uniq", False)])
def test_dist_heavy_keys_other_k_and_strands(k, mode, rc, monkeypatch):
    """The heavy-key table at other widths of the key rest (k 15 .. 31: 4- and
    8-byte pass-1 items, tables of longer rests) and with both strands (-r),
    forced on, with every 5th region left out and redone from pass 1's
    output, across 3 simulated ranks in 2+ rounds: the rows equal the
    oracle's."""
    import inputs
    import np_oracle

    monkeypatch.setenv("KMAN_HEAVY", "1")
    monkeypatch.setenv("KMAN_TEST_LEAVE_OUT", "5")
    monkeypatch.setenv("KMAN_DROUND_MIN_G", "1")
    text = inputs.grch38_like(17, n_bases=800_000, n_records=2)
    keys, pos = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k, rc=rc)
    sk, sp = np_oracle.stable_sort(keys, pos)
    wk, wv = np_oracle.rle_count(sk) if mode == "count" else np_oracle.rle_uniq(sk, sp)
    kw = {"rc": rc, "max_round_items": 300_000 if not rc else 600_000}
    outs, pipes, _ = _run(text, k, mode, 3, **kw)
    try:
        if mode == "count":
            assert sum(p.heavy_keys for p in pipes) > 0
        for kk, vv in outs:
            np.testing.assert_array_equal(kk, wk)
            np.testing.assert_array_equal(vv, wv)
    finally:
        _close(pipes)


def test_dist_heavy_keys_eight_ranks_canonical(monkeypatch):
    """Config 5's shape across 8 simulated ranks: canonical counts of the
    repeat-rich input with the heavy-key table forced on; each rank samples
    the items it received, so the tables differ by rank -- the rows equal
    the oracle's, in key order and as the mixed multiset, and the
    all-reduced spectrum is exact."""
    import inputs
    import np_oracle

    monkeypatch.setenv("KMAN_HEAVY", "1")
    text = inputs.grch38_like(13, n_bases=2_000_000, n_records=3)
    wk, wc = _oracle(text, 21, "count", canonical=True)
    outs, pipes, _ = _run(text, 21, "count", 8, canonical=True)
    try:
        assert sum(p.heavy_keys for p in pipes) > 0
        for keys, counts in outs:
            np.testing.assert_array_equal(keys, wk)
            np.testing.assert_array_equal(counts, wc)
    finally:
        _close(pipes)
    outs, pipes, grp = _run(text, 21, "count", 8, canonical=True, ordered=False)
    try:
        mk = np_oracle.mix_keys(wk, 21)
        o = np.argsort(mk, kind="stable")
        for keys, counts in outs:
            q = np.argsort(keys, kind="stable")
            np.testing.assert_array_equal(keys[q], mk[o])
            np.testing.assert_array_equal(counts[q], wc[o])
        hs = grp.run(lambda p: p.hist_gen(1001))
        want = np.bincount(np.minimum(wc.astype(np.int64), 1000), minlength=1001).astype(np.uint64)
        want[0] = 0
        for h in hs:
            np.testing.assert_array_equal(h, want)
    finally:
        _close(pipes)


@pytest.mark.parametrize("G", [1, 2, 3])
@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("ordered", [True, False], ids=["ordered", "multiset"])
def test_dist_left_out_regions_redone_locally(G, mode, ordered, monkeypatch):
    """kman_dround_left: the regions a round's finish left out are redone
    from its pass-1 output (no re-extraction from the codes, no exchange),
    the heavy keys' dropped copies added back (kman_dround_heavy_fix).  Every
    7th region is left out (KMAN_TEST_LEAVE_OUT, as if it had overflowed) on
    the repeat-rich grch38_like input, with the heavy-key table on and off and
    in 1 or 3 rounds: the rows equal the oracle's (as a multiset when
    unordered) and equal those of the marked-extraction redo
    (KMAN_LOCAL_REDO=0)."""
    import inputs

    text = inputs.grch38_like(12, n_bases=1_500_000, n_records=2)
    wk, wv = _oracle(text, 21, mode)
    monkeypatch.setenv("KMAN_TEST_LEAVE_OUT", "7")
    monkeypatch.setenv("KMAN_DROUND_MIN_G", "1")  # (the leave-out hook acts on pass 1b's regions)
    for hv in ("1", "0"):
        monkeypatch.setenv("KMAN_HEAVY", hv)
        for mri in (None, 250_000):
            for loc in ("1", "0"):
                monkeypatch.setenv("KMAN_LOCAL_REDO", loc)
                kw = {"ordered": ordered}
                if mri:
                    kw["max_round_items"] = mri
                outs, pipes, _ = _run(text, 21, mode, G, **kw)
                try:
                    for keys, vals in outs:
                        if not ordered:
                            q = np.lexsort((vals, keys))
                            keys, vals = keys[q], vals[q]
                        np.testing.assert_array_equal(keys, wk)
                        np.testing.assert_array_equal(vals, wv)
                    assert sum(p.partial_rounds for p in pipes) > 0
                    local = sum(p.local_redo_kmers for p in pipes)
                    assert (local > 0) == (loc == "1"), (local, loc)
                    if hv == "1":
                        assert sum(p.heavy_keys for p in pipes) > 0
                finally:
                    _close(pipes)
