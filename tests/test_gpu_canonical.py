"""GPU parity of canonical k-mers and the abundance spectrum (BASELINE config
5; neither is in the reference).

Pinning: the reference's own `kmer count -r` outputs (tests/golden/ref_outputs,
produced by the reference) give canonical counts for odd k: -r emits both
strands (seq.py:274-282), so count(x) = occ(x) + occ(rc x), and the rows with
x <= rc(x) are exactly the canonical count table.  Everything else is checked
bit-exact against np_oracle (stream_kmers(canonical=True) -> sort -> RLE)."""

from __future__ import annotations

import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

_RC = bytes.maketrans(b"ACGT", b"TGCA")


@pytest.fixture(scope="module")
def dev():
    from kman_amd import engine

    return engine.default_device()


def _ref_cases():
    import json

    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        cases = json.load(fh)["cases"]
    return [c for c in cases if c["cmd"] == "count" and "-r" in c["flags"] and c["k"] % 2 == 1
            and os.path.isfile(os.path.join(GOLDEN, "ref_outputs", c["name"] + ".txt"))]


@pytest.mark.parametrize("case", _ref_cases(), ids=lambda c: c["name"])
def test_canonical_counts_pinned_by_reference_rc_counts(dev, golden_inputs, case):
    from kman_amd import engine

    with open(os.path.join(GOLDEN, "ref_outputs", case["name"] + ".txt"), "rb") as fh:
        ref = fh.read()
    want = b"".join(line + b"\n" for line in ref.splitlines()
                    if line.split(b"\t")[0] <= line.split(b"\t")[0][::-1].translate(_RC))
    p = engine.parse(dev, engine.read_input(golden_inputs[case["input"]]))
    try:
        r = engine.count_groups(p, case["k"], canonical=True)
        if r is None:
            got = b""
        elif isinstance(r, engine.WordsResult):  # (k > 32: word keys)
            got = bytes(engine._emit_words(p, r))
            engine.free_result(r)
        else:
            got = engine.format_count(*engine.download_count(dev, r), case["k"])
    finally:
        p.free()
    assert got == want


def _texts():
    import inputs

    return [inputs.messy_records(21, n_records=50, max_len=20000), inputs.syn_numpy(2_000_000, 8, record_len=300_000),
            b">r\n" + (b"ACGTTGCAAC" * 3000) + b"\n>s\n" + inputs.syn_numpy(200_000, 9).split(b"\n", 1)[1]]


@pytest.mark.parametrize("k", [15, 21, 25, 31])
@pytest.mark.parametrize("mode", ["count", "uniq"])
def test_canonical_groups_match_oracle(dev, k, mode):
    import np_oracle
    from kman_amd import engine

    for text in _texts():
        keys, pos = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k, canonical=True)
        sk, sp = np_oracle.stable_sort(keys, pos)
        want = np_oracle.rle_count(sk) if mode == "count" else np_oracle.rle_uniq(sk, sp)
        p = engine.parse(dev, text)
        try:
            if mode == "count":
                r = engine.count_groups(p, k, canonical=True)
                got = engine.download_count(dev, r)
                r.ukeys.free()
                r.counts.free()
            else:
                r = engine.groups(p, k, False, "uniq", canonical=True)
                if r is None:  # k = 31: the prefix-split path
                    km = engine.extract_sorted(p, k, False, want_pos=True, canonical=True)
                    r = engine.rle_uniq(km, dev)
                    km.free()
                got = engine.download_uniq(dev, r)
                r.keys.free()
                r.pos.free()
        finally:
            p.free()
        np.testing.assert_array_equal(got[0], want[0])
        np.testing.assert_array_equal(got[1].astype(np.uint64), want[1])


@pytest.mark.parametrize("canonical", [True, False])
@pytest.mark.parametrize("nbins", [3, 50, 10001])
def test_abundance_hist_matches_oracle(dev, canonical, nbins):
    import np_oracle
    from kman_amd import engine

    text = _texts()[2]
    keys, _ = np_oracle.stream_kmers(np_oracle.parse_fasta(text), 21, canonical=canonical)
    _, counts = np_oracle.rle_count(np.sort(keys))
    want = np.bincount(np.minimum(counts, nbins - 1).astype(np.int64), minlength=nbins).astype(np.uint64)
    got = engine.abundance_hist(text, 21, canonical=canonical, nbins=nbins, dev=dev)
    np.testing.assert_array_equal(got, want)
    lines = engine.format_hist(got).decode().splitlines()
    assert sum(int(x.split("\t")[1]) for x in lines) == len(counts)


def test_hist_cli(tmp_path):
    import subprocess
    import sys

    import np_oracle

    text = _texts()[0]
    src, out = tmp_path / "in.fa", tmp_path / "h.txt"
    src.write_bytes(text)
    root = os.path.dirname(GOLDEN.rstrip("/").rsplit("/", 1)[0])
    subprocess.run([sys.executable, "-m", "kman_amd", "hist", str(src), str(out), "21"], check=True,
                   cwd=os.path.dirname(os.path.dirname(GOLDEN)))
    keys, _ = np_oracle.stream_kmers(np_oracle.parse_fasta(text), 21, canonical=True)
    _, counts = np_oracle.rle_count(np.sort(keys))
    h = np.bincount(counts.astype(np.int64))
    want = "".join("%d\t%d\n" % (c, h[c]) for c in np.nonzero(h)[0])
    assert out.read_text() == want
    del root


@pytest.mark.parametrize("k", [15, 21, 31])
def test_mixed_canonical_spectrum_keys(dev, k):
    """ordered=False (a spectrum) counts canonical keys through KMAN_MIXED's
    bijection: the rows are exactly {mix(x): occ(x)} over the oracle's
    canonical keys -- the same counts, so the same spectrum -- including the
    repeat-heavy input whose regions overflow and are redone."""
    import np_oracle
    from kman_amd import engine

    for text in _texts():
        keys, _ = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k, canonical=True)
        wk, wc = np.unique(np_oracle.mix_keys(keys, k), return_counts=True)
        p = engine.parse(dev, text)
        try:
            r = engine.count_groups(p, k, canonical=True, ordered=False)
            gk, gc = engine.download_count(dev, r)
            r.ukeys.free()
            r.counts.free()
        finally:
            p.free()
        o = np.argsort(gk, kind="stable")
        np.testing.assert_array_equal(gk[o], wk)
        np.testing.assert_array_equal(np.asarray(gc)[o].astype(np.int64), wc)
