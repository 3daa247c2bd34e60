"""The drop-in surface on the GPU: the ``kmer`` CLI and the FastaBatcher /
Batch / Crawler / KJoiner API produce the reference's bytes (golden sha256 /
batch-file contents from tests/golden/manifest.json)."""

from __future__ import annotations

import gzip
import hashlib
import json
import os

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)


def _cli(argv):
    from kman_amd.scripts.kmer import main

    main(argv, standalone_mode=False)


def _sha(path):
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


@pytest.mark.parametrize("case", [c for c in _manifest()["cases"] ], ids=lambda c: c["name"])
def test_cli_matches_reference(case, golden_inputs, tmp_path):
    out = str(tmp_path / "out.txt")
    _cli([case["cmd"], golden_inputs[case["input"]], out, str(case["k"])] + case["flags"])
    assert _sha(out) == case["sha256"]


@pytest.mark.parametrize("case", _manifest()["batch_cases"], ids=lambda c: c["name"])
def test_cli_batch_files_match_reference(case, golden_inputs, tmp_path):
    outdir = str(tmp_path / "batches")
    _cli(["batch", golden_inputs[case["input"]], outdir, str(case["k"])] + case["flags"])
    got = []
    for fn in sorted(os.listdir(outdir)):
        with open(os.path.join(outdir, fn)) as fh:
            got.append(fh.read())
    assert sorted(got) == case["files"]


def test_cli_batch_compressed(golden_inputs, tmp_path):
    case = _manifest()["batch_cases"][0]
    outdir = str(tmp_path / "b")
    _cli(["batch", golden_inputs[case["input"]], outdir, str(case["k"]), "-C"] + case["flags"])
    got = []
    for fn in os.listdir(outdir):
        assert fn.endswith(".fa.gz")
        with gzip.open(os.path.join(outdir, fn), "rt") as fh:
            got.append(fh.read())
    assert sorted(got) == case["files"]


@pytest.mark.parametrize("cmd", ["count", "uniq"])
def test_previous_batches_roundtrip(cmd, golden_inputs, tmp_path):
    """-B: batches written by `kmer batch`, loaded back, joined == joining the
    FASTA directly (the reference's loader is broken, §A-5: evident intent)."""
    case = [c for c in _manifest()["cases"] if c["name"] == "messy2__%s__k21__r" % cmd][0]
    outdir = str(tmp_path / "batches")
    _cli(["batch", golden_inputs["messy2"], outdir, "21", "-r", "-b", "777"])
    out = str(tmp_path / "out.txt")
    _cli([cmd, golden_inputs["messy2"], out, "21", "-B", outdir])
    assert _sha(out) == case["sha256"]


@pytest.mark.parametrize("cmd", ["count", "uniq"])
def test_records_scan_mode_same_output(cmd, golden_inputs, tmp_path):
    case = [c for c in _manifest()["cases"] if c["name"] == "messy1__%s__k5__r" % cmd][0]
    out = str(tmp_path / "out.txt")
    _cli([cmd, golden_inputs["messy1"], out, "5", "-r", "-s", "RECORDS", "-b", "50"])
    assert _sha(out) == case["sha256"]


def test_cli_errors(golden_inputs, tmp_path):
    out = str(tmp_path / "o.txt")
    with pytest.raises(AssertionError, match="k must be >= 1, got 1 instead."):
        _cli(["count", golden_inputs["edge"], out, "1"])
    with pytest.raises(AssertionError, match="premature end of file or empty file"):
        _cli(["count", golden_inputs["empty"], out, "3"])
    with pytest.raises(AssertionError, match="premature end of file or empty file"):
        _cli(["uniq", golden_inputs["noheader"], out, "3"])
    with pytest.raises(AssertionError, match="incompatible string"):
        _cli(["count", golden_inputs["emptyname"], out, "3"])
    assert not os.path.exists(out)
    d = tmp_path / "full"
    d.mkdir()
    (d / "x").write_text("x")
    with pytest.raises(AssertionError, match="output folder must be empty"):
        _cli(["batch", golden_inputs["edge"], str(d), "3"])


def test_crawler_groups_match_oracle(golden_inputs):
    """Crawler.do_batch: every group with all its headers, in merged order
    (join.py:95-130), against the numpy restatement."""
    import numpy as np
    import np_oracle

    from kman_amd.batcher import FastaBatcher
    from kman_amd.join import Crawler

    path = golden_inputs["messy1"]
    batches = FastaBatcher(reverse=True, size=101).do(path, 5).collection
    got = list(Crawler().do_batch(batches))
    with open(path, "rb") as fh:
        recs = np_oracle.parse_fasta(fh.read())
    keys, pos = np_oracle.stream_kmers(recs, 5, rc=True)
    order = np.argsort(keys, kind="stable")
    names = [np_oracle.record_name(t).decode() for t, _ in recs]
    starts = np.cumsum([0] + [len(s) for _, s in recs])
    want = []
    for i in order:
        g = int(pos[i]) >> 1
        r = int(np.searchsorted(starts, g, side="right")) - 1
        hdr = "%s:%d-%d:%s" % (names[r], g - starts[r], g - starts[r] + 5, "-" if int(pos[i]) & 1 else "+")
        seq = np_oracle.decode(keys[i], 5).decode()
        if want and want[-1][1] == seq:
            want[-1][0].append(hdr)
        else:
            want.append(([hdr], seq))
    assert got == want


def test_batch_objects(golden_inputs):
    from kman_amd.batcher import FastaBatcher

    fb = FastaBatcher(size=40).do(golden_inputs["edge"], 3)
    col = fb.collection
    assert col[0].current_size == 0  # the batcher's own initial batch, as in the reference
    sizes = [b.current_size for b in col[1:]]
    assert sum(sizes) == fb.source.n_kmers and all(s == 40 for s in sizes[:-1])
    recs = col[1].sorted()
    assert [r.seq for r in recs] == sorted(r.seq for r in recs)
    assert list(col[1].record_gen()) == recs


def test_sequence_kmerator_known_answers():
    """Known answers of the reference's tests/test_seq.py:117-181."""
    from kman_amd.seq import NATYPES, KMer, Sequence, SequenceCoords

    s = Sequence("ACGAT", NATYPES.DNA, "stest")
    assert list(s.kmers(4)) == [KMer("stest", 0, 4, "ACGA"), KMer("stest", 1, 5, "CGAT")]
    s = Sequence("ACGATCGATCG", NATYPES.DNA, "ref")
    m = SequenceCoords.STRAND.MINUS
    want = [
        [KMer("ref", 0, 4, "ACGA"), KMer("ref", 0, 4, "TCGT", strand=m),
         KMer("ref", 1, 5, "CGAT"), KMer("ref", 1, 5, "ATCG", strand=m)],
        [KMer("ref", 2, 6, "GATC"), KMer("ref", 2, 6, "GATC", strand=m),
         KMer("ref", 3, 7, "ATCG"), KMer("ref", 3, 7, "CGAT", strand=m)],
        [KMer("ref", 4, 8, "TCGA"), KMer("ref", 4, 8, "TCGA", strand=m),
         KMer("ref", 5, 9, "CGAT"), KMer("ref", 5, 9, "ATCG", strand=m)],
        [KMer("ref", 6, 10, "GATC"), KMer("ref", 6, 10, "GATC", strand=m),
         KMer("ref", 7, 11, "ATCG"), KMer("ref", 7, 11, "CGAT", strand=m)],
    ]
    assert [list(g) for g in s.kmerator_batched(s.text, 4, s.natype, 5, s.name, True)] == want
    assert [k.seq for k in Sequence.kmerator("ACGNACGT", 3, NATYPES.DNA)] == ["ACG", "ACG", "CGT"]


@pytest.mark.parametrize("case", [c for c in _manifest()["cases"] if c["k"] <= 32 and c["cmd"] in ("count", "uniq")
                                  and "-B" not in c["flags"]][::3], ids=lambda c: c["name"])
def test_cli_multi_gpu_path_world1(case, golden_inputs, tmp_path, monkeypatch):
    """The CLI's multi-GPU path (kman_amd/launch.py) without SimGroup: with
    KMAN_DIST=1 at world size 1, FastaBatcher.do loads the byte-range shard,
    KJoiner.join builds a real RCCL communicator (one rank), runs the key
    rounds with every exchange through RCCL (exchange forced) and writes the
    output through DistPipeline.emit_gen -- byte-identical to the reference's
    golden output."""
    monkeypatch.setenv("KMAN_DIST", "1")
    monkeypatch.setenv("KMAN_DIST_EXCHANGE", "1")
    out = str(tmp_path / "out.txt")
    _cli([case["cmd"], golden_inputs[case["input"]], out, str(case["k"])] + case["flags"])
    assert _sha(out) == case["sha256"]


def test_cli_hist_multi_gpu_path_world1(golden_inputs, tmp_path, monkeypatch):
    """`kmer hist` through the multi-GPU path at world size 1 equals the
    single-GPU spectrum."""
    out1, out2 = str(tmp_path / "h1.txt"), str(tmp_path / "h2.txt")
    _cli(["hist", golden_inputs["messy1"], out1, "21"])
    monkeypatch.setenv("KMAN_DIST", "1")
    monkeypatch.setenv("KMAN_DIST_EXCHANGE", "1")
    _cli(["hist", golden_inputs["messy1"], out2, "21"])
    assert open(out1, "rb").read() == open(out2, "rb").read() and os.path.getsize(out1) > 0


@pytest.mark.parametrize("case", _manifest().get("vec_cases", []), ids=lambda c: c["name"])
def test_cli_vec_masked_matches_reference(case, golden_inputs, tmp_path, monkeypatch):
    """`kmer count --count-mode VEC_COUNT_MASKED` (default: the reference's
    behaviour) raises where the reference raised -- a group holding records
    of two names reaches add_count, join.py:318-335 -- and otherwise leaves
    the same (empty) vector folder; k > 32 through the word-key path."""
    import builtins

    monkeypatch.delenv("KMAN_VEC_COUNT", raising=False)
    out = str(tmp_path / "vec.out")
    argv = ["count", golden_inputs[case["input"]], out, str(case["k"]), "--count-mode", "VEC_COUNT_MASKED"] + case["flags"]
    if case["result"]["ok"]:
        _cli(argv)
        assert sorted(os.listdir(str(tmp_path / "vec"))) == case["folder"]
    else:
        with pytest.raises(getattr(builtins, case["result"]["type"])):
            _cli(argv)


@pytest.mark.parametrize("k", [21, 40])
def test_cli_vec_masked_previous_batches(k, golden_inputs, tmp_path, monkeypatch):
    """-B: the VEC_COUNT_MASKED decision from reloaded batch files (refs read
    from the batch records' titles) is the one the FASTA gives (the
    reference's loader rejects every non-empty folder, SURVEY §A-5: evident
    intent), at k <= 32 and k > 32."""
    monkeypatch.delenv("KMAN_VEC_COUNT", raising=False)
    want = {c["input"]: c["result"]["ok"] for c in _manifest()["vec_cases"] if c["k"] == 40 and not c["flags"]}
    for inp in ("vecshare", "vecsame"):
        outdir = str(tmp_path / ("b_%s" % inp))
        _cli(["batch", golden_inputs[inp], outdir, str(k), "-b", "50"])
        out = str(tmp_path / ("%s.out" % inp))
        argv = ["count", golden_inputs[inp], out, str(k), "--count-mode", "VEC_COUNT_MASKED", "-B", outdir]
        if want[inp]:
            _cli(argv)
            assert os.listdir(str(tmp_path / inp)) == []
        else:
            with pytest.raises(NotImplementedError):
                _cli(argv)
