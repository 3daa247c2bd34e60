"""KJoiner VEC_COUNT / VEC_COUNT_MASKED on the GPU (kman_vec_fill) against a
restatement of the reference's vector code with its abstract-base call
removed (join.py:288-335 join_vector_count[_masked] over Crawler.do_batch
groups -> AbundanceVector.add_count / add_ref / write_to,
abundance.py:103-168).  The reference itself raises NotImplementedError at
the first add_count (abundance.py:60), so these semantics are parity
unpinned: the restatement below is the check."""

from __future__ import annotations

import gzip
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expected(text: bytes, k: int, rc: bool, masked: bool):
    """{(ref, strand): [counts]} as AbundanceVector would hold them."""
    import np_oracle

    recs = np_oracle.parse_fasta(text)
    names = [np_oracle.record_name(t).decode("utf-8", "surrogateescape") for t, _ in recs]
    _, rec_seq = np_oracle.codes_of(recs)
    keys, pos = np_oracle.stream_kmers(recs, k, rc=rc)
    sk, sp = np_oracle.stable_sort(keys, pos)
    rec_of = np.searchsorted(rec_seq.astype(np.int64), (sp >> np.uint64(1)).astype(np.int64), side="right") - 1
    vec = {}

    def add(ref, strand, p, count):  # AbundanceVector.add_count (replace=False)
        v = vec.setdefault((ref, strand), np.zeros(p + 1, np.int64))
        if len(v) < p + 1:
            v = np.concatenate([v, np.zeros(p + 1 - len(v), np.int64)])
            vec[(ref, strand)] = v
        assert v[p] == 0
        v[p] = count

    i, n = 0, len(sk)
    while i < n:  # Crawler.do_batch: the groups of equal k-mers, in order
        j = i
        while j < n and sk[j] == sk[i]:
            j += 1
        grp = range(i, j)
        coords = [(names[rec_of[g]], "+-"[int(sp[g]) & 1], int(sp[g] >> np.uint64(1)) - int(rec_seq[rec_of[g]]))
                  for g in grp]
        if not masked:
            for ref, strand, st in coords:
                add(ref, strand, st, len(coords))
        elif len(coords) != 1:
            refs = [c[0] for c in coords]
            if len(set(refs)) != 1:
                for ref, strand, st in coords:
                    add(ref, strand, st, sum(1 for x in refs if x != ref))
        i = j
    return vec


def _read_dir(d):
    out = {}
    for f in os.listdir(d):
        assert f.endswith(".gz")
        ref, strand = f[:-3].rsplit("___", 1)
        lines = gzip.open(os.path.join(d, f), "rb").read().decode().split("\n")
        assert lines[-1] == ""
        out[(ref, strand)] = (lines[0], np.array([int(x) for x in lines[1:-1]], np.int64))
    return out


def _texts():
    import inputs

    rep = "ACGTTGCAGGCATTACGATTAC"
    a = b">chrA desc\n" + (rep * 40).encode() + b"NNACGT\n" + b"ACGTACGTAC" * 30 + b"\n"
    b = b">chrB\n" + (rep * 7).encode() + b"\n>chrC x\nACGTNACGTACGTTTT\n>chrD\nAC\n"
    return [a + b, inputs.messy_records(5, n_records=12, max_len=3000), inputs.syn_numpy(20_000, 3)]


@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("rc", [False, True])
@pytest.mark.parametrize("k", [3, 9, 21])
def test_vectors_match_restatement(tmp_path, monkeypatch, masked, rc, k):
    import np_oracle

    monkeypatch.setenv("KMAN_VEC_COUNT", "1")  # (this engine's vector writer; the default raises as the reference)

    from kman_amd.batcher import FastaBatcher
    from kman_amd.join import KJoiner

    for ti, text in enumerate(_texts()):
        names = [np_oracle.record_name(t) for t, _ in np_oracle.parse_fasta(text)]
        if len(set(names)) != len(names):
            continue
        fa = tmp_path / ("in%d.fa" % ti)
        fa.write_bytes(text)
        batches = FastaBatcher(reverse=rc, size=777).do(str(fa), k).collection
        mode = KJoiner.MODE.VEC_COUNT_MASKED if masked else KJoiner.MODE.VEC_COUNT
        out = tmp_path / ("vec%d_%d%d%d.out" % (ti, k, rc, masked))
        KJoiner(mode).join(batches, str(out))
        got = _read_dir(str(out)[:-4])
        want = _expected(text, k, rc, masked)
        assert set(got) == set(want)
        for key, (head, v) in got.items():
            assert head == "# k=%d" % k
            np.testing.assert_array_equal(v, want[key])


def _add_count_called(text: bytes, k: int, masked: bool) -> bool:
    """Would the reference's join call AbundanceVector.add_count at all?
    VEC_COUNT: for every k-mer; VEC_COUNT_MASKED: for a group whose headers
    name two refs or more (join.py:318-335)."""
    import np_oracle

    recs = np_oracle.parse_fasta(text)
    names = [np_oracle.record_name(t) for t, _ in recs]
    _, rec_seq = np_oracle.codes_of(recs)
    keys, pos = np_oracle.stream_kmers(recs, k)
    if not masked:
        return len(keys) > 0
    rec_of = np.searchsorted(rec_seq.astype(np.int64), (pos >> np.uint64(1)).astype(np.int64), side="right") - 1
    refs = {}
    for key, r in zip(keys.tolist(), rec_of.tolist()):
        refs.setdefault(key, set()).add(names[r])
    return any(len(v) > 1 for v in refs.values())


@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("k", [3, 21])
def test_vectors_default_raise_like_reference(tmp_path, monkeypatch, masked, k):
    """Without KMAN_VEC_COUNT=1, VEC_* do what the reference does: the first
    AbundanceVector.add_count raises NotImplementedError (abundance.py:60,
    via :123) -- VEC_COUNT at any k-mer, VEC_COUNT_MASKED at a k-mer shared by
    records of different names (join.py:318-335) -- and a join that never
    calls it writes the empty vector folder (abundance.py:151-165)."""
    from kman_amd.batcher import FastaBatcher
    from kman_amd.join import KJoiner

    monkeypatch.delenv("KMAN_VEC_COUNT", raising=False)
    texts = _texts() + [b">same\nACGTACGTAC\n>same\nACGTACGTAC\n", b">solo\n" + b"ACGTTGCA" * 50 + b"\n"]
    for ti, text in enumerate(texts):
        fa = tmp_path / ("in%d.fa" % ti)
        fa.write_bytes(text)
        batches = FastaBatcher(size=1000).do(str(fa), k).collection
        mode = KJoiner.MODE.VEC_COUNT_MASKED if masked else KJoiner.MODE.VEC_COUNT
        out = tmp_path / ("vec%d_%d%d.out" % (ti, k, masked))
        calls = _add_count_called(text, k, masked)
        if calls:
            with pytest.raises(NotImplementedError):
                KJoiner(mode).join(batches, str(out))
        else:
            KJoiner(mode).join(batches, str(out))
            assert os.path.isdir(str(out)[:-4]) and os.listdir(str(out)[:-4]) == []
