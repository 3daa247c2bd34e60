"""Host-side API surface (CPU only): record types and the generic Batch
container behave like the reference's (kmermaid/seq.py, batch.py), as its own
unit tests pin them (tests/test_seq.py, tests/test_batch.py of the reference,
restated here)."""

from __future__ import annotations

import os

import pytest

from kman_amd.batch import Batch
from kman_amd.seq import NATYPES, KMer, Sequence, SequenceCoords, SequenceCount


def test_coords_validation_and_roundtrip():
    for args in [("chr1", -1, 1), ("chr1", 0, -1)]:
        with pytest.raises(AssertionError):
            SequenceCoords(*args, SequenceCoords.STRAND.MINUS)
    with pytest.raises(AssertionError):
        SequenceCoords("chr1", 0, 1, "minus")
    sc = SequenceCoords("chr1", 0, 1000, SequenceCoords.STRAND.PLUS)
    assert str(sc) == "chr1:0-1000:+"
    assert SequenceCoords.from_str(str(sc)) == sc
    assert SequenceCoords.rev(SequenceCoords.STRAND.PLUS) == SequenceCoords.STRAND.MINUS
    assert SequenceCoords.from_str("a:b:3-9:-") == SequenceCoords("a:b", 3, 9, SequenceCoords.STRAND.MINUS)
    with pytest.raises(AssertionError, match="incompatible string: :0-3:\\+"):
        SequenceCoords.from_str(":0-3:+")


def test_kmer_record():
    with pytest.raises(AssertionError):
        KMer("chr1", 0, 1, "ACGATCGATCG")
    with pytest.raises(AssertionError):
        KMer("chr1", 0, 11, "ACGATCGATCG", t="DNA")
    k = KMer("chr1", 0, 11, "ACGATCGATCG")
    assert k.header == "chr1:0-11:+"
    assert k.as_fasta() == ">chr1:0-11:+\nACGATCGATCG\n"
    assert str(k) == "chr1:0-11:+\tACGATCGATCG"
    assert KMer.from_fasta((k.header, k.seq)) == k
    assert k.is_ab_checked()
    assert not KMer("c", 0, 4, "ACNT").is_ab_checked()


def test_sequence_helpers():
    with pytest.raises(AssertionError):
        Sequence("ACGAT", "DNA")
    s = Sequence("ACGATCGATCG", NATYPES.DNA)
    assert s == Sequence("acgatcgatcg", NATYPES.DNA)
    assert s != Sequence("ACGATCGATCG", NATYPES.RNA)
    assert list(s.batches(3, 5)) == [("ACGAT", 0), ("ATCGA", 3), ("GATCG", 6)]
    assert Sequence.mkrc("ACGA", NATYPES.DNA) == "TCGT"
    assert Sequence.mkrc("GATC", NATYPES.DNA) == "GATC"


def test_sequence_count_text():
    with pytest.raises(AssertionError):
        SequenceCount("ACGT", [1, 2], NATYPES.DNA)
    sc = SequenceCount("ACGATCGATCG", ["chr1:0-1000:+", "chr1:1000-2000:+"])
    assert str(sc) == "ACGATCGATCG\tchr1:0-1000:+ chr1:1000-2000:+"
    assert SequenceCount.from_text(str(sc)) == sc
    assert sc.as_text() == str(sc) + "\n"


def test_host_batch_lifecycle(tmp_path):
    b = Batch(str, str(tmp_path), 5)
    b.isFasta = False
    b.fwrite = b.fread = b.keyAttr = "__str__"
    assert (b.size, b.remaining, b.current_size, b.is_written) == (5, 5, 0, False)
    assert list(b.record_gen()) == [] and list(b.sorted()) == []
    with pytest.raises(AssertionError):
        b.add(1)
    b.add("First record")
    b.add_all(["Second record", "Third record"])
    b.add_all(["4th record"])
    assert b.current_size == 4 and b.remaining == 1
    assert list(b.record_gen()) == list(b.to_write())
    b.write()
    assert os.path.isfile(b.tmp) and b.is_written and b.collection == [None]
    assert len(list(b.record_gen())) == 4
    b2 = Batch.from_file(b.tmp, str, False)
    b2.isFasta = False
    b2.fwrite = b2.fread = b2.keyAttr = "__str__"
    assert b2.current_size == 4 and b2.tmp == b.tmp and b2.is_written
    assert list(b.record_gen()) == list(b2.record_gen())
    b.unwrite()
    assert b.current_size == 4 and not b.is_written
    b.add("5th record")
    assert b.is_full()
    assert list(b.sorted()) == ["4th record\n", "5th record", "First record\n", "Second record\n",
                                "Third record\n"]
    b.write()
    b.reset()
    assert (b.current_size, b.size, b.remaining, b.is_written) == (0, 5, 5, False)
    assert not os.path.isfile(b.tmp)


def test_batcher_validation(tmp_path):
    from kman_amd.batcher import FastaBatcher, load_batches

    fb = FastaBatcher(size=10)
    with pytest.raises(AssertionError, match="input file not found"):
        fb.do(str(tmp_path / "missing.fa"), 5)
    p = tmp_path / "x.fa"
    p.write_text(">a\nACGT\n")
    with pytest.raises(AssertionError, match="k must be >= 1, got 1 instead."):
        fb.do(str(p), 1)
    with pytest.raises(AssertionError):
        FastaBatcher(size=0)
    with pytest.raises(AssertionError):
        FastaBatcher(reverse="yes")
    with pytest.raises(AssertionError):
        load_batches(str(tmp_path / "nope"))
    empty = tmp_path / "empty_dir"
    empty.mkdir()
    with pytest.raises(AssertionError):
        load_batches(str(empty))


def test_joiner_modes(tmp_path):
    from kman_amd.join import KJoiner, KJoinerThreading

    j = KJoinerThreading()
    assert j.mode == KJoiner.MODE.UNIQUE and j.memory == KJoiner.MEMORY.NORMAL
    with pytest.raises(AssertionError):
        KJoiner("UNIQUE")
    with pytest.raises(AssertionError):
        j.batch_size = 1
    j.batch_size = 4
    # abundance vectors of nothing: the output directory (extension dropped),
    # no vector files (AbundanceVector.write_to over an empty crawl)
    KJoiner(KJoiner.MODE.VEC_COUNT).join([], str(tmp_path / "vec.out"))
    assert (tmp_path / "vec").is_dir() and not list((tmp_path / "vec").iterdir())
    (tmp_path / "file").write_text("")
    with pytest.raises(AssertionError):  # the directory path is a file
        KJoiner(KJoiner.MODE.VEC_COUNT_MASKED).join([], str(tmp_path / "file.txt"))


def test_pipelined_writer_pwrite_only_into_regular_non_append_files(tmp_path):
    """The pipelined writer (engine._format_dev) puts slices at computed
    offsets with os.pwrite only where that is the file's order: a regular
    file opened without O_APPEND; an append-mode file, a pipe or a sink
    without a descriptor are written in order by the calling thread."""
    import io

    from kman_amd import engine

    with open(tmp_path / "w.txt", "wb") as fh:
        fh.write(b"abc")
        fd, base = engine._pwrite_target(fh)
        assert fd == fh.fileno() and base == 3
    with open(tmp_path / "a.txt", "ab") as fh:
        assert engine._pwrite_target(fh) == (None, 0)
    assert engine._pwrite_target(io.BytesIO()) == (None, 0)
    r, w = os.pipe()
    try:
        with os.fdopen(w, "wb", closefd=False) as fh:
            assert engine._pwrite_target(fh) == (None, 0)
    finally:
        os.close(r)
        os.close(w)
