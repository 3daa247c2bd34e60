"""The C-ABI library loads and exports every symbol include/kman.h declares,
and the host-only parts of it (plan, formatters) behave.  CPU only: no call
here touches a GPU."""

from __future__ import annotations

import ctypes

import numpy as np
import pytest

from kman_amd import _native as N


def test_library_loads_and_exports_header_symbols():
    L = N.lib()
    declared = N.header_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    # the ctypes signatures cover exactly what the header declares
    assert sorted(N.SIGNATURES) == declared
    assert L.kman_abi_version() == 1


def test_sort_plan_splits_bits_evenly():
    L = N.lib()
    for key_bits, want in [(42, [7] * 6), (62, [8, 8, 8, 8, 8, 8, 7, 7]), (8, [8]), (4, [4]), (64, [8] * 8)]:
        np_, sh, bi = ctypes.c_uint32(), (ctypes.c_uint32 * 8)(), (ctypes.c_uint32 * 8)()
        assert L.kman_sort_plan(key_bits, ctypes.byref(np_), sh, bi) == 0
        bits = [bi[i] for i in range(np_.value)]
        assert sorted(bits, reverse=True) == want
        assert sum(bits) == key_bits
        assert [sh[i] for i in range(np_.value)] == list(np.cumsum([0] + bits[:-1]))


def test_format_count_is_reference_format():
    from kman_amd import engine

    keys = np.array([0, 1, 27, (1 << 42) - 1], dtype=np.uint64)
    counts = np.array([1, 22, 333, 4444], dtype=np.uint32)
    out = engine.format_count(keys, counts, 21)
    want = "".join("%s\t%d\n" % (s, c) for s, c in zip(
        ["A" * 21, "A" * 20 + "C", "A" * 18 + "CGT", "T" * 21], [1, 22, 333, 4444]))
    assert out == want.encode()


def test_format_fasta_headers():
    from kman_amd import engine
    from kman_amd.engine import Parsed

    names = [b"chr0\tx", b"r2"]
    p = Parsed(None, None, 30, 2, np.array([0, 9], np.uint64), np.array([0, 10], np.uint64), names,
               b"".join(names), np.array([0, 6, 8], np.uint64))
    keys = np.array([0b00011011, 0b11100100], dtype=np.uint64)  # ACGT, TGCA
    pos = np.array([(3 << 1) | 0, (12 << 1) | 1], dtype=np.uint32)
    out = engine.format_fasta(keys, pos, 4, p)
    assert out == b">chr0\tx:3-7:+\nACGT\n>r2:2-6:-\nTGCA\n"


def test_title_name_matches_python_rules():
    from kman_amd.engine import _title_name

    text = b">chr0\tx y  \r\nACGT\n>  lead\n>\xc2\xa0nbsp \xc2\xa0\n"
    assert _title_name(text, 0) == b"chr0\tx"
    i = text.index(b">  lead")
    assert _title_name(text, i) == b""
    j = text.index(b">\xc2\xa0")
    assert _title_name(text, j) == " nbsp".encode()


@pytest.mark.parametrize("k", [1, 0, -3])
def test_k_validation_message(k):
    from kman_amd import engine

    with pytest.raises(AssertionError, match="k must be >= 1, got %d instead." % k):
        engine._check_k(k)


def _words_of(seqs, k):
    """(W, n) word planes of k-mer strings (words.hip layout)."""
    import numpy as np

    W = (k + 31) // 32
    h = k - 32 * (W - 1)
    out = np.zeros((W, len(seqs)), np.uint64)
    for i, sq in enumerate(seqs):
        parts = [sq[:h]] + [sq[h + 32 * j:h + 32 * (j + 1)] for j in range(W - 1)]
        for j, part in enumerate(parts):
            v = 0
            for c in part:
                v = (v << 2) | "ACGT".index(c)
            out[j, i] = v
    return out


def test_host_word_writers_match_reference_formats():
    """format.cpp's word-key writers (any k) print the reference's lines:
    "%s\\t%d\\n" (join.py:283-284) and ">%s\\n%s\\n" with "%s:%d-%d:%s"
    headers (join.py:261-262, seq.py:103-104) -- no GPU needed."""
    import ctypes
    from ctypes import byref, c_size_t, c_void_p

    import numpy as np

    from kman_amd import _native as N

    L = N.lib()
    rng = np.random.default_rng(3)
    for k in (2, 31, 32, 33, 64, 65, 100, 129):
        seqs = ["".join(rng.choice(list("ACGT"), k)) for _ in range(50)]
        planes = np.ascontiguousarray(_words_of(seqs, k))
        counts = rng.integers(1, 10 ** 6, 50).astype(np.uint32)
        used = c_size_t(0)
        args = (planes.ctypes.data_as(c_void_p), 50, counts.ctypes.data_as(c_void_p), 4, 50, k)
        assert L.kman_format_count_words(*args, None, 0, byref(used), 2) == N.KMAN_ECAP
        buf = ctypes.create_string_buffer(used.value)
        assert L.kman_format_count_words(*args, buf, used.value, byref(used), 2) == N.KMAN_OK
        assert buf.raw.decode() == "".join("%s\t%d\n" % (s, c) for s, c in zip(seqs, counts.tolist()))
        # uniq over a record table: names r0, r1 at bases 0 and 1000
        names = b"r0chrX\ty"
        off = np.array([0, 2, len(names)], np.uint64)
        rec = np.array([0, 1000], np.uint64)
        pos = np.sort(rng.integers(0, 2000, 50)).astype(np.uint64) << np.uint64(1) | rng.integers(0, 2, 50).astype(
            np.uint64)
        nb = ctypes.create_string_buffer(names, len(names))
        args = (planes.ctypes.data_as(c_void_p), 50, pos.ctypes.data_as(c_void_p), 8, 50, k, nb,
                off.ctypes.data_as(c_void_p), rec.ctypes.data_as(c_void_p), 2)
        assert L.kman_format_uniq_words(*args, None, 0, byref(used), 2) == N.KMAN_ECAP
        buf = ctypes.create_string_buffer(used.value)
        assert L.kman_format_uniq_words(*args, buf, used.value, byref(used), 2) == N.KMAN_OK
        want = []
        for s, v in zip(seqs, pos.tolist()):
            g = v >> 1
            r = 0 if g < 1000 else 1
            st = g - (0 if r == 0 else 1000)
            nm = ["r0", "chrX\ty"][r]
            want.append(">%s:%d-%d:%s\n%s\n" % (nm, st, st + k, "-" if v & 1 else "+", s))
        assert buf.raw.decode() == "".join(want)
        kinds = np.array([0, 1], np.uint8)
        args = (planes.ctypes.data_as(c_void_p), 50, pos.ctypes.data_as(c_void_p), 50, k, nb,
                off.ctypes.data_as(c_void_p), rec.ctypes.data_as(c_void_p), kinds.ctypes.data_as(c_void_p), 2)
        assert L.kman_format_uniq_mixed_words(*args, None, 0, byref(used), 2) == N.KMAN_ECAP
        buf = ctypes.create_string_buffer(used.value)
        assert L.kman_format_uniq_mixed_words(*args, buf, used.value, byref(used), 2) == N.KMAN_OK
        want = []
        for s, v in zip(seqs, pos.tolist()):
            g = v >> 1
            if g < 1000:
                want.append(">r0:%d-%d:%s\n%s\n" % (g, g + k, "-" if v & 1 else "+", s))
            else:  # a batch-file record: printed by its title
                want.append(">chrX\ty\n%s\n" % s)
        assert buf.raw.decode() == "".join(want)
