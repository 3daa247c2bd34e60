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
