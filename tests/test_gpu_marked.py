"""GPU parity of kman_extract_marked (the partial redo's extraction: the
k-mers whose top map_bits key bits map to one destination; dist._redo_ranges),
including its LDS coarse bitmap (map_coarse): exact when the map has at most
16 key bits (or 2k), a prefilter before the HBM map otherwise.

Bar: the extracted keys (and their pos) as a multiset equal the numpy
restatement's windows (np_oracle.stream_kmers, seq.py:285-328) filtered by
the same map."""

from __future__ import annotations

from ctypes import byref, c_uint64, c_void_p

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,map_bits", [(7, 6), (7, 14), (13, 16), (21, 12), (21, 17), (21, 20), (21, 24)])
@pytest.mark.parametrize("variant", ["fwd", "rc", "canonical"])
def test_extract_marked_matches_oracle(k, map_bits, variant):
    import inputs
    import np_oracle
    from kman_amd import _native as N
    from kman_amd import engine

    rc, canon = variant == "rc", variant == "canonical"
    text = inputs.messy_records(7, n_records=40, max_len=20_000)
    keys, pos = np_oracle.stream_kmers(np_oracle.parse_fasta(text), k, rc=rc, canonical=canon)
    rng = np.random.default_rng(map_bits * 100 + k)
    pm = rng.integers(0, 4, 1 << map_bits, dtype=np.uint8)  # values 0..3: destination 2 wanted
    shift = np.uint64(2 * k - map_bits)
    want = np.sort(keys[pm[(keys >> shift).astype(np.int64)] == 2])
    dev = engine.default_device()
    p = engine.parse(dev, text)
    d_map = dev.alloc(len(pm))
    cap = max(1, 2 * p.n_bases)
    d_keys, d_pos = dev.alloc(8 * cap), dev.alloc(8 * cap)
    try:
        dev.upload(d_map, pm)
        fl = engine.flags_for(rc, True, canon)
        n = c_uint64(0)
        N.check(dev.ctx, N.lib().kman_extract_marked(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k, fl,
                                                     c_void_p(d_map.ptr), map_bits, 2, c_void_p(d_keys.ptr),
                                                     c_void_p(d_pos.ptr), 8, cap, byref(n)), "kman_extract_marked")
        got = dev.download(d_keys, n.value, np.uint64)
        gpos = dev.download(d_pos, n.value, np.uint64)
        np.testing.assert_array_equal(np.sort(got), want)
        # each key sits at its window (pos = window << 1 | strand, as the oracle's)
        sel = pm[(keys >> shift).astype(np.int64)] == 2
        o1 = np.lexsort((pos[sel], keys[sel]))
        o2 = np.lexsort((gpos, got))
        np.testing.assert_array_equal(gpos[o2], pos[sel][o1])
    finally:
        for b in (d_map, d_keys, d_pos):
            b.free()
        p.free()
