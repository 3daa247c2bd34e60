"""Host logic of the multi-batch device join (engine.key_ranges): key ranges
cover the key space in order, each holds at most max_keys k-mers, a single
8-bit prefix larger than a batch is refused."""

from __future__ import annotations

import numpy as np
import pytest


def _check(h, k, mk):
    from kman_amd import engine

    rs = engine.key_ranges(h, k, mk)
    sh = max(0, 2 * k - 8)
    assert sum(r[2] for r in rs) == int(h.sum())
    prev_hi = -1
    for lo, hi, n in rs:
        assert 0 < n <= mk
        assert lo > prev_hi and lo <= hi
        assert (lo >> sh) << sh == lo and ((hi + 1) >> sh) << sh == hi + 1
        assert n == int(h[lo >> sh : (hi >> sh) + 1].sum())
        prev_hi = hi
    if rs:
        assert rs[-1][1] <= (1 << (2 * k)) - 1
    return rs


@pytest.mark.parametrize("k", [2, 3, 4, 13, 21, 31, 32])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_key_ranges(k, seed):
    rng = np.random.default_rng(seed)
    bins = 256 if 2 * k >= 8 else 1 << (2 * k)
    h = rng.integers(0, 1000, bins).astype(np.uint64)
    h[rng.integers(0, bins, bins // 4)] = 0
    for mk in (int(h.max()), int(h.sum()) // 5 + 1, int(h.sum()) + 10):
        rs = _check(h, k, mk)
        if mk >= int(h.sum()):
            assert len(rs) == 1


def test_key_ranges_edges():
    from kman_amd import engine

    assert engine.key_ranges(np.zeros(256, np.uint64), 21, 10) == []
    h = np.zeros(256, np.uint64)
    h[255] = 7
    assert engine.key_ranges(h, 21, 7) == [(0, (1 << 42) - 1, 7)]
    h[3] = 8
    with pytest.raises(MemoryError):
        engine.key_ranges(h, 21, 7)
    assert engine.key_ranges(h, 32, 8) == [(0, (255 << 56) - 1, 8), (255 << 56, (1 << 64) - 1, 7)]
