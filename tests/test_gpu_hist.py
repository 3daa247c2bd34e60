"""GPU parity of kman_count_hist (the abundance spectrum of config 5): h[c] =
rows whose count is c, the last bin every count >= nbins - 1, for u32 and
u64 counts; counts of 1 and 2 are summed in registers, the rest by LDS
atomics.  Bar: equal to numpy's bincount of the same counts."""

from __future__ import annotations

from ctypes import c_void_p

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbins", [2, 3, 17, 1001, 16384])
@pytest.mark.parametrize("dtype", [np.uint32, np.uint64])
def test_count_hist_matches_bincount(nbins, dtype):
    from kman_amd import _native as N
    from kman_amd import engine

    rng = np.random.default_rng(nbins)
    n = 3_000_017
    counts = np.where(rng.random(n) < 0.9, 1, rng.integers(1, 40_000, n)).astype(dtype)
    counts[::7] = 2
    want = np.bincount(np.minimum(counts.astype(np.int64), nbins - 1), minlength=nbins).astype(np.uint64)
    dev = engine.default_device()
    d_c, d_h = dev.alloc(counts.nbytes), dev.alloc(8 * nbins)
    try:
        dev.upload(d_c, counts)
        N.check(dev.ctx, N.lib().kman_count_hist(dev.ctx, c_void_p(d_c.ptr), counts.itemsize, n, c_void_p(d_h.ptr),
                                                 nbins), "kman_count_hist")
        np.testing.assert_array_equal(dev.download(d_h, nbins, np.uint64), want)
    finally:
        d_c.free()
        d_h.free()
