"""Pinned H2D async copies of the loader's chunks, byte-compared (debug)."""
import sys
from ctypes import c_void_p

import numpy as np

sys.path.insert(0, "tests/golden")
sys.path.insert(0, ".")
import inputs  # noqa: E402

from kman_amd import _native as N  # noqa: E402
from kman_amd import engine, shard  # noqa: E402

dev = engine.default_device()
text = inputs.syn_numpy(3_000_000, 11, record_len=700_000, width=61)
rd = shard.PinnedReader(dev, text)
cuts = shard.chunk_cuts(rd, 0, len(text), 333_333)
bufs = [dev.alloc(400_000), dev.alloc(400_000)]
L = N.lib()
for rep in range(2):
    for i, (lo, hi) in enumerate(zip(cuts, cuts[1:])):
        s = i & 1
        N.check(dev.ctx, L.kman_copy_h2d_async(dev.ctx, c_void_p(bufs[s].ptr), c_void_p(rd.ptr(lo)), hi - lo, s), "cp")
        N.check(dev.ctx, L.kman_copy_sync(dev.ctx), "sync")
        got = dev.download(bufs[s], hi - lo, np.uint8)
        bad = np.nonzero(got != np.frombuffer(text[lo:hi], np.uint8))[0]
        print("rep", rep, "chunk", i, "lo", lo, "lo%16", lo % 16, "n", hi - lo, "bad", len(bad), bad[:2], bad[-2:],
              flush=True)
# the same through a plain synchronous hipMemcpy of the pinned range
for i, (lo, hi) in enumerate(zip(cuts, cuts[1:])):
    dev.upload(bufs[0], rd.array[lo:hi])
    got = dev.download(bufs[0], hi - lo, np.uint8)
    print("upload chunk", i, "bad", int((got != np.frombuffer(text[lo:hi], np.uint8)).sum()), flush=True)
