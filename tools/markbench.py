#!/usr/bin/env python3
"""Time the redo path's marked extraction (kman_extract_marked: a byte map
over the top key bits in HBM) against kman_extract_range over one narrow
range and over every key, on the bench's 1 GB synthetic FASTA (k=21):
where the GRCh38-shaped line's redo extraction spends its time."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import numpy as np
import inputs
from ctypes import byref, c_void_p, c_uint64
from kman_amd import engine, _native as N

dev = engine.Device(0)
text = inputs.syn_numpy(1_000_000_000, 1)
p = engine.parse(dev, text)
del text
L = N.lib()
k = 21
cap = p.n_bases
keys = dev.alloc(8 * cap)
pos = dev.alloc(8 * cap)
fl = engine.flags_for(False, False, False)


def timed(f, reps=5):
    f()
    dev.sync()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    dev.sync()
    return (time.perf_counter() - t) / reps * 1e3


def rng(lo, hi):
    n = c_uint64(0)
    N.check(dev.ctx, L.kman_extract_range(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k, fl, lo, hi,
                                          c_void_p(keys.ptr), None, 8, cap, None, byref(n)), "range")
    return n.value


for bits, nmark in ((17, 300), (20, 300), (24, 3000)):
    pm = np.zeros(1 << bits, np.uint8)
    pm[np.random.default_rng(1).choice(1 << bits, nmark, replace=False)] = 1
    d = dev.alloc(len(pm))
    dev.upload(d, pm)

    def marked():
        n = c_uint64(0)
        N.check(dev.ctx, L.kman_extract_marked(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k, fl, c_void_p(d.ptr), bits,
                                               1, c_void_p(keys.ptr), None, 8, cap, byref(n)), "marked")
        return n.value

    print("marked %2d-bit map, %5d entries: %.2f ms (%d k-mers)" % (bits, nmark, timed(marked), marked()), flush=True)
    d.free()
print("range, narrow: %.2f ms (%d)" % (timed(lambda: rng(0, (1 << 30) - 1)), rng(0, (1 << 30) - 1)), flush=True)
print("range, every key: %.2f ms (%d)" % (timed(lambda: rng(0, ~0 & ((1 << 64) - 1))), rng(0, (1 << 64) - 1)),
      flush=True)
