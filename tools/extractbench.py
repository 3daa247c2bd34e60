#!/usr/bin/env python3
"""Time kman_extract (bench workload: 1 GB synthetic FASTA, k=21, pos u32,
prefix histograms) with the library at KMAN_LIB (ablation builds)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import inputs
from kman_amd import engine
dev = engine.Device(0)
text = inputs.syn_numpy(1_000_000_000, 1)
pipe = engine.ResidentPipeline(dev, text, 21, mode="uniq")
del text
import ctypes
from ctypes import byref, c_void_p, c_uint64
from kman_amd import _native as N
L = N.lib()


def run():
    info = N.ParseInfo()
    N.check(dev.ctx, L.kman_parse_fasta(dev.ctx, c_void_p(pipe.text.ptr), pipe.n_bytes, c_void_p(pipe.codes.ptr),
                                        c_void_p(pipe.rec_hdr.ptr), c_void_p(pipe.rec_seq.ptr), pipe.rec_cap,
                                        byref(info)), "parse")
    N.check(dev.ctx, L.kman_memset(dev.ctx, c_void_p(pipe.hist.ptr), 0, 8 * 256 * 8), "memset")
    n = c_uint64(0)
    N.check(dev.ctx, L.kman_extract(dev.ctx, c_void_p(pipe.codes.ptr), info.n_bases, 21, pipe.flags,
                                    c_void_p(pipe.keys.ptr), c_void_p(pipe.pos.ptr), pipe.pos_bytes, pipe.bound,
                                    c_void_p(pipe.hist.ptr), byref(n)), "extract")


for _ in range(2):
    run()
pipe.timing(True)
for _ in range(5):
    run()
pipe.dev.sync()
n, ms = pipe.timed("extract")
print("%s: extract %.3f ms/launch (%d launches)" % (os.environ.get("KMAN_LIB", "default"), ms / n, n))
