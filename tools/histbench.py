#!/usr/bin/env python3
"""Time the k-mer digit-histogram pre-pass of kman_extract_sorted alone on the
bench workload (1 GB synthetic FASTA, k=21); prints ms per launch and a digest
of the histogram + count so builds (KMAN_LIB) can be compared."""
import ctypes, hashlib, os, sys
from ctypes import byref, c_void_p, c_uint64
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import numpy as np
import inputs
from kman_amd import engine, _native as N
k = int(os.environ.get("K", "21"))
dev = engine.Device(0)
text = inputs.syn_numpy(1_000_000_000, 1)
pipe = engine.ResidentPipeline(dev, text, k, mode="uniq")
del text
L = N.lib()
info = N.ParseInfo()
N.check(dev.ctx, L.kman_parse_fasta(dev.ctx, c_void_p(pipe.text.ptr), pipe.n_bytes, c_void_p(pipe.codes.ptr),
                                    c_void_p(pipe.rec_hdr.ptr), c_void_p(pipe.rec_seq.ptr), pipe.rec_cap,
                                    byref(info)), "parse")
L.kman_debug_kmer_hist.argtypes = [c_void_p, c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_uint32, c_void_p, ctypes.POINTER(c_uint64)]
n = c_uint64(0)
for rc in (0, 1):
    flags = pipe.flags | (N.KMAN_RC if rc else 0)
    L.kman_timing_enable(dev.ctx, 1)
    reps = 5
    for _ in range(reps):
        N.check(dev.ctx, L.kman_debug_kmer_hist(dev.ctx, c_void_p(pipe.codes.ptr), info.n_bases, k, flags, pipe.lo_bit,
                                                c_void_p(pipe.hist.ptr), byref(n)), "kmer_hist")
    cnt, ms = c_uint64(), ctypes.c_double()
    L.kman_timing_query(dev.ctx, b"kmer_hist", byref(cnt), byref(ms))
    h = dev.download(pipe.hist, 8 * 256, np.uint64)
    print("rc %d k %d lo %d: kmer_hist %.3f ms/launch, %d k-mers, digest %s" % (
        rc, k, pipe.lo_bit, ms.value / max(cnt.value, 1), n.value, hashlib.sha1(h.tobytes()).hexdigest()[:12]),
        flush=True)
