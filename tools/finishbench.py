#!/usr/bin/env python3
"""Time kman_finish alone (uniq / count / sort over the bench key distribution).

Random 42-bit keys + u32 payload are prefix-sorted with kman_sort_range, then
kman_finish runs --reps times (uniq and count only read the keys).  Prints the
time per launch and a digest of the output so builds can be compared.
Set KMAN_LIB to time another build of libkman.so."""
import argparse, ctypes, hashlib, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kman_amd import _native as N, engine

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000_000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--modes", default="uniq,count")
ap.add_argument("--bits", type=int, default=42)
a = ap.parse_args()
dev = engine.Device(0)
L = N.lib()
rng = np.random.default_rng(1)
n = a.n
kb = [dev.alloc(8 * n), dev.alloc(8 * n)]
vb = [dev.alloc(4 * n), dev.alloc(4 * n)]
ok, ov = dev.alloc(8 * n), dev.alloc(8 * n)
for o in range(0, n, 1 << 26):
    m = min(1 << 26, n - o)
    dev.upload(kb[0], rng.integers(0, 1 << a.bits, size=m, dtype=np.uint64), offset=8 * o)
    dev.upload(vb[0], np.arange(o, o + m, dtype=np.uint32), offset=4 * o)
lo = engine.split_bits(n, a.bits)
res = ctypes.c_int()
P = lambda b: ctypes.c_void_p(b.ptr)  # noqa: E731
N.check(dev.ctx, L.kman_sort_range(dev.ctx, P(kb[0]), P(kb[1]), P(vb[0]), P(vb[1]), 4, n, lo, a.bits, None,
                                   ctypes.byref(res)), "sort_range")
c = res.value
L.kman_timing_enable(dev.ctx, 1)
modes = {"sort": 0, "count": 1, "uniq": 2}
for name in a.modes.split(","):
    md = modes[name]
    out = ctypes.c_uint64()
    for r in range(a.reps):
        N.check(dev.ctx, L.kman_finish(dev.ctx, P(kb[c]), P(kb[c ^ 1]), P(vb[c]), P(vb[c ^ 1]), 4, n, a.bits, lo, md,
                                       P(ok), P(ov), 4, ctypes.byref(out)), "finish")
    cnt, ms = ctypes.c_uint64(), ctypes.c_double()
    L.kman_timing_query(dev.ctx, b"finish", ctypes.byref(cnt), ctypes.byref(ms))
    no = out.value if md else n
    h = hashlib.sha1()
    for off in (0, max(0, no - (1 << 20))):
        m = min(1 << 20, no)
        h.update(dev.download(ok if md else kb[c], m, np.uint64, offset=8 * off).tobytes())
        h.update(dev.download(ov if md else vb[c], m, np.uint32, offset=4 * off).tobytes())
    print("%s n %d lo %d: %.3f ms/launch (%d launches), %d out, digest %s" % (
        name, n, lo, ms.value / max(cnt.value, 1), cnt.value, no, h.hexdigest()[:12]), flush=True)
    L.kman_timing_enable(dev.ctx, 0)
    L.kman_timing_enable(dev.ctx, 1)
