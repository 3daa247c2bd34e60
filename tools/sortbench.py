#!/usr/bin/env python3
"""Micro-benchmark of kman_sort on device-resident random keys (+ u32 payload).

Times every onesweep pass with the library's HIP-event timer.  KMAN_LIB may
point at an ablation build (see kman_amd/csrc/Makefile ABL=...)."""
import argparse, ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kman_amd import _native as N, engine

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000_000)
ap.add_argument("--bits", type=int, default=42)
ap.add_argument("--vals", type=int, default=4)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = engine.Device(0)
L = N.lib()
rng = np.random.default_rng(1)
keys = dev.alloc(8 * a.n); alt = dev.alloc(8 * a.n)
chunk = 1 << 26
for o in range(0, a.n, chunk):
    m = min(chunk, a.n - o)
    dev.upload(keys, rng.integers(0, 1 << a.bits, size=m, dtype=np.uint64), offset=8 * o)
src = dev.download(keys, a.n, np.uint64)
v = v2 = None
if a.vals:
    v = dev.alloc(a.vals * a.n); v2 = dev.alloc(a.vals * a.n)
for r in range(a.reps):
    dev.upload(keys, src)
    L.kman_timing_enable(dev.ctx, 1)
    res = ctypes.c_int(0)
    t0 = time.perf_counter()
    rc = L.kman_sort(dev.ctx, ctypes.c_void_p(keys.ptr), ctypes.c_void_p(alt.ptr), ctypes.c_void_p(v.ptr if v else None),
                     ctypes.c_void_p(v2.ptr if v2 else None), a.vals, a.n, a.bits, None, ctypes.byref(res))
    dev.sync()
    t1 = time.perf_counter()
    N.check(dev.ctx, rc, "sort")
    n, ms = ctypes.c_uint64(), ctypes.c_double()
    L.kman_timing_query(dev.ctx, b"sort_pass", ctypes.byref(n), ctypes.byref(ms))
    per = ms.value / max(1, n.value)
    gbs = (16 + 2 * a.vals) * a.n / (per / 1e3) / 1e9
    print("rep %d: total %.2f ms, %d passes, %.3f ms/pass, %.0f GB/s/pass (%.1f%% of 8 TB/s)" % (
        r, (t1 - t0) * 1e3, n.value, per, gbs, gbs / 80), flush=True)
if os.environ.get("KMAN_CHECK", "1") == "1" and not os.environ.get("KMAN_LIB"):
    out = dev.download(alt if res.value else keys, a.n, np.uint64)
    assert (out[1:] >= out[:-1]).all(), "not sorted"
    print("sorted ok")
