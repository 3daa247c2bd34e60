#!/usr/bin/env python3
"""Phase breakdown of onesweep tiles from a diagnostic build (ABL=4).

Runs one kman_sort over random 42-bit keys + u32 payload with the library at
KMAN_LIB (built with `make ABL=4`), reads the per-tile s_memrealtime stamps
(100 MHz) of the LAST pass and prints per-phase medians/percentiles:
  0 start  1 keys landed  2 ranked  3 looked back  4 keys written  5 done"""
import argparse, ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kman_amd import _native as N, engine

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000_000)
ap.add_argument("--tile", type=int, default=6144)
a = ap.parse_args()
dev = engine.Device(0)
L = N.lib()
rng = np.random.default_rng(1)
keys, alt = dev.alloc(8 * a.n), dev.alloc(8 * a.n)
v, v2 = dev.alloc(4 * a.n), dev.alloc(4 * a.n)
for o in range(0, a.n, 1 << 26):
    m = min(1 << 26, a.n - o)
    dev.upload(keys, rng.integers(0, 1 << 42, size=m, dtype=np.uint64), offset=8 * o)
tiles = (a.n + a.tile - 1) // a.tile
dbg = dev.alloc(8 * 8 * tiles)
dev.memset(dbg, 0, 8 * 8 * tiles)
L.kman_debug_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
L.kman_debug_set(dev.ctx, ctypes.c_void_p(dbg.ptr))
res = ctypes.c_int()
N.check(dev.ctx, L.kman_sort(dev.ctx, ctypes.c_void_p(keys.ptr), ctypes.c_void_p(alt.ptr), ctypes.c_void_p(v.ptr),
                             ctypes.c_void_p(v2.ptr), 4, a.n, 42, None, ctypes.byref(res)), "sort")
dev.sync()
s = dev.download(dbg, 8 * tiles, np.uint64).reshape(tiles, 8)[:, :6].astype(np.int64)
s = s[(s > 0).all(axis=1)]
d = np.diff(s, axis=1) * 10.0  # ns
names = ["load", "rank", "lookback", "scatter+write keys", "vals"]
print("tiles %d, kernel span %.3f ms" % (len(s), (s[:, 5].max() - s[:, 0].min()) / 1e5))
for i, nm in enumerate(names):
    q = np.percentile(d[:, i], [10, 50, 90, 99])
    print("%-20s p10 %7.0f  p50 %7.0f  p90 %7.0f  p99 %8.0f ns" % (nm, *q))
tot = (s[:, 5] - s[:, 0]) * 10.0
print("%-20s p10 %7.0f  p50 %7.0f  p90 %7.0f  p99 %8.0f ns" % ("tile total", *np.percentile(tot, [10, 50, 90, 99])))
# concurrency: tiles in flight at the midpoint of the kernel
mid = (s[:, 0].min() + s[:, 5].max()) // 2
print("tiles in flight at mid-kernel: %d" % int(((s[:, 0] <= mid) & (s[:, 5] >= mid)).sum()))
r = dev.download(dbg, 8 * tiles, np.uint64).reshape(tiles, 8)[:, 6:].astype(np.int64)
print("look-back rounds p50 %d p90 %d p99 %d max %d; stall spins p50 %d p90 %d p99 %d" % (
    *np.percentile(r[:, 0], [50, 90, 99]), r[:, 0].max(), *np.percentile(r[:, 1], [50, 90, 99])))
