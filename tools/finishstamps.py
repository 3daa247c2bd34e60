#!/usr/bin/env python3
"""Phase breakdown of kman_finish chunks from a diagnostic build (ABL=4).

Uniq mode over the bench workload's key distribution: random 42-bit keys +
u32 payload, prefix-sorted with kman_sort_range, then one kman_finish with
per-chunk s_memrealtime stamps (100 MHz):
  0 start 1 chunk+starts 2 tail 3 LDS sort 7 RLE+scan 4 look-back+gather
  5 key staging 6 writes"""
import argparse, ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kman_amd import _native as N, engine

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000_000)
a = ap.parse_args()
dev = engine.Device(0)
L = N.lib()
rng = np.random.default_rng(1)
n = a.n
kb = [dev.alloc(8 * n), dev.alloc(8 * n)]
vb = [dev.alloc(4 * n), dev.alloc(4 * n)]
ok, ov = dev.alloc(8 * n), dev.alloc(4 * n)
for o in range(0, n, 1 << 26):
    m = min(1 << 26, n - o)
    dev.upload(kb[0], rng.integers(0, 1 << 42, size=m, dtype=np.uint64), offset=8 * o)
lo = engine.split_bits(n, 42)
res = ctypes.c_int()
P = lambda b: ctypes.c_void_p(b.ptr)  # noqa: E731
N.check(dev.ctx, L.kman_sort_range(dev.ctx, P(kb[0]), P(kb[1]), P(vb[0]), P(vb[1]), 4, n, lo, 42, None,
                                   ctypes.byref(res)), "sort_range")
c = res.value
T = (n + 4095) // 4096
dbg = dev.alloc(8 * 8 * T)
dev.memset(dbg, 0, 8 * 8 * T)
L.kman_debug_set_finish.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
L.kman_debug_set_finish(dev.ctx, ctypes.c_void_p(dbg.ptr))
out = ctypes.c_uint64()
L.kman_timing_enable(dev.ctx, 1)
N.check(dev.ctx, L.kman_finish(dev.ctx, P(kb[c]), P(kb[c ^ 1]), P(vb[c]), P(vb[c ^ 1]), 4, n, 42, lo, 2, P(ok), P(ov),
                               4, ctypes.byref(out)), "finish")
cnt, ms = ctypes.c_uint64(), ctypes.c_double()
L.kman_timing_query(dev.ctx, b"finish", ctypes.byref(cnt), ctypes.byref(ms))
print("n %d lo_bit %d: finish %.3f ms (%d launches), %d singles" % (n, lo, ms.value, cnt.value, out.value))
s = dev.download(dbg, 8 * T, np.uint64).reshape(T, 8).astype(np.int64)
s = s[(s > 0).all(axis=1)]
order = [0, 1, 2, 3, 7, 4, 5, 6]
names = ["chunk load+starts", "tail scan", "LDS sort", "RLE+scan", "look-back+gather", "key staging", "writes"]
d = np.diff(s[:, order], axis=1) * 10.0
print("chunks %d, kernel span %.3f ms" % (len(s), (s[:, 6].max() - s[:, 0].min()) / 1e5))
for i, nm in enumerate(names):
    q = np.percentile(d[:, i], [10, 50, 90, 99])
    print("%-20s p10 %7.0f  p50 %7.0f  p90 %7.0f  p99 %8.0f ns" % (nm, *q))
tot = (s[:, 6] - s[:, 0]) * 10.0
print("%-20s p10 %7.0f  p50 %7.0f  p90 %7.0f  p99 %8.0f ns" % ("chunk total", *np.percentile(tot, [10, 50, 90, 99])))
st = (ctypes.c_ulonglong * 4)()
L.kman_debug_finish_stats(dev.ctx, st)
print("wave-path chunks %d, block-path chunks %d, segments %d, sorted keys %d" % tuple(st))
mid = (s[:, 0].min() + s[:, 6].max()) // 2
print("chunks in flight at mid-kernel: %d" % int(((s[:, 0] <= mid) & (s[:, 6] >= mid)).sum()))
