#!/usr/bin/env python3
"""The uniq writer of config 2 (1e9 rows, 49 GB of text) into /dev/null,
three times in one process: the first (cold) against the warm ones, and the
format kernels' own time (KTimer "format").  usage: fmtcold.py [bases]"""
import os
import sys
import time
from ctypes import byref, c_double, c_uint64

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import inputs
    from kman_amd import _native as N
    from kman_amd import engine

    bases = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    text = inputs.syn_numpy(bases, 1)
    dev = engine.Device(0)
    p = engine.parse(dev, text)
    del text
    r = engine.groups(p, 21, False, "uniq")
    if os.environ.get("FMT_SLICES"):  # per-slice host timeline of the first (cold) and a warm run
        import concurrent.futures  # noqa: F401
        orig = N.lib().kman_copy_d2h_wait
        marks = []

        def traced(ctx, b):
            t = time.perf_counter()
            rc = orig(ctx, b)
            marks.append((t, time.perf_counter()))
            return rc
        N.lib().kman_copy_d2h_wait = traced
        for i in range(2):
            marks.clear()
            t0 = time.perf_counter()
            with open(os.devnull, "wb") as sink:
                engine.emit_uniq(p, r, sink)
            w = [b - a for a, b in marks]
            gaps = [marks[j + 1][0] - marks[j][1] for j in range(len(marks) - 1)]
            print("trace run %d: %.3f s, %d waits: wait ms first10 %s last5 %s sum %.1f; between-waits ms first10 %s "
                  "sum %.1f" % (i, time.perf_counter() - t0, len(w), [round(x * 1e3, 2) for x in w[:10]],
                                [round(x * 1e3, 2) for x in w[-5:]], sum(w) * 1e3,
                                [round(x * 1e3, 2) for x in gaps[:10]], sum(gaps) * 1e3), flush=True)
        N.lib().kman_copy_d2h_wait = orig
    for i in range(3):
        with open(os.devnull, "wb") as sink:
            N.lib().kman_timing_enable(dev.ctx, 1)
            t0 = time.perf_counter()
            engine.emit_uniq(p, r, sink)
            el = time.perf_counter() - t0
            c, ms = c_uint64(0), c_double(0)
            N.lib().kman_timing_query(dev.ctx, b"format", byref(c), byref(ms))
            N.lib().kman_timing_enable(dev.ctx, 0)
        print("run %d: %.3f s, format kernels %.1f ms in %d launches" % (i, el, ms.value, c.value), flush=True)


if __name__ == "__main__":
    main()
