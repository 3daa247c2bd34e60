"""Output formatting cost, 1 GB synthetic FASTA k=21 (BASELINE config 2):
device writers (kman_format_*_dev + D2H of the text, into one host buffer or streamed
through a pinned buffer to a file, here /dev/null) against the host
writers (D2H of the result arrays + kman_format_* on host threads).  Prints
one JSON line of seconds per call and text bytes."""

from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main() -> None:
    import inputs
    from ctypes import byref, c_double, c_uint64

    from kman_amd import _native as N
    from kman_amd import engine

    bases = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    text = inputs.syn_numpy(bases, 1)
    dev = engine.Device(0)
    p = engine.parse(dev, text)
    del text
    res = {"bases": bases, "host_threads": engine.host_threads()}
    for mode in ("count", "uniq"):
        r = engine.groups(p, 21, False, mode)
        for fmt in ("device", "device_sink", "host"):
            sink = open(os.devnull, "wb") if fmt == "device_sink" else None
            emit = ((lambda: engine.emit_count(dev, r, sink)) if mode == "count" else
                    (lambda: engine.emit_uniq(p, r, sink)))
            os.environ["KMAN_HOST_FORMAT"] = "1" if fmt == "host" else "0"
            emit()
            N.lib().kman_timing_enable(dev.ctx, 1)
            t0 = time.perf_counter()
            out = emit()
            el = time.perf_counter() - t0
            c, ms = c_uint64(0), c_double(0)
            N.lib().kman_timing_query(dev.ctx, b"format", byref(c), byref(ms))
            N.lib().kman_timing_enable(dev.ctx, 0)
            res["%s_%s_s" % (mode, fmt)] = round(el, 3)
            if fmt == "device":
                res["%s_kernel_ms" % mode] = round(ms.value, 2)
                res["%s_kernel_launches" % mode] = c.value
            if out is not None:
                res["%s_bytes" % mode] = len(out)
            print(mode, fmt, el, file=sys.stderr, flush=True)
            del out
        for b in ((r.ukeys, r.counts) if mode == "count" else (r.keys, r.pos)):
            b.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
