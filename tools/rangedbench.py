"""BASELINE config 3 timing: 10 GB synthetic FASTA (numpy PCG64 seed 2),
k=31, multi-batch device join (engine.ranged_groups: key ranges of at most
--max-keys k-mers, each extracted from the resident codes, prefix-sorted and
finished on the device).  Prints one JSON line: k-mers/s over the timed steps
(codes resident in HBM, buffers allocated once; range planning, extraction,
sort and join inside the timed region) and per-stage ms."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bases", type=int, default=10_000_000_000)
    ap.add_argument("--k", type=int, default=31)
    ap.add_argument("--mode", choices=["count", "uniq"], default="count")
    ap.add_argument("--max-keys", type=int, default=1_000_000_000, help="k-mers per batch (0: as HBM allows)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()

    import inputs
    from ctypes import byref, c_double, c_uint64

    from kman_amd import _native as N
    from kman_amd import engine

    t0 = time.time()
    text = inputs.syn_numpy(args.bases, 2)
    print("generated %.2f GB in %.1f s" % (len(text) / 1e9, time.time() - t0), file=sys.stderr, flush=True)
    dev = engine.Device(0)
    p = engine.parse(dev, text)
    fasta = len(text)
    del text
    mk = args.max_keys or None
    L = N.lib()

    t0 = time.time()
    job = engine.RangedJoin(p, args.k, False, args.mode, mk)
    print("planned + allocated in %.1f s" % (time.time() - t0), file=sys.stderr, flush=True)

    def step():
        job.step()
        return job.n_out

    for _ in range(args.warmup):
        step()
        print("warmup step done", file=sys.stderr, flush=True)
    N.check(dev.ctx, L.kman_timing_enable(dev.ctx, 1), "timing")
    dev.sync()
    t0 = time.perf_counter()
    outs = [step() for _ in range(args.steps)]
    dev.sync()
    el = time.perf_counter() - t0
    n, ranges = job.n_kmers, job.ranges
    stages = {}
    for tag in ("kmer_hist", "extract", "prefix_hist", "partition", "sort_hist", "sort_pass", "finish"):
        c, ms = c_uint64(0), c_double(0)
        N.check(dev.ctx, L.kman_timing_query(dev.ctx, tag.encode(), byref(c), byref(ms)), "timing")
        if c.value:
            stages[tag] = {"launches_per_step": c.value / args.steps, "ms_per_step": round(ms.value / args.steps, 2)}
    print(json.dumps({
        "metric": "k-mers/s extract+sort+join, config 3 (multi-batch device join)",
        "value": n * args.steps / el, "unit": "k-mers/s", "ms_per_step": el / args.steps * 1e3,
        "config": {"workload": "%.2f GB synthetic FASTA, k=%d, %s, key-range batches" % (fasta / 1e9, args.k, args.mode),
                   "kmers": n, "batches": len(ranges), "max_keys": job.max_keys, "n_out": outs[-1]},
        "stages": stages}), flush=True)
    job.free()
    p.free()


if __name__ == "__main__":
    main()
