#!/usr/bin/env python3
"""Bench lines for the inputs outside the headline config (VERDICT r01 item 7
/ BASELINE configs 3 and 5), each timed on the device from codes already in
HBM (parse + count / uniq), results device-resident:

  config3   10 GB synthetic FASTA, k = 31, count (kman_groups takes k <= 32
            count items; > 1 G k-mers go through the key rounds, dist.local_groups)
  rc1g      1 GB synthetic FASTA, k = 21, count -r (2 G k-mers: key rounds)
  grch38    GRCh38-shaped synthetic (inputs.grch38_like: N runs, soft-masking,
            repeats, satellites), k = 21, canonical count + abundance spectrum,
            then the spectrum alone (count rows as a multiset)
  grch38s   the same on inputs.grch38_skewed (a ~1 M-copy 10 %-diverged
            Alu-like family, Mbp satellite arrays, poly-A runs, N gaps)
  grch38s_spectrum   its spectrum line alone
  grch38u   the grch38 spectrum line alone

Each line: k-mers/s, ms per step, the path taken and rounds.  Usage:
widebench.py [config3|rc1g|grch38 ...] [--steps N] [--gb G]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import numpy as np  # noqa: E402

import inputs  # noqa: E402
from kman_amd import dist, engine, shard  # noqa: E402


def run(name, dev, text_reader, k, mode, rc=False, canonical=False, steps=3, hist=False, ordered=True):
    t0 = time.time()
    sp = shard.shard_specs(text_reader, 1, k)[0]
    ld = shard.ShardLoader(dev, text_reader, sp, k, chunk_bytes=1 << 30)
    sh = ld.load()
    names = sh.names
    off = np.concatenate([[0], np.cumsum([len(x) for x in names])]).astype(np.uint64)
    p = engine.Parsed(dev, sh.codes, sh.n_own, len(names), np.zeros(len(names), np.uint64), sh.rec_seq, names,
                      b"".join(names), off)
    print("%s: %.2f GB loaded + parsed in %.1f s" % (name, text_reader.size / 1e9, time.time() - t0), file=sys.stderr,
          flush=True)
    times, n_k, n_out, path = [], 0, 0, None
    from ctypes import byref, c_uint64

    from kman_amd import _native as N
    fl = engine.flags_for(rc, mode == "uniq", canonical)
    fm = N.KMAN_FINISH_UNIQ if mode == "uniq" else N.KMAN_FINISH_COUNT
    in_groups = N.lib().kman_groups_plan(p.n_bases, k, fl, fm, byref(c_uint64(0))) == N.KMAN_OK
    # outside kman_groups: the key rounds with their buffers held across
    # steps (as bench.py holds ResidentPipeline's)
    lr = None if in_groups else dist.LocalRounds(p, k, rc, mode, canonical, ordered=ordered)
    tags = ("region_extract", "region_pass", "region_pass1b", "region_finish", "heavy_sample", "left_gather",
            "extract_marked", "extract", "sort_pass", "sort_hist", "heavy_fix")
    if lr is not None:
        lr.pipe.timing(True)
    for s in range(steps + 1):
        dev.sync()
        t = time.perf_counter()
        if lr is not None:
            lr.step()
            r = lr.result()
        elif mode == "count":
            r = engine.count_groups(p, k, rc, canonical, ordered=ordered)
        else:
            r = engine.join_groups(p, k, rc, mode)
        h = None
        if hist and r is not None:
            from ctypes import c_void_p

            from kman_amd import _native as N
            d_h = dev.alloc(8 * 10001)
            N.check(dev.ctx, N.lib().kman_count_hist(dev.ctx, c_void_p(r.counts.ptr), r.count_bytes, r.n,
                                                     c_void_p(d_h.ptr), 10001), "hist")
            h = dev.download(d_h, 10001, np.uint64)
            d_h.free()
        dev.sync()
        el = time.perf_counter() - t
        if s:
            times.append(el)
        if r is not None:
            n_out = r.n
            vals = r.counts if mode == "count" else r.pos
            vb = r.count_bytes if mode == "count" else r.pos_bytes
            if mode == "count":
                n_k = int(dev.download(vals, r.n, np.uint32 if vb == 4 else np.uint64).sum(dtype=np.uint64))
            if lr is None:
                engine.free_result(r)
    path = "kman_groups" if in_groups else "key rounds (dist.LocalRounds)"
    if lr is not None:
        dist.LAST_LOCAL.clear()
        dist.LAST_LOCAL.update(rounds=lr.pipe.rounds, fallback_rounds=lr.pipe.fallback_rounds,
                               partial_rounds=lr.pipe.partial_rounds, redone_kmers=lr.pipe.redone_kmers,
                               heavy_keys=lr.pipe.heavy_keys,
                               plan=getattr(lr.pipe, "plan_info", None), phases_ms=dict(lr.pipe.phase_ms))
        kern = {t: lr.pipe.timed(t)[1] / (steps + 1) for t in tags}
        dist.LAST_LOCAL["kernels_ms_per_step"] = {t: round(v, 3) for t, v in kern.items() if v}
        lr.free()
    ms = 1e3 * sum(times) / len(times)
    out = {"line": name, "value": n_k / (ms / 1e3) if n_k else None, "unit": "k-mers/s", "ms_per_step": ms,
           "kmers": n_k, "rows": n_out, "k": k, "mode": mode, "rc": rc, "canonical": canonical, "rows_in_key_order": ordered,
           "fasta_bytes": text_reader.size, "path": path,
           "note": "parse done once; a step = count/uniq of the resident codes to device-resident rows"}
    if h is not None:
        out["hist_head"] = {int(c): int(h[c]) for c in np.nonzero(h)[0][:8]}
    if path.startswith("key"):
        out["rounds"] = dict(dist.LAST_LOCAL)
    print(json.dumps(out), flush=True)
    ld.free()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lines", nargs="*", default=["rc1g", "grch38", "config3"])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--gb", type=float, default=10.0, help="config3 size")
    a = ap.parse_args()
    dev = engine.Device(0)
    for ln in a.lines:
        if ln == "config3":
            lay = inputs.SynthLayout(int(a.gb * 1e9), 2)
            run("config3: %.0f GB synthetic, k=31, count" % a.gb, dev, shard.SynthReader(lay), 31, "count",
                steps=a.steps)
        elif ln == "rc1g":
            lay = inputs.SynthLayout(1_000_000_000, 1)
            run("1 GB synthetic, k=21, count -r", dev, shard.SynthReader(lay), 21, "count", rc=True, steps=a.steps)
        elif ln in ("grch38", "grch38u"):
            t0 = time.time()
            text = inputs.grch38_like(38, n_bases=3_100_000_000, n_records=25)
            print("grch38-like generated in %.0f s" % (time.time() - t0), file=sys.stderr, flush=True)
            if ln == "grch38":
                run("GRCh38-shaped 3.1 Gbp synthetic, k=21, canonical count + hist", dev, shard.BytesReader(text), 21,
                    "count", canonical=True, steps=a.steps, hist=True)
            # config 5 asks for the spectrum only: the rows as a multiset (a
            # redone key range appended, not merged into key order)
            run("GRCh38-shaped 3.1 Gbp synthetic, k=21, canonical abundance spectrum (rows unordered)", dev,
                shard.BytesReader(text), 21, "count", canonical=True, steps=a.steps, hist=True, ordered=False)
            del text
        elif ln in ("grch38s", "grch38s_spectrum"):
            t0 = time.time()
            text = inputs.grch38_skewed(38, n_bases=3_100_000_000, n_records=25)
            print("grch38-skewed generated in %.0f s" % (time.time() - t0), file=sys.stderr, flush=True)
            if ln == "grch38s":
                run("GRCh38-skewed 3.1 Gbp synthetic (Alu family, satellite arrays, poly-A, N gaps), k=21, canonical "
                    "count + hist", dev, shard.BytesReader(text), 21, "count", canonical=True, steps=a.steps, hist=True)
            run("GRCh38-skewed 3.1 Gbp synthetic, k=21, canonical abundance spectrum (rows as a multiset, mixed "
                "keys)", dev, shard.BytesReader(text), 21, "count", canonical=True, steps=a.steps, hist=True,
                ordered=False)
            del text
    dev.close()


if __name__ == "__main__":
    main()
