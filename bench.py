#!/usr/bin/env python3
"""Headline benchmark: k-mers/s extract+sort+join, k=21 synthetic FASTA.

Workload (BASELINE.json configs[1]): 1 GB synthetic FASTA (numpy PCG64 seed
1 + rank, i.i.d. uniform ACGT, 80 columns, records of <= 256 Mbp named
syn<i>), k=21, extract + radix sort + uniq (``kmer uniq``: keys and their
pos payload) as one device batch.  A "step" is one full pass of the hot path
over the FASTA bytes that are already resident in HBM:
    parse -> k-mer digit histograms -> extraction fused with the first prefix
    pass -> 2 more onesweep digit passes over the top 21 key bits -> finish
    (segments sorted in LDS + uniq, one pass)
leaving the (k-mer, header pos) result device-resident.  Text formatting and
the file write are not part of the step (reported separately by the CLI).

Prints ONE JSON line (rank 0).  ``roofline`` is measured live: the average
duration of the onesweep sort-pass kernel from HIP events recorded on the
engine's own stream around every launch in the timed steps.
``cpu_baseline`` times the C restatement of the reference algorithm
(oracle/kman_oracle, 1 thread) on a bounded sample of the same workload.

Multi-GPU: ``python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N``; every rank holds its own 1 GB shard (weak scaling).
"""

from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

METRIC = "k-mers/s extract+sort+join, k=21 synthetic FASTA, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(k: int, mode: str, target_s: float = 12.0) -> dict:
    """oracle/kman_oracle (C restatement, 1 thread) on a sample of the same
    synthetic workload; the sample is scaled to ~target_s seconds."""
    import inputs

    exe = os.path.join(ROOT, "oracle", "kman_oracle")
    if not os.path.isfile(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    with tempfile.TemporaryDirectory() as d:
        def run(nbases):
            src = os.path.join(d, "s.fa")
            with open(src, "wb") as fh:
                fh.write(inputs.syn_numpy(nbases, 1))
            r = subprocess.run([exe, mode, src, os.path.join(d, "o.txt"), str(k), "-t"], capture_output=True,
                               text=True, check=True)
            m = re.search(r"kmers=(\d+) seconds=([0-9.]+)", r.stdout)
            return int(m.group(1)), float(m.group(2))

        n, s = run(2_000_000)
        scale = max(1.0, min(32.0, target_s / max(s, 1e-3)))
        nb = int(2_000_000 * scale)
        n, s = run(nb)
    return {"value": n / s, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": "%d-base prefix-shaped sample of the same generator (seed 1), %s k=%d, %d k-mers in %.2f s"
                      % (nb, mode, k, n, s)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--mode", choices=["uniq", "count"], default="uniq")
    ap.add_argument("--bases", type=int, default=1_000_000_000, help="synthetic bases per GPU (1 GB FASTA)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", choices=["region", "split", "full"], default="region",
                    help="engine path (region falls back to split outside its domain)")
    ap.add_argument("--dist", action="store_true", help="run the multi-GPU pipeline even at world size 1")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo, host-side barrier / max only

        dist.init_process_group("gloo")

    import inputs
    from kman_amd import engine

    t0 = time.time()
    text = inputs.syn_numpy(args.bases, 1 + rank)
    log("rank %d: generated %.2f GB FASTA in %.1f s" % (rank, len(text) / 1e9, time.time() - t0))
    dev = engine.Device(local)
    if world > 1 or args.dist:
        # region path across ranks: one RCCL all-to-all of packed items over
        # xGMI (kman_amd/dist.py), prefix-range path as the fallback
        from kman_amd import dist as kd

        uid = [kd.unique_id() if rank == 0 else None]
        if dist:
            dist.broadcast_object_list(uid, src=0)
        pipe = kd.DistPipeline(dev, text, args.k, args.mode, world, rank, uid[0],
                               path="split" if args.path == "split" else "region")
    else:
        pipe = engine.ResidentPipeline(dev, text, args.k, mode=args.mode, path=args.path)
    fasta_bytes = len(text)
    del text

    for _ in range(args.warmup):
        pipe.step()
    pipe.timing(True)
    if dist:
        dist.barrier()
    dev.sync()
    t0 = time.perf_counter()
    kmers = 0
    for _ in range(args.steps):
        kmers += pipe.step()
    dev.sync()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist:
        import torch

        t = torch.tensor([elapsed, float(kmers)], dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, total_kmers = float(mx[0]), float(sm[1])
    else:
        total_kmers = float(kmers)

    # live roofline of the dominant kernel (the digit pass), from HIP events
    # recorded on the engine's own stream around every launch
    region = getattr(pipe, "path", "split") == "region"
    n_pass, pass_ms = pipe.timed("region_pass" if region else "sort_pass")
    stages = {}
    for tag in ("parse", "region_extract", "dist_gather", "region_pass", "region_pass1b", "region_finish", "kmer_hist",
                "extract_pass", "extract",
                "prefix_hist", "partition", "sort_hist", "sort_pass", "finish", "rle_count", "rle_uniq"):
        c, ms = pipe.timed(tag)
        if c:
            stages[tag] = round(ms / args.steps, 3)
    avg_pass_s = pass_ms / n_pass / 1e3
    # region path: one packed u64 item read + written per k-mer; LSD path: the
    # key read + written, plus the pos payload read + written (uniq)
    bytes_per_key = 16 if region else 16 + (2 * pipe.pos_bytes if args.mode == "uniq" else 0)
    achieved = bytes_per_key * pipe.n_sorted / avg_pass_s / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_sort_pass.json")
    if os.path.isfile(pmc):
        with open(pmc) as fh:
            p = json.load(fh)
        if (p.get("mode") == args.mode and p.get("k") == args.k and p.get("bases") == args.bases
                and p.get("kernel", "onesweep_pass") == ("rg_pass" if region else "onesweep_pass")):
            traffic = p.get("hbm_bytes_per_launch")

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    out = {
        "metric": METRIC,
        "value": total_kmers / elapsed,
        "unit": "k-mers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (numpy PCG64 seed 1+rank, uniform ACGT, 80 col)",
        "config": {
            "workload": "%.2f GB synthetic FASTA per GPU, k=%d, extract+radix-sort+%s single batch"
                        % (fasta_bytes / 1e9, args.k, args.mode),
            "fasta_bytes_per_gpu": fasta_bytes,
            "kmers_per_step_per_gpu": pipe.n_kmers,
            "k": args.k,
            "mode": args.mode,
            "parallelism": ("dp%d: top-8-bit bucket ranges + one RCCL all-to-all" % world
                            if world > 1 or args.dist else "single"),
            "path": getattr(pipe, "path", "dist"),
            "stages_ms_per_step": stages,
        },
        "roofline": {
            "kernel": ("rg_pass (per-bucket MSD digit pass over packed u64 items, %d per step)" if region else
                       "onesweep_pass (LSD digit pass, %d per step)") % (n_pass // args.steps),
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "algorithmic_bytes_per_key": bytes_per_key,
            "avg_launch_ms": avg_pass_s * 1e3,
        },
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.k, args.mode)
        except Exception as e:  # reported, never fatal to the GPU number
            out["cpu_baseline"] = {"error": repr(e)}
    print(json.dumps(out), flush=True)
    pipe.free()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
