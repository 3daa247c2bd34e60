#!/usr/bin/env python3
"""Headline benchmark: k-mers/s extract+sort+join, k=21 synthetic FASTA.

N = 1 (BASELINE.json configs[1]): 1 GB synthetic FASTA (numpy PCG64 seed 1,
i.i.d. uniform ACGT, 80 columns, records of <= 256 Mbp named syn<i>), k=21,
``kmer uniq`` (extract + radix sort + join: keys that occur once, with their
header pos) as one device batch.  A "step" is one pass of the hot path over
the FASTA bytes already resident in HBM:
    parse -> rg_extract (windows scattered by the top 8 key bits into
    regions) -> rg_pass (per bucket, by the next 9 bits) -> rg_finish (one
    LDS block per region: sort the rest, run-length uniq, compacted output)
leaving the (k-mer, pos) rows device-resident.  ``value`` is that rate.
Reported beside it:
  * ``pinned_host``: the same step starting from pinned host bytes: chunked
    H2D copies on a copy stream overlapping the parse and the first region
    pass of the previous chunk (shard.StreamedPipeline), beside the serial
    variant and the plain H2D time of the text;
  * ``output``: device text formatting and the file write of a bounded
    slice of the rows, as rates and as ms extrapolated to all rows, beside
    the plain D2H rate (``output.d2h``) that bounds them;
  * ``file_to_file``: the CLI (`kmer count`) on a bounded FASTA file;
    ``file_to_file_config2``: the CLI (`kmer uniq`) on config 2's whole 1 GB
    FASTA into /dev/null and into a file;
  * ``roofline``: the dominant kernel of the step (largest stage), its
    algorithmic bytes per launch over its HIP-event duration, against the
    8 TB/s HBM peak; ``sort_pass_roofline``: the digit pass (the north star's
    >= 60 % bar); ``traffic`` from the committed rocprofv3 PMC passes;
  * ``cpu_baseline``: the C restatement of the reference algorithm
    (oracle/kman_oracle) on a bounded sample, 1 core and one process per
    core on the host's cores (count stated).

N > 1 (``python -m torch.distributed.run --nproc-per-node N bench.py --gpus
N``; or plain ``python bench.py --gpus N``, which starts the N rank processes
itself -- see ``spawn_ranks``; or ``--dist`` at N = 1): ONE global synthetic
FASTA of N x 1 GB (seed 1,
kman_synth_fasta / inputs.SynthLayout), byte-range sharded (each rank
generates its own bytes + halo on its GPU); per step every rank runs the
shard histogram, the key rounds (extraction into the send buffer, one RCCL
all-to-all of packed items over xGMI, per-bucket passes + LDS finish).  The
rendezvous is RCCL only: rank 0 writes the RCCL id to a file, the barrier and
the max-over-ranks time are RCCL collectives (no torch.distributed).
``--shard-gb 12.5`` gives the per-rank shape of BASELINE config 4
(100 GB over 8 GPUs).
"""

from __future__ import annotations

import argparse
import json
import os
import re
import shutil
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


def cgroup_cpu_quota(path: str = "/sys/fs/cgroup/cpu.max"):
    """The cgroup v2 CPU quota in CPUs (quota / period), None when unlimited
    or absent."""
    try:
        with open(path) as fh:
            q, per = fh.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def effective_cores(affinity: int, quota) -> int:
    """CPUs the process can actually keep busy: min(affinity, cgroup quota)."""
    if quota is None:
        return max(1, affinity)
    return max(1, min(affinity, int(quota + 0.5)))


def cpu_baseline(k: int, mode: str, target_s: float = 10.0) -> dict:
    """oracle/kman_oracle (C restatement of the reference algorithm) on a
    sample of the same synthetic workload scaled to ~target_s seconds: one
    process (1 core), then one process per core on independent samples of
    the same size (aggregate k-mers / wall time)."""
    import inputs

    exe = os.path.join(ROOT, "oracle", "kman_oracle")
    if not os.path.isfile(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    # the CPUs this process may run on (nproc shows the whole machine); the
    # effective count is capped by the cgroup CPU quota (the box's share)
    affinity = max(1, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1)
    quota = cgroup_cpu_quota()
    cores = effective_cores(affinity, quota)
    with tempfile.TemporaryDirectory() as d:
        def sample(nbases, seed):
            src = os.path.join(d, "s%d.fa" % seed)
            with open(src, "wb") as fh:
                fh.write(inputs.syn_numpy(nbases, seed))
            return src

        def run(srcs):
            t0 = time.perf_counter()
            ps = [subprocess.Popen([exe, mode, s, s + ".out", str(k), "-t"], stdout=subprocess.PIPE, text=True)
                  for s in srcs]
            outs = [p.communicate()[0] for p in ps]
            wall = time.perf_counter() - t0
            n = sum(int(re.search(r"kmers=(\d+)", o).group(1)) for o in outs)
            s = max(float(re.search(r"seconds=([0-9.]+)", o).group(1)) for o in outs)
            return n, s, wall

        n, s, _ = run([sample(2_000_000, 1)])
        nb = int(2_000_000 * max(1.0, min(32.0, target_s / max(s, 1e-3))))
        n1, s1, _ = run([sample(nb, 1)])
        # one process per core on independent samples; the total work is
        # bounded (8 x the 1-core sample) so many cores do not stretch the run
        nbp = max(1_000_000, min(nb // 2, 8 * nb // cores))
        srcs = [sample(nbp, 1 + i) for i in range(cores)]
        nP, _, wallP = run(srcs)
    return {"value": n1 / s1, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": "%d-base sample of the same generator (seed 1), %s k=%d, %d k-mers in %.2f s, 1 thread"
                      % (nb, mode, k, n1, s1),
            "all_cores": {"value": nP / wallP, "cores": cores, "affinity_cpus": affinity, "nproc": os.cpu_count(),
                          "cgroup_cpu_quota": quota,
                          "sample": "%d processes on independent %d-base samples (seeds 1..%d), %d k-mers in %.2f s "
                                    "wall" % (cores, nbp, cores, nP, wallP)}}


def pmc_traffic(kernel: str, mode: str, k: int, bases: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary of this workload (profiles/pmc_current.json), else None."""
    p = os.path.join(ROOT, "profiles", "pmc_current.json")
    if not os.path.isfile(p):
        return None
    with open(p) as fh:
        d = json.load(fh)
    meta = d.get("_meta", {})
    if meta.get("mode") != mode or meta.get("k") != k or meta.get("bases") != bases:
        return None
    # (summary names are rocprofv3's: "void rg_finish<2, unsigned int, true, false>")
    def base(n):
        return n.replace("void ", "", 1).split("<")[0].split("(")[0]

    hits = [v for n, v in d.items() if n != "_meta" and base(n) == kernel]
    return max(hits, key=lambda v: v["launches"])["hbm_bytes_per_launch"] if hits else None


def roofline(pipe, stages, steps, mode, k, bases):
    """(dominant-kernel roofline, digit-pass roofline) of the region path.
    Algorithmic bytes per k-mer: rg_extract 1 code read + 8 B
    item write; rg_pass 8 + 8; rg_finish 8 B item read + 12 B per output row
    (8 B key + 4 B count | pos)."""
    n, rows = pipe.n_kmers, pipe.n_out
    per = {"region_extract": ("rg_extract", 9.0 * n), "region_pass": ("rg_pass", 16.0 * n),
           "region_finish": ("rg_finish", 8.0 * n + 12.0 * rows)}

    def line(tag):
        kern, alg = per[tag]
        c, ms = pipe.timed(tag)
        avg = ms / max(c, 1) / 1e3
        a = alg / avg / 1e9
        return {"kernel": kern, "bound": "hbm", "achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": a / HBM_PEAK_GBS, "traffic": pmc_traffic(kern, mode, k, bases),
                "algorithmic_bytes_per_launch": alg, "avg_launch_ms": avg * 1e3, "launches_per_step": c // steps}

    dom = max(per, key=lambda t: stages.get(t, 0.0))
    return line(dom), line("region_pass")


class _CountingSink:
    """A sink that keeps nothing: the text reaches pinned host memory and is
    counted (the format + D2H pipeline's own rate)."""

    def __init__(self):
        self.n = 0

    def write(self, b):
        self.n += len(b)
        return len(b)


def output_lines(dev, pipe, k, mode, rows_max=100_000_000):
    """The output text of the first rows_max rows of the result through the
    pipelined writer (engine._format_dev: device formatting of slice i, D2H
    of slice i - 1 into a pinned stage on the copy stream, host copies of
    slice i - 2 by 8 threads): (a) into pinned host memory only, (b) into a
    file (pwrite into the page cache), then fsync.  Rates, and ms
    extrapolated to every row."""
    from kman_amd import engine

    m = min(pipe.n_out, rows_max)
    if m == 0:
        return None
    ob = pipe.count_bytes if mode == "count" else pipe.pos_bytes
    if mode == "count":
        res = engine.CountResult(pipe.out_keys, pipe.out_vals, ob, m, k)
        run = lambda sink: engine.format_count_dev(dev, res, sink)  # noqa: E731
    else:
        import numpy as np

        # the generator's record table: syn<i> of 256 Mbp each (inputs.syn_numpy)
        R = (pipe.n_bases + (256 << 20) - 1) // (256 << 20)
        names = [b"syn%d" % i for i in range(R)]
        off = np.concatenate([[0], np.cumsum([len(x) for x in names])]).astype(np.uint64)
        p = engine.Parsed(dev, None, pipe.n_bases, R, None, np.arange(R, dtype=np.uint64) * np.uint64(256 << 20),
                          names, b"".join(names), off)
        res = engine.UniqResult(pipe.out_keys, pipe.out_vals, ob, m, k)
        run = lambda sink: engine.format_uniq_dev(p, res, sink)  # noqa: E731
    cs = _CountingSink()
    run(cs)  # (warm: pinned stages, code objects)
    cs = _CountingSink()
    t0 = time.perf_counter()
    run(cs)
    t1 = time.perf_counter()
    nbytes = cs.n
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp"), delete=True) as fh:
        t2 = time.perf_counter()
        run(fh)
        fh.flush()
        t3 = time.perf_counter()
        os.fsync(fh.fileno())
        t4 = time.perf_counter()
        assert os.path.getsize(fh.name) == nbytes
    scale = pipe.n_out / m
    return {"rows": m, "text_bytes": nbytes, "format_ms": (t1 - t0) * 1e3 * scale,
            "format_gbs": nbytes / (t1 - t0) / 1e9,
            "file_ms": (t3 - t2) * 1e3 * scale, "file_gbs": nbytes / (t3 - t2) / 1e9,
            "fsync_ms": (t4 - t3) * 1e3 * scale, "write_ms": (t4 - t2) * 1e3 * scale,
            "write_gbs": nbytes / (t4 - t2) / 1e9,
            "note": "the first %d of %d rows through the pipelined writer (device formatting of slice i | D2H of "
                    "slice i-1 into a pinned stage on the copy stream | host copies of slice i-2): format_* = the "
                    "text reaching pinned host memory; file_* = the same into a file (8 pwrite threads, page "
                    "cache); write_* = file + fsync; ms scaled to all rows" % (m, pipe.n_out)}


def file_to_file(k: int, nbases: int = 100_000_000):
    """`kmer count IN OUT k` through the CLI on a bounded synthetic file."""
    import inputs

    with tempfile.TemporaryDirectory() as d:
        src, out = os.path.join(d, "in.fa"), os.path.join(d, "out.txt")
        with open(src, "wb") as fh:
            fh.write(inputs.syn_numpy(nbases, 3))
        t0 = time.perf_counter()
        subprocess.run([sys.executable, "-m", "kman_amd", "count", src, out, str(k)], check=True, cwd=ROOT,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        s = time.perf_counter() - t0
        size = os.path.getsize(out)
    n = nbases - k + 1
    return {"value": n / s, "unit": "k-mers/s", "seconds": s, "output_bytes": size,
            "sample": "%d-base FASTA, `python -m kman_amd count` k=%d, process start to output file closed "
                      "(includes interpreter + device init)" % (nbases, k)}


def d2h_probe(dev, total: int = 8 << 30) -> dict:
    """Device -> pinned host copies in the pipelined writer's own pattern
    (engine._format_dev without the formatting): slices of _FMT_SLICE bytes
    through two pinned stages on the copy stream (kman_copy_d2h_async into
    stage i % 2, then the wait for slice i - 1), `total` bytes, warm: the
    ceiling of any output line that leaves the GPU.  Also one whole 1 GiB
    copy, as earlier rounds reported it."""
    from ctypes import byref, c_void_p

    from kman_amd import _native as N
    from kman_amd import engine

    L = N.lib()
    sl = engine._FMT_SLICE
    bufs = [dev.alloc(sl) for _ in range(2)]
    stages = []
    try:
        for _ in range(2):
            hp = c_void_p()
            N.check(dev.ctx, L.kman_host_alloc(dev.ctx, byref(hp), sl), "kman_host_alloc")
            stages.append(hp)

        def sliced():
            last = None
            for i in range(total // sl):
                b = i % 2
                N.check(dev.ctx, L.kman_copy_d2h_async(dev.ctx, stages[b], c_void_p(bufs[b].ptr), sl, b),
                        "kman_copy_d2h_async")
                if last is not None:
                    N.check(dev.ctx, L.kman_copy_d2h_wait(dev.ctx, last), "kman_copy_d2h_wait")
                last = b
            N.check(dev.ctx, L.kman_copy_d2h_wait(dev.ctx, last), "kman_copy_d2h_wait")

        sliced()  # (warm: maps the pages)
        t0 = time.perf_counter()
        sliced()
        dt = time.perf_counter() - t0
    finally:
        for hp in stages:
            L.kman_host_free(dev.ctx, hp)
        for b_ in bufs:
            b_.free()
    nb1 = 1 << 30
    buf = dev.alloc(nb1)
    hp = c_void_p()
    N.check(dev.ctx, L.kman_host_alloc(dev.ctx, byref(hp), nb1), "kman_host_alloc")
    try:
        def once():
            N.check(dev.ctx, L.kman_copy_d2h_async(dev.ctx, hp, c_void_p(buf.ptr), nb1, 0), "kman_copy_d2h_async")
            N.check(dev.ctx, L.kman_copy_d2h_wait(dev.ctx, 0), "kman_copy_d2h_wait")

        once()
        t0 = time.perf_counter()
        for _ in range(3):
            once()
        d1 = (time.perf_counter() - t0) / 3
    finally:
        L.kman_host_free(dev.ctx, hp)
        buf.free()
    return {"bytes": total, "slice_bytes": sl, "ms": dt * 1e3, "gbs": total / dt / 1e9,
            "single_1gib_gbs": nb1 / d1 / 1e9,
            "note": "the writer's pattern: %d MiB slices through two pinned stages on the copy stream" % (sl >> 20)}


def file_to_file_config2(path: str, k: int, mode: str, text_bytes_est: int) -> dict:
    """`python -m kman_amd MODE IN OUT k` on config 2's whole 1 GB FASTA, what
    a kmermaid user runs (kmer_uniq.py:73-92 / kmer_count.py): process start
    to exit, into /dev/null (parse, sort, join, device formatting, D2H; no
    disk) and into a file (+ the page cache; when the disk has room)."""
    out = {}

    def run(dst, phases_out=None):
        from kman_amd import phases

        fd_, ph = tempfile.mkstemp(suffix=".json")
        os.close(fd_)
        try:
            t0 = time.perf_counter()
            env = dict(os.environ, KMAN_PHASES=ph, KMAN_T0=repr(time.time()))
            subprocess.run([sys.executable, "-m", "kman_amd", mode, path, dst, str(k)], check=True, cwd=ROOT,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env)
            dt = time.perf_counter() - t0
            if phases_out is not None:
                try:
                    phases_out.update(phases.breakdown(ph))
                except (OSError, ValueError, KeyError):
                    pass
            return dt
        finally:
            os.remove(ph)

    ph = {}
    s = run("/dev/null", ph)
    out["devnull"] = {"seconds": s, "phases_s": ph}
    d = os.environ.get("TMPDIR", "/tmp")
    free = shutil.disk_usage(d).free
    if free > 1.3 * text_bytes_est + (8 << 30):
        dst = os.path.join(d, "kman_cfg2_out.txt")
        try:
            ph2 = {}
            s2 = run(dst, ph2)
            out["file"] = {"seconds": s2, "output_bytes": os.path.getsize(dst), "gbs": os.path.getsize(dst) / s2 / 1e9,
                           "phases_s": ph2}
        finally:
            try:
                os.remove(dst)
            except OSError:
                pass
    else:
        out["file"] = {"skipped": "%.1f GB free in %s for ~%.1f GB of text" % (free / 1e9, d, text_bytes_est / 1e9)}
    out["note"] = ("`python -m kman_amd %s <1 GB FASTA> OUT %d`, process start to exit (interpreter, device init, "
                   "file read, H2D, the step, device formatting, D2H, write); phases_s: wall seconds from one mark "
                   "to the next (kman_amd/phases.py, KMAN_PHASES)" % (mode, k))
    return out


def extra_lines(args, dev, pipe, out, text, cfg2_path):
    """The non-quick lines after the headline: the same step from pinned host
    bytes, the 100 Mbp and config-2 file-to-file CLI lines (each recorded in
    `out`, an error string when it fails)."""
    from kman_amd import shard

    # the same step from pinned host bytes (chunked H2D overlapping the parse)
    rd = None
    try:
        rd = shard.PinnedReader(dev, text)
        buf = dev.alloc(rd.size + 64)
        from ctypes import c_void_p as _vp

        from kman_amd import _native as _N

        def _copy():  # one async copy on the copy stream (what the chunked loader issues)
            _N.check(dev.ctx, _N.lib().kman_copy_h2d_async(dev.ctx, _vp(buf.ptr), _vp(rd.ptr(0)), rd.size, 0),
                     "kman_copy_h2d_async")
            _N.check(dev.ctx, _N.lib().kman_copy_sync(dev.ctx), "kman_copy_sync")

        _copy()  # (warm: the first copy also maps the pages)
        t0 = time.perf_counter()
        _copy()
        h2d = time.perf_counter() - t0
        buf.free()
        lines = {}
        for ov in (True, False):
            sp_ = shard.StreamedPipeline(dev, rd, args.k, args.mode, chunk_bytes=args.chunk_mb << 20, overlap=ov)
            for _ in range(args.warmup):
                sp_.step()
            dev.sync()
            t0 = time.perf_counter()
            n = 0
            for _ in range(args.steps):
                n += sp_.step()
            dev.sync()
            lines[ov] = (n / (time.perf_counter() - t0), (time.perf_counter() - t0) / args.steps * 1e3)
            sp_.free()
        out["pinned_host"] = {"value": lines[True][0], "unit": "k-mers/s", "ms_per_step": lines[True][1],
                              "serial_value": lines[False][0], "serial_ms_per_step": lines[False][1],
                              "h2d_ms": h2d * 1e3, "h2d_gbs": rd.size / h2d / 1e9, "chunk_mb": args.chunk_mb,
                              "note": "step from pinned host bytes: %d MiB chunks copied on a copy stream; the "
                                      "parse and the region path's first pass (kman_groups_begin / _extract) "
                                      "of chunk i run behind the copy of chunk i + 1, pass 1 + finish after "
                                      "the last chunk (kman_groups_end); serial_* = the whole load, then "
                                      "kman_groups; h2d_ms = one warm async copy of the whole text on the "
                                      "copy stream" % args.chunk_mb}
    except Exception as e:
        out["pinned_host"] = {"error": repr(e)}
    finally:
        if rd is not None:
            rd.free()
    try:
        out["file_to_file"] = file_to_file(args.k)
    except Exception as e:
        out["file_to_file"] = {"error": repr(e)}
    try:
        o = out.get("output") or {}
        est = int(o.get("text_bytes", 0) * pipe.n_out / max(1, o.get("rows", 1))) if "rows" in o else 60 << 30
        if cfg2_path is None:
            raise RuntimeError("no room in TMPDIR for config 2's FASTA")
        out["file_to_file_config2"] = file_to_file_config2(cfg2_path, args.k, args.mode, est)
        f2 = out["file_to_file_config2"]
        for key in ("devnull", "file"):
            if "seconds" in f2.get(key, {}):
                f2[key]["kmers_per_s"] = out["config"]["kmers_per_step_per_gpu"] / f2[key]["seconds"]
    except Exception as e:
        out["file_to_file_config2"] = {"error": repr(e)}


def run_single(args):
    import numpy as np  # noqa: F401
    import inputs
    from kman_amd import engine, shard

    t0 = time.time()
    text = inputs.syn_numpy(args.bases, 1)
    log("generated %.2f GB FASTA in %.1f s" % (len(text) / 1e9, time.time() - t0))
    dev = engine.Device(0)
    pipe = engine.ResidentPipeline(dev, text, args.k, mode=args.mode, path=args.path)
    fasta_bytes = len(text)
    for _ in range(args.warmup):
        pipe.step()
    pipe.timing(True)
    dev.sync()
    t0 = time.perf_counter()
    kmers = 0
    for _ in range(args.steps):
        kmers += pipe.step()
    dev.sync()
    elapsed = time.perf_counter() - t0
    stages = {}
    for tag in ("parse", "region_extract", "region_pass", "region_finish", "kmer_hist", "extract_pass", "extract",
                "sort_hist", "sort_pass", "finish", "rle_count", "rle_uniq"):
        c, ms = pipe.timed(tag)
        if c:
            stages[tag] = round(ms / args.steps, 3)
    region = pipe.path == "region"
    dom, sp = roofline(pipe, stages, args.steps, args.mode, args.k, args.bases) if region else (None, None)
    out = {
        "metric": METRIC, "value": kmers / elapsed, "unit": "k-mers/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (numpy PCG64 seed 1, uniform ACGT, 80 col), HBM-resident at the start of a step",
        "config": {"workload": "%.2f GB synthetic FASTA, k=%d, extract+radix-sort+%s single batch"
                               % (fasta_bytes / 1e9, args.k, args.mode),
                   "fasta_bytes_per_gpu": fasta_bytes, "kmers_per_step_per_gpu": pipe.n_kmers, "k": args.k,
                   "mode": args.mode, "parallelism": "single", "path": pipe.path, "stages_ms_per_step": stages,
                   "value_scope": "FASTA bytes resident in HBM at the start of a step -> device-resident rows (the "
                                  "harness contract); SURVEY 8(d)'s pinned-host -> device-resident region is the "
                                  "pinned_host line, H2D included"},
        "roofline": dom, "sort_pass_roofline": sp, "cpu_baseline": None,
    }
    pipe.timing(False)
    if not args.quick:
        try:
            out["output"] = output_lines(dev, pipe, args.k, args.mode)
            d2h = d2h_probe(dev)
            out["output"]["d2h"] = d2h
            out["output"]["format_vs_d2h"] = out["output"]["format_gbs"] / d2h["gbs"]
        except Exception as e:  # reported, never fatal to the GPU number
            out["output"] = {"error": repr(e)}
    pipe.free()
    cfg2_path = None
    if not args.quick:
        try:
            # config 2's FASTA as a file, for the end-to-end CLI line below
            # (never fatal to the GPU number: any failure is reported in the
            # line, and the file is removed whatever happens)
            tdir = os.environ.get("TMPDIR", "/tmp")
            if shutil.disk_usage(tdir).free > 2 * len(text) + (1 << 30):
                fd, cfg2_path = tempfile.mkstemp(suffix=".fa", dir=tdir)
                with os.fdopen(fd, "wb") as fh:
                    fh.write(text)
            extra_lines(args, dev, pipe, out, text, cfg2_path)
        finally:
            if cfg2_path is not None:
                try:
                    os.remove(cfg2_path)
                except OSError:
                    pass
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.k, args.mode)
        except Exception as e:  # reported, never fatal to the GPU number
            out["cpu_baseline"] = {"error": repr(e)}
    emit(out)
    dev.close()


def dist_line(args, dev, world: int, rank: int, per: int, mode: str, canon: bool, reparse: bool, steps: int,
              warmup: int, tag: str, also_overlap: bool = False):
    """One multi-GPU measurement: ONE global synthetic FASTA of `per` bytes
    per rank, byte-range sharded; `warmup` untimed steps, then `steps` timed
    ones between barriers, max over ranks.  also_overlap: then the same
    pipeline with overlapped rounds (each round's all-to-all in pieces on the
    communication stream, piece s sorted while piece s + 1 is exchanged), one
    untimed step and `steps` timed ones -- the line's "overlapped" entry, so
    one N > 1 run settles which default is faster.  Returns rank 0's line
    (None on the other ranks); the pipeline is freed before it returns."""
    import numpy as np
    import inputs
    from kman_amd import dist, launch, shard

    lay = inputs.SynthLayout(per * world, 1)
    rd = shard.SynthReader(lay)
    uid = launch.rendezvous(rank, world, tag)
    t_setup = time.time()
    pipe = dist.DistPipeline(dev, rd, args.k, mode, world, rank, uid, chunk_bytes=1 << 30, reparse=reparse,
                             canonical=canon, ordered=not canon, exchange=args.exchange == "on")
    if rank == 0:
        launch.remove_id(tag)  # (every rank has joined the communicator)
    comm = pipe.comm
    rccl_ranks, rccl_rank = comm.count()
    log("rank %d (RCCL rank %d of %d): shard %d..%d (%.2f GB) generated + parsed on the device, setup %.1f s"
        % (rank, rccl_rank, rccl_ranks, pipe.spec.start, pipe.spec.own_end, (pipe.spec.own_end - pipe.spec.start) / 1e9,
           time.time() - t_setup))
    hist = [None]

    def one_step():
        n = pipe.step()
        if canon:  # config 5: the abundance spectrum of the global canonical counts, all-reduced
            hist[0] = comm.run(pipe.hist_gen(10001))
        return n

    def timed_steps(n):
        """n steps between barriers: (max elapsed over ranks, k-mers of all ranks)"""
        comm.allreduce(np.zeros(1, np.uint64))  # barrier
        dev.sync()
        t0 = time.perf_counter()
        kmers = 0
        for _ in range(n):
            kmers += one_step()
        dev.sync()
        elapsed = time.perf_counter() - t0
        el = comm.allgather(np.array([int(elapsed * 1e9)], np.uint64))
        tot = comm.allreduce(np.array([kmers], np.uint64))
        return float(el.max()) / 1e9, int(tot[0])

    try:
        for _ in range(warmup):
            one_step()
        setup_s = time.time() - t_setup
        pipe.timing(True)
        elapsed, total = timed_steps(steps)
        out = None
        if rank == 0:
            stages = {}
            for st in ("parse", "shard_hist", "region_extract", "exchange", "region_pass", "region_pass1b",
                       "region_finish", "extract", "sort_pass", "finish"):
                c, ms = pipe.timed(st)
                if c:
                    stages[st] = round(ms / steps, 3)
            dom, sp = dist_roofline(pipe, steps, mode, args.k, per, world, canon)
            stage_alg = {}
            for st, (kern, alg_step) in dist_stage_bytes(pipe, steps, mode).items():
                c, _ = pipe.timed(st)
                if c:
                    stage_alg[st] = {"kernel": kern, "alg_bytes_per_launch": alg_step / max(1, c // steps),
                                     "launches_per_step": c // steps}
            out = {"value": total / elapsed, "ms_per_step": elapsed / steps * 1e3, "steps": steps, "warmup": warmup,
                   "kmers_per_step": total // max(steps, 1), "rccl_ranks": rccl_ranks, "setup_s": round(setup_s, 2),
                   "fasta_bytes": lay.size, "fasta_bytes_per_rank": per, "path": pipe.path, "rounds": pipe.rounds,
                   "fallback_rounds": pipe.fallback_rounds, "partial_rounds": pipe.partial_rounds,
                   "memory_plan": getattr(pipe, "plan_info", None), "stages_ms_per_step_rank0": stages,
                   "stage_alg_bytes_rank0": stage_alg, "roofline": dom, "sort_pass_roofline": sp,
                   "spectrum_distinct": int(hist[0].sum()) if canon else None,
                   # the data path: the all-to-all runs on every rank at N > 1;
                   # at world 1 only with --exchange on (RCCL send/recv to self,
                   # the per-rank step the N > 1 run takes), else the rank
                   # extracts straight into its receive buffer / once for all
                   # rounds (a one-GPU-only shortcut)
                   "exchange": bool(pipe.exchanged_items),
                   "exchanged_bytes_per_step": 8 * pipe.exchanged_items,
                   "max_message_bytes": pipe.max_message,
                   "exchange_gbs_rank0": (8 * pipe.exchanged_items / (stages["exchange"] / 1e3) / 1e9
                                          if stages.get("exchange") else None)}
        if also_overlap:
            pipe.timing(False)
            pipe.overlap = True
            one_step()  # (untimed: the overlapped plan's arenas grow here)
            e2, t2 = timed_steps(steps)
            if rank == 0:
                out["overlapped"] = {"value": t2 / e2, "ms_per_step": e2 / steps * 1e3, "steps": steps,
                                     "overlapped_rounds": pipe.overlapped_rounds, "rounds": pipe.rounds,
                                     "pieces": pipe.pieces,
                                     "vs_sequential": (elapsed / steps) / (e2 / steps)}
            pipe.overlap = False
        comm.allreduce(np.zeros(1, np.uint64))  # every rank is done with this line
        return out
    finally:
        pipe.free()


def run_dist(args, world: int, rank: int, local: int):
    from kman_amd import engine

    dev = engine.Device(local)
    per = int(args.shard_gb * 1e9) if args.shard_gb else args.bases
    # the 1 GB-per-rank line keeps each rank's text in HBM and parses it in
    # every step (the single-GPU step's scope); config 4's 12.5 GB shards
    # stream through two 1 GiB staging buffers, parsed once at setup
    reparse = args.shard_gb is None
    canon = args.canonical
    if canon and args.mode != "count":
        raise SystemExit("--canonical counts (config 5): use --mode count")
    # N > 1: each line also timed with overlapped rounds (opt-in in the
    # product until an N > 1 run shows which is faster)
    ov = world > 1 and not canon
    ln = dist_line(args, dev, world, rank, per, args.mode, canon, reparse, args.steps, args.warmup, "bench",
                   also_overlap=ov)
    # BASELINE config 4 (100 GB synthetic FASTA, k=21, N GPUs): after the
    # weak-scaling line, the same job at 100 / N GB per rank, count mode,
    # parsed at setup -- so the driver's plain `--gpus N` run measures it too
    sub = None
    if world > 1 and args.config4 and args.shard_gb is None and not canon:
        per4 = int(100e9 / world)
        sub = dist_line(args, dev, world, rank, per4, "count", False, False, args.config4_steps, 1, "bench4",
                        also_overlap=ov)
    dev.close()
    if rank == 0:
        out = {
            "metric": METRIC, "value": ln["value"], "unit": "k-mers/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ln["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic: ONE global FASTA (kman_synth_fasta seed 1, uniform ACGT, 80 col) of %d x %.2f GB, "
                    "byte-range sharded, each rank's bytes generated in its HBM; a step = %s shard histogram + key "
                    "rounds" % (world, per / 1e9, "parse of the resident text +" if reparse else "(parsed at setup)"),
            "config": {"workload": "%.2f GB synthetic FASTA in %d byte-range shards of %.2f GB per rank, k=%d, "
                                   "extract+radix-sort+%s, key rounds%s%s"
                                   % (ln["fasta_bytes"] / 1e9, world, per / 1e9, args.k,
                                      "canonical count + all-reduced abundance spectrum (config 5's pipeline)"
                                      if canon else args.mode,
                                      (" + one all-to-all per round (kman_alltoallv: RCCL send/recv between "
                                       "ranks, each rank's own part a device-to-device copy%s)"
                                       % ("; at one rank the whole exchange is that copy"
                                          if world == 1 and os.environ.get("KMAN_RCCL_SELF") != "1" else
                                          "; KMAN_RCCL_SELF=1: the own part through RCCL too"
                                          if os.environ.get("KMAN_RCCL_SELF") == "1" else ""))
                                      if ln.get("exchange") else
                                      " without an exchange (one rank, --exchange off: a one-GPU-only shortcut, "
                                      "not the per-rank step of an N > 1 run)",
                                      "" if not canon else "; the synthetic input stands in for GRCh38"),
                       "exchange": ln.get("exchange"), "exchanged_bytes_per_step": ln.get("exchanged_bytes_per_step"),
                       "max_message_bytes": ln.get("max_message_bytes"),
                       "exchange_gbs_rank0": ln.get("exchange_gbs_rank0"), "overlapped": ln.get("overlapped"),
                       "canonical": canon, "spectrum_distinct": ln["spectrum_distinct"],
                       "fasta_bytes": ln["fasta_bytes"], "fasta_bytes_per_rank": per,
                       "kmers_per_step": ln["kmers_per_step"], "k": args.k,
                       "mode": args.mode, "parallelism": "dp%d: top-8-bit bucket parts + RCCL all-to-all" % world,
                       "rccl_ranks": ln["rccl_ranks"], "setup_s": ln["setup_s"],
                       "path": ln["path"], "rounds": ln["rounds"], "fallback_rounds": ln["fallback_rounds"],
                       "partial_rounds": ln["partial_rounds"], "memory_plan": ln["memory_plan"],
                       "stages_ms_per_step_rank0": ln["stages_ms_per_step_rank0"],
                       "stage_alg_bytes_rank0": ln["stage_alg_bytes_rank0"]},
            "roofline": ln["roofline"], "sort_pass_roofline": ln["sort_pass_roofline"], "cpu_baseline": None,
        }
        if sub is not None:
            out["config4"] = dict(sub, metric=METRIC, unit="k-mers/s", n_gpus=world,
                                  workload="BASELINE config 4: 100 GB synthetic FASTA, k=21, count, %d x %.2f GB "
                                           "byte-range shards, key rounds + RCCL all-to-all" % (world, 100.0 / world))
        # the C port on the host's cores, after every rank has left the GPU
        # work (the other ranks exit; the GPUs are idle while it runs)
        if not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.k, args.mode)
            except Exception as e:  # reported, never fatal to the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        emit(out)


def dist_pmc_traffic(kernel: str, mode: str, k: int, per_rank: int, canonical: bool, alg_bytes: float):
    """HBM bytes per launch of `kernel` on the multi-GPU path, from the
    committed world-1 PMC summary of the same per-rank workload
    (profiles/pmc_dist_current.json: HBM bytes and algorithmic bytes per
    launch there): that run's measured/algorithmic ratio times this launch's
    algorithmic bytes (at world 1: the measured bytes themselves).  None if
    no summary of this workload is committed."""
    p = os.path.join(ROOT, "profiles", "pmc_dist_current.json")
    if not os.path.isfile(p):
        return None
    with open(p) as fh:
        d = json.load(fh)
    m = d.get("_meta", {})
    if (m.get("mode"), m.get("k"), m.get("bases_per_rank"), bool(m.get("canonical"))) != (mode, k, per_rank,
                                                                                         canonical):
        return None
    e = d.get(kernel)
    if not e or not e.get("alg_bytes_per_launch"):
        return None
    return e["hbm_bytes_per_launch"] / e["alg_bytes_per_launch"] * alg_bytes


def dist_stage_bytes(pipe, steps: int, mode: str) -> dict:
    """Algorithmic HBM bytes per step of each region-path stage on this rank
    (multi-GPU rows): shard_hist 1 code read per base;
    rg_extract R code reads per base (every round re-rolls the shard) + 8 B
    per item sent; rg_pass and pass 1b 8 + 8 B per received item; rg_finish
    8 B per received item + 8 B key and the value (u32 count | u64 pos) per
    row."""
    sh = pipe.shard
    R = max(1, int(pipe.rounds or 1))
    vb = pipe._out[2] if getattr(pipe, "_out", None) else (4 if mode == "count" else 8)
    nb = float(sh.n_eff)
    return {"shard_hist": ("rg_hist", nb),
            "region_extract": ("rg_extract", R * nb + 8.0 * pipe.n_local),
            "region_pass": ("rg_pass", 16.0 * pipe.n_recv),
            "region_pass1b": ("rg_pass", 16.0 * pipe.n_recv),
            "region_finish": ("rg_finish", 8.0 * pipe.n_recv + (8.0 + vb) * pipe.n_out)}


def dist_roofline(pipe, steps: int, mode: str, k: int, per_rank: int, world: int, canonical: bool):
    """(dominant-stage roofline, digit-pass roofline) of rank 0's step: the
    stage with the most kernel time, its algorithmic bytes per launch over
    its HIP-event average launch time."""
    per = dist_stage_bytes(pipe, steps, mode)

    def line(tag):
        kern, alg_step = per[tag]
        c, ms = pipe.timed(tag)
        if not c:
            return None
        launches = max(1, c // steps)
        alg = alg_step / launches
        avg = ms / c / 1e3
        a = alg / avg / 1e9
        tr = dist_pmc_traffic(tag, mode, k, per_rank, canonical, alg)
        return {"kernel": "%s (%s, rank 0 of %d)" % (kern, tag, world), "bound": "hbm", "achieved": a,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": a / HBM_PEAK_GBS, "traffic": tr,
                "algorithmic_bytes_per_launch": alg, "avg_launch_ms": avg * 1e3, "launches_per_step": launches,
                "traffic_basis": None if tr is None else
                "profiles/pmc_dist_current.json: world-1 PMC bytes per algorithmic byte x this launch's "
                "algorithmic bytes"}

    timed = {t: pipe.timed(t)[1] for t in per}
    dom = max(timed, key=lambda t: timed[t])
    return line(dom), line("region_pass")


_RESULT_FD = None  # stdout as the driver sees it (main() points fd 1 at stderr)


def emit(out: dict) -> None:
    """The ONE JSON line, on the real stdout: libraries (RCCL prints a
    version banner at communicator init) only ever see fd 1 -> stderr."""
    line = (json.dumps(out) + "\n").encode()
    if _RESULT_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_RESULT_FD, line)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--mode", choices=["uniq", "count"], default="uniq")
    ap.add_argument("--bases", type=int, default=1_000_000_000, help="synthetic bases per GPU (1 GB FASTA)")
    ap.add_argument("--shard-gb", type=float, default=None, help="FASTA GB per rank on the multi-GPU path "
                                                                 "(12.5 = BASELINE config 4's shape)")
    ap.add_argument("--chunk-mb", type=int, default=128, help="chunk size of the pinned-host line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quick", action="store_true", help="HBM-resident line only (profiling runs)")
    ap.add_argument("--path", choices=["region", "split", "full"], default="region",
                    help="single-GPU engine path (region falls back to split outside its domain)")
    ap.add_argument("--dist", action="store_true", help="run the multi-GPU pipeline even at world size 1")
    ap.add_argument("--no-config4", dest="config4", action="store_false",
                    help="N > 1: skip the config-4 sub-line (100 GB / N per rank, count) after the main line")
    ap.add_argument("--config4-steps", type=int, default=3, help="timed steps of the config-4 sub-line")
    ap.add_argument("--exchange", choices=["on", "off"], default="on",
                    help="multi-GPU path at world 1: on (default) runs each round's all-to-all (RCCL send/recv to "
                         "self), i.e. the per-rank step of an N > 1 run; off extracts straight into the receive "
                         "buffer (for R > 1 rounds once for all of them: a one-GPU-only shortcut).  N > 1 always "
                         "exchanges")
    ap.add_argument("--canonical", action="store_true",
                    help="multi-GPU path: canonical k-mers + the all-reduced abundance spectrum (config 5; "
                         "with --mode count)")
    return ap.parse_args(argv)


def main() -> None:
    global _RESULT_FD
    sys.stdout.flush()
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)  # everything else printed to fd 1 (ours or a library's) goes to stderr
    args = parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.dist or args.canonical):
        # no launcher: start the ranks here (this process never touches the GPU)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d ranks (WORLD_SIZE)" % (args.gpus, world))
    if world > 1 or args.dist or args.canonical:
        run_dist(args, world, rank, local)
    else:
        run_single(args)


_COUNT_GPUS = r"""
import ctypes, sys
for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
    try:
        hip = ctypes.CDLL(name)
        break
    except OSError:
        hip = None
n = ctypes.c_int(0)
print(n.value if hip is not None and hip.hipGetDeviceCount(ctypes.byref(n)) == 0 else 0)
"""


def visible_gpus(timeout: float = 180.0) -> int:
    """GPUs visible to a rank, counted in a short-lived child process: the
    spawning process itself never initialises the GPU."""
    try:
        r = subprocess.run([sys.executable, "-c", _COUNT_GPUS], capture_output=True, text=True, timeout=timeout)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else 0
    except (subprocess.TimeoutExpired, ValueError, IndexError):
        return 0


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base: dict, world: int, rank: int, port: int, run_id: str) -> dict:
    """The launcher environment of rank `rank` (what torch.distributed.run
    sets: one process per GPU, LOCAL_RANK = the GPU)."""
    e = dict(base)
    e.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(world),
              "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "KMAN_RUN_ID": run_id})
    return e


def spawn_ranks(n: int, argv, cmd=None, gpus=None, poll_s: float = 0.2, grace_s: float = 10.0) -> int:
    """Run the N-rank benchmark without an external launcher: N child
    processes of this script (or `cmd`), each with WORLD_SIZE / RANK /
    LOCAL_RANK / MASTER_* set, started before this process makes any GPU
    call (it never makes one; it does not re-exec itself).  Rank 0's stdout
    (the JSON line) is passed to this process's result stream; the others'
    stdout goes to stderr.  Returns the exit status: non-zero, with a
    message, if fewer than N GPUs are visible or any rank fails (the other
    ranks are then terminated, by PID)."""
    import secrets
    import signal
    import threading

    have = visible_gpus() if gpus is None else gpus
    if have < n:
        log("bench.py: --gpus %d needs %d visible GPUs, %d visible; no result" % (n, n, have))
        return 2
    cmd = list(cmd) if cmd is not None else [sys.executable, os.path.abspath(__file__)]
    port, run_id = free_port(), secrets.token_hex(8)
    procs = []
    chunks = []

    def pump(fh):  # rank 0's stdout, read as it comes (no pipe back-pressure)
        for line in iter(fh.readline, b""):
            chunks.append(line)
        fh.close()

    reader = None
    try:
        for r in range(n):
            p = subprocess.Popen(cmd + list(argv), env=rank_env(os.environ, n, r, port, run_id),
                                 stdout=subprocess.PIPE if r == 0 else 2, stdin=subprocess.DEVNULL)
            procs.append(p)
            if r == 0:
                reader = threading.Thread(target=pump, args=(p.stdout,), daemon=True)
                reader.start()
        failed = None
        while failed is None:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.send_signal(signal.SIGTERM)
        t_end = time.time() + grace_s
        for p in live:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if reader is not None:
        reader.join(timeout=grace_s)
    if failed is not None:
        log("bench.py: rank %d of %d exited with status %d; no result" % (failed[0], n, failed[1]))
        return failed[1] if failed[1] > 0 else 1
    text = b"".join(chunks).decode(errors="replace")
    lines = [ln for ln in text.splitlines() if ln.strip().startswith("{")]
    if not lines:
        log("bench.py: rank 0 printed no result line")
        return 1
    emit(json.loads(lines[-1]))
    return 0


if __name__ == "__main__":
    main()
