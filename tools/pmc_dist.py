#!/usr/bin/env python3
"""profiles/pmc_dist_current.json for bench.py's multi-GPU roofline traffic:
the world-1 multi-GPU bench line's rocprofv3 FETCH_SIZE and WRITE_SIZE passes
(HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024, the gfx950
FETCH_SIZE correction, as tools/pmc_summary.py) per stage, beside the stage's
algorithmic bytes per launch from the same line's JSON
(config.stage_alg_bytes_rank0).  usage: pmc_dist.py FETCH_DIR WRITE_DIR BENCH_JSON TAG"""
import collections, csv, json, os, sys


def load(d, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
bench = json.load(open(sys.argv[3]))
tag = sys.argv[4]
cfg = bench["config"]


def base(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    return n.split("<")[0].split("(")[0]


out = {"_meta": {"mode": cfg["mode"], "k": cfg["k"], "bases_per_rank": cfg["fasta_bytes_per_rank"],
                 "canonical": bool(cfg.get("canonical")), "world": bench["n_gpus"], "tag": tag}}
for stage, st in cfg["stage_alg_bytes_rank0"].items():
    f = [v for k, vs in fetch.items() if base(k) == st["kernel"] for v in vs]
    w = [v for k, vs in write.items() if base(k) == st["kernel"] for v in vs]
    if not f or not w:
        continue
    hbm = (2 * sum(f) / len(f) + sum(w) / len(w)) * 1024
    out[stage] = {"kernel": st["kernel"], "hbm_bytes_per_launch": hbm,
                  "alg_bytes_per_launch": st["alg_bytes_per_launch"], "ratio": hbm / st["alg_bytes_per_launch"]}
    print("%-16s %-10s hbm/launch %8.3f GB  alg %8.3f GB  ratio %.3f" % (
        stage, st["kernel"], hbm / 1e9, st["alg_bytes_per_launch"] / 1e9, hbm / st["alg_bytes_per_launch"]))
with open(os.path.join(ROOT, "profiles", "pmc_dist_%s.json" % tag), "w") as fh:
    json.dump(out, fh, indent=1, sort_keys=True)
with open(os.path.join(ROOT, "profiles", "pmc_dist_current.json"), "w") as fh:
    json.dump(out, fh, indent=1, sort_keys=True)
