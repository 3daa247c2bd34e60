#!/usr/bin/env python3
"""Summarise rocprofv3 output (kernel-trace stats + separate FETCH_SIZE and
WRITE_SIZE passes) into profiles/pmc_<tag>.json and profiles/pmc_sort_pass.json.

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
streaming read (MI355X_MICROARCH.md, HBM section), WRITE_SIZE counts them
exactly.  Usage: pmc_summary.py FETCH_DIR WRITE_DIR TAG [mode k bases]"""
import csv, collections, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(d, counter):
    f = os.path.join(d, "run_counter_collection.csv")
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def short(name):
    s = name.replace("(anonymous namespace)::", "")
    return s.split("(")[0] if "<" not in s.split("(")[0] else s[: s.index(">") + 1]


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
out = {}
for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, []), write.get(k, [])
    if not f or not w:
        continue
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    out[short(k)] = {"launches": len(f), "fetch_kib": fk, "write_kib": wk,
                     "hbm_bytes_per_launch": (2 * fk + wk) * 1024}
tag = sys.argv[3]
with open(os.path.join(ROOT, "profiles", "pmc_%s.json" % tag), "w") as fh:
    json.dump(out, fh, indent=1, sort_keys=True)
for k, v in out.items():
    print("%-60s %3d  fetch %12.0f KiB  write %12.0f KiB  hbm/launch %8.3f GB" % (
        k[:60], v["launches"], v["fetch_kib"], v["write_kib"], v["hbm_bytes_per_launch"] / 1e9))
if len(sys.argv) > 6:
    # every kernel of this workload, for bench.py's roofline traffic fields
    cur = dict(out)
    cur["_meta"] = {"mode": sys.argv[4], "k": int(sys.argv[5]), "bases": int(sys.argv[6]), "tag": tag}
    with open(os.path.join(ROOT, "profiles", "pmc_current.json"), "w") as fh:
        json.dump(cur, fh, indent=1, sort_keys=True)
    # the bench's roofline kernel: the region path's digit pass (rg_pass), else
    # the LSD onesweep pass
    for name in ("rg_pass", "onesweep_pass"):
        sp = [v for k, v in out.items() if name in k]
        if sp:
            best = max(sp, key=lambda v: v["launches"])
            with open(os.path.join(ROOT, "profiles", "pmc_sort_pass.json"), "w") as fh:
                json.dump({"mode": sys.argv[4], "k": int(sys.argv[5]), "bases": int(sys.argv[6]), "tag": tag,
                           "kernel": name, "hbm_bytes_per_launch": best["hbm_bytes_per_launch"]}, fh, indent=1)
            break
