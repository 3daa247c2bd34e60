#!/usr/bin/env python3
"""Per-launch kernel durations from a rocprofv3 --kernel-trace csv directory,
beside the HIP-event stage times the bench line of the same process printed.

usage: kernel_launches.py TRACE_DIR BENCH_JSON [kernel substrings...]

For each kernel: every launch's duration (end - start, ns -> ms) in launch
order, and the average / minimum over the last `steps` launches (the bench's
timed loop: bench.py does `warmup` untimed steps, then `steps` timed ones,
one launch per kernel per step), against the bench's HIP-event stage time."""
import csv
import glob
import json
import os
import sys

STAGE = {"rg_extract": "region_extract", "rg_pass": "region_pass", "rg_finish": "region_finish"}


def main():
    d, bj = sys.argv[1], sys.argv[2]
    kerns = sys.argv[3:] or list(STAGE)
    bench = json.load(open(bj))
    steps = int(bench["steps"])
    stages = bench["config"].get("stages_ms_per_step", {})
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    out = {}
    for k in kerns:
        ls = [r for r in rows if k in r["Kernel_Name"]]
        ls.sort(key=lambda r: int(r["Start_Timestamp"]))
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ls]
        if not ms:
            continue
        timed = ms[-steps:]
        ev = stages.get(STAGE.get(k, ""), None)
        out[k] = {"launches_ms": [round(x, 4) for x in ms], "timed_avg_ms": sum(timed) / len(timed),
                  "timed_min_ms": min(timed), "all_avg_ms": sum(ms) / len(ms), "hip_event_ms": ev,
                  "rocprof_over_event": (sum(timed) / len(timed)) / ev if ev else None}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
