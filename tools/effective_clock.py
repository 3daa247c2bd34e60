#!/usr/bin/env python3
"""Effective shader clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE
run (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE counts GPU-busy cycles summed over
the 8 XCDs): GHz = GRBM_GUI_ACTIVE / 8 / the dispatch's duration.
usage: effective_clock.py DIR/run_counter_collection.csv > clock.json"""
import csv
import json
import sys
from collections import defaultdict

acc = defaultdict(lambda: [0, 0.0, 0.0])  # launches, grbm, ns
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    a = acc[r["Kernel_Name"]]
    a[0] += 1
    a[1] += float(r["Counter_Value"])
    a[2] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
out = {}
for k, (n, g, ns) in acc.items():
    if ns <= 0:
        continue
    out[k] = {"launches": n, "grbm_gui_active_avg": g / n, "avg_ms": ns / n / 1e6,
              "effective_clock_ghz": (g / n) / 8 / (ns / n)}
json.dump(out, sys.stdout, indent=1)
print()
