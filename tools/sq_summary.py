#!/usr/bin/env python3
"""Print per-kernel SQ counter averages from rocprofv3 --pmc output dirs."""
import collections, csv, os, sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        print("missing", f)
        continue
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = name.split("(")[0][:70]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    print("==", k)
    for c, v in sorted(cs.items()):
        print("   %-24s %16.4g  (x%d)" % (c, sum(v) / len(v), len(v)))
