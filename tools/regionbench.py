#!/usr/bin/env python3
"""Stage timings of the region path (kman_groups) with timing ablations
(KMAN_RG_DBG, region.hip): 1 = finish without its LDS sort passes, 2 = finish
without output writes, 4 = finish without look-back (regions placed in
completion order), 8 = finish on synthetic items (no HBM reads), 16 = rg_pass
without look-back, 256 = rg_extract
without look-back.  Results of ablated
runs are wrong by construction; only their timings are read."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import inputs  # noqa: E402
from kman_amd import engine  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "uniq"
text = inputs.syn_numpy(1_000_000_000, 1)
dev = engine.Device(0)
pipe = engine.ResidentPipeline(dev, text, 21, mode=mode)
del text
for dbg in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "3", "16", "256", "0"]):
    if ":" in dbg:  # NAME=VALUE:dbg also sets another knob (empty VALUE = unset)
        kv, dbg = dbg.split(":")
        os.environ[kv.split("=")[0]] = kv.split("=")[1]
    os.environ["KMAN_RG_DBG"] = dbg
    pipe.step()
    pipe.timing(True)
    steps = 4
    for _ in range(steps):
        pipe.step()
    row = {}
    for tag in ("parse", "region_extract", "region_pass", "region_finish"):
        c, ms = pipe.timed(tag)
        row[tag] = round(ms / max(c, 1), 3)
    pipe.timing(False)
    print("dbg=%-3s %s" % (dbg, row), flush=True)
