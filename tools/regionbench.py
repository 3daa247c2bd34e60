#!/usr/bin/env python3
"""Stage timings of the region path (kman_groups) on BASELINE config 2 (1 GB
synthetic FASTA, k=21): ms per launch of parse, rg_extract, rg_pass and
rg_finish over a few steps.  The round-1..3 timing ablations (KMAN_RG_DBG)
are gone with the variants they timed; compare builds instead
(KMAN_LIB=kman_amd/lib_ab_<name>/libkman.so, tools/ab/build_variants.sh).
usage: regionbench.py [uniq|count] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import inputs  # noqa: E402
from kman_amd import engine  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "uniq"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
text = inputs.syn_numpy(1_000_000_000, 1)
dev = engine.Device(0)
pipe = engine.ResidentPipeline(dev, text, 21, mode=mode)
del text
pipe.step()
pipe.timing(True)
for _ in range(steps):
    pipe.step()
row = {}
for tag in ("parse", "region_extract", "region_pass", "region_finish"):
    c, ms = pipe.timed(tag)
    row[tag] = round(ms / max(c, 1), 3)
pipe.timing(False)
print("%s %s" % (os.environ.get("KMAN_LIB", "kman_amd/lib/libkman.so"), row), flush=True)
