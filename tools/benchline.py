#!/usr/bin/env python3
"""Print value / ms per step / stage times / roofline of a bench.py JSON line (stdin)."""
import json, sys
for line in sys.stdin:
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    c = d.get("config", {})
    print("value %.4g %s  ms/step %.3f  frac %s" % (d["value"], d["unit"], d["ms_per_step"],
                                                   d.get("roofline", {}).get("frac")))
    print("stages", c.get("stages_ms_per_step") or d.get("stages_ms_per_step"))
