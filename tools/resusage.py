#!/usr/bin/env python3
"""Per-kernel VGPRs / spills / LDS / occupancy of one HIP source for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage).  usage: resusage.py FILE.hip
[filter] [-- extra hipcc flags]"""
import re, subprocess, sys

args = sys.argv[1:]
extra = []
if "--" in args:
    i = args.index("--")
    args, extra = args[:i], args[i + 1:]
src = args[0]
flt = args[1] if len(args) > 1 else ""
p = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
                    "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + extra,
                   capture_output=True, text=True, cwd=None)
cur, rows = None, []
for line in p.stderr.splitlines():
    m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    key, val = m.group(1).strip(), m.group(2).strip()
    if key == "Function Name":
        cur = {"name": val}
        rows.append(cur)
    elif cur is not None:
        cur[key] = val
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    if flt and flt not in d:
        continue
    d = d.replace("(anonymous namespace)::", "")
    d = d[: d.index("(")] if "(" in d else d
    print("%-72s vgpr %4s spill %3s sgpr-spill %3s lds %6s occ %s" % (
        d[:72], r.get("VGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"), r.get("LDS Size [bytes/block]"),
        r.get("Occupancy [waves/SIMD]")))
if p.returncode:
    print(p.stderr[-3000:])
