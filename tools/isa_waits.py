#!/usr/bin/env python3
"""Stores the compiler serialised: per kernel of one HIP source, the global
stores and the `s_waitcnt vmcnt` that follow a store before the next barrier.
On gfx950 vmcnt counts loads and stores in order, so a vmcnt wait between two
stores of a loop makes each store wait for the previous one's write
acknowledgement (found in rg_extract, round 4: the region-cursor atomic's
return looked pending on the waves that skipped it; 3.29 -> 3.09 ms once
waited for once).  usage: isa_waits.py FILE.hip [filter] [-- extra hipcc flags]"""
import os
import re
import subprocess
import sys
import tempfile


def kernel_waits(src: str, extra=()) -> dict:
    """{demangled kernel: (stores, vmcnt waits after a store before the next
    barrier)} of `src` compiled for gfx950 as the Makefile does."""
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "--cuda-device-only", "-S", os.path.abspath(src), "-o", asm] + list(extra),
                       check=True, capture_output=True, cwd=os.path.dirname(os.path.abspath(src)))
        lines = open(asm).read().split("\n")
    res, kern, after = {}, None, False
    for line in lines:
        m = re.match(r"^(_Z\S+):", line)
        if m:
            kern, after = m.group(1), False
            res[kern] = [0, 0]
            continue
        if kern is None:
            continue
        t = line.strip()
        if t.startswith(("global_store", "buffer_store")):
            res[kern][0] += 1
            after = True
        elif t.startswith("s_waitcnt") and "vmcnt" in t and after:
            res[kern][1] += 1
        elif t.startswith(("s_barrier", "s_endpgm")):
            after = False
    names = list(res)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return {d: tuple(res[n]) for n, d in zip(names, dem)}


if __name__ == "__main__":
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    flt = args[1] if len(args) > 1 else ""
    for name, (st, w) in kernel_waits(args[0], extra).items():
        if flt in name and st:
            print(f"{name[:100]:100s} stores {st:4d} vmcnt-after-store {w:4d}")
