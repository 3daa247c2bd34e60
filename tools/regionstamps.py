#!/usr/bin/env python3
"""Per-phase mean durations of the region kernels (KMAN_RG_STAMPS: one
s_memrealtime stamp per phase boundary per tile, printed by kman_groups).
Needs the diagnostic build: make -C kman_amd/csrc EXTRA=-DKMAN_RG_STAMPS OUT=../lib_stamps,
run with KMAN_LIB=kman_amd/lib_stamps/libkman.so."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import inputs  # noqa: E402
from kman_amd import engine  # noqa: E402

text = inputs.syn_numpy(1_000_000_000, 1)
dev = engine.Device(0)
pipe = engine.ResidentPipeline(dev, text, 21, mode=sys.argv[1] if len(sys.argv) > 1 else "uniq")
del text
pipe.step()
os.environ["KMAN_RG_STAMPS"] = "1"
pipe.step()
