"""The streaming kernels of the region path issue their stores back to back:
no `s_waitcnt vmcnt` between two stores of pass 0 or pass 1 (gfx950 counts
loads and stores in order, so such a wait makes each store wait for the last
one's write acknowledgement -- rg_extract had one per store until round 4,
3.29 vs 3.09 ms).  Compiles region.hip to gfx950 assembly (~30 s, CPU only)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or not shutil.which("c++filt"),
                    reason="needs hipcc")
def test_region_stores_not_serialised():
    import isa_waits
    got = isa_waits.kernel_waits(os.path.join(ROOT, "kman_amd", "csrc", "region.hip"))
    # (the 0-bit merge instance, rg_pass<..., ZB = true>, is left out: pass 1b
    # at N > 1 only; the compiler places its scatter's out-of-line branch
    # blocks after the store loop, where this linear scan reads their key
    # waits as waits after a store)
    hot = {k: v for k, v in got.items()
           if "rg_extract<" in k or ("rg_pass" in k and "false, true>" not in k)}
    assert len([k for k in hot if "rg_extract<" in k]) >= 8 and any("rg_pass" in k for k in hot)
    bad = {k: v for k, v in hot.items() if v[1]}
    assert not bad, bad
