"""The bit-parallel window roll (kman_amd/csrc/rollfast.h, used by every
extraction kernel) against a per-base roll, on the host: random codes with
not-ACGT and record-start flags, k = 2..32, all four word alignments, and
the 8- and 16-byte vector reads roll() uses when the base is that aligned."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_rollfast_matches_per_base_roll(tmp_path):
    exe = str(tmp_path / "rollfast_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-o", exe,
                    os.path.join(HERE, "native", "rollfast_check.cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout + r.stderr
