"""The stable ranks of the LSD passes (rg_finish, kman_sort, the split path)
use same-word LDS atomics that return in lane order -- an observed property of
gfx950 that kman_create probes, not an architectural one.  KMAN_RANK=ballot
forces the probe-free ranking (ballot match-any); this runs the CLI outputs
in a child process under it (the setting is read once per context) and
requires them byte-identical to the C oracle's `kmer count|uniq` outputs, as
the default ranking's are (test_gpu_parity.py): either ranking alone gives
the reference's rows."""

from __future__ import annotations

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
from kman_amd import engine
text = open(sys.argv[2], "rb").read()
k, mode, rc, path, out = int(sys.argv[3]), sys.argv[4], sys.argv[5] == "1", sys.argv[6], sys.argv[7]
fn = engine.count_text if mode == "count" else engine.uniq_text
open(out, "wb").write(fn(text, k, rc, engine.default_device()))
"""


@pytest.mark.parametrize("path", ["region", "split"])
@pytest.mark.parametrize("mode,k,rc", [("count", 21, False), ("uniq", 13, True), ("count", 9, True), ("uniq", 25, False)])
def test_ballot_ranks_match_oracle(tmp_path, oracle_bin, mode, k, rc, path):
    import inputs

    text = inputs.syn_numpy(600_000, 7, record_len=150_000, width=63) + inputs.messy_records(9, n_records=20)
    src = tmp_path / "in.fa"
    src.write_bytes(text)
    want = tmp_path / "want.txt"
    subprocess.run([oracle_bin, mode, str(src), str(want), str(k)] + (["-r"] if rc else []), check=True)
    got = tmp_path / "got.txt"
    env = dict(os.environ, KMAN_RANK="ballot")
    if path == "split":
        env["KMAN_NO_REGION"] = "1"  # the general path: kman_extract_sorted + kman_finish
    subprocess.run([sys.executable, "-c", CHILD, ROOT, str(src), str(k), mode, "1" if rc else "0", path, str(got)],
                   env=env, check=True, timeout=300)
    assert got.read_bytes() == want.read_bytes()
