"""kman_amd/phases.py: the wall-clock marks of the user-visible command
(bench.py's file_to_file_config2 breakdown), in a child process as bench.py
starts the CLI; without KMAN_PHASES nothing is written."""

from __future__ import annotations

import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import time
from kman_amd import phases
time.sleep(0.2)
phases.mark("file_read")
time.sleep(0.1)
phases.mark("step")
phases.mark("step")
"""


def test_phase_marks_written_at_exit(tmp_path):
    from kman_amd import phases

    out = tmp_path / "ph.json"
    env = dict(os.environ, KMAN_PHASES=str(out), KMAN_T0=repr(time.time()), PYTHONPATH=ROOT)
    subprocess.run([sys.executable, "-c", CHILD], check=True, env=env, cwd=ROOT)
    b = phases.breakdown(str(out))
    assert list(b) == ["interpreter+import", "file_read", "step", "exit"]
    assert b["interpreter+import"] > 0 and 0.18 < b["file_read"] < 2.0 and 0.08 < b["step"] < 2.0
    env.pop("KMAN_PHASES")
    out.unlink()
    subprocess.run([sys.executable, "-c", CHILD], check=True, env=env, cwd=ROOT)
    assert not out.exists()
