"""Wall-clock phase marks of one process (the user-visible `kmer` command):
with ``KMAN_PHASES=<path>`` in the environment every ``mark(name)`` records
the time it was reached, and at exit the marks are written to <path> as JSON
(``KMAN_T0``: the launcher's time.time() just before it started the process,
so the first mark also gives interpreter start + imports).  Without
KMAN_PHASES a mark costs one dict lookup.  bench.py's file_to_file_config2
reads them into its per-phase breakdown."""

from __future__ import annotations

import atexit
import json
import os
import time

_PATH = os.environ.get("KMAN_PHASES")
_MARKS = []


def mark(name: str) -> None:
    if _PATH:
        _MARKS.append((name, time.time()))


def _dump() -> None:
    mark("exit")
    try:
        t0 = float(os.environ.get("KMAN_T0", "0") or 0) or None
        with open(_PATH, "w") as fh:
            json.dump({"t0": t0, "marks": _MARKS}, fh)
    except OSError:
        pass


def breakdown(path: str) -> dict:
    """Seconds per phase from a KMAN_PHASES file: each phase runs from the
    previous mark (the first from KMAN_T0) to its own mark; phases reached
    more than once are summed."""
    with open(path) as fh:
        d = json.load(fh)
    out, prev = {}, d.get("t0")
    for name, t in d["marks"]:
        if prev is not None:
            out[name] = round(out.get(name, 0.0) + t - prev, 4)
        prev = t
    return out


if _PATH:
    atexit.register(_dump)
