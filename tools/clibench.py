#!/usr/bin/env python3
"""The user-visible `kmer uniq|count` on BASELINE config 2's 1 GB FASTA,
process start to exit, with the per-phase wall times of kman_amd/phases.py:
usage: clibench.py [uniq|count] [runs] [dst]   (dst default /dev/null)."""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import inputs
    from kman_amd import phases

    mode = sys.argv[1] if len(sys.argv) > 1 else "uniq"
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dst = sys.argv[3] if len(sys.argv) > 3 else "/dev/null"
    fd, path = tempfile.mkstemp(suffix=".fa")
    with os.fdopen(fd, "wb") as fh:
        fh.write(inputs.syn_numpy(1_000_000_000, 1))
    try:
        for r in range(runs):
            fd2, ph = tempfile.mkstemp(suffix=".json")
            os.close(fd2)
            t0 = time.perf_counter()
            env = dict(os.environ, KMAN_PHASES=ph, KMAN_T0=repr(time.time()))
            subprocess.run([sys.executable, "-m", "kman_amd", mode, path, dst, "21"], check=True, cwd=ROOT, env=env,
                           stdout=subprocess.DEVNULL)
            dt = time.perf_counter() - t0
            b = phases.breakdown(ph)
            os.remove(ph)
            print("run %d: %.3f s  %s" % (r, dt, " ".join("%s=%.3f" % kv for kv in b.items())), flush=True)
    finally:
        os.remove(path)


if __name__ == "__main__":
    main()
