#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Runs only in the build container (it needs /root/reference, which never travels
to the GPU box).  The reference (kmermaid 1.0.0, pure Python) imports three
third-party modules that are not installed here:

* ``oligo_melting`` — an un-vendored git dependency
  (github.com/ggirelli/oligo-melting rev 301b2c8, version 2.0.1.post3;
  /root/reference/poetry.lock:290-310).  Only ``NATYPES``, ``AB_NA``,
  ``Sequence``, ``check_ab`` and ``mkrc`` are used on the k-mer path
  (kmermaid/seq.py:130,279,318).  The throw-away stand-in written below restates
  them with the semantics the reference's own tests pin
  (tests/test_seq.py:114,133-134,152-181): DNA alphabet "ACGT", complement
  "TGCA", ``check_ab`` = every char in the alphabet, ``mkrc`` = reverse +
  translate.  Whether the real alphabet admits N/IUPAC is *parity unpinned*
  (SURVEY §8c); the fixtures that contain N only pin the "skip" policy.
* ``Bio.SeqIO.FastaIO.SimpleFastaParser`` (biopython 1.79) — used only to
  re-read the reference's own temp batch files; restated here.
* ``h5py`` — imported by the out-of-scope abundance module only; empty stub.

The stand-ins live in a scratch directory outside the repo and are never
shipped.  Each case runs the reference CLI (``kmermaid.scripts.kmer:main``) in
its own subprocess from a scratch cwd with its own TMPDIR, with
PYTHONDONTWRITEBYTECODE=1 so nothing is written into /root/reference.

Usage:  python tests/golden/gen_golden.py [--quick]
"""

from __future__ import annotations

import argparse
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import textwrap
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import inputs  # noqa: E402

REFERENCE = "/root/reference"

STANDIN_OM = textwrap.dedent(
    '''
    from enum import Enum

    class NATYPES(Enum):
        DNA = 1
        RNA = 2

    AB_NA = {NATYPES.DNA: ["ACGT", "TGCA"], NATYPES.RNA: ["ACGU", "UGCA"]}

    class Sequence:
        def __init__(self, seq, t, name=None):
            assert t in NATYPES
            self.text = seq.upper()
            self.natype = t
            self.name = name
            self.ab = AB_NA[t]

        def __eq__(self, other):
            return self.text == other.text and self.natype == other.natype

        @staticmethod
        def check_ab(s, ab):
            return all(c in ab[0] for c in s)

        @staticmethod
        def mkrc(s, t):
            ab = AB_NA[t]
            return s[::-1].translate(str.maketrans(ab[0], ab[1]))
    '''
)

STANDIN_FASTAIO = textwrap.dedent(
    '''
    def SimpleFastaParser(handle):
        for line in handle:
            if line[0] == ">":
                title = line[1:].rstrip()
                break
        else:
            return
        lines = []
        for line in handle:
            if line[0] == ">":
                yield title, "".join(lines).replace(" ", "").replace("\\r", "")
                lines = []
                title = line[1:].rstrip()
                continue
            lines.append(line.rstrip())
        yield title, "".join(lines).replace(" ", "").replace("\\r", "")
    '''
)

RUNNER = textwrap.dedent(
    '''
    import json, sys, traceback
    from kmermaid.scripts.kmer import main
    try:
        main(sys.argv[1:], standalone_mode=False)
        print(json.dumps({"ok": True}))
    except BaseException as e:
        print(json.dumps({"ok": False, "type": type(e).__name__, "msg": str(e)}))
    '''
)


def make_standins(root: str) -> None:
    os.makedirs(os.path.join(root, "oligo_melting"))
    with open(os.path.join(root, "oligo_melting", "__init__.py"), "w") as fh:
        fh.write(STANDIN_OM)
    os.makedirs(os.path.join(root, "Bio", "SeqIO"))
    for sub in ("Bio", "Bio/SeqIO"):
        open(os.path.join(root, sub, "__init__.py"), "w").close()
    with open(os.path.join(root, "Bio", "SeqIO", "FastaIO.py"), "w") as fh:
        fh.write(STANDIN_FASTAIO)
    open(os.path.join(root, "h5py.py"), "w").close()
    dist = os.path.join(root, "kmermaid-1.0.0.dist-info")
    os.makedirs(dist)
    with open(os.path.join(dist, "METADATA"), "w") as fh:
        fh.write("Metadata-Version: 2.1\nName: kmermaid\nVersion: 1.0.0\n")
    with open(os.path.join(root, "runner.py"), "w") as fh:
        fh.write(RUNNER)


def run_reference(standins: str, argv: list, workdir: str, timeout: int = 240) -> dict:
    tmp = os.path.join(workdir, "tmp")
    os.makedirs(tmp, exist_ok=True)
    env = dict(os.environ)
    env["PYTHONPATH"] = standins + os.pathsep + REFERENCE
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    env["TMPDIR"] = tmp
    t0 = time.time()
    try:
        p = subprocess.run(
            [sys.executable, os.path.join(standins, "runner.py")] + argv,
            cwd=workdir,
            env=env,
            capture_output=True,
            text=True,
            timeout=timeout,
        )
    except subprocess.TimeoutExpired:
        shutil.rmtree(tmp, ignore_errors=True)
        return {"ok": False, "type": "timeout", "msg": "no result within %ds" % timeout}
    dt = time.time() - t0
    last = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    res = json.loads(last[-1]) if last else {"ok": False, "type": "crash", "msg": p.stderr[-2000:]}
    res["seconds"] = round(dt, 3)
    shutil.rmtree(tmp, ignore_errors=True)
    return res


def sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for chunk in iter(lambda: fh.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


# (case id, input id, subcommand, k, extra flags)
CASES_SMALL = []
for inp in ("edge", "messy1", "messy2"):
    for k in (2, 3, 5, 21):
        for cmd in ("count", "uniq"):
            for rc in (False, True):
                CASES_SMALL.append((inp, cmd, k, ["-r"] if rc else []))
for inp in ("messy1",):
    for k in (31, 32, 33, 40):
        for cmd in ("count", "uniq"):
            CASES_SMALL.append((inp, cmd, k, []))
for inp in ("syn64k_a", "syn64k_b"):
    for k in (21, 31):
        for cmd in ("count", "uniq"):
            for rc in (False, True):
                CASES_SMALL.append((inp, cmd, k, ["-r"] if rc else []))
# k > 32 (word-pair keys, k <= 64) and k > 64 (multi-word keys); round 3
for inp, cmd, k, extra in (("messy1", "count", 65, []), ("messy1", "uniq", 65, []), ("messy1", "count", 80, []),
                           ("messy1", "uniq", 80, []), ("messy2", "count", 33, ["-r"]), ("messy2", "uniq", 64, ["-r"]),
                           ("messy2", "count", 100, ["-r"]), ("messy2", "uniq", 127, [])):
    CASES_SMALL.append((inp, cmd, k, extra))
# batch-size invariance and gzip input
CASES_SMALL.append(("messy1", "count", 5, ["-b", "37"]))
CASES_SMALL.append(("messy1", "uniq", 5, ["-b", "37", "-r"]))
CASES_SMALL.append(("messy1.gz", "count", 5, []))

BATCH_CASES = [
    ("edge", 3, ["-b", "25"]),
    ("edge", 4, ["-b", "25", "-r"]),
    ("messy1", 5, ["-b", "500"]),
    ("messy2", 21, ["-b", "1000", "-r"]),
    # k > 32 batch files (round 3)
    ("messy1", 33, ["-b", "500"]),
    ("messy2", 40, ["-b", "1000", "-r"]),
    ("messy1", 70, ["-b", "300"]),
]

# VEC_COUNT_MASKED (round 4): the reference's add_count raises
# NotImplementedError at the first group whose records carry two names
# (join.py:311-335, abundance.py:60 via :123), else it writes the empty
# vector folder; k > 32 and k <= 32, with and without -r
VEC_CASES = [
    ("vecshare", 40, []),
    ("vecshare", 40, ["-r"]),
    ("vecshare", 21, []),
    ("vecsame", 40, []),
    ("vecsame", 21, ["-r"]),
    ("messy1", 40, []),
    ("messy2", 33, ["-r"]),
    ("edge", 5, []),
]

ERROR_CASES = [
    ("empty", "count", 3, []),
    ("noheader", "count", 3, []),
    ("edge", "count", 1, []),
    ("emptyname", "count", 3, []),
    ("emptyname_short", "count", 5, []),
]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="skip the 1 MB config-1 runs")
    ap.add_argument("--only-new", action="store_true",
                    help="keep the committed manifest and run only the cases it does not hold yet")
    args = ap.parse_args()
    if not os.path.isdir(REFERENCE):
        sys.exit("reference not present: fixtures can only be generated in the build container")

    scratch = tempfile.mkdtemp(prefix="kman_golden_")
    standins = os.path.join(scratch, "standins")
    make_standins(standins)
    inp_dir = os.path.join(scratch, "inputs")
    os.makedirs(inp_dir)
    paths = inputs.build_inputs(inp_dir)

    out_root = os.path.join(HERE, "ref_outputs")
    os.makedirs(out_root, exist_ok=True)
    manifest = {"cases": [], "batch_cases": [], "error_cases": [], "config1": [], "vec_cases": []}
    have = set()
    if args.only_new:
        with open(os.path.join(HERE, "manifest.json")) as fh:
            manifest = json.load(fh)
        manifest.setdefault("vec_cases", [])
        have = {e["name"] for part in ("cases", "batch_cases", "error_cases", "config1", "vec_cases")
                for e in manifest[part]}

    def case_name(inp, cmd, k, extra):
        tag = "".join(x.strip("-") for x in extra)
        return "%s__%s__k%d%s" % (inp.replace(".", "_"), cmd, k, ("__" + tag) if tag else "")

    for inp, cmd, k, extra in CASES_SMALL:
        name = case_name(inp, cmd, k, extra)
        if name in have:
            continue
        work = os.path.join(scratch, "w_" + name)
        os.makedirs(work)
        out = os.path.join(work, "out.txt")
        res = run_reference(standins, [cmd, paths[inp], out, str(k)] + extra, work)
        entry = {"name": name, "input": inp, "cmd": cmd, "k": k, "flags": extra, "result": res}
        if res["ok"]:
            dst = os.path.join(out_root, name + ".txt")
            shutil.copy(out, dst)
            entry["sha256"] = sha256(dst)
        manifest["cases"].append(entry)
        print(name, res, flush=True)

    for inp, k, extra in BATCH_CASES:
        name = case_name(inp, "batch", k, extra)
        if name in have:
            continue
        work = os.path.join(scratch, "w_" + name)
        os.makedirs(work)
        outdir = os.path.join(work, "batches")
        res = run_reference(standins, ["batch", paths[inp], outdir, str(k)] + extra, work)
        entry = {"name": name, "input": inp, "k": k, "flags": extra, "result": res}
        if res["ok"]:
            contents = []
            for fn in sorted(os.listdir(outdir)):
                with open(os.path.join(outdir, fn)) as fh:
                    contents.append(fh.read())
            entry["files"] = sorted(contents)
        manifest["batch_cases"].append(entry)
        print(name, res, len(entry.get("files", [])), flush=True)

    for inp, k, extra in VEC_CASES:
        name = case_name(inp, "vecmasked", k, extra)
        if name in have:
            continue
        work = os.path.join(scratch, "w_" + name)
        os.makedirs(work)
        out = os.path.join(work, "vec.out")
        res = run_reference(standins, ["count", paths[inp], out, str(k), "--count-mode", "VEC_COUNT_MASKED"] + extra,
                            work)
        folder = os.path.join(work, "vec")
        entry = {"name": name, "input": inp, "k": k, "flags": extra, "result": res,
                 "folder": sorted(os.listdir(folder)) if os.path.isdir(folder) else None}
        manifest["vec_cases"].append(entry)
        print(name, res, entry["folder"], flush=True)

    for inp, cmd, k, extra in ERROR_CASES:
        name = case_name(inp, cmd, k, extra)
        if name in have:
            continue
        work = os.path.join(scratch, "w_" + name)
        os.makedirs(work)
        out = os.path.join(work, "out.txt")
        res = run_reference(standins, [cmd, paths[inp], out, str(k)] + extra, work)
        entry = {"name": name, "input": inp, "cmd": cmd, "k": k, "flags": extra, "result": res,
                 "output_created": os.path.exists(out)}
        manifest["error_cases"].append(entry)
        print(name, res, flush=True)

    if not args.quick and not args.only_new:
        for cmd, k in (("count", 4), ("count", 21), ("uniq", 21)):
            name = "syn1m__%s__k%d" % (cmd, k)
            work = os.path.join(scratch, "w_" + name)
            os.makedirs(work)
            out = os.path.join(work, "out.txt")
            res = run_reference(standins, [cmd, paths["syn1m"], out, str(k)], work)
            entry = {"name": name, "input": "syn1m", "cmd": cmd, "k": k, "result": res}
            if res["ok"]:
                entry["sha256"] = sha256(out)
                with open(out, "rb") as fh:
                    entry["lines"] = sum(1 for _ in fh)
                if k == 4:
                    shutil.copy(out, os.path.join(out_root, name + ".txt"))
            manifest["config1"].append(entry)
            print(name, res, flush=True)

    manifest["input_sha256"] = {k: sha256(v) for k, v in paths.items()}
    manifest["generated_with"] = {
        "python": sys.version.split()[0],
        "reference": "kmermaid 1.0.0 @ /root/reference (read-only), stand-ins per SURVEY §8c",
    }
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    shutil.rmtree(scratch, ignore_errors=True)


if __name__ == "__main__":
    main()
