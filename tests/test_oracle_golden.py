"""Pin the CPU oracle to the reference: every golden fixture in tests/golden/
(outputs of the reference itself, tests/golden/gen_golden.py) must be
reproduced byte for byte by oracle/kman_oracle.c.  CPU only."""

from __future__ import annotations

import hashlib
import os
import subprocess

import pytest

from conftest import GOLDEN, sha256_bytes


def _file_sha(path):
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def test_inputs_match_reference_inputs(manifest, golden_inputs):
    for name, sha in manifest["input_sha256"].items():
        if name.endswith(".gz"):
            continue  # gzip headers carry an mtime
        assert _file_sha(golden_inputs[name]) == sha, name


def _cases(manifest_key):
    import json

    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        m = json.load(fh)
    return m[manifest_key]


def _run_oracle(oracle_bin, cmd, inp, out, k, flags):
    return subprocess.run([oracle_bin, cmd, inp, out, str(k)] + list(flags), capture_output=True, text=True)


def _plain(path, tmp_path):
    if path.endswith(".gz"):
        import gzip

        p = str(tmp_path / "in.fa")
        with gzip.open(path, "rb") as fh, open(p, "wb") as out:
            out.write(fh.read())
        return p
    return path


@pytest.mark.parametrize("case", _cases("cases"), ids=lambda c: c["name"])
def test_oracle_matches_reference(case, golden_inputs, oracle_bin, tmp_path):
    assert case["result"]["ok"], case
    out = str(tmp_path / "out.txt")
    r = _run_oracle(oracle_bin, case["cmd"], _plain(golden_inputs[case["input"]], tmp_path), out, case["k"],
                    case["flags"])
    assert r.returncode == 0, r.stderr
    assert _file_sha(out) == case["sha256"]
    ref = os.path.join(GOLDEN, "ref_outputs", case["name"] + ".txt")
    if os.path.isfile(ref):
        with open(ref, "rb") as a, open(out, "rb") as b:
            assert a.read() == b.read()


@pytest.mark.parametrize("case", _cases("config1"), ids=lambda c: c["name"])
def test_oracle_config1(case, golden_inputs, oracle_bin, tmp_path):
    out = str(tmp_path / "out.txt")
    r = _run_oracle(oracle_bin, case["cmd"], golden_inputs[case["input"]], out, case["k"], [])
    assert r.returncode == 0, r.stderr
    assert _file_sha(out) == case["sha256"]


@pytest.mark.parametrize("case", _cases("batch_cases"), ids=lambda c: c["name"])
def test_oracle_batch_files(case, golden_inputs, oracle_bin, tmp_path):
    outdir = str(tmp_path / "batches")
    r = _run_oracle(oracle_bin, "batch", golden_inputs[case["input"]], outdir, case["k"], case["flags"])
    assert r.returncode == 0, r.stderr
    got = []
    for fn in sorted(os.listdir(outdir)):
        with open(os.path.join(outdir, fn)) as fh:
            got.append(fh.read())
    assert sorted(got) == case["files"]


EXIT = {"premature end of file or empty file": 3, "k must be >= 1": 2, "incompatible string": 4}


@pytest.mark.parametrize("case", _cases("error_cases"), ids=lambda c: c["name"])
def test_oracle_errors(case, golden_inputs, oracle_bin, tmp_path):
    out = str(tmp_path / "out.txt")
    r = _run_oracle(oracle_bin, case["cmd"], golden_inputs[case["input"]], out, case["k"], case["flags"])
    res = case["result"]
    if res["ok"]:
        assert r.returncode == 0
        return
    assert res["type"] == "AssertionError"
    code = [v for key, v in EXIT.items() if res["msg"].startswith(key)]
    assert code and r.returncode == code[0], (r.returncode, r.stderr, res)
    assert res["msg"] in r.stderr or res["msg"].split(":")[0] in r.stderr
    assert not case["output_created"] and not os.path.exists(out)


def test_oracle_batch_size_invariance(golden_inputs, oracle_bin, tmp_path):
    """outputs do not depend on -b."""
    outs = []
    for b in ("1", "7", "1000000"):
        out = str(tmp_path / ("o%s.txt" % b))
        r = _run_oracle(oracle_bin, "uniq", golden_inputs["messy2"], out, 5, ["-b", b, "-r"])
        assert r.returncode == 0
        with open(out, "rb") as fh:
            outs.append(sha256_bytes(fh.read()))
    assert len(set(outs)) == 1
