"""Shared fixtures: golden manifest, deterministic inputs, oracle binary."""

from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLDEN)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


# The uniq finish's early row count is checked on the device in every GPU
# test (KMAN_RG_CHECK=1: each singleton mark against the rows its sorted keys
# give; a disagreement fails the call).  The check costs 0.25-0.3 ms per 1 GB
# step (profiles/archive/r04a_check_ab.txt), so the product default is off; tests
# that pin the default kernel set KMAN_RG_CHECK=0 themselves.
os.environ.setdefault("KMAN_RG_CHECK", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    # `kmer count` declares -m twice, exactly as the reference CLI does
    # (arguments.py:104-115 and 134-149); click warns at every parse
    config.addinivalue_line("filterwarnings", "ignore:The parameter -m is used more than once")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def golden_inputs(tmp_path_factory):
    """Rebuild every golden input from its seed; check it against the sha256
    recorded when the reference ran on it."""
    import inputs

    d = tmp_path_factory.mktemp("inputs")
    paths = inputs.build_inputs(str(d))
    return paths


@pytest.fixture(scope="session")
def oracle_bin():
    exe = os.path.join(ROOT, "oracle", "kman_oracle")
    if not os.path.isfile(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return exe


def sha256_bytes(data: bytes) -> str:
    import hashlib

    return hashlib.sha256(data).hexdigest()
