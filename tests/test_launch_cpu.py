"""kman_amd/launch.py on the CPU: the launcher environment, the file reader
the ranks cut their byte ranges from, and the RCCL-id rendezvous (a fake id
maker: no GPU, no RCCL) across real processes, including a stale id file
left by an earlier launch."""

from __future__ import annotations

import gzip
import multiprocessing as mp
import os
import time

import pytest


def test_world_env(monkeypatch):
    from kman_amd import launch

    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "KMAN_DIST"):
        monkeypatch.delenv(v, raising=False)
    assert launch.world_env() == (1, 0, 0) and not launch.distributed() and launch.solo_rank()
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "2")
    monkeypatch.setenv("LOCAL_RANK", "2")
    assert launch.world_env() == (4, 2, 2) and launch.distributed() and not launch.solo_rank()
    monkeypatch.setenv("KMAN_DIST", "0")
    assert not launch.distributed()
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("KMAN_DIST", "1")
    assert launch.distributed()  # (forced at world size 1: the RCCL path with one rank)
    monkeypatch.setenv("RANK", "5")
    with pytest.raises(RuntimeError):
        launch.world_env()


@pytest.mark.parametrize("gz", [False, True])
def test_file_reader_cuts_like_bytes(tmp_path, gz):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import inputs
    from kman_amd import launch, shard

    text = inputs.messy_records(3, n_records=25, max_len=5000)
    p = tmp_path / ("in.fa.gz" if gz else "in.fa")
    if gz:
        with gzip.open(p, "wb") as fh:
            fh.write(text)
    else:
        p.write_bytes(text)
    rd = launch.FileReader(str(p))
    try:
        assert rd.size == len(text) and rd.read(-5, 10) == text[:10] and rd.read(len(text) - 3, 10 ** 9) == text[-3:]
        for G in (1, 3, 8):
            assert shard.shard_specs(rd, G, 13) == shard.shard_specs(shard.BytesReader(text), G, 13)
    finally:
        rd.close()
    e = tmp_path / "empty.fa"
    e.write_bytes(b"")
    rd = launch.FileReader(str(e))
    assert rd.size == 0 and rd.read(0, 10) == b""
    with pytest.raises(AssertionError):  # parsers.py:105-107, on every rank
        shard.shard_specs(rd, 2, 5)
    rd.close()


def _rank(rank, world, d, q, delay):
    from kman_amd import launch

    time.sleep(delay)
    uid = launch.rendezvous(rank, world, "t", make_uid=lambda: bytes([7]) * 100 + os.urandom(28), directory=d,
                            timeout=30)
    q.put((rank, uid))


def test_rendezvous_processes_and_stale_file(tmp_path):
    """Rank 0 writes the id; peers started before or after it read that id,
    never the stale one an earlier (crashed) launch left under the same key."""
    from kman_amd import launch

    d = str(tmp_path)
    stale = launch._id_path("t", d)
    with open(stale, "wb") as fh:  # an id file from a launch that started long ago
        import struct

        fh.write(launch._MAGIC + struct.pack("<d", time.time() - 3600) + b"\0" * 8 + b"\x01" * 128)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 4
    # peers start first (they must wait for rank 0's fresh id), rank 0 last
    ps = [ctx.Process(target=_rank, args=(r, world, d, q, 0.0 if r else 1.0)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=60) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    assert len(set(got.values())) == 1 and got[0][:100] == bytes([7]) * 100
    launch.remove_id("t", d)
    assert not os.path.exists(stale)


def test_rendezvous_back_to_back_relaunch(tmp_path, monkeypatch):
    """A launch that crashed seconds ago (its id file is fresh, so the
    start-time check alone would take it) is keyed by its own run id: a new
    launch on the same port never reads it."""
    import struct

    from kman_amd import launch

    d = str(tmp_path)
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.setenv("KMAN_RUN_ID", "old")
    stale = launch._id_path("t", d)
    with open(stale, "wb") as fh:
        fh.write(launch._MAGIC + struct.pack("<d", time.time()) + b"\0" * 8 + b"\x01" * 128)
    monkeypatch.setenv("KMAN_RUN_ID", "new")
    assert launch._id_path("t", d) != stale
    with pytest.raises(RuntimeError):  # no rank 0 of the new launch: the old id is not taken
        launch.rendezvous(1, 2, "t", make_uid=lambda: b"\2" * 128, directory=d, timeout=0.5)
    # under torch.distributed.run: its run id and restart count when the id
    # is a real one; the constant "none" keys nothing (start-time check only)
    monkeypatch.delenv("KMAN_RUN_ID")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "abc")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "2")
    assert launch.launch_nonce() == "abc-2"
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    assert launch.launch_nonce() == ""


def _wrapped_rank(rank, world, d, q, delay):
    # one more process between the "launcher" and the rank (a shell or a
    # wrapper script): every rank then has a parent of its own
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_rank, args=(rank, world, d, q, delay))
    p.start()
    p.join(timeout=60)


def test_rendezvous_ranks_with_different_parents(tmp_path, monkeypatch):
    """torchrun with a wrapper between the agent and Python
    (TORCHELASTIC_RUN_ID "none"): the ranks' parents differ, and they still
    meet on one id file."""
    from kman_amd import launch

    monkeypatch.delenv("KMAN_RUN_ID", raising=False)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    monkeypatch.setenv("MASTER_PORT", "29501")
    d = str(tmp_path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 3
    ps = [ctx.Process(target=_wrapped_rank, args=(r, world, d, q, 0.0 if r else 0.5)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=90) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    assert len(got) == world and len(set(got.values())) == 1
    launch.remove_id("t", d)


def test_cli_leaves_solo_work_to_rank_zero(tmp_path, monkeypatch):
    """Outside the multi-GPU domain (k > 32 here), ranks other than 0 leave
    without touching the GPU or the output; k <= 1 still raises everywhere."""
    from click.testing import CliRunner

    from kman_amd.scripts.kmer import main

    src = tmp_path / "in.fa"
    src.write_bytes(b">a\nACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGT\n")
    out = tmp_path / "o.txt"
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    r = CliRunner().invoke(main, ["count", str(src), str(out), "40"])
    assert r.exit_code == 0, r.output
    assert not out.exists()
    r = CliRunner().invoke(main, ["batch", str(src), str(tmp_path / "bd"), "5"])
    assert r.exit_code == 0 and not (tmp_path / "bd").exists()
    r = CliRunner().invoke(main, ["count", str(src), str(out), "1"])
    assert isinstance(r.exception, AssertionError)


def _gz_rank(rank, world, path, d, q, chunk):
    import hashlib
    import resource

    from kman_amd import launch, shard

    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024
    rd = launch.FileReader(path, world, rank, directory=d, timeout=120)
    spec = shard.shard_specs(rd, world, 21)[rank]
    h = hashlib.sha256()
    for lo in range(spec.start, spec.halo_end, chunk):  # the loader's chunked reads
        h.update(rd.read(lo, min(spec.halo_end, lo + chunk)))
    peak = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024 - rss0
    q.put((rank, spec.start, spec.halo_end, h.hexdigest(), peak, rd.size))
    # rank 0 keeps its reader (and the temp file) until every peer has read
    time.sleep(3.0 if rank == 0 else 0.0)
    rd.close()


def test_gzip_input_inflated_once_and_memory_mapped_by_every_rank(tmp_path):
    """A gzipped FASTA under a 4-rank launch: rank 0 inflates it once into a
    shared temp file, every rank maps it and reads only its byte range; each
    rank's peak RSS grows by at most 1.5x its shard, the shards are the plain
    file's bytes, and the temp file is gone once rank 0 closes its reader."""
    import hashlib

    import numpy as np

    from kman_amd import shard

    rng = np.random.default_rng(5)
    recs = []
    for r in range(24):  # ~10 MB records of 80-column lines
        seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 10_000_000)].tobytes()
        recs.append(b">rec%d some description\n" % r + b"\n".join(seq[i:i + 80] for i in range(0, len(seq), 80)) + b"\n")
    text = b"".join(recs)
    gz = tmp_path / "big.fa.gz"
    with gzip.open(gz, "wb", compresslevel=1) as fh:
        fh.write(text)
    world, chunk = 4, 16 << 20
    specs = shard.shard_specs(shard.BytesReader(text), world, 21)
    d = str(tmp_path / "tmp")
    os.mkdir(d)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gz_rank, args=(r, world, str(gz), d, q, chunk)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(world):
        rank, lo, hi, digest, peak, size = q.get(timeout=300)
        got[rank] = (lo, hi, digest, peak, size)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    del recs
    for r, s in enumerate(specs):
        lo, hi, digest, peak, size = got[r]
        assert size == len(text) and (lo, hi) == (s.start, s.halo_end)
        assert digest == hashlib.sha256(text[lo:hi]).hexdigest()
        assert peak <= 1.5 * (hi - lo), (r, peak, hi - lo)
    assert os.listdir(d) == []


def test_nonce_from_torchrun_log_dir(monkeypatch):
    """torch.distributed.run with the default run id "none": the workers of one
    launch share its per-launch log directory (TORCHELASTIC_ERROR_FILE =
    <dir>/<run id>_<random>/attempt_<n>/<local rank>/error.json), so the id
    file is keyed by it -- and a later launch has another."""
    from kman_amd import launch

    monkeypatch.delenv("KMAN_RUN_ID", raising=False)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    base = "/tmp/torchelastic_ab12/none_x9y8/attempt_0/%d/error.json"
    monkeypatch.setenv("TORCHELASTIC_ERROR_FILE", base % 0)
    n0 = launch.launch_nonce()
    monkeypatch.setenv("TORCHELASTIC_ERROR_FILE", base % 3)
    assert launch.launch_nonce() == n0 and n0
    monkeypatch.setenv("TORCHELASTIC_ERROR_FILE", "/tmp/torchelastic_cd34/none_q1w2/attempt_0/3/error.json")
    assert launch.launch_nonce() != n0
    monkeypatch.setenv("TORCHELASTIC_ERROR_FILE", "")  # (logs to /dev/null: nothing to key on)
    assert launch.launch_nonce() == ""


def _gz_peer(path, d, q):
    from kman_amd import launch

    t0 = time.time()
    try:
        launch.FileReader(path, 2, 1, directory=d, timeout=120)
        q.put(("ok", time.time() - t0))
    except RuntimeError as e:
        q.put((str(e), time.time() - t0))


def test_gzip_failure_reaches_the_peers_at_once(tmp_path, monkeypatch):
    """A corrupt gzip: rank 0 raises and writes a failure marker, so its peer
    raises with rank 0's error within seconds instead of waiting out its
    timeout (120 s here)."""
    from kman_amd import launch

    monkeypatch.setattr(launch, "_START", time.time())  # (this process plays a rank 0 started with its peer)

    gz = tmp_path / "bad.fa.gz"
    good = gzip.compress(b">a\n" + b"ACGT" * 100000 + b"\n")
    gz.write_bytes(good[:len(good) // 2] + b"\0" * 64 + good[-8:])  # truncated body, intact ISIZE trailer
    d = str(tmp_path / "tmp")
    os.mkdir(d)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_gz_peer, args=(str(gz), d, q))
    p.start()
    time.sleep(1.0)
    with pytest.raises(Exception):
        launch.FileReader(str(gz), 2, 0, directory=d, timeout=120)
    msg, dt = q.get(timeout=60)
    p.join(timeout=30)
    assert msg != "ok" and "failed to decompress" in msg and dt < 30
    assert not [f for f in os.listdir(d) if not f.endswith(".done")]
