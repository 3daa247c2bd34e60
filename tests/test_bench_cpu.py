"""bench.py's host logic on the CPU: the N-rank spawner (environment of each
rank, rank 0's line passed through, a failing rank ends the run with a
non-zero status and the others terminated), the refusal to report a 1-GPU
number for --gpus N when fewer GPUs are visible, and the effective core
count of the CPU baseline."""

from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

FAKE_RANK = r"""
import json, os, sys, time
env = {k: os.environ.get(k) for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                                      "KMAN_RUN_ID")}
mode = sys.argv[1]
rank = int(env["RANK"])
if mode == "fail" and rank == 1:
    time.sleep(0.5)
    sys.exit(3)
if mode == "fail":
    time.sleep(60)  # (a rank stuck in a collective: must be terminated)
with open(os.path.join(sys.argv[2], "rank%d.json" % rank), "w") as fh:
    json.dump(env, fh)
print("banner text a library printed")
if rank == 0:
    print(json.dumps({"metric": "m", "value": 1.0, "argv": sys.argv[1:]}))
"""


def _fake(tmp_path):
    p = tmp_path / "fake_rank.py"
    p.write_text(FAKE_RANK)
    return [sys.executable, str(p)]


def test_spawner_sets_each_rank_env_and_passes_rank0_line(tmp_path, capsys):
    rc = bench.spawn_ranks(3, ["ok", str(tmp_path)], cmd=_fake(tmp_path), gpus=8)
    assert rc == 0
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0])["argv"] == ["ok", str(tmp_path)]
    envs = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] and [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"} and {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and len({e["KMAN_RUN_ID"] for e in envs}) == 1


def test_spawner_failing_rank_terminates_the_others(tmp_path, capsys):
    t0 = time.time()
    rc = bench.spawn_ranks(3, ["fail", str(tmp_path)], cmd=_fake(tmp_path), gpus=8, grace_s=5)
    assert rc == 3 and time.time() - t0 < 30  # (rank 0 / 2 would sleep 60 s)
    assert capsys.readouterr().out.strip() == ""  # no result line
    assert not list(tmp_path.glob("rank*.json"))


def test_spawner_refuses_too_few_gpus(tmp_path, capsys):
    assert bench.spawn_ranks(4, ["ok", str(tmp_path)], cmd=_fake(tmp_path), gpus=2) != 0
    assert capsys.readouterr().out.strip() == "" and not list(tmp_path.glob("rank*.json"))


def test_bench_gpus_2_without_gpus_exits_nonzero():
    """`python bench.py --gpus 2` with no launcher and no visible GPU (this
    container) prints no result line and exits non-zero."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert "needs 2 visible GPUs" in r.stderr


def test_bench_rejects_gpus_mismatch_with_launcher():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr and r.stdout.strip() == ""


def test_effective_cores(tmp_path):
    assert bench.effective_cores(256, 16.0) == 16
    assert bench.effective_cores(8, 16.0) == 8
    assert bench.effective_cores(12, None) == 12
    assert bench.effective_cores(4, 0.2) == 1
    p = tmp_path / "cpu.max"
    p.write_text("1600000 100000\n")
    assert bench.cgroup_cpu_quota(str(p)) == 16.0
    p.write_text("max 100000\n")
    assert bench.cgroup_cpu_quota(str(p)) is None
    assert bench.cgroup_cpu_quota(str(tmp_path / "absent")) is None


class _FakePipe:
    """The attributes dist_roofline reads from a DistPipeline."""

    class _Shard:
        n_eff = 1_000_000_000

    def __init__(self):
        self.shard, self.rounds, self.n_local, self.n_recv, self.n_out = self._Shard(), 1, 999_999_980, 10 ** 9, 9 * 10 ** 8
        self._out = (None, None, 8)
        self.t = {"region_extract": (2, 6.0), "region_pass": (2, 7.0), "region_finish": (2, 12.0)}

    def timed(self, tag):
        return self.t.get(tag, (0, 0.0))


def test_dist_roofline_picks_the_dominant_stage():
    dom, sp = bench.dist_roofline(_FakePipe(), 2, "uniq", 21, 10 ** 9, 2, False)
    assert dom["kernel"].startswith("rg_finish") and sp["kernel"].startswith("rg_pass")
    alg = 8.0 * 10 ** 9 + 16.0 * 9 * 10 ** 8
    assert abs(dom["algorithmic_bytes_per_launch"] - alg) < 1 and abs(dom["avg_launch_ms"] - 6.0) < 1e-9
    assert abs(dom["achieved"] - alg / 6e-3 / 1e9) < 1e-6 and abs(sp["achieved"] - 16e9 / 3.5e-3 / 1e9) < 1e-6


def test_committed_pmc_summary_matches_the_default_workload():
    """bench.py's roofline `traffic` comes from profiles/pmc_current.json only
    when its metadata names the default workload (uniq, k 21, 1 G bases): a
    copy without it silently turns the field into null."""
    import bench
    for kern in ("rg_finish", "rg_pass", "rg_extract"):
        t = bench.pmc_traffic(kern, "uniq", 21, 1_000_000_000)
        assert t is not None and t > 0, kern


def _fake_line(calls):
    def line(args, dev, world, rank, per, mode, canon, reparse, steps, warmup, tag, also_overlap=False):
        calls.append({"per": per, "mode": mode, "canon": canon, "reparse": reparse, "steps": steps,
                      "warmup": warmup, "tag": tag, "also_overlap": also_overlap})
        if rank:
            return None
        out = {"value": 1e9 * world, "ms_per_step": 10.0, "steps": steps, "warmup": warmup,
               "kmers_per_step": per * world, "rccl_ranks": world, "setup_s": 1.0, "fasta_bytes": per * world,
               "fasta_bytes_per_rank": per, "path": "region", "rounds": 3 if mode == "count" else 1,
               "fallback_rounds": 0, "partial_rounds": 0, "memory_plan": None, "stages_ms_per_step_rank0": {},
               "stage_alg_bytes_rank0": {}, "roofline": {"frac": 0.5}, "sort_pass_roofline": {"frac": 0.6},
               "spectrum_distinct": None, "exchange": args.exchange == "on", "exchanged_bytes_per_step": 8 * per,
               "max_message_bytes": per, "exchange_gbs_rank0": 100.0}
        if also_overlap:
            out["overlapped"] = {"value": 1.1e9 * world, "ms_per_step": 9.0, "steps": steps,
                                 "overlapped_rounds": out["rounds"], "rounds": out["rounds"], "pieces": 4,
                                 "vs_sequential": 10.0 / 9.0}
        return out
    return line


class _Dev:
    def __init__(self, i):
        pass

    def close(self):
        pass


def test_multi_gpu_line_carries_config4_and_rccl_ranks(monkeypatch, capsys):
    """`bench.py --gpus N` (N > 1, the driver's plain run): after the
    1 GB-per-rank weak-scaling line, a config4 sub-line of BASELINE config 4
    (100 GB over N ranks: 100/N GB per rank, count, parsed at setup), each with
    the RCCL communicator's own rank count."""
    from kman_amd import engine

    calls = []
    monkeypatch.setattr(bench, "dist_line", _fake_line(calls))
    monkeypatch.setattr(engine, "Device", _Dev)
    args = bench.parse_args(["--gpus", "8", "--steps", "4", "--warmup", "1", "--no-cpu-baseline"])
    bench.run_dist(args, 8, 0, 0)
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["n_gpus"] == 8 and out["config"]["rccl_ranks"] == 8 and out["steps"] == 4
    c4 = out["config4"]
    assert c4["rccl_ranks"] == 8 and c4["fasta_bytes_per_rank"] == int(100e9 / 8) and c4["rounds"] == 3
    assert "roofline" in c4 and c4["ms_per_step"] > 0 and c4["setup_s"] >= 0
    assert [(c["mode"], c["per"], c["reparse"], c["tag"], c["also_overlap"]) for c in calls] == [
        ("uniq", 10 ** 9, True, "bench", True), ("count", int(100e9 / 8), False, "bench4", True)]
    # both sub-lines of each: the sequential step (the line itself) and the
    # overlapped one, for the N > 1 run to settle the default
    for ln in (out["config"], c4):
        assert ln["overlapped"]["ms_per_step"] > 0 and ln["overlapped"]["overlapped_rounds"] >= 1
    assert c4["overlapped"]["rounds"] == 3 and out["config"]["exchange"] is True
    assert "one all-to-all per round (kman_alltoallv: RCCL send/recv between ranks" in out["config"]["workload"]
    assert "at one rank" not in out["config"]["workload"]
    # the other ranks run both lines and print nothing
    calls.clear()
    bench.run_dist(args, 8, 3, 3)
    assert capsys.readouterr().out.strip() == "" and len(calls) == 2
    # --no-config4, an explicit --shard-gb and world 1 run the main line only
    for argv, world in ((["--gpus", "2", "--no-config4"], 2), (["--gpus", "2", "--shard-gb", "12.5"], 2),
                        (["--dist"], 1)):
        calls.clear()
        bench.run_dist(bench.parse_args(argv + ["--no-cpu-baseline"]), world, 0, 0)
        out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
        assert len(calls) == 1 and "config4" not in out and out["config"]["rccl_ranks"] == world
        assert calls[0]["also_overlap"] == (world > 1)
        if world == 1:
            assert "at one rank the whole exchange is that copy" in out["config"]["workload"]
