"""bench.py's own launcher (`--gpus N` must run N ranks): the decision logic, the
command it builds, and a real two-rank launch on CPU that stops before any GPU call."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_launch_decision():
    assert bench.launch_decision(1, {}) == "run"
    assert bench.launch_decision(8, {}) == "spawn"
    assert bench.launch_decision(8, {"WORLD_SIZE": "8"}) == "run"
    msg = bench.launch_decision(8, {"WORLD_SIZE": "1"})
    assert msg not in ("run", "spawn") and "WORLD_SIZE=1" in msg and "--gpus 8" in msg


def test_launch_command():
    cmd = bench.launch_command(4, ["--gpus", "4", "--steps", "5"], 29999)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd and "29999" in cmd
    assert cmd[-3:] == ["--gpus", "4", "--steps", "5"][-3:]


def test_two_ranks_spawned_on_cpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["gpus"] == 2 and x["launched_by_bench"] for x in lines)
    # the host group is gloo, so each rank holds one RCCL communicator (the
    # engine's own); the group was really created (and barriered) by the launched ranks
    assert all(x["host_group"] == "gloo" for x in lines)
    # the headline at N = 2 is BASELINE configs[2] itself: 10,000 instances in total, split over the
    # ranks; the weak-scaling run and the 1M-peer flood ride along
    for x in lines:
        h = x["headline"]
        assert h["peers_total"] == 10_000 and h["bounds"] == [0, 5000, 10_000] and h["scaling"] == "strong"
        assert h["weak_per_gpu_peers_total"] == 20_000 and h["at_1M_peers_total"] == 1_000_000
        # the CPU oracle is timed beside the N > 1 line too (rank 0's host cores)
        assert h["cpu_baseline_ranks"] == [0]


def test_world_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr
