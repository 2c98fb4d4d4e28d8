"""bench.py's multi-rank launcher (CPU): ``bench.py --gpus N`` run directly starts N ranks of itself
through torch.distributed.run; every rank sees WORLD_SIZE = N (checked with a gloo all-reduce in
--dry-run mode, which exits before any GPU call)."""
import json
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def test_launch_command_plumbing():
    import bench
    cmd = bench.launch_command(["--gpus", "4", "--workload", "c3", "--steps", "7"], 4, 29512)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    assert cmd[-6:] == ["--gpus", "4", "--workload", "c3", "--steps", "7"]
    assert Path(cmd[-7]).name == "bench.py"


def test_no_launch_inside_a_rank(monkeypatch):
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch(["--gpus", "2"], 2) is None
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.maybe_launch(["--gpus", "1"], 1) is None


@pytest.mark.timeout(180)
def test_gpus_two_starts_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                       capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    # the two ranks share the terminal: their lines may interleave
    lines = [json.loads(x) for x in re.findall(r"\{[^{}]*\"dry_run\"[^{}]*\}", r.stdout)]
    assert sorted(l["rank"] for l in lines) == [0, 1]
    assert all(l["world"] == 2 and l["world_seen"] == 2 for l in lines)


def test_world_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)
