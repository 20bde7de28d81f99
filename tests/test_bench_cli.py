"""CPU: bench.py's --gpus contract. `--gpus N` without a launcher starts N ranks itself (one
process per GPU through torch.distributed.run), a launcher whose WORLD_SIZE disagrees with --gpus
is refused with a non-zero exit before any GPU is touched, and every line's n_gpus is the rank
count (asserted in bench.py before printing)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_world_plan_without_launcher():
    assert bench.world_plan(1, {}) == "run"
    assert bench.world_plan(2, {}) == "launch"
    assert bench.world_plan(8, {}) == "launch"


def test_world_plan_under_launcher():
    assert bench.world_plan(2, {"WORLD_SIZE": "2"}) == "run"
    assert bench.world_plan(1, {"WORLD_SIZE": "1"}) == "run"
    with pytest.raises(SystemExit) as e:
        bench.world_plan(8, {"WORLD_SIZE": "1"})
    assert e.value.code == 2
    with pytest.raises(SystemExit) as e:
        bench.world_plan(1, {"WORLD_SIZE": "2"})
    assert e.value.code == 2
    with pytest.raises(SystemExit):
        bench.world_plan(0, {})


def test_rank_launch_command_is_one_rank_per_gpu():
    cmd = bench.rank_launch_command(4, ["--gpus", "4", "--steps", "7"], 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29999"
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "7"]


@pytest.mark.parametrize("ws,gpus", [("2", "1"), ("1", "8")])
def test_mismatched_world_exits_nonzero(ws, gpus):
    env = dict(os.environ, WORLD_SIZE=ws, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", gpus],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "refusing" in r.stderr
    assert not r.stdout.strip()   # no JSON line


def test_gpus_beyond_visible_devices_exits_nonzero():
    """--gpus 2 with no launcher on a host without 2 GPUs (this container has none): the
    launcher is not started and the exit status is non-zero (no 1-GPU line passes for 2)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MAXCOVER_BENCH_DEVICE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not r.stdout.strip()
