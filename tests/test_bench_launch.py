"""bench.py's launcher (CPU): ``--gpus N`` starts N ranks itself when no launcher did, and a
WORLD_SIZE that disagrees with ``--gpus`` is refused, so the printed ``n_gpus`` always equals
``--gpus`` (reference: one DDP process per GPU, main.py:85 / utils/misc.py:436-458)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, ["--steps", "3"]) is None


def test_launcher_rank_runs_in_process():
    assert bench.launch_plan(4, {"WORLD_SIZE": "4", "RANK": "2"}, []) is None


def test_multi_gpu_spawns_torchrun():
    cmd = bench.launch_plan(8, {}, ["--gpus", "8", "--steps", "5", "--warmup", "2"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    port = int(cmd[cmd.index("--master-port") + 1])
    assert 0 < port < 65536
    assert cmd[-7] == os.path.join(ROOT, "bench.py")
    assert cmd[-6:] == ["--gpus", "8", "--steps", "5", "--warmup", "2"]


def test_mismatch_refused():
    with pytest.raises(SystemExit) as e:
        bench.launch_plan(2, {"WORLD_SIZE": "1"}, [])
    assert e.value.code == 2
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {}, [])


def test_mismatch_exits_nonzero_before_any_device_work():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=1" in r.stderr
    assert r.stdout.strip() == ""
