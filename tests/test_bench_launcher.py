"""bench.py --gpus N without a launcher: the process spawns torch.distributed.run as a
child (never an exec), forwards rank 0's JSON line and exits with the launcher's status.  Run end to end on
CPU through the hidden --launch-selftest mode (gloo, no GPU call), plus the pure helpers."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env():
    env = dict(os.environ)
    for k in bench._RANK_ENV:
        env.pop(k, None)
    env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_launcher_cmd_and_env():
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "20"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "20"]
    assert cmd[-5] == os.path.join(ROOT, "bench.py")
    env = bench.launcher_env({"RANK": "3", "WORLD_SIZE": "8", "LOCAL_RANK": "3", "MASTER_PORT": "1", "PATH": "/x"})
    assert "RANK" not in env and "WORLD_SIZE" not in env and "MASTER_PORT" not in env
    assert env["PATH"] == "/x" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_self_launch_two_ranks_end_to_end():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-selftest", "ok"],
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["selftest"] and d["world"] == 2 and d["sum"] == 3.0
    assert sorted(r["rank"] for r in d["ranks"]) == [0, 1]
    assert sorted(r["local_rank"] for r in d["ranks"]) == [0, 1]
    assert all(r["master"].startswith("127.0.0.1:") and r["ipc_legacy"] == "0" for r in d["ranks"])
    assert "torch.distributed.run" in p.stderr


def test_self_launch_propagates_failure():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-selftest", "fail"],
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert p.returncode != 0
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
