"""The N > 1 exchange path over real RCCL on a one-GPU box.  RCCL refuses two ranks on one device
("Duplicate GPU detected", profiles/r03_rccl_same_gpu_probe.txt), so the multi-rank semantics are tested
over gloo (tests/test_gpu_mlp_dist.py, tests/test_dist_*.py); here a ONE-rank nccl group runs
WorkerExchange with the split path forced -- phase A, the loss all_gather_into_tensor, the on-device alpha,
the gradient all_reduce and the side-stream E-share all_reduce all go through RCCL on the step's streams,
eager and graph-replayed phases alternating -- and must leave every parameter, moment and running statistic
bitwise equal to the same rounds run without a group (alpha = 1 and one-rank sums are exact)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_exchange_over_rccl_world1():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "rccl_world1_worker.py")]
    env = dict(os.environ)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "RCCL-WORLD1 OK" in out, out[-4000:]
