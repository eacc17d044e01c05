"""The N > 1 exchange path over real RCCL on a one-GPU box.  RCCL refuses two ranks on one device
("Duplicate GPU detected", profiles/r03_rccl_same_gpu_probe.txt), so the multi-rank semantics are tested
over gloo (tests/test_gpu_mlp_dist.py, tests/test_gpu_conv_dist.py, tests/test_dist_*.py); here a ONE-rank
nccl group runs every collective of the exchange layer with the split path forced (tests/rccl_world1_worker.py):
the MLP round (phase A, loss all_gather_into_tensor, on-device alpha, gradient all_reduce, side-stream E-share
all_reduce, phase B; eager and graph-replayed phases alternating), the Cloud FedAvg in both scopes ("all" on
CAPGAN, "trunk" with BatchNorm running statistics on Mix-G; segema 0.3), and the conv round with phase A / B
replayed as hipGraphs and the side-stream E-share of D's parameters and running statistics.  Each must leave
every parameter, moment and running statistic bitwise equal to the same rounds run without a group (alpha = 1
and one-rank sums are exact).  A one-rank D-swap is the identity (no send / recv is issued): not covered here."""
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
    if r.returncode != 0:
        print(out[-12000:])          # (the worker's traceback, whole, in the test log)
    assert r.returncode == 0 and "RCCL-WORLD1 OK" in out, out[-4000:]
