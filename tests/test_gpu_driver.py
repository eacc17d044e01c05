"""cglgan.driver on the HIP path (one worker, no process group): every algorithm builds its fused
round from the driver knobs, runs, and two drivers with the same knobs stay bitwise identical (the
replicated-server premise of the multi-GPU driver); checkpoints come out in the reference's format.
The multi-worker topology (server groups, Cloud, D-swap) is covered over gloo by test_driver_gloo.py."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo", ["capgan", "mixg", "mdgan"])
def test_driver_single_worker(algo, tmp_path):
    from cglgan.checkpoint import load_generator
    from cglgan.driver import Driver, DriverConfig
    cfg = DriverConfig(algo=algo, num_workers=1, num_servers=1, batch_size=64, num_communication=4,
                       dataset_rows=4000, num_sample=100, iid=1 if algo == "mdgan" else 0,
                       checkpoint_dir=str(tmp_path), log_every=2)
    logs = []
    a, b = Driver(cfg), Driver(cfg)
    sa, sb = a.run(log=logs.append), b.run(log=None)
    assert sa["round"] == sb["round"] == 4
    assert all(math.isfinite(x) for x in sa["d_loss"]) and math.isfinite(sa["g_loss"])
    assert torch.equal(a.step.g_params, b.step.g_params) and torch.equal(a.step.d_params, b.step.d_params)
    assert len(logs) == 2
    pts = list(tmp_path.glob("*.pt"))
    assert len(pts) == 1 and (tmp_path / ("config" + pts[0].stem + ".pkl")).exists()
    sd = load_generator(str(pts[0]))
    assert set(sd) >= set(a.step.g_views)
