"""D's hidden-layer weights read fragment-packed by the D forward GEMMs (round 5, plan_d_pack, CGL_DPACK=0 off): D's
Adam launch writes P(V_j; fo, fi) beside each updated matrix (cgl_adam_pack), so the next local D step's forward and
the G-loss pass through the updated D read two contiguous 1 KB wave loads per 16-k chunk.  D parameters written from
outside the round (E-share, D-swap, a state-dict load) move d_params' version counter and GanStep refreshes the packed
copies before the next round (cgl_gan_sync_params).

The packed B operand changes the D forward GEMMs' tile choice (cost model), so the packed and the row-major rounds
agree to fp32 tolerance, not bitwise."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(dpack, B=256, kind="capgan", epoch=1):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    old = os.environ.get("CGL_DPACK")
    os.environ["CGL_DPACK"] = "1" if dpack else "0"
    try:
        if kind == "mixg":
            gm, extra = specs.mixgen_worker(0), dict(weighting="mix_single", exchange_layer=specs.MIXGEN_HEAD_LAYER)
        else:
            gm, extra = specs.mnist_generator(), dict(weighting="capgan")
        dm = specs.mnist_discriminator()
        g = torch.Generator().manual_seed(5)
        real = (torch.rand(4 * B + 9, 784, generator=g) * 2 - 1).cuda()
        st = GanStep(gm, dm, batch=B, epoch=epoch, loss="ce", gen_z=True, real=real, sample_n=real.shape[0],
                     seed=41, **extra)
    finally:
        if old is None:
            os.environ.pop("CGL_DPACK", None)
        else:
            os.environ["CGL_DPACK"] = old
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(99)
    default_init(dm, st.d_views)
    st.reset()
    return st


def _close(a, b, rtol):
    for k in ("g_loss", "F"):
        x, y = a.stats()[k], b.stats()[k]
        assert abs(x - y) <= rtol * abs(y) + 1e-6, (k, x, y)
    for x, y in zip(a.stats()["d_loss"], b.stats()["d_loss"]):
        assert abs(x - y) <= rtol * abs(y) + 1e-6, ("d_loss", x, y)
    rel = float((a.d_params - b.d_params).norm() / b.d_params.norm())
    assert rel <= 1e-4, rel


def test_plan_d_adam_carries_the_packing():
    a, b = _step(True), _step(False)
    la, lb = a.launches(), b.launches()
    assert [k for k, _, _ in la] == [k for k, _, _ in lb]
    adam_a = [g for k, _, g in la if k == "adam"]
    adam_b = [g for k, _, g in lb if k == "adam"]
    assert adam_a[0] != adam_b[0]            # the D Adam launch runs in the packing form (cgl_adam_pack)
    assert adam_a[1:] == adam_b[1:]


@pytest.mark.parametrize("kind,epoch", [("capgan", 1), ("capgan", 2), ("mixg", 1)])
def test_d_pack_matches_row_major(kind, epoch):
    a, b = _step(True, kind=kind, epoch=epoch), _step(False, kind=kind, epoch=epoch)
    for r in range(4):
        a.run(graph=r >= 2)
        b.run(graph=r >= 2)
    torch.cuda.synchronize()
    _close(a, b, 1e-4)


def test_d_written_outside_the_round_refreshes_the_packed_copy():
    """An in-place write of D's parameters between rounds (what an E-share / D-swap does) must reach the packed
    copies: with a stale copy the next D forward would use the old weights and the losses would split."""
    a, b = _step(True), _step(False)
    for r in range(2):
        a.run(graph=True)
        b.run(graph=True)
    for s in (a, b):
        with torch.no_grad():
            s.d_params.mul_(0.5)
    for r in range(2):
        a.run(graph=True)
        b.run(graph=True)
    torch.cuda.synchronize()
    _close(a, b, 1e-4)
