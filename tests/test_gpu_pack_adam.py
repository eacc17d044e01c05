"""G's packed weight copies written by the G Adam launch (cgl_round.h cgl_adam_pack, plan_pack_adam; round 5;
opt-in CGL_PACK_ADAM=1, measured slower than the default) instead of re-packed by every round's prologue
(CGL_PACK_ADAM=0, the default): bitwise the same rounds.

The packed operands P(W; fo, fi) (forward B) and P(W^T; fi, fo) (input-gradient B) of the MNIST G's wide
layers are written from the updated parameters in 4 x 4 tiles by the Adam launch; every other parameter
runs through cgl_adam_at.  Covered: fp32 CAPGAN (B = 64, 256, eager and graph-replayed), a Mix-G worker
(trunk + head), f16 operands with dynamic loss scaling (clean steps, and a scale that overflows so both
Adam steps are skipped), and G parameters written from outside the round between rounds (a FedAvg-style
in-place update through a state-dict view, and cloud averaging): GanStep notices the version counter of its
parameter buffer and refreshes the packed copies (cgl_gan_sync_params) before the next round."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

NAMES = ("g_params", "g_grads", "g_m", "g_v", "d_params", "d_m", "d_v", "g_running", "z")


def _step(on, B=256, kind="capgan", carry=1, **kw):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    os.environ["CGL_PACK_ADAM"] = "1" if on else "0"
    os.environ["CGL_PACK_CARRY"] = str(carry)
    try:
        if kind == "mixg":
            gm, extra = specs.mixgen_worker(0), dict(weighting="mix_single", exchange_layer=specs.MIXGEN_HEAD_LAYER)
        else:
            gm, extra = specs.mnist_generator(), dict(weighting="capgan")
        dm = specs.mnist_discriminator()
        g = torch.Generator().manual_seed(3)
        real = (torch.rand(4 * B + 17, 784, generator=g) * 2 - 1).cuda()
        st = GanStep(gm, dm, batch=B, loss="ce", gen_z=True, real=real, sample_n=real.shape[0], seed=99,
                     **extra, **kw)
    finally:
        os.environ.pop("CGL_PACK_ADAM", None)
        os.environ.pop("CGL_PACK_CARRY", None)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(4242)
    default_init(dm, st.d_views)
    st.reset()
    return st


def _same(a, b, tag=""):
    torch.cuda.synchronize()
    for name in NAMES:
        x, y = getattr(a, name), getattr(b, name)
        same = (x == y) | (torch.isnan(x) & torch.isnan(y))      # (an overflowing f16 round stores NaN gradients)
        assert bool(same.all()), (tag, name, (x - y).abs().max().item())
    sa, sb = a.stats(), b.stats()
    for k in ("round", "g_loss", "F", "lambda", "d_loss", "loss_scale", "skipped"):
        assert sa[k] == sb[k], (tag, k, sa[k], sb[k])


def test_plan_moves_packing_into_adam():
    a, b = _step(True), _step(False, carry=0)
    la, lb = a.launches(), b.launches()
    assert [k for k, _, _ in la] == [k for k, _, _ in lb]
    assert la[0][2] < lb[0][2], (la[0], lb[0])       # the prologue launch lost its packing blocks


def test_plan_carries_packing_in_small_launches():
    """Default plan (CGL_PACK_CARRY=1): the packing jobs ride in the forward cgl_bn_apply launches and the
    deferred loss heads; the prologue keeps none, and the plan's launch sequence is unchanged."""
    c, b = _step(False), _step(False, carry=0)
    lc, lb = c.launches(), b.launches()
    assert [k for k, _, _ in lc] == [k for k, _, _ in lb]
    assert lc[0][2] < lb[0][2], (lc[0], lb[0])
    grew = [k for (k, _, gc), (_, _, gb) in zip(lc, lb) if gc > gb]
    assert grew and set(grew) <= {"bn_apply", "head"}, grew
    assert sum(gc - gb for (_, _, gc), (_, _, gb) in zip(lc[1:], lb[1:])) == lb[0][2] - lc[0][2]


@pytest.mark.parametrize("kind", ["capgan", "mixg"])
def test_pack_carry_bitwise(kind):
    a, b = _step(False, 256, kind), _step(False, 256, kind, carry=0)
    for r in range(5):
        a.run(graph=r >= 2)
        b.run(graph=r >= 2)
    _same(a, b, kind)


@pytest.mark.parametrize("B", [64, 256])
@pytest.mark.parametrize("kind", ["capgan", "mixg"])
def test_pack_adam_bitwise(B, kind):
    a, b = _step(True, B, kind), _step(False, B, kind)
    for r in range(6):
        a.run(graph=r >= 2)
        b.run(graph=r >= 2)
    _same(a, b, f"{kind} B={B}")


@pytest.mark.parametrize("scale", [65536.0, 2.0 ** 40])
def test_pack_adam_bitwise_f16_scaled(scale):
    a = _step(True, 256, gemm_dtype="f16", loss_scale=scale)
    b = _step(False, 256, gemm_dtype="f16", loss_scale=scale)
    for r in range(5):
        a.run(graph=r >= 2)
        b.run(graph=r >= 2)
    _same(a, b, f"f16 S={scale}")
    if scale > 1e10:
        assert a.stats()["skipped"][1] >= 1          # the skipped-step path ran


def test_external_parameter_writes_refresh_the_packed_copies():
    from cglgan.exchange import local_cloud_average
    a, b = _step(True), _step(False)
    for r in range(2):
        a.run()
        b.run()
    for s in (a, b):          # an in-place update through a state-dict view (a FedAvg / load_state_dict write)
        with torch.no_grad():
            s.g_views["model.11.weight"].mul_(0.75)
            s.g_views["model.8.weight"].add_(1e-3)
    for r in range(2):
        a.run(graph=r >= 1)
        b.run(graph=r >= 1)
    _same(a, b, "view write")
    c, d = _step(True), _step(False)          # cloud averaging of two replicas with different histories
    for s in (c, d):
        s.run()
    local_cloud_average([a, c], [0.25, 0.75], cloud_scope="all")
    local_cloud_average([b, d], [0.25, 0.75], cloud_scope="all")
    for r in range(2):
        a.run()
        b.run()
    _same(a, b, "cloud average")


def test_stale_packed_copy_would_be_caught():
    """Control: skipping the refresh after an external write changes the round (so the test above has power)."""
    a, b = _step(True), _step(False)
    a.run()
    b.run()
    for s in (a, b):
        with torch.no_grad():
            s.g_views["model.11.weight"].mul_(0.5)
    a._pk_ver = a._pver()                     # pretend the write was seen: the packed copies stay stale
    a.run()
    b.run()
    torch.cuda.synchronize()
    assert not torch.equal(a.g_params, b.g_params)
