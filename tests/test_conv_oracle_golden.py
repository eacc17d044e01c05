"""Pin oracle/conv_oracle.py (the model/lsgan.py restatement) against fixtures generated from the
reference's own model/lsgan.py modules (tests/golden/make_golden.py, ``lsgan`` section): module
structure and state-dict keys, the construction-order init, a train-mode G forward / backward, a
D forward with the reference's Dropout2d draws, eval-mode sampling, and 3 CAPGAN-shaped rounds per
objective.  Bitwise (sha256) on the generating host, within fp32 reduction-order tolerance otherwise
(see tests/test_oracle_golden.py)."""
import math

import pytest
import torch

from golden_replay import load_golden, sha
from oracle import conv_oracle as CV


@pytest.fixture(scope="module", autouse=True)
def one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


@pytest.fixture(scope="module")
def fx():
    return load_golden()["lsgan"]


def _same(t, ent, rtol=1e-4, atol=1e-6):
    if "int" in ent:
        assert int(t) == ent["int"]
        return
    assert t.numel() == math.prod(ent["shape"])
    if sha(t) == ent["sha256"]:
        return
    assert math.isclose(float(t.double().norm()), ent["norm"], rel_tol=rtol, abs_tol=atol * math.sqrt(t.numel()))
    head = t.detach().flatten()[:16].double()
    assert torch.allclose(head, torch.tensor(ent["head"], dtype=torch.float64), rtol=rtol, atol=atol)


def _init():
    torch.manual_seed(20211212)
    gp, gb = CV.init_params(CV.G_SPEC)
    dp, db = CV.init_params(CV.D_SPEC)
    return gp, gb, dp, db


def test_structure_and_init(fx):
    gp, gb, dp, db = _init()
    gsd = {**gp, **gb}
    dsd = {**dp, **db}
    keys_g = [k for k, _ in fx["keys_G"]]
    keys_d = [k for k, _ in fx["keys_D"]]
    assert sorted(keys_g) == sorted(gsd) and sorted(keys_d) == sorted(dsd)
    for k, shp in fx["keys_G"]:
        assert list(gsd[k].shape) == shp, k
    for k, shp in fx["keys_D"]:
        assert list(dsd[k].shape) == shp, k
    for k, ent in fx["init_G"].items():
        _same(gsd[k], ent)
    for k, ent in fx["init_D"].items():
        _same(dsd[k], ent)


def test_forward_backward_and_eval(fx):
    gp, gb, dp, db = _init()
    for p in list(gp.values()) + list(dp.values()):
        p.requires_grad_(True)
    gen = torch.Generator().manual_seed(fx["g_fwd"]["z_seed"])
    z = torch.randn(4, 100, generator=gen)
    img = CV.g_forward(gp, gb, z)
    dy = torch.randn(img.shape, generator=gen)
    (img * dy).sum().backward()
    _same(img.detach(), fx["g_fwd"]["img"])
    assert torch.allclose(img.detach().flatten().double(), torch.tensor(fx["g_fwd"]["img"]["full"], dtype=torch.float64),
                          rtol=1e-5, atol=1e-6)
    for k, ent in fx["g_fwd"]["grads"].items():
        if k in ("conv_blocks.1.bias", "conv_blocks.5.bias"):   # feed BatchNorm: gradient is rounding noise
            continue
        _same(gp[k].grad, ent, rtol=1e-3)
    for k, ent in fx["g_fwd"]["running"].items():
        _same(gb[k], ent)
    torch.manual_seed(fx["d_fwd"]["rng_seed"])
    real = torch.rand(4, 1, 32, 32, generator=gen) * 2 - 1
    masks = CV.draw_masks(4)
    v = CV.d_forward(dp, db, real, masks)
    v.sum().backward()
    assert torch.allclose(v.detach().flatten().double(), torch.tensor(fx["d_fwd"]["v"], dtype=torch.float64),
                          rtol=1e-5, atol=1e-6)
    for k, ent in fx["d_fwd"]["grads"].items():
        _same(dp[k].grad, ent, rtol=1e-3)
    with torch.no_grad():
        ev = CV.g_forward(gp, gb, z, train=False)
    assert torch.allclose(ev.flatten().double(), torch.tensor(fx["g_eval"]["full"], dtype=torch.float64),
                          rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("kind", ["mse", "bce"])
def test_rounds(fx, kind):
    ent = fx[f"round_{kind}"]
    cfg = ent["config"]
    gp, gb, dp, db = _init()
    o = CV.ConvGan(gp, gb, dp, db, loss=kind, dtype=torch.float32)
    B = cfg["B"]
    for step in range(cfg["steps"]):
        gg = torch.Generator().manual_seed(cfg["input_seed0"] + step)
        z1 = torch.randn(B, 100, generator=gg)
        z2 = torch.randn(B, 100, generator=gg)
        real = torch.rand(B, 1, 32, 32, generator=gg) * 2 - 1
        torch.manual_seed(cfg["rng_seed0"] + step)
        mr, mf, mg = CV.draw_masks(B), CV.draw_masks(B), CV.draw_masks(B)
        r = o.round(z1, z2, real, mr, mf, mg)
        for key in ("d_loss", "g_loss"):
            ref = ent["trajectory"][key][step]
            assert abs(r[key] - ref) <= 4e-6 * max(abs(ref), 1e-3), (key, step, r[key], ref)
        assert abs(o.lam - ent["trajectory"]["lambda"][step]) <= 1e-9
    sdg = {**{k: v.detach() for k, v in o.gp.items()}, **o.gb}
    sdd = {**{k: v.detach() for k, v in o.dp.items()}, **o.db}
    for k, e in ent["final_G"].items():
        if k in ("conv_blocks.1.bias", "conv_blocks.5.bias"):
            continue   # Adam on a rounding-noise gradient (feeds BatchNorm): bounded by lr per step
        _same(sdg[k], e, rtol=1e-4, atol=2 * 2e-4 * cfg["steps"] if "running_mean" in k else 1e-6)
    for k, e in ent["final_D"].items():
        _same(sdd[k], e)


def test_dropin_modules_have_reference_keys(fx):
    """cglgan.lsgan modules build the reference's module tree: identical state-dict keys and shapes
    (checkpoint compatibility); constructing them needs no GPU."""
    from cglgan import lsgan
    g, d = lsgan.Generator((1, 32, 32)), lsgan.Discriminator((1, 32, 32))
    assert [[k, list(v.shape)] for k, v in g.state_dict().items()] == fx["keys_G"]
    assert [[k, list(v.shape)] for k, v in d.state_dict().items()] == fx["keys_D"]
    torch.manual_seed(20211212)
    g2, d2 = lsgan.Generator(), lsgan.Discriminator()
    for k, ent in fx["init_G"].items():
        _same(g2.state_dict()[k], ent)
    for k, ent in fx["init_D"].items():
        _same(d2.state_dict()[k], ent)
    m = lsgan.MixGenerator((1, 32, 32), 3)
    keys = list(m.state_dict())
    assert keys[:2] == ["model.0.0.weight", "model.0.0.bias"] and "paths.2.2.weight" in keys


def test_dropin_modules_refuse_cpu_tensors():
    from cglgan import lsgan
    g = lsgan.Generator()
    with pytest.raises(RuntimeError, match="GPU only"):
        g(torch.randn(2, 100))
