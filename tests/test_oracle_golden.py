"""Pin the CPU oracle against the reference-generated fixtures (1 thread).

The fixtures come from ``tests/golden/make_golden.py``, which drives the reference's own
model modules (model/mnist_model.py, MDGAN/MNIST/mnist_model.py, CGLGAN/2DMG/{model,data}.py)
with torch.optim.  Passing here means oracle/ computes what the reference's step computes.

On the CPU that generated the fixtures the match is bit-for-bit (sha256 of every tensor, exact
scalars).  torch's CPU kernels pick their vector width from the host ISA (AVX2 vs AVX-512), which
reorders a few fp32 reductions by one ulp, so on another host the comparison falls back to fp32
reduction-order tolerance: scalars within 4e-6 relative, tensors by float64 norm within 1e-4
relative (1e-3 for step-1 gradients, which pass through BatchNorm backward's cancellations) and
the first 16 values within the same relative / 1e-5 absolute tolerance.  Either way a wrong operation (order of Adam ops,
BN eps, loss weighting) fails by orders of magnitude more.
"""
import math

import pytest
import torch

from golden_replay import capgan_replay, load_golden, mixg_replay, ring_replay, sha
from oracle import gan_oracle as O


@pytest.fixture(scope="module", autouse=True)
def one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


@pytest.fixture(scope="module")
def golden():
    return load_golden()


def _flat(x):
    if isinstance(x, (list, tuple)):
        out = []
        for y in x:
            out += _flat(y)
        return out
    return [float(x)]


def _same_traj(a, b, key):
    """Exact, or within fp32 reduction-order tolerance (see module docstring)."""
    if a == b:
        return
    fa, fb = _flat(a), _flat(b)
    assert len(fa) == len(fb), key
    for x, y in zip(fa, fb):
        assert abs(x - y) <= 4e-6 * max(abs(y), 1e-3), (key, x, y)


def _pre_bn_biases(keys):
    """Biases of Linear layers that feed a BatchNorm (e.g. model.2.bias before model.3): their
    gradient is exactly zero in real arithmetic and pure fp32 rounding noise in practice, which
    Adam then turns into lr-sized steps of arbitrary sign -- these tensors cannot be pinned across
    host ISAs and do not influence any output (the BatchNorm removes them)."""
    out = set()
    for k in keys:
        if k.endswith(".bias"):
            head, idx = k[:-5].rsplit(".", 1)
            if f"{head}.{int(idx) + 1}.running_mean" in keys:
                out.add(k)
    return out


NOISE = set()


def _check_sd(summary, sd, rtol=1e-4, atol=1e-5):
    noise = _pre_bn_biases(set(summary)) | NOISE
    for k, ent in summary.items():
        v = sd[k]
        if "int" in ent:
            assert int(v.item()) == ent["int"], k
            continue
        assert v.numel() == math.prod(ent["shape"]), k
        if v.dim() > 1 and k not in ("Xd", "Xg"):
            assert list(v.shape) == ent["shape"], k
        if sha(v) == ent["sha256"]:
            continue
        if k in noise:
            continue
        head, idx = (k.rsplit(".", 2)[0], k.rsplit(".", 2)[1]) if k.count(".") >= 2 else (None, None)
        if k.endswith(".running_mean") and f"{head}.{int(idx) - 1}.bias" in noise:
            # tracks the mean of (W x + noisy bias): off by at most the bias drift, 2 lr per Adam step
            ref = torch.tensor(ent["head"], dtype=torch.float64)
            assert torch.allclose(v.detach().flatten()[:16].double(), ref, rtol=0, atol=2e-3), k
            continue
        nrm = float(v.double().norm())
        assert math.isclose(nrm, ent["norm"], rel_tol=rtol, abs_tol=atol * math.sqrt(v.numel())), (k, nrm, ent["norm"])
        head = v.detach().flatten()[:16].double()
        ref = torch.tensor(ent["head"], dtype=torch.float64)
        assert torch.allclose(head, ref, rtol=rtol, atol=atol), k


def test_init_recipe(golden):
    g = golden["init"]
    G, ws = O.build_capgan(1)
    _check_sd(g["capgan_G"], G.state_dict())
    _check_sd(g["capgan_D"], ws[0].D.state_dict())
    mg, _ = O.build_mixg(2)
    _check_sd(g["mixg2_G"], mg.state_dict())


@pytest.mark.parametrize("name", ["capgan_b64_n1", "capgan_b256_n1", "capgan_b64_n3",
                                  "capgan_b64_n1_ep2_partial", "mdgan_b64_n2"])
def test_capgan_family_bitwise(golden, name):
    fx = golden[name]
    NOISE.update(_pre_bn_biases(set(fx["final_G"])))
    traj, first, G, workers = capgan_replay(fx["config"])
    for key in ("d_loss", "g_loss", "F", "lambda", "alpha"):
        _same_traj(traj[key], fx["trajectory"][key], key)
    if "Xd" in fx["step1"]:
        _check_sd({"Xd": fx["step1"]["Xd"], "Xg": fx["step1"]["Xg"]}, {"Xd": first["Xd"], "Xg": first["Xg"]})
    if "g_grads" in fx["step1"]:
        _check_sd(fx["step1"]["g_grads"], first["g_grads"], rtol=1e-3)
    _check_sd(fx["final_G"], G.state_dict())
    for w, summ in zip(workers, fx["final_D"]):
        _check_sd(summ, w.D.state_dict())


@pytest.mark.parametrize("name", ["mixg_b64_n2", "mixg_b64_n2_double"])
def test_mixg_bitwise(golden, name):
    fx = golden[name]
    NOISE.update(_pre_bn_biases(set(fx["final_G"])))
    traj, first, G, workers = mixg_replay(fx["config"])
    for key in ("d_loss", "g_loss", "F", "lambda"):
        _same_traj(traj[key], fx["trajectory"][key], key)
    _check_sd(fx["step1"]["g_grads"], first["g_grads"], rtol=1e-3)
    # Mix-G trunk gradients are ~1e-6 per element, so off the generating host Adam's normalised
    # step can differ by up to its full size (lr) per round: bound by 2 lr per step
    steps = fx["config"]["steps"]
    _check_sd(fx["final_G"], G.state_dict(), atol=2 * 2e-4 * steps)
    for w, summ in zip(workers, fx["final_D"]):
        _check_sd(summ, w.D.state_dict())


def test_ring_bitwise(golden):
    fx = golden["ring_b64"]
    data, init, traj, G, workers = ring_replay(fx["config"])
    assert sha(data) == fx["data_sha256"]
    _check_sd(fx["init_G"], init[0])
    _check_sd(fx["init_D"], init[1])
    for key in ("d_loss", "g_loss", "F", "lambda"):
        _same_traj(traj[key], fx["trajectory"][key], key)
    _check_sd(fx["final_G"], G.state_dict())
    _check_sd(fx["final_D"], workers[0].D.state_dict())


def test_capgan_lambda_closed_form(golden):
    """N=1: alpha == 1 exactly and lambda grows by the SGD step each round."""
    traj = golden["capgan_b64_n1"]["trajectory"]
    assert all(a == [1.0] for a in traj["alpha"])
    lam = torch.tensor(0.0)
    for v in traj["lambda"]:
        lam = lam + torch.tensor(-0.1) * torch.tensor(-0.001)
        assert abs(float(lam) - v) <= 1e-9


def test_fedavg_restatement():
    """mixed-gan.py:114-124 weighted mean; S=1 is the identity; segema mix (:198-199)."""
    a = {"w": torch.tensor([1.0, 2.0]), "n": torch.tensor(3)}
    b = {"w": torch.tensor([3.0, 6.0]), "n": torch.tensor(3)}
    p = O.fedavg([a, b], [100, 300])
    assert "n" not in p
    torch.testing.assert_close(p["w"], torch.tensor([2.5, 5.0]))
    p1 = O.fedavg([a], [7])
    torch.testing.assert_close(p1["w"], a["w"])
    pm = O.fedavg([a, b], [100, 300], segema=0.5, self_sd=a)
    torch.testing.assert_close(pm["w"], 0.5 * a["w"] + 0.5 * torch.tensor([2.5, 5.0]))
