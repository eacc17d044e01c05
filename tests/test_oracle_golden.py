"""Pin the CPU oracle bit-for-bit (1 thread) against the reference-generated fixtures.

The fixtures come from ``tests/golden/make_golden.py``, which drives the reference's own
model modules (model/mnist_model.py, MDGAN/MNIST/mnist_model.py, CGLGAN/2DMG/{model,data}.py)
with torch.optim.  Passing here means oracle/ computes exactly what the reference's step computes.
"""
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


def _check_sd(summary, sd):
    for k, ent in summary.items():
        v = sd[k]
        if "int" in ent:
            assert int(v.item()) == ent["int"], k
            continue
        assert list(v.shape) == ent["shape"], k
        assert sha(v) == ent["sha256"], k


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
    traj, first, G, workers = capgan_replay(fx["config"])
    for key in ("d_loss", "g_loss", "F", "lambda", "alpha"):
        assert traj[key] == fx["trajectory"][key], key
    if "Xd" in fx["step1"]:
        assert sha(first["Xd"]) == fx["step1"]["Xd"]["sha256"]
        assert sha(first["Xg"]) == fx["step1"]["Xg"]["sha256"]
    if "g_grads" in fx["step1"]:
        _check_sd(fx["step1"]["g_grads"], first["g_grads"])
    _check_sd(fx["final_G"], G.state_dict())
    for w, summ in zip(workers, fx["final_D"]):
        _check_sd(summ, w.D.state_dict())


@pytest.mark.parametrize("name", ["mixg_b64_n2", "mixg_b64_n2_double"])
def test_mixg_bitwise(golden, name):
    fx = golden[name]
    traj, first, G, workers = mixg_replay(fx["config"])
    for key in ("d_loss", "g_loss", "F", "lambda"):
        assert traj[key] == fx["trajectory"][key], key
    _check_sd(fx["step1"]["g_grads"], first["g_grads"])
    _check_sd(fx["final_G"], G.state_dict())
    for w, summ in zip(workers, fx["final_D"]):
        _check_sd(summ, w.D.state_dict())


def test_ring_bitwise(golden):
    fx = golden["ring_b64"]
    data, init, traj, G, workers = ring_replay(fx["config"])
    assert sha(data) == fx["data_sha256"]
    _check_sd(fx["init_G"], init[0])
    _check_sd(fx["init_D"], init[1])
    for key in ("d_loss", "g_loss", "F", "lambda"):
        assert traj[key] == fx["trajectory"][key], key
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
