"""N workers on one GPU in lockstep (cglgan.exchange.LocalComm): the HIP rounds of N worker
contexts, exchanged through the same phase A / alpha / sum / phase B sequence the RCCL path
runs, vs the oracle in which the reference's Server backpropagates F_max through every D
(CAPGAN capgan.py:211-262 with data-size weights beta; Mix-G mixed-gan.py:238-292 with one
head per worker).  Same tolerance rule as the single-worker parity tests (parity_helpers).
"""
import copy

import pytest
import torch

from cglgan import GanStep, specs
from cglgan.exchange import LocalComm
from oracle import gan_oracle as O
from parity_helpers import g_params, to_double, within

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _threads():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


def _round64(srv64, workers64, z1, z2, reals, **kw):
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return srv64.round(workers64, z1.double(), z2.double(), [[r.double() for r in rs] for rs in reals], **kw)
    finally:
        torch.set_default_dtype(prev)


def _check_params(step, G32, G64, names):
    """Updated G params of one replica vs the fp32/fp64 oracle (+ Adam step-1 sensitivity)."""
    p32, p64 = g_params(G32), g_params(G64)
    fails = []
    for k in names:
        v = step.g_views[k]
        g64 = p64[k].grad.detach().double().flatten()
        dg = (step.g_grad_views[k].detach().double().cpu().flatten() - g64).abs()
        extra = 1.5 * float((2e-4 * dg / (g64.abs() + 1e-8)).norm())
        ok, e, a = within(v, p32[k], p64[k], extra)
        if not ok:
            fails.append((k, e, a))
    return fails


def _seed_ok(G, workers, z1, z2, reals, margin=1e-6):
    """Kink margin of every LeakyReLU input of the round (see parity_helpers)."""
    tr = []
    with torch.no_grad():
        Gc = copy.deepcopy(G)
        xd = Gc.forward(z1, trace=tr)
        xg = Gc.forward(z2, trace=tr)
        n = len(workers)
        for i, (w, rs) in enumerate(zip(workers, reals)):
            D = copy.deepcopy(w.D)
            xs = [xd, xg] if not hasattr(G, "trunk") else [xd.chunk(n)[i], xg.chunk(n)[i]]
            for r in rs:
                D.forward(r, trace=tr)
            for x in xs:
                D.forward(x, trace=tr)
    return min(float(t.abs().min() / (t.std() + 1e-30)) for t in tr) >= margin


def test_capgan_three_workers_beta_weighted():
    N, B = 3, 64
    beta = [0.2, 0.3, 0.5]
    G, workers = O.build_capgan(N)
    srv = O.CapganServer(G, torch.tensor(beta))
    steps = []
    for r in range(N):
        s = GanStep(specs.mnist_generator(), specs.mnist_discriminator(), batch=B, n_workers=N, rank=r)
        s.load_state_dicts(G.state_dict(), workers[r].D.state_dict())
        s.reset(beta=beta)
        steps.append(s)
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    for seed in range(40, 104):
        z1, z2, reals = O.synthetic_inputs(B, N, 1, seed=seed)
        if _seed_ok(G, workers, z1, z2, reals):
            break
    for r, s in enumerate(steps):
        s.z[:B].copy_(z1)
        s.z[B:].copy_(z2)
        s.real.copy_(reals[r][0])
    LocalComm(steps).round(0)
    torch.cuda.synchronize()
    r32 = srv.round(workers, z1, z2, reals)
    r64 = _round64(srv64, workers64, z1, z2, reals)
    for s in steps[1:]:   # replicated G stays bitwise identical
        assert torch.equal(s.g_params, steps[0].g_params)
    st = steps[0].stats()
    assert abs(st["F"] - float(r64["F"])) <= max(1e-5 * abs(float(r64["F"])), 2 * abs(float(r32["F"] - r64["F"])))
    assert abs(st["lambda"] - float(r32["lam"])) <= 1e-7
    fails = _check_params(steps[0], srv.G, srv64.G, list(steps[0].g_views))
    assert not fails, fails
    for r, s in enumerate(steps):
        for k, v in s.d_views.items():
            ok, e, a = within(v, workers[r].D.params[k], workers64[r].D.params[k])
            assert ok, (r, k, e, a)


def test_mixg_two_heads_trunk_exchange():
    N, B = 2, 64
    G, workers = O.build_mixg(N)
    srv = O.MixgServer(G, torch.full((N,), 1.0 / N))
    steps = []
    for h in range(N):
        s = GanStep(specs.mixgen_worker(h), specs.mnist_discriminator(), batch=B, n_workers=N, rank=h,
                    weighting="mix_single", exchange_layer=specs.MIXGEN_HEAD_LAYER)
        s.load_state_dicts(G.state_dict(), workers[h].D.state_dict())
        s.reset()
        steps.append(s)
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    for seed in range(60, 124):
        z1, z2, reals = O.synthetic_inputs(B, N, 1, seed=seed)
        if _seed_ok(G, workers, z1, z2, reals):
            break
    for h, s in enumerate(steps):
        s.z[:B].copy_(z1)
        s.z[B:].copy_(z2)
        s.real.copy_(reals[h][0])
    LocalComm(steps).round(0)
    torch.cuda.synchronize()
    srv.round(workers, z1, z2, reals)
    _round64(srv64, workers64, z1, z2, reals)
    trunk = [k for k in steps[0].g_views if k.startswith("model.")]
    p0, _ = steps[0].trunk_slices()
    p1, _ = steps[1].trunk_slices()
    assert torch.equal(p0, p1)        # the shared trunk stays identical on every worker
    for h, s in enumerate(steps):
        names = trunk + [k for k in s.g_views if k.startswith(f"paths.{h}.")]
        fails = _check_params(s, srv.G, srv64.G, names)
        assert not fails, (h, fails)
