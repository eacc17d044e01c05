"""nn.Module drop-ins of the CGLGAN drivers and the asynchronous single-op path.

* Structure (CPU): ``cglgan.cglgan_2dmg`` / ``cglgan.cglgan_mnist`` build the module trees of
  CGLGAN/2DMG/model.py:26-71 and CGLGAN/MNIST/mnist_model.py:30-86 -- constructor signatures
  ``Generator(img_shape, num_client)``, ``Discriminator(ns=1)`` / ``Discriminator(img_shape, ns=1)``,
  the ``.model`` / ``.paths`` attributes the driver toggles, and the reference's state-dict keys.
* A CGLGAN ring round through the modules (GPU): the reference driver's own loop
  (CGLGAN/2DMG/main.py:225-278 server with 2 heads, :344-375 workers) written with these modules,
  ``nn.BCELoss`` and ``torch.optim.Adam`` -- judged against the oracle's ``CglganServer`` round in fp32
  and fp64 from the same state with the tolerance of tests/parity_helpers.py (<= 1e-5 relative to
  fp64, or 2x the fp32 reference's own error; updated parameters add Adam's step-1 sensitivity term).
* Graph capture (GPU): a ``torch.cuda.graph`` capture of an MLP Generator / Discriminator forward +
  backward (model/mnist_model.py modules; the single ops pass their descriptors as kernel arguments,
  no upload, no host synchronisation) replays bitwise equal to the same step run eagerly.
"""
import copy

import pytest
import torch

from oracle import gan_oracle as O
from parity_helpers import STEP_TOL, dist, lambda_within, to_double, within

RING_KEYS_G = ["model.0.weight", "model.0.bias", "paths.0.0.weight", "paths.0.0.bias", "paths.1.0.weight",
               "paths.1.0.bias"]


def test_cglgan_module_structure():
    from cglgan import cglgan_2dmg as R
    from cglgan import cglgan_mnist as M
    g = R.Generator((2,), 2)
    assert list(g.state_dict()) == RING_KEYS_G
    assert list(g.state_dict()) == list(O.MixNet(O.ring_generator_trunk_spec(),
                                                 [O.ring_generator_head_spec(h) for h in range(2)]).state_dict())
    d = R.Discriminator(3)                         # ns accepted, unused (CGLGAN/2DMG/model.py:54)
    assert list(d.state_dict()) == list(O.SeqNet(O.ring_discriminator_spec()).state_dict())
    gm = M.Generator((1, 28, 28), 3)
    assert len(gm.paths) == 3 and hasattr(gm, "model")
    ref = O.MixNet(O.mnist_mixgen_trunk_spec(), [O.mnist_mixgen_head_spec(h) for h in range(3)])
    assert list(gm.state_dict()) == list(ref.state_dict())
    dm = M.Discriminator((1, 28, 28), ns=2)
    assert list(dm.state_dict()) == list(O.SeqNet(O.mnist_discriminator_spec(sigmoid=True)).state_dict())
    # the reference modules' shapes
    assert tuple(dm.model[4].weight.shape) == (1, 256) and tuple(d.model[0].weight.shape) == (128, 2)


def _load_oracle(net, mod):
    """Copy a module's state into an oracle net (SeqNet / MixNet), fp32."""
    sd = mod.state_dict()
    nets = [net.trunk] + list(net.heads) if hasattr(net, "trunk") else [net]
    for n in nets:
        for k in list(n.params):
            n.params[k] = sd[k].detach().cpu().clone().requires_grad_(True)


def _ring_inputs(srv, workers, B, seed0):
    """z1, z2 and one real batch per worker whose LeakyReLU inputs lie >= 1e-6 sigma from the kink."""
    for s in range(seed0, seed0 + 64):
        g = torch.Generator().manual_seed(s)
        z1, z2 = torch.randn(B, 100, generator=g), torch.randn(B, 100, generator=g)
        reals = [torch.randn(B, 2, generator=g) * 0.7 for _ in workers]
        tr = []
        with torch.no_grad():
            G = copy.deepcopy(srv.G)
            xd, xg = G.forward(z1, trace=tr), G.forward(z2, trace=tr)
            for w, r, a, b in zip(workers, reals, torch.chunk(xd, len(workers)), torch.chunk(xg, len(workers))):
                D = copy.deepcopy(w.D)
                for x in (r, a, b):
                    D.forward(x, trace=tr)
        if min(float(t.abs().min() / (t.std() + 1e-30)) for t in tr) >= 1e-6:
            return z1, z2, reals
    raise RuntimeError("no well-conditioned seed")


def _reference_round(net_g, opti_g, nets_d, optis_d, lam, beta, z1, z2, reals, d_step=True):
    """One round of CGLGAN/2DMG/main.py with iid != 0 (one head per worker), written as the reference
    driver writes it: Server.train :225-278 around Worker.train :344-375 (one local step, epoch = 1).
    The MNIST driver (CGLGAN/MNIST/main.py:203-296 around :363-394) is the same round, except that its
    Worker.train iterates its D step over an always-empty list (``Xs = []`` at :365, ``for idx, X in Xs``
    at :376): the literal driver never updates D (``d_step=False``)."""
    loss_fn = torch.nn.BCELoss()
    N = len(nets_d)
    with torch.no_grad():
        Xd = torch.chunk(net_g(z1), N, dim=0)
    Xg = torch.chunk(net_g(z2), N, dim=0)
    d_losses = []
    for i in range(N if d_step else 0):                   # Worker.train: the D step on (real, Xd_i)
        net_d, opti_d = nets_d[i], optis_d[i]
        valid = torch.ones(reals[i].shape[0], 1, device=z1.device)
        opti_d.zero_grad()
        real_loss = loss_fn(net_d(reals[i]), valid)
        fake = torch.zeros(Xd[i].shape[0], 1, device=z1.device)
        fake_loss = loss_fn(net_d(Xd[i].clone()), fake)
        D_loss = real_loss + fake_loss
        D_loss.backward()
        opti_d.step()
        d_losses.append(D_loss.detach())
    opti_g.zero_grad()
    loss = torch.zeros(N, device=z1.device)
    for i in range(N):                                    # Worker.train: G_loss through the updated D
        valid = torch.ones(Xg[i].shape[0], 1, device=z1.device)
        loss[i] = loss_fn(nets_d[i](Xg[i].clone()), valid).clone()
    losses = loss.sum()
    net_g.model.requires_grad_(False)
    losses.backward(retain_graph=True)
    net_g.model.requires_grad_(True)
    gamma = torch.softmax(lam * loss, dim=0).detach()
    F_beta = (beta * loss).sum()
    F_gamma = (gamma * loss).sum()
    F_max = (F_beta + F_gamma) / 2
    net_g.paths.requires_grad_(False)
    F_max.backward()
    net_g.paths.requires_grad_(True)
    grad = (loss * loss * gamma).sum() - (loss * gamma * F_gamma).sum()
    lam = lam + 10 * grad
    opti_g.step()
    return dict(d_losses=torch.stack(d_losses).detach() if d_losses else torch.zeros(0), g_losses=loss.detach(),
                F=F_max.detach(), lam=lam.detach())


@pytest.mark.gpu
def test_cglgan_ring_round_through_modules_vs_oracle():
    from cglgan import cglgan_2dmg as R
    N, B = 2, 64
    torch.manual_seed(20211212)
    net_g = R.Generator((2,), N).cuda()
    nets_d = [R.Discriminator(N).cuda() for _ in range(N)]
    srv = O.CglganServer(O.MixNet(O.ring_generator_trunk_spec(), [O.ring_generator_head_spec(h) for h in range(N)]),
                         torch.full((N,), 1.0 / N))
    _load_oracle(srv.G, net_g)
    workers = []
    for d in nets_d:
        w = O.Worker(O.SeqNet(O.ring_discriminator_spec()), "bce")
        _load_oracle(w.D, d)
        w.opt = O.Adam(w.D.parameters())
        workers.append(w)
    srv.opt = O.Adam(srv.G.parameters())
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    z1, z2, reals = _ring_inputs(srv, workers, B, 31)
    opti_g = torch.optim.Adam(net_g.parameters(), lr=O.LR, betas=(O.B1, O.B2))
    optis_d = [torch.optim.Adam(d.parameters(), lr=O.LR, betas=(O.B1, O.B2)) for d in nets_d]
    lam0 = torch.tensor(0.0, device="cuda")
    out = _reference_round(net_g, opti_g, nets_d, optis_d, lam0, torch.full((N,), 1.0 / N, device="cuda"),
                           z1.cuda(), z2.cuda(), [r.cuda() for r in reals])
    torch.cuda.synchronize()
    r32 = srv.round(workers, z1, z2, [[r] for r in reals])
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        r64 = srv64.round(workers64, z1.double(), z2.double(), [[r.double()] for r in reals])
    finally:
        torch.set_default_dtype(prev)
    fails = []
    for name, key in (("d_losses", "d_losses"), ("g_losses", "g_losses"), ("F", "F")):
        ok, e, a = within(out[name].cpu().reshape(-1), r32[key].reshape(-1), r64[key].reshape(-1), tol=STEP_TOL)
        if not ok:
            fails.append((name, e, a))
    # lambda = 10 (sum l^2 gamma - sum l gamma F_gamma) (CGLGAN/2DMG/main.py:273-274), a difference of two
    # nearly equal sums: judged against the fp64 oracle's lambda with the explicit cancellation bound of
    # parity_helpers.lambda_within (propagated loss error + fp32 evaluation of the formula)
    ok, e, a = lambda_within(out["lam"].cpu(), out["g_losses"].cpu(), r64["lam"], r64["g_losses"])
    if not ok:
        fails.append(("lam", e, a))
    g32 = {k: v for n in [srv.G.trunk] + list(srv.G.heads) for k, v in n.params.items()}
    g64 = {k: v for n in [srv64.G.trunk] + list(srv64.G.heads) for k, v in n.params.items()}
    for k, p in net_g.named_parameters():
        gd = p.grad.detach().double().cpu().flatten() - g64[k].grad.detach().double().flatten()
        ok, e, a = within(p.grad, g32[k].grad, g64[k].grad)
        if not ok:
            fails.append(("G grad", k, e, a))
        extra = 1.5 * float((2e-4 * gd.abs() / (g64[k].grad.detach().double().flatten().abs() + 1e-8)).norm())
        ok, e, a = within(p, g32[k], g64[k], extra)
        if not ok:
            fails.append(("G param", k, e, a))
    for i, d in enumerate(nets_d):
        for k, p in d.named_parameters():
            q32, q64 = workers[i].D.params[k], workers64[i].D.params[k]
            gd = p.grad.detach().double().cpu().flatten() - q64.grad.detach().double().flatten()
            extra = 1.5 * float((2e-4 * gd.abs() / (q64.grad.detach().double().flatten().abs() + 1e-8)).norm())
            ok, e, a = within(p, q32, q64, extra)
            if not ok:
                fails.append(("D param", i, k, e, a))
    assert not fails, fails


def _mnist_inputs(srv, workers, B, seed0):
    """z1, z2 and one real batch per worker (uniform(-1, 1) 28x28 images) whose LeakyReLU inputs lie
    >= 1e-6 sigma from the kink in the fp32 oracle's forward calls of the round."""
    for s in range(seed0, seed0 + 64):
        g = torch.Generator().manual_seed(s)
        z1, z2 = torch.randn(B, 100, generator=g), torch.randn(B, 100, generator=g)
        reals = [torch.rand(B, 784, generator=g) * 2 - 1 for _ in workers]
        tr = []
        with torch.no_grad():
            G = copy.deepcopy(srv.G)
            xd, xg = G.forward(z1, trace=tr), G.forward(z2, trace=tr)
            for w, r, a, b in zip(workers, reals, torch.chunk(xd, len(workers)), torch.chunk(xg, len(workers))):
                D = copy.deepcopy(w.D)
                for x in (r, a, b):
                    D.forward(x, trace=tr)
        if min(float(t.abs().min() / (t.std() + 1e-30)) for t in tr) >= 1e-6:
            return z1, z2, reals
    raise RuntimeError("no well-conditioned seed")


@pytest.mark.gpu
@pytest.mark.parametrize("d_step", [True, False], ids=["d_step", "literal_no_d_step"])
def test_cglgan_mnist_round_through_modules_vs_oracle(d_step):
    """The CGLGAN MNIST round through ``cglgan.cglgan_mnist`` (CGLGAN/MNIST/mnist_model.py:30-86: MixGenerator
    trunk + one head per worker, Sigmoid D) driven as CGLGAN/MNIST/main.py:203-296 / :363-394 drive it -- BCE,
    torch.optim.Adam, the two-phase backward with the ``requires_grad_`` toggles (heads from sum(l), trunk from
    F_max) -- against the oracle's CglganServer round in fp32 and fp64 at the 1e-5 step tolerance.  d_step:
    the intended worker D step (as the 2DMG worker); literal_no_d_step: the MNIST worker's D loop never runs."""
    from cglgan import cglgan_mnist as M
    N, B = 2, 64
    torch.manual_seed(20211213)
    net_g = M.Generator((1, 28, 28), N).cuda()
    nets_d = [M.Discriminator((1, 28, 28), N).cuda() for _ in range(N)]
    srv = O.CglganServer(O.MixNet(O.mnist_mixgen_trunk_spec(), [O.mnist_mixgen_head_spec(h) for h in range(N)]),
                         torch.full((N,), 1.0 / N))
    _load_oracle(srv.G, net_g)
    for n in [srv.G.trunk] + list(srv.G.heads):          # BatchNorm running statistics too
        for k in list(n.buffers):
            n.buffers[k] = net_g.state_dict()[k].detach().cpu().clone()
    workers = []
    for d in nets_d:
        w = O.Worker(O.SeqNet(O.mnist_discriminator_spec(sigmoid=True)), "bce")
        _load_oracle(w.D, d)
        w.opt = O.Adam(w.D.parameters())
        workers.append(w)
    srv.opt = O.Adam(srv.G.parameters())
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    z1, z2, reals = _mnist_inputs(srv, workers, B, 101)
    opti_g = torch.optim.Adam(net_g.parameters(), lr=O.LR, betas=(O.B1, O.B2))
    optis_d = [torch.optim.Adam(d.parameters(), lr=O.LR, betas=(O.B1, O.B2)) for d in nets_d]
    lam0 = torch.tensor(0.0, device="cuda")
    out = _reference_round(net_g, opti_g, nets_d, optis_d, lam0, torch.full((N,), 1.0 / N, device="cuda"),
                           z1.cuda(), z2.cuda(), [r.cuda() for r in reals], d_step=d_step)
    torch.cuda.synchronize()
    orc = [[r] for r in reals] if d_step else [[] for _ in reals]
    r32 = srv.round(workers, z1, z2, orc)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        r64 = srv64.round(workers64, z1.double(), z2.double(), [[r.double() for r in rs] for rs in orc])
    finally:
        torch.set_default_dtype(prev)
    fails = []
    names = (("d_losses", "d_losses"),) if d_step else ()
    for name, key in names + (("g_losses", "g_losses"), ("F", "F")):
        ok, e, a = within(out[name].cpu().reshape(-1), r32[key].reshape(-1), r64[key].reshape(-1), tol=STEP_TOL)
        if not ok:
            fails.append((name, e, a))
    ok, e, a = lambda_within(out["lam"].cpu(), out["g_losses"].cpu(), r64["lam"], r64["g_losses"])
    if not ok:
        fails.append(("lam", e, a))
    g32 = {k: v for n in [srv.G.trunk] + list(srv.G.heads) for k, v in n.params.items()}
    g64 = {k: v for n in [srv64.G.trunk] + list(srv64.G.heads) for k, v in n.params.items()}
    for k, p in net_g.named_parameters():
        gd = p.grad.detach().double().cpu().flatten() - g64[k].grad.detach().double().flatten()
        ok, e, a = within(p.grad, g32[k].grad, g64[k].grad)
        if not ok:
            fails.append(("G grad", k, e, a))
        extra = 1.5 * float((2e-4 * gd.abs() / (g64[k].grad.detach().double().flatten().abs() + 1e-8)).norm())
        ok, e, a = within(p, g32[k], g64[k], extra)
        if not ok:
            fails.append(("G param", k, e, a))
    b32 = {k: v for n in [srv.G.trunk] + list(srv.G.heads) for k, v in n.buffers.items()}
    b64 = {k: v for n in [srv64.G.trunk] + list(srv64.G.heads) for k, v in n.buffers.items()}
    for k, v in net_g.state_dict().items():
        if k in b32 and "running" in k:
            ok, e, a = within(v, b32[k], b64[k])
            if not ok:
                fails.append(("G buffer", k, e, a))
    for i, d in enumerate(nets_d):
        for k, p in d.named_parameters():
            q32, q64 = workers[i].D.params[k], workers64[i].D.params[k]
            if not d_step:
                if not torch.equal(p.detach().cpu(), q32.detach()):
                    fails.append(("D param moved", i, k))
                continue
            gd = p.grad.detach().double().cpu().flatten() - q64.grad.detach().double().flatten()
            extra = 1.5 * float((2e-4 * gd.abs() / (q64.grad.detach().double().flatten().abs() + 1e-8)).norm())
            ok, e, a = within(p, q32, q64, extra)
            if not ok:
                fails.append(("D param", i, k, e, a))
    assert not fails, fails


def _snapshot(mods):
    return [copy.deepcopy(m.state_dict()) for m in mods]


def _restore(mods, snaps):
    for m, s in zip(mods, snaps):
        m.load_state_dict(s)


@pytest.mark.gpu
def test_module_forward_backward_graph_capture_bitwise():
    """torch.cuda.graph of G(z) -> D -> loss -> backward (MLP modules, BatchNorm in train mode) replays
    bitwise equal to the eager step: outputs, every parameter gradient, BatchNorm running statistics."""
    from cglgan import model as CM
    torch.manual_seed(5)
    G = CM.Generator((1, 28, 28)).cuda()
    D = CM.Discriminator((1, 28, 28)).cuda()
    z = torch.randn(128, 100, device="cuda")
    snaps = _snapshot([G, D])

    def step():
        out = D(G(z))
        loss = torch.nn.functional.cross_entropy(out, torch.ones(out.shape[0], dtype=torch.long, device="cuda"))
        loss.backward()
        return out, loss

    # eager
    for p in list(G.parameters()) + list(D.parameters()):
        p.grad = None
    out_e, loss_e = step()
    eager = {"out": out_e.detach().clone(), "loss": loss_e.detach().clone(),
             "grads": [p.grad.detach().clone() for p in list(G.parameters()) + list(D.parameters())],
             "sd": copy.deepcopy(G.state_dict())}
    # drop the eager autograd graph: its AccumulateGrad nodes (bound to the default stream) would otherwise
    # be reused by the captured backward (torch's capture recipe: no graph kept alive across the capture)
    del out_e, loss_e
    # capture (torch's recipe: warm up on a side stream first), then restore the state and replay
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            for p in list(G.parameters()) + list(D.parameters()):
                p.grad = None
            step()
    torch.cuda.current_stream().wait_stream(s)
    for p in list(G.parameters()) + list(D.parameters()):
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out_g, loss_g = step()
    _restore([G, D], snaps)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out_g, eager["out"]) and torch.equal(loss_g, eager["loss"])
    for p, ge in zip(list(G.parameters()) + list(D.parameters()), eager["grads"]):
        assert torch.equal(p.grad, ge)
    sd = G.state_dict()
    for k, v in eager["sd"].items():
        assert torch.equal(sd[k], v), k
    # a second replay from the same restored state is bitwise the same again
    _restore([G, D], snaps)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out_g, eager["out"])
    assert dist(out_g, eager["out"]) == 0.0
