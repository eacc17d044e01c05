"""Shared helpers for the GPU parity tests: build an oracle run and the HIP GanStep from the
same seeded initial state and inputs, and compare them with the tolerances SURVEY F8 sets
(single step <= 1e-5 relative; <= 10-step trajectory <= 1e-4 relative).

Single-step comparisons are made against the oracle run in float64, with the fp32 oracle
(= the reference's own CPU arithmetic, pinned bitwise by tests/golden) as the yardstick: the
HIP result must be within 1e-5 relative of fp64, or at least as close to fp64 as 2x the fp32
reference's own error.  Two properties of the reference computation make this necessary:
  * the bias of a Linear that feeds BatchNorm has an analytically zero gradient (BN removes
    the batch mean), so every fp32 implementation returns rounding noise there, and Adam's
    first step turns noise g into an update lr*g/(|g|+eps) -- bounded by lr/eps*|g|;
  * LeakyReLU' is discontinuous at 0: an activation within rounding distance of 0 flips the
    mask under ANY reordering of fp32 sums.  Inputs are therefore drawn from seeds whose
    LeakyReLU inputs all lie >= 1e-6 standard deviations from the kink (searched, seeded).
"""
import copy

import torch

from cglgan import GanStep, specs
from oracle import gan_oracle as O

STEP_TOL = 1e-5     # single step from identical state: losses, grads, updated params
TRAJ_TOL = 1e-4     # free-running trajectory, <= 10 steps
KINK_MARGIN = 1e-6  # min |LeakyReLU input| / std of its tensor for a well-conditioned input


def rel(a, b, floor=1e-30):
    """||a - b|| / max(||b||, floor)."""
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return float((a - b).norm() / max(float(b.norm()), floor))


def dist(a, b):
    return float((a.detach().double().cpu().flatten() - b.detach().double().cpu().flatten()).norm())


def rel_scalar(a, b):
    return abs(float(a) - float(b)) / max(abs(float(b)), 1e-30)


def make_pair(kind, B, Br=None, epoch=1, seed=20211212, gen_z=False, gemm_dtype="f32", **step_kw):
    """(oracle server, oracle workers, HIP step) with identical initial parameters."""
    if kind == "capgan":
        G, workers = O.build_capgan(1)
        srv = O.CapganServer(G, torch.tensor([1.0]))
        gm, dm, loss, weighting, xl = specs.mnist_generator(), specs.mnist_discriminator(), "ce", "capgan", -1
    elif kind == "mdgan":
        G, workers = O.build_capgan(1, loss="bce")
        srv = O.CapganServer(G, torch.tensor([1.0]))
        gm, dm, loss, weighting, xl = (specs.mnist_generator(), specs.mnist_discriminator(sigmoid=True), "bce",
                                       "mean", -1)
    elif kind == "ring":
        G, workers = O.build_ring(1, 1)
        srv = O.CglganServer(G, torch.tensor([1.0]))
        gm, dm, loss, weighting, xl = specs.ring_generator(0), specs.ring_discriminator(), "bce", "cglgan", -1
    elif kind in ("mixg1", "mixg1x"):
        # Mix-G with a single head: the full reference two-phase backward on one worker
        # (mixg1x: same model/init, planned without the trunk/head exchange split)
        G, workers = O.build_mixg(1)
        srv = O.MixgServer(G, torch.tensor([1.0]))
        gm, dm, loss, weighting, xl = (specs.mixgen_worker(0), specs.mnist_discriminator(), "ce", "mix_single",
                                       specs.MIXGEN_HEAD_LAYER if kind == "mixg1" else -1)
    else:
        raise ValueError(kind)
    step = GanStep(gm, dm, batch=B, batch_real=Br or B, epoch=epoch, loss=loss, weighting=weighting,
                   exchange_layer=xl, seed=seed, gen_z=gen_z, gemm_dtype=gemm_dtype, **step_kw)
    step.load_state_dicts(G.state_dict(), workers[0].D.state_dict())
    step.reset()
    return srv, workers, step


def make_pair_oracle_only(kind, B=64):
    """The oracle server + workers of make_pair (no GPU)."""
    if kind == "capgan":
        G, workers = O.build_capgan(1)
        return O.CapganServer(G, torch.tensor([1.0])), workers
    if kind == "mdgan":
        G, workers = O.build_capgan(1, loss="bce")
        return O.CapganServer(G, torch.tensor([1.0])), workers
    raise ValueError(kind)


def feed(step, z1, z2, reals):
    """Copy one round's explicit inputs into the step's device buffers."""
    step.z[: step.B].copy_(z1)
    step.z[step.B:].copy_(z2)
    step.real.copy_(torch.cat([r.reshape(r.shape[0], -1) for r in reals], 0))


def oracle_round(kind, srv, workers, z1, z2, reals):
    if kind == "capgan":
        return srv.round(workers, z1, z2, [reals], weighting="capgan")
    if kind == "mdgan":
        return srv.round(workers, z1, z2, [reals], weighting="mean")
    return srv.round(workers, z1, z2, [reals])


def inputs(kind, B, Br, epoch, seed):
    if kind == "ring":
        g = torch.Generator().manual_seed(seed)
        z1 = torch.randn(B, 100, generator=g)
        z2 = torch.randn(B, 100, generator=g)
        reals = [torch.randn(Br, 2, generator=g) * 0.7 for _ in range(epoch)]
        return z1, z2, reals
    z1, z2, reals = O.synthetic_inputs(B, 1, epoch, seed=seed, B_real=Br)
    return z1, z2, reals[0]


def kink_margin(srv, workers, z1, z2, reals):
    """min over every LeakyReLU input of the round's forwards of |x| / std(x) (initial D)."""
    G = copy.deepcopy(srv.G)
    D = copy.deepcopy(workers[0].D)
    tr = []
    with torch.no_grad():
        xd = G.forward(z1, trace=tr)
        xg = G.forward(z2, trace=tr)
        for r in reals:
            D.forward(r, trace=tr)
        D.forward(xd, trace=tr)
        D.forward(xg, trace=tr)
    return min(float(t.abs().min() / (t.std() + 1e-30)) for t in tr)


def well_conditioned_inputs(kind, srv, workers, B, Br, epoch, seed0):
    for s in range(seed0, seed0 + 64):
        z1, z2, reals = inputs(kind, B, Br, epoch, s)
        if kink_margin(srv, workers, z1, z2, reals) >= KINK_MARGIN:
            return z1, z2, reals, s
    raise RuntimeError("no well-conditioned seed found")


def to_double(srv, workers):
    """Convert an oracle server + workers (params, buffers, optimiser state) to float64."""
    def conv_net(n):
        nets = [n.trunk] + list(n.heads) if hasattr(n, "trunk") else [n]
        for net in nets:
            for k in list(net.params):
                net.params[k] = net.params[k].detach().double().requires_grad_(True)
            for k in list(net.buffers):
                if net.buffers[k].dtype == torch.float32:
                    net.buffers[k] = net.buffers[k].double()
    conv_net(srv.G)
    srv.opt.params = srv.G.parameters()
    srv.opt.m = [m.double() for m in srv.opt.m]
    srv.opt.v = [v.double() for v in srv.opt.v]
    srv.beta = srv.beta.double()
    for w in workers:
        conv_net(w.D)
        w.opt.params = w.D.parameters()
        w.opt.m = [m.double() for m in w.opt.m]
        w.opt.v = [v.double() for v in w.opt.v]


def oracle_round64(kind, srv64, workers64, z1, z2, reals):
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return oracle_round(kind, srv64, workers64, z1.double(), z2.double(), [r.double() for r in reals])
    finally:
        torch.set_default_dtype(prev)


def g_params(G):
    nets = [G.trunk] + list(G.heads) if hasattr(G, "trunk") else [G]
    out = {}
    for n in nets:
        out.update(n.params)
    return out


def within(gpu, t32, t64, extra=0.0, tol=STEP_TOL):
    """HIP error vs fp64 <= max(tol * |fp64|, 2 * fp32-reference error vs fp64, extra, 1e-9 sqrt(n))."""
    e_gpu = dist(gpu, t64)
    allowed = max(tol * float(t64.detach().double().norm()), 2.0 * dist(t32, t64), extra,
                  1e-9 * (t64.numel() ** 0.5))
    return e_gpu <= allowed, e_gpu, allowed


def _scalar_ok(gpu, s32, s64):
    e = abs(float(gpu) - float(s64))
    return e <= max(STEP_TOL * abs(float(s64)), 2 * abs(float(s32) - float(s64)), 1e-12), (gpu, s32, s64)


def cglgan_lambda(lam0, losses):
    """CGLGAN/2DMG/main.py:261-274 (= CGLGAN/MNIST/main.py:271-290) in fp64: lambda0 + 10 (sum l^2 gamma -
    sum l gamma F_gamma), gamma = softmax(lambda0 l).  Returns (lambda, the six-term sum of |terms|)."""
    l = torch.as_tensor(losses).double().flatten()
    g = torch.softmax(float(lam0) * l, dim=0)
    fg = (g * l).sum()
    a, b = l * l * g, l * g * fg
    return float(lam0) + 10.0 * float(a.sum() - b.sum()), float(a.abs().sum() + b.abs().sum())


def lambda_within(lam_gpu, l_gpu, lam64, l64, lam0=0.0, k=8):
    """The closed-form lambda judged against the fp64 oracle's lambda (not against itself).  lambda is a
    difference of two nearly equal sums, so its error budget is explicit: (1) the propagated loss error --
    the fp64 formula applied to the round's own losses minus the fp64 oracle's lambda (exact propagation
    of the already-judged loss differences), plus (2) the fp32 evaluation of the formula, bounded by
    10 k eps_32 sum |terms| (k ~ the rounding steps per term: square, exp / softmax, products, the sums).
    Returns (ok, error, allowed)."""
    lam_prop, mag = cglgan_lambda(lam0, l_gpu)
    err = abs(float(lam_gpu) - float(lam64))
    allowed = abs(lam_prop - float(lam64)) + 10.0 * k * 2.0 ** -24 * mag + 1e-12
    return err <= allowed, err, allowed


def check_single_round(kind, B, Br=None, epoch=1, seed0=7):
    """Run one round on the HIP path and on the fp32 + fp64 oracles from identical state; return
    (failures, stats).  Every tensor is judged with ``within`` (module docstring)."""
    Br = Br or B
    fail = []
    srv, workers, step = make_pair(kind, B, Br, epoch)
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    z1, z2, reals, _ = well_conditioned_inputs(kind, srv, workers, B, Br, epoch, seed0)
    feed(step, z1, z2, reals)
    step.run()
    torch.cuda.synchronize()
    r32 = oracle_round(kind, srv, workers, z1, z2, reals)
    r64 = oracle_round64(kind, srv64, workers64, z1, z2, reals)
    st = step.stats()
    if st["round"] != 1:
        fail.append(("round", st["round"]))
    # G output of the round (Xd rows then Xg rows)
    out = step.g_output().cpu()
    for name, o in (("Xd", out[:B]), ("Xg", out[B:])):
        ok, e, a = within(o, r32[name].reshape(B, -1), r64[name].reshape(B, -1))
        if not ok: fail.append((name, e, a))
    # losses
    for e in range(epoch):
        ok, info = _scalar_ok(st["d_loss"][e], r32["d_losses"][e], r64["d_losses"][e])
        if not ok: fail.append(("d_loss", e, info))
    ok, info = _scalar_ok(st["g_loss"], r32["g_losses"][0], r64["g_losses"][0])
    if not ok: fail.append(("g_loss", info))
    ok, info = _scalar_ok(st["F"], r32["F"], r64["F"])
    if not ok: fail.append(("F", info))
    # G gradients of the round and updated parameters
    p32, p64 = g_params(srv.G), g_params(srv64.G)
    for k, v in step.g_grad_views.items():
        ok, e, a = within(v, p32[k].grad, p64[k].grad)
        if not ok: fail.append(("grad", k, e, a))
    for k, v in step.g_views.items():
        # Adam's first step maps g to -lr*g/(|g|+eps): a gradient error dg (itself checked
        # above) moves the parameter by at most lr*|dg|/(|g|+eps) per element -- the bound that
        # governs the analytically-zero grads of Linear biases feeding BatchNorm, and the
        # small-|g| elements of every tensor
        g64 = p64[k].grad.detach().double().flatten()
        dg = (step.g_grad_views[k].detach().double().cpu().flatten() - g64).abs()
        extra = 1.5 * float((2e-4 * dg / (g64.abs() + 1e-8)).norm())
        ok, e, a = within(v, p32[k], p64[k], extra)
        if not ok: fail.append(("param", k, e, a))
    for k, v in step.d_views.items():
        ok, e, a = within(v, workers[0].D.params[k], workers64[0].D.params[k])
        if not ok: fail.append(("D param", k, e, a))
    # BatchNorm running statistics (two train-mode forward calls per round)
    sd32, sd64 = srv.G.state_dict(), srv64.G.state_dict()
    for k, v in step.running.items():
        ok, e, a = within(v, sd32[k], sd64[k])
        if not ok: fail.append(("running", k, e, a))
    gsd = step.g_state_dict()
    for k in sd32:
        if k.endswith("num_batches_tracked"):
            if int(gsd[k]) != int(sd32[k]):
                fail.append(("num_batches_tracked", k))
    return fail, st


def gpu_kink_margin(step, slope=0.2):
    """min over every LeakyReLU input of the round the HIP step just ran of |x| / std(x), read from
    the step's own activations (cgl_gan_tensor: G layers' LeakyReLU outputs, the D-step and G-loss
    hidden layers through the D actually used -- the updated D for the G loss).  LeakyReLU keeps the
    sign, so x = y (y > 0) or y / slope.  A LeakyReLU' mask can differ from the fp64 oracle's only
    where |x| is within rounding distance of 0 (fp32 pre-activation errors are ~3e-7 std, up to a
    few 1e-6 std), so rounds whose margin is >= KINK_MARGIN are comparable at the 1e-5 bound."""
    gm, dm = step.gm, step.dm
    codes = [(48 + l) if gm.bn[l] else (64 + l) for l in range(gm.n_layers - 1)]
    codes += [112 + j for j in range(dm.n_layers - 1)] + [128 + j for j in range(dm.n_layers - 1)]
    m = float("inf")
    for c in codes:
        y = step.internal(c)
        x = torch.where(y > 0, y, y / slope)
        m = min(m, float(x.abs().min() / (x.std() + 1e-30)))
    return m


def gpu_masks(step):
    """The LeakyReLU branch decisions (x > 0) the HIP round just took, per oracle forward call:
    ``g`` -- [G(z1) call, G(z2) call], one mask per hidden G layer; ``d`` -- [D(real), D(fake) of the
    (last) local D step, D(Xg) of the G loss], one mask per hidden D layer (cgl_gan_tensor 48+/64+,
    112+, 128+; LeakyReLU keeps the sign, so y > 0 <=> x > 0)."""
    gm, dm, B, Br = step.gm, step.dm, step.B, step.Br
    gt = [step.internal((48 + l) if gm.bn[l] else (64 + l)).view(2 * B, -1) > 0 for l in range(gm.n_layers - 1)]
    P = [step.internal(112 + j).view(Br + B, -1) > 0 for j in range(dm.n_layers - 1)]
    S = [step.internal(128 + j).view(B, -1) > 0 for j in range(dm.n_layers - 1)]
    return {"g": [[t[:B].cpu() for t in gt], [t[B:].cpu() for t in gt]],
            "d": [[p[:Br].cpu() for p in P], [p[Br:].cpu() for p in P], [s.cpu() for s in S]]}


class MaskedRun:
    """Make oracle runs follow the HIP round's branch decisions at the LeakyReLU kinks.

    A mask can only differ from the fp64 oracle's own sign where |x| is at rounding level (fp32
    pre-activation errors are ~3e-7 std, at most a few 1e-6 std), and such a flip -- a legitimate fp32
    outcome -- moves the gradients by O(1/sqrt(rows x features)), far above the 1e-5 bound.  So the
    oracle runs are fed the GPU's masks (SeqNet.mask_feed), which makes the 1e-5 comparison a test of
    everything but those decisions, and the decisions themselves are checked by ``check_signs``: every
    fed mask agrees with the sign of the fp64 run's own LeakyReLU input wherever |x| > SIGN_TOL std."""

    SIGN_TOL = 2e-5

    def __init__(self, G, workers, masks, head_layer=None):
        """``masks``: gpu_masks() of each worker (the replicated G's from worker 0, or, with a Mix-G
        ``head_layer``, the trunk's from worker 0 and head h's from worker h)."""
        self.fed = []
        if head_layer is None:
            self._feed(G, masks[0]["g"])
        else:
            self._feed(G.trunk, [c[:head_layer] for c in masks[0]["g"]])
            for h, hd in enumerate(G.heads):
                self._feed(hd, [c[head_layer:] for c in masks[h]["g"]])
        for w, m in zip(workers, masks):
            self._feed(w.D, m["d"])

    def _feed(self, net, calls):
        net.mask_feed = [list(c) for c in calls]
        net.trace_sink = []
        self.fed.append((net, [m for c in calls for m in c]))

    def check_signs(self):
        worst = 0.0
        for net, fed in self.fed:
            assert not net.mask_feed, "oracle made fewer forward calls than the HIP round"
            assert len(net.trace_sink) == len(fed)
            for x, m in zip(net.trace_sink, fed):
                x = x.reshape(m.shape)
                bad = (x > 0) != m
                if bool(bad.any()):
                    worst = max(worst, float(x[bad].abs().max() / x.std()))
        assert worst <= self.SIGN_TOL, f"GPU LeakyReLU branch differs from fp64 at |x| = {worst:.2e} std"
        return worst


def masked_pair(G32, workers32, G64, workers64, masks, head_layer=None):
    """Feed the same GPU masks to the fp32 and the fp64 oracle (see MaskedRun)."""
    return MaskedRun(G32, workers32, masks, head_layer), MaskedRun(G64, workers64, masks, head_layer)
