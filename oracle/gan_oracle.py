"""torch-CPU restatement of the CGL-GAN worker step (TEST INFRASTRUCTURE ONLY).

See ``oracle/__init__.py``: only tests, ``__graft_entry__.smoke`` and bench.py's
``cpu_baseline`` leg use this module.  Every function cites the reference
file:line it restates (paths relative to the reference repository root).

The models are expressed as a flat "sequential spec" so that the same
interpreter covers the reference's MLP ``Generator`` / ``MixGenerator`` /
``Discriminator`` (model/mnist_model.py:5-88), the Sigmoid/BCE discriminator of
MDGAN/MNIST/mnist_model.py:31-50 and the CGLGAN 2-D-ring models
(CGLGAN/2DMG/model.py:26-71).  Parameter keys are the reference state-dict keys
(``model.0.weight`` ...).  Backward uses torch autograd exactly as the reference
does; Adam is restated op-for-op from torch 2.10's ``_single_tensor_adam``
(the CPU default path the reference's ``optim.Adam`` takes).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

LR = 0.0002          # capgan.py:122 (lr_g / lr_d defaults)
B1, B2 = 0.5, 0.999  # capgan.py:52-53
ADAM_EPS = 1e-8      # torch.optim.Adam default
BN_EPS = 0.8         # model/mnist_model.py:13  nn.BatchNorm1d(out_feat, 0.8): 0.8 is eps
BN_MOMENTUM = 0.1    # torch default
SLOPE = 0.2          # nn.LeakyReLU(0.2)
LAMBDA_LR = 0.1      # capgan.py:141  optim.SGD([Lambda], lr=0.1)
LAMBDA_REG = 0.001   # capgan.py:249  F_max = ... - 0.001 * Lambda
SEED = 20211212      # capgan.py:26


# --------------------------------------------------------------------------
# Sequential specs (what nn.Sequential in the reference builds)
# --------------------------------------------------------------------------
def _block(prefix, idx, fin, fout, normalize):
    """``block()`` of model/mnist_model.py:10-15: Linear -> [BatchNorm1d(eps=0.8)] -> LeakyReLU(0.2)."""
    spec = [("linear", f"{prefix}{idx}", fin, fout)]
    idx += 1
    if normalize:
        spec.append(("bn", f"{prefix}{idx}", fout))
        idx += 1
    spec.append(("leaky",))
    idx += 1
    return spec, idx


def mnist_generator_spec(img_dim=784, z_dim=100):
    """``Generator`` model/mnist_model.py:17-24 (100->128->256->512->1024->784, Tanh)."""
    spec, i = [], 0
    for fin, fout, bn in ((z_dim, 128, False), (128, 256, True), (256, 512, True), (512, 1024, True)):
        s, i = _block("model.", i, fin, fout, bn)
        spec += s
    spec.append(("linear", f"model.{i}", 1024, img_dim))
    spec.append(("tanh",))
    return spec


def mnist_mixgen_trunk_spec(z_dim=100):
    """``MixGenerator.model`` model/mnist_model.py:44-48 (100->128->256->512)."""
    spec, i = [], 0
    for fin, fout, bn in ((z_dim, 128, False), (128, 256, True), (256, 512, True)):
        s, i = _block("model.", i, fin, fout, bn)
        spec += s
    return spec


def mnist_mixgen_head_spec(h, img_dim=784):
    """``MixGenerator.paths[h]`` model/mnist_model.py:50-56 (512->1024 BN ->784 Tanh)."""
    s, i = _block(f"paths.{h}.", 0, 512, 1024, True)
    return s + [("linear", f"paths.{h}.{i}", 1024, img_dim), ("tanh",)]


def mnist_discriminator_spec(img_dim=784, sigmoid=False):
    """``Discriminator`` model/mnist_model.py:76-83 (784->512->256->2 logits).

    ``sigmoid=True`` gives MDGAN/MNIST/mnist_model.py:36-43 / CGLGAN/MNIST (->1, Sigmoid)."""
    out = 1 if sigmoid else 2
    spec = [("linear", "model.0", img_dim, 512), ("leaky",),
            ("linear", "model.2", 512, 256), ("leaky",),
            ("linear", "model.4", 256, out)]
    if sigmoid:
        spec.append(("sigmoid",))
    return spec


def ring_generator_trunk_spec():
    """CGLGAN/2DMG/model.py:30-33: Linear(100,32) -> LeakyReLU(0.2)."""
    return [("linear", "model.0", 100, 32), ("leaky",)]


def ring_generator_head_spec(h):
    """CGLGAN/2DMG/model.py:36-41: Linear(32,2) -> Tanh."""
    return [("linear", f"paths.{h}.0", 32, 2), ("tanh",)]


def ring_discriminator_spec():
    """CGLGAN/2DMG/model.py:58-66: 2->128->256->1, Sigmoid."""
    return [("linear", "model.0", 2, 128), ("leaky",), ("linear", "model.2", 128, 256), ("leaky",),
            ("linear", "model.4", 256, 1), ("sigmoid",)]


# --------------------------------------------------------------------------
# 16-bit GEMM operand emulation (test infrastructure for cgl_gan_config.gemm_dtype).  The
# reference computes in fp32 only, so this has no reference counterpart: the 16-bit path's parity
# is unpinned, and this restates what the HIP path computes (every GEMM operand rounded to 16
# bits, exact products, wide accumulation) so that tests can check it at fp32-level tolerance.
# --------------------------------------------------------------------------
class _LowpLinear(torch.autograd.Function):
    """y = r(x) r(W)^T + b; dx = r(dy) r(W); dW = r(dy)^T r(x); db = sum r(dy), r = round to
    ``dt`` (round-to-nearest-even) and back.  ``full`` False: forward and input gradient in full
    precision (the HIP loss head computes the D output layer outside the GEMMs)."""

    @staticmethod
    def forward(ctx, x, w, b, dt, full):
        ctx.save_for_backward(x, w)
        ctx.dt, ctx.full = dt, full
        r = (lambda t: t.to(dt).to(x.dtype)) if full else (lambda t: t)
        return r(x) @ r(w).t() + b

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        rr = lambda t: t.to(ctx.dt).to(gy.dtype)
        r = rr if ctx.full else (lambda t: t)
        return r(gy) @ r(w), rr(gy).t() @ rr(x), rr(gy).sum(0), None, None


# --------------------------------------------------------------------------
# Functional network
# --------------------------------------------------------------------------
class SeqNet:
    """Parameters + buffers of one ``nn.Sequential`` spec, run functionally."""

    def __init__(self, spec, init="default", generator=None):
        self.spec = list(spec)
        self.params = OrderedDict()
        self.buffers = OrderedDict()
        for ent in self.spec:
            if ent[0] == "linear":
                _, key, fin, fout = ent
                w = torch.empty(fout, fin)
                b = torch.empty(fout)
                # nn.Linear.reset_parameters: kaiming_uniform_(a=sqrt(5)) then U(-1/sqrt(fan_in), ..)
                torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5), generator=generator)
                bound = 1.0 / math.sqrt(fin) if fin > 0 else 0.0
                torch.nn.init.uniform_(b, -bound, bound, generator=generator)
                self.params[key + ".weight"] = w
                self.params[key + ".bias"] = b
            elif ent[0] == "bn":
                _, key, n = ent
                self.params[key + ".weight"] = torch.ones(n)
                self.params[key + ".bias"] = torch.zeros(n)
                self.buffers[key + ".running_mean"] = torch.zeros(n)
                self.buffers[key + ".running_var"] = torch.ones(n)
                self.buffers[key + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
        for p in self.params.values():
            p.requires_grad_(True)
        # test hooks (unset = the plain reference arithmetic): ``mask_feed`` -- per forward call, one
        # bool tensor per LeakyReLU (x > 0) imposed instead of the sign of this run's own x, so that a
        # comparison run can follow another implementation's branch decisions at the kink;
        # ``trace_sink`` -- a list collecting every LeakyReLU input (see ``forward``)
        self.mask_feed = []
        self.trace_sink = None
        # ``lowp`` = (dtype, head_key): emulate 16-bit GEMM operands (_LowpLinear); the Linear
        # ``head_key`` (the D output layer) keeps a full-precision forward / input gradient
        self.lowp = None

    # weights_init of mixed-gan.py:68-77 (Linear W~N(0,.02), b=0; BN g~N(1,.02), b=0),
    # applied in nn.Module.apply's post-order == spec order for a flat Sequential.
    def apply_weights_init(self, generator=None):
        with torch.no_grad():
            for ent in self.spec:
                if ent[0] == "linear":
                    torch.nn.init.normal_(self.params[ent[1] + ".weight"], 0.0, 0.02, generator=generator)
                    torch.nn.init.constant_(self.params[ent[1] + ".bias"], 0)
                elif ent[0] == "bn":
                    torch.nn.init.normal_(self.params[ent[1] + ".weight"], 1.0, 0.02, generator=generator)
                    torch.nn.init.constant_(self.params[ent[1] + ".bias"], 0)

    def forward(self, x, train=True, trace=None, masks=None):
        """nn.Sequential forward of the spec (train-mode BatchNorm updates running stats).

        ``trace`` (a list) collects the input of every LeakyReLU (conditioning checks in tests).
        ``masks``: one bool tensor per LeakyReLU, the branch taken (x > 0); by default the next entry
        of ``mask_feed`` if any, else the sign of x itself (= F.leaky_relu, the reference)."""
        h = x.reshape(x.shape[0], -1)
        if masks is None and self.mask_feed:
            masks = self.mask_feed.pop(0)
        if trace is None:
            trace = self.trace_sink
        li = 0
        for ent in self.spec:
            if trace is not None and ent[0] == "leaky":
                trace.append(h.detach())
            kind = ent[0]
            if kind == "leaky" and masks is not None:
                m = masks[li].to(h.device).reshape(h.shape)
                h = torch.where(m, h, h * SLOPE)
                li += 1
                continue
            if kind == "linear" and self.lowp is not None:
                h = _LowpLinear.apply(h, self.params[ent[1] + ".weight"], self.params[ent[1] + ".bias"],
                                      self.lowp[0], ent[1] != self.lowp[1])
            elif kind == "linear":
                h = F.linear(h, self.params[ent[1] + ".weight"], self.params[ent[1] + ".bias"])
            elif kind == "bn":
                k = ent[1]
                if train:
                    self.buffers[k + ".num_batches_tracked"].add_(1)
                h = F.batch_norm(h, self.buffers[k + ".running_mean"], self.buffers[k + ".running_var"],
                                 self.params[k + ".weight"], self.params[k + ".bias"], train, BN_MOMENTUM, BN_EPS)
            elif kind == "leaky":
                h = F.leaky_relu(h, SLOPE)
            elif kind == "tanh":
                h = torch.tanh(h)
            elif kind == "sigmoid":
                h = torch.sigmoid(h)
            else:
                raise ValueError(kind)
        return h

    def parameters(self):
        return list(self.params.values())

    def zero_grad(self):
        for p in self.params.values():
            p.grad = None

    def requires_grad_(self, flag):
        for p in self.params.values():
            p.requires_grad_(flag)

    def state_dict(self):
        sd = OrderedDict()
        for ent in self.spec:
            if ent[0] in ("linear", "bn"):
                sd[ent[1] + ".weight"] = self.params[ent[1] + ".weight"].detach()
                sd[ent[1] + ".bias"] = self.params[ent[1] + ".bias"].detach()
            if ent[0] == "bn":
                for s in ("running_mean", "running_var", "num_batches_tracked"):
                    sd[ent[1] + "." + s] = self.buffers[ent[1] + "." + s]
        return sd


class MixNet:
    """``MixGenerator`` (model/mnist_model.py:32-66, CGLGAN/2DMG/model.py:26-50): trunk + N heads.

    forward returns ``torch.cat([head_i(trunk(z))], 0)`` (model/mnist_model.py:59-66)."""

    def __init__(self, trunk_spec, head_specs, generator=None):
        self.trunk = SeqNet(trunk_spec, generator=generator)
        self.heads = [SeqNet(s, generator=generator) for s in head_specs]

    def forward(self, z, train=True, trace=None):
        h = self.trunk.forward(z, train, trace)
        return torch.cat([hd.forward(h, train, trace) for hd in self.heads], dim=0)

    def apply_weights_init(self, generator=None):
        self.trunk.apply_weights_init(generator)
        for hd in self.heads:
            hd.apply_weights_init(generator)

    def parameters(self):
        ps = self.trunk.parameters()
        for hd in self.heads:
            ps += hd.parameters()
        return ps

    def zero_grad(self):
        self.trunk.zero_grad()
        for hd in self.heads:
            hd.zero_grad()

    def state_dict(self):
        sd = OrderedDict(self.trunk.state_dict())
        for hd in self.heads:
            sd.update(hd.state_dict())
        return sd


# --------------------------------------------------------------------------
# Optimisers
# --------------------------------------------------------------------------
class Adam:
    """torch 2.10 ``_single_tensor_adam`` (CPU, non-capturable, no amsgrad/weight decay), op for op.

    Used by every driver: ``optim.Adam(params, lr=2e-4, betas=(b1, b2))`` (capgan.py:158,312)."""

    def __init__(self, params, lr=LR, betas=(B1, B2), eps=ADAM_EPS):
        self.params = list(params)
        self.lr, (self.b1, self.b2), self.eps = lr, betas, eps
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.step_t = [torch.tensor(0.0) for _ in self.params]

    @torch.no_grad()
    def step(self):
        for p, m, v, st in zip(self.params, self.m, self.v, self.step_t):
            g = p.grad
            if g is None:
                continue
            st += 1
            m.lerp_(g, 1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            step = st.item()
            bias_correction1 = 1 - self.b1 ** step
            bias_correction2 = 1 - self.b2 ** step
            step_size = self.lr / bias_correction1
            bias_correction2_sqrt = bias_correction2 ** 0.5
            denom = (v.sqrt() / bias_correction2_sqrt).add_(self.eps)
            p.addcdiv_(m, denom, value=-step_size)


class LambdaSGD:
    """``self.Lambda = tensor(0., requires_grad=True); opti_L = optim.SGD([Lambda], lr=0.1)`` (capgan.py:140-141)."""

    def __init__(self):
        self.lam = torch.tensor(0.0, requires_grad=True)

    @torch.no_grad()
    def step(self):
        if self.lam.grad is not None:
            self.lam.add_(self.lam.grad, alpha=-LAMBDA_LR)

    def zero_grad(self):
        self.lam.grad = None


# --------------------------------------------------------------------------
# Losses
# --------------------------------------------------------------------------
def ce_loss(logits, target_value):
    """``nn.CrossEntropyLoss()`` with int64 targets filled with 1 (valid) / 0 (fake) (capgan.py:311,331,336)."""
    t = torch.full((logits.shape[0],), target_value, dtype=torch.long)
    return F.cross_entropy(logits, t)


def bce_loss(probs, target_value):
    """``nn.BCELoss()`` on Sigmoid outputs with [B,1] targets (CGLGAN/2DMG/main.py:336,357,362)."""
    t = torch.full((probs.shape[0], 1), float(target_value))
    return F.binary_cross_entropy(probs, t)


# --------------------------------------------------------------------------
# Rounds
# --------------------------------------------------------------------------
def _scaled_backward(loss, scale, params, extra=()):
    """loss.backward(), or (S * loss).backward() with every gradient of ``params`` / ``extra`` then
    divided by S (GradScaler.scale + unscale_; test hook, see Worker.loss_scale)."""
    if not scale:
        loss.backward()
        return
    (loss * scale).backward()
    with torch.no_grad():
        for p in list(params) + list(extra):
            if p.grad is not None:
                p.grad.div_(scale)


class Worker:
    """Worker role: holds D, its Adam and its shard (capgan.py:265-349)."""

    def __init__(self, dnet, loss="ce"):
        self.D = dnet
        self.opt = Adam(self.D.parameters())
        self.loss = loss
        # test hook (None = the reference arithmetic): a static loss scale S, GradScaler-style -- the
        # backward runs on S * loss and the gradients are divided by S before the optimiser step; with
        # ``SeqNet.lowp`` this restates the 16-bit path's dynamic loss scaling on a round without
        # overflow (cgl_gan_config.loss_scale; no reference counterpart, parity unpinned)
        self.loss_scale = None

    def d_step(self, real, X, half=True):
        """One local D step.  CE/0.5 form: capgan.py:331-341; BCE/no-0.5 form: CGLGAN/2DMG/main.py:357-366."""
        lossf = ce_loss if self.loss == "ce" else bce_loss
        self.D.zero_grad()
        real_loss = lossf(self.D.forward(real), 1)
        fake_loss = lossf(self.D.forward(X), 0)
        D_loss = (real_loss + fake_loss) * 0.5 if half else (real_loss + fake_loss)
        _scaled_backward(D_loss, self.loss_scale, self.D.parameters())
        self.opt.step()
        return D_loss.detach()

    def g_loss(self, Xg):
        """capgan.py:343-347: G_loss = loss(net_d(Xg), valid) with the post-update D, graph kept."""
        lossf = ce_loss if self.loss == "ce" else bce_loss
        return lossf(self.D.forward(Xg), 1)


class CapganServer:
    """Server role of capgan.py:120-262 (holds G, lambda, beta)."""

    def __init__(self, gnet, beta):
        self.G = gnet
        self.opt = Adam(self.G.parameters())
        self.L = LambdaSGD()
        self.beta = beta.clone()
        self.loss_scale = None   # test hook: see Worker.loss_scale

    def round(self, workers, z1, z2, reals, weighting="capgan"):
        """One communication round: Server.train capgan.py:211-262 + every Worker.train capgan.py:316-349.

        ``reals[i]`` is the list of ``epoch`` real batches of worker i.
        ``weighting``: "capgan" (capgan.py:247-249, CAPGAN/MNIST/capgan.py:241-243),
        "mean" (MDGAN/MNIST/mdgan.py:203)."""
        N = len(workers)
        with torch.no_grad():
            Xd = self.G.forward(z1)
        Xg = self.G.forward(z2)
        d_losses = []
        for w, rs in zip(workers, reals):
            for r in rs:
                d_losses.append(w.d_step(r, Xd.detach(), half=(w.loss == "ce")))
        self.G.zero_grad()
        loss = torch.zeros(N)
        for i, w in enumerate(workers):
            loss[i] = w.g_loss(Xg.clone()).clone()
        self.L.zero_grad()
        if weighting == "capgan":
            alpha = F.softmax(self.L.lam.detach() * loss.detach(), dim=0)
            alpha = F.softmax(alpha * self.beta, dim=0)
            F_max = (alpha * loss).sum() - LAMBDA_REG * self.L.lam
        elif weighting == "mean":
            alpha = torch.full((N,), 1.0 / N)
            F_max = loss.mean()
        else:
            raise ValueError(weighting)
        _scaled_backward(F_max, self.loss_scale, self.G.parameters(), [self.L.lam])
        self.L.step()
        self.opt.step()
        return dict(Xd=Xd.detach(), Xg=Xg.detach(), d_losses=torch.stack(d_losses), g_losses=loss.detach(),
                    alpha=alpha.detach(), F=F_max.detach(), lam=self.L.lam.detach().clone())


class MixgServer:
    """Server role of mixed-gan.py:127-292: MixGenerator with one head per worker."""

    def __init__(self, mixnet, beta, weighting="mix_single"):
        self.G = mixnet
        self.opt = Adam(self.G.parameters())
        self.L = LambdaSGD()
        self.beta = beta.clone()
        self.weighting = weighting

    def round(self, workers, z1, z2, reals):
        """mixed-gan.py:238-292 (+ worker mixed-gan.py:355-392).

        Phase 1 (heads, trunk frozen) then phase 2 (trunk, heads frozen), exactly as :263-281."""
        N = len(workers)
        with torch.no_grad():
            Xd = torch.chunk(self.G.forward(z1), N, dim=0)
        Xg = torch.chunk(self.G.forward(z2), N, dim=0)
        d_losses = []
        for i, (w, rs) in enumerate(zip(workers, reals)):
            for r in rs:
                d_losses.append(w.d_step(r, Xd[i].clone()))
        self.G.zero_grad()
        loss = torch.zeros(N)
        for i, w in enumerate(workers):
            loss[i] = w.g_loss(Xg[i].clone()).clone()
        losses = loss.sum()
        self.G.trunk.requires_grad_(False)
        losses.backward(retain_graph=True)
        self.G.trunk.requires_grad_(True)
        self.L.zero_grad()
        if self.weighting == "mix_single":      # mixed-gan.py:276
            alpha = F.softmax(self.beta * self.L.lam.detach() * loss.detach(), dim=0)
        elif self.weighting == "mix_double":    # CAPGAN/MNIST/mixed-gan.py:276-278
            alpha = F.softmax(self.beta * F.softmax(self.L.lam.detach() * loss.detach(), dim=0), dim=0)
        else:
            raise ValueError(self.weighting)
        F_max = (alpha * loss).sum() - LAMBDA_REG * self.L.lam
        for hd in self.G.heads:
            hd.requires_grad_(False)
        F_max.backward()
        for hd in self.G.heads:
            hd.requires_grad_(True)
        self.L.step()
        self.opt.step()
        return dict(Xd=torch.cat(Xd).detach(), Xg=torch.cat(Xg).detach(), d_losses=torch.stack(d_losses),
                    g_losses=loss.detach(), alpha=alpha.detach(), F=F_max.detach(), lam=self.L.lam.detach().clone())


class CglganServer:
    """Server role of CGLGAN/2DMG/main.py:139-278 (closed-form lambda ascent, BCE workers).

    The reference's lambda update builds on the live graph (:273-274, a leak); here it is computed
    from detached values, which gives the same numbers."""

    def __init__(self, mixnet, beta):
        self.G = mixnet
        self.opt = Adam(self.G.parameters())
        self.lam = torch.tensor(0.0)
        self.beta = beta.clone()

    def round(self, workers, z1, z2, reals):
        N = len(workers)
        multi = len(self.G.heads) > 1
        with torch.no_grad():
            out = self.G.forward(z1)
            Xd = torch.chunk(out, N, dim=0) if multi else [out] * N
        outg = self.G.forward(z2)
        Xg = torch.chunk(outg, N, dim=0) if multi else [outg] * N
        d_losses = []
        for i, (w, rs) in enumerate(zip(workers, reals)):
            for r in rs:
                d_losses.append(w.d_step(r, Xd[i].clone(), half=False))
        self.G.zero_grad()
        loss = torch.zeros(N)
        for i, w in enumerate(workers):
            loss[i] = w.g_loss(Xg[i].clone()).clone()
        if multi:
            losses = loss.sum()
            self.G.trunk.requires_grad_(False)
            losses.backward(retain_graph=True)
            self.G.trunk.requires_grad_(True)
        gamma = F.softmax(self.lam * loss, dim=0).detach()
        F_beta = (self.beta * loss).sum()
        F_gamma = (gamma * loss).sum()
        F_max = (F_beta + F_gamma) / 2
        if multi:
            for hd in self.G.heads:
                hd.requires_grad_(False)
            F_max.backward()
            for hd in self.G.heads:
                hd.requires_grad_(True)
        else:
            F_max.backward()
        ld, Fg = loss.detach(), F_gamma.detach()
        grad = (ld * ld * gamma).sum() - (ld * gamma * Fg).sum()
        self.lam = self.lam + 10 * grad
        self.opt.step()
        return dict(Xd=torch.cat(list(Xd)).detach(), Xg=outg.detach(),
                    d_losses=torch.stack(d_losses) if d_losses else torch.zeros(0),   # (no D step: [[]] reals)
                    g_losses=ld, gamma=gamma, F=F_max.detach(), lam=self.lam.clone())


# --------------------------------------------------------------------------
# Aggregation restatements (cross-server / cross-worker exchanges)
# --------------------------------------------------------------------------
def fedavg(state_dicts, data_lens, segema=0.0, self_sd=None):
    """Cloud FedAvg: mixed-gan.py:114-124 (p = sum_s A_s p_s, A_s = data_len_s / sum) and the
    segema mix of mixed-gan.py:198-199.  Tensors with ``len(size) == 0`` are skipped (:155)."""
    A = torch.tensor([float(x) for x in data_lens])
    A = A / A.sum()
    p = OrderedDict()
    for s, sd in enumerate(state_dicts):
        for key, var in sd.items():
            if var.dim() == 0:
                continue
            p[key] = p[key] + var * A[s] if key in p else var * A[s]
    if self_sd is not None:
        for key in p:
            p[key] = segema * self_sd[key] + (1 - segema) * p[key]
    return p


@torch.no_grad()
def eshare_mean(workers):
    """E-share of D: every worker's D <- the mean of the N discriminators,
    summed in worker order.  The only reference code for it is commented out and broken
    (ACGAN/MNIST/acgan.py:240-263), so this is the build's definition: parity unpinned."""
    n = len(workers)
    for k in workers[0].D.params:
        tot = workers[0].D.params[k].detach().clone()
        for w in workers[1:]:
            tot += w.D.params[k]
        tot /= n
        for w in workers:
            w.D.params[k].copy_(tot)


@torch.no_grad()
def dswap(workers, perm):
    """MD-GAN D-swap (MDGAN/MNIST/mdgan.py:158-164 with copy_parameters :233-238, commented out in
    the reference: parity unpinned): worker i continues with D_{perm[i]}'s parameters and keeps its
    own optimiser state."""
    old = [{k: v.detach().clone() for k, v in w.D.params.items()} for w in workers]
    for i, w in enumerate(workers):
        for k, v in w.D.params.items():
            v.copy_(old[perm[i]][k])


def capgan_alpha(lam, losses, beta):
    """capgan.py:247-248: alpha = softmax(softmax(lam*l) * beta)."""
    a = F.softmax(lam * losses, dim=0)
    return F.softmax(a * beta, dim=0)


# --------------------------------------------------------------------------
# 2-D Gaussian ring data (CGLGAN/2DMG/data.py:5-38)
# --------------------------------------------------------------------------
def gmm_ring(n_class=8, x=2000, np_seed=SEED):
    """``gmm(n_class, x)``: n_class modes on the unit circle, std 0.01, sorted by label.

    Reseeds numpy with the value data.py:4 sets at import; the per-sample ``torch.normal`` draws use
    the torch global RNG, as the reference does."""
    rs = np.random.RandomState(np_seed)
    thetas = np.linspace(0, 2 * (1 - 1 / n_class) * np.pi, n_class)
    xs, ys = np.sin(thetas), np.cos(thetas)
    n = x * n_class
    data = torch.zeros(n, 2)
    labels = torch.zeros(n)
    std = 0.01
    for i in range(n):
        coin = rs.randint(0, n_class)
        data[i, :] = torch.normal(mean=torch.Tensor([xs[coin], ys[coin]]), std=std * torch.ones(1, 2))
        labels[i] = coin
    targets, idx = torch.sort(labels)
    return data[idx], targets


# --------------------------------------------------------------------------
# Convenience builders (seed recipe used by the golden fixtures)
# --------------------------------------------------------------------------
def build_capgan(n_workers=1, seed=SEED, loss="ce", img_dim=784):
    """torch.manual_seed(seed); G = Generator(ims); then one D per worker (capgan.py:28,156,309)."""
    torch.manual_seed(seed)
    G = SeqNet(mnist_generator_spec(img_dim))
    workers = [Worker(SeqNet(mnist_discriminator_spec(img_dim, sigmoid=(loss == "bce"))), loss)
               for _ in range(n_workers)]
    return G, workers


def build_mixg(n_heads=2, seed=SEED, img_dim=784):
    """torch.manual_seed(seed); MixGenerator(ims, N).apply(weights_init); D_i with weights_init
    (mixed-gan.py:34,180-181,347-348)."""
    torch.manual_seed(seed)
    G = MixNet(mnist_mixgen_trunk_spec(), [mnist_mixgen_head_spec(h, img_dim) for h in range(n_heads)])
    G.apply_weights_init()
    workers = []
    for _ in range(n_heads):
        d = SeqNet(mnist_discriminator_spec(img_dim))
        d.apply_weights_init()
        workers.append(Worker(d, "ce"))
    return G, workers


def build_ring(n_heads=1, n_workers=1, seed=SEED):
    """CGLGAN 2DMG: torch.manual_seed(seed); Generator(ims, N if iid else 1); Discriminator()
    (CGLGAN/2DMG/main.py:43,191,335)."""
    torch.manual_seed(seed)
    G = MixNet(ring_generator_trunk_spec(), [ring_generator_head_spec(h) for h in range(n_heads)])
    workers = [Worker(SeqNet(ring_discriminator_spec()), "bce") for _ in range(n_workers)]
    return G, workers


def synthetic_inputs(B, n_workers=1, epoch=1, seed=1, img_dim=784, z_dim=100, B_real=None):
    """Explicit step inputs: z ~ N(0,1) [B,100] x2, real ~ U(-1,1) [B_r, img_dim]
    (the range Normalize([0.5],[0.5]) produces, capgan.py:469)."""
    g = torch.Generator().manual_seed(seed)
    z1 = torch.randn(B, z_dim, generator=g)
    z2 = torch.randn(B, z_dim, generator=g)
    br = B if B_real is None else B_real
    reals = [[torch.rand(br, img_dim, generator=g) * 2 - 1 for _ in range(epoch)] for _ in range(n_workers)]
    return z1, z2, reals
