"""torch-CPU restatement of the model/lsgan.py conv GAN and its worker round (TEST INFRASTRUCTURE ONLY).

See ``oracle/__init__.py``: only tests, ``__graft_entry__.smoke`` and bench.py's ``cpu_baseline`` leg
use this module; the product path never imports it.

Models (reference model/lsgan.py, paths relative to the reference root):
  * ``Generator``      :3-27  -- l1 = Linear(100, 128*8*8), view(B,128,8,8) (:25), conv_blocks =
    Upsample(2) Conv(128,128) BN2d(128,.8) LReLU(.2) Upsample(2) Conv(128,64) BN2d(64,.8) LReLU
    Conv(64,1) Tanh (:10-21)
  * ``Discriminator``  :73-99 -- 4 x [Conv(k3,s2,p1) LReLU(.2) Dropout2d(.25) (BN2d(.8) but block 1)]
    (:77-88), view(B,-1) (:96), adv_layer = Linear(128*2*2, 1) (:92,97)
  * ``MixGenerator``   :37-70 -- the intended trunk/heads split (the reference's forward cannot run:
    ``self.img_shape`` is never set, :68) -- parity unpinned by the reference.

The functional forward takes the Dropout2d scales explicitly (``masks``: one [B, C] tensor per
Dropout2d, value 0 or 1/(1-p)); ``draw_masks`` reproduces torch's own draw (``_dropout_impl``:
``empty(n, c, 1, 1).bernoulli_(1 - p).div_(1 - p)``) so that a reference module run under the same
seed and this oracle agree bit for bit (tests/golden/make_golden.py pins it).

The worker round restates capgan.py:211-262 (Server.train) + :316-349 (Worker.train) with these
models.  The reference never trains model/lsgan.py; the losses offered are the
LSGAN objective (MSELoss; north_star "LSGAN/BCE adversarial loss") and Sigmoid + BCELoss on the
logit -- both parity-unpinned by the reference, pinned against torch's own loss modules.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

from .gan_oracle import ADAM_EPS, B1, B2, BN_EPS, BN_MOMENTUM, LAMBDA_LR, LAMBDA_REG, LR, SLOPE, Adam

DROP_P = 0.25   # nn.Dropout2d(0.25) model/lsgan.py:78

# (key, kind, shape) in the reference's construction (= state-dict) order
G_SPEC = [
    ("l1.0", "linear", (128 * 8 * 8, 100)),
    ("conv_blocks.1", "conv", (128, 128)),
    ("conv_blocks.2", "bn", 128),
    ("conv_blocks.5", "conv", (64, 128)),
    ("conv_blocks.6", "bn", 64),
    ("conv_blocks.8", "conv", (1, 64)),
]
D_SPEC = [
    ("model.0", "conv", (16, 1)),
    ("model.3", "conv", (32, 16)),
    ("model.6", "bn", 32),
    ("model.7", "conv", (64, 32)),
    ("model.10", "bn", 64),
    ("model.11", "conv", (128, 64)),
    ("model.14", "bn", 128),
    ("adv_layer", "linear", (1, 128 * 2 * 2)),
]
D_CHANNELS = [16, 32, 64, 128]


def init_params(spec, generator=None):
    """nn.Linear / nn.Conv2d reset_parameters (kaiming_uniform_(a=sqrt(5)), bias U(+-1/sqrt(fan_in)))
    and BatchNorm (1, 0; running 0 / 1), drawn in construction order from the torch CPU RNG, so that
    ``torch.manual_seed(s); init_params(G_SPEC)`` equals ``torch.manual_seed(s); Generator(ims)``."""
    params, buffers = OrderedDict(), OrderedDict()
    for key, kind, shp in spec:
        if kind in ("linear", "conv"):
            w = torch.empty(*shp) if kind == "linear" else torch.empty(shp[0], shp[1], 3, 3)
            b = torch.empty(shp[0])
            torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5), generator=generator)
            fan_in = w[0].numel()
            bound = 1.0 / math.sqrt(fan_in)
            torch.nn.init.uniform_(b, -bound, bound, generator=generator)
            params[key + ".weight"], params[key + ".bias"] = w, b
        else:
            params[key + ".weight"], params[key + ".bias"] = torch.ones(shp), torch.zeros(shp)
            buffers[key + ".running_mean"] = torch.zeros(shp)
            buffers[key + ".running_var"] = torch.ones(shp)
            buffers[key + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return params, buffers


def draw_masks(n, channels=D_CHANNELS, p=DROP_P):
    """torch's Dropout2d noise for one D forward call, in call order (one bernoulli per block)."""
    return [torch.empty(n, c, 1, 1).bernoulli_(1 - p).div_(1 - p).view(n, c) for c in channels]


def _bn(x, P, Bf, key, train):
    if train:
        Bf[key + ".num_batches_tracked"].add_(1)
    return F.batch_norm(x, Bf[key + ".running_mean"], Bf[key + ".running_var"], P[key + ".weight"],
                        P[key + ".bias"], train, BN_MOMENTUM, BN_EPS)


def _leaky(x, signs=None, trace=None):
    """LeakyReLU(0.2).  ``signs`` (a list, consumed in call order): the branch decisions (x > 0) to
    follow instead of x's own sign -- used by the parity tests to make an oracle run take the GPU
    round's decisions at the kinks (a flip there is a legitimate fp32 outcome, checked separately);
    ``trace`` (a list) collects every LeakyReLU input."""
    if trace is not None:
        trace.append(x.detach())
    if signs:
        m = signs.pop(0).to(x.device).reshape(x.shape)
        return torch.where(m, x, x * SLOPE)
    return F.leaky_relu(x, SLOPE)


def g_forward(P, Bf, z, train=True, signs=None, trace=None):
    """Generator.forward model/lsgan.py:23-27 (+ conv_blocks :10-21)."""
    out = F.linear(z, P["l1.0.weight"], P["l1.0.bias"])
    x = out.view(out.shape[0], 128, 8, 8)
    x = F.interpolate(x, scale_factor=2, mode="nearest")
    x = F.conv2d(x, P["conv_blocks.1.weight"], P["conv_blocks.1.bias"], 1, 1)
    x = _leaky(_bn(x, P, Bf, "conv_blocks.2", train), signs, trace)
    x = F.interpolate(x, scale_factor=2, mode="nearest")
    x = F.conv2d(x, P["conv_blocks.5.weight"], P["conv_blocks.5.bias"], 1, 1)
    x = _leaky(_bn(x, P, Bf, "conv_blocks.6", train), signs, trace)
    x = F.conv2d(x, P["conv_blocks.8.weight"], P["conv_blocks.8.bias"], 1, 1)
    return torch.tanh(x)


def d_forward(P, Bf, img, masks=None, train=True, signs=None, trace=None):
    """Discriminator.forward model/lsgan.py:94-99; ``masks`` = the 4 Dropout2d scales [B, C]
    (None in eval mode: Dropout2d is the identity)."""
    x = img
    convs = ["model.0", "model.3", "model.7", "model.11"]
    bns = [None, "model.6", "model.10", "model.14"]
    for i, (ck, bk) in enumerate(zip(convs, bns)):
        x = F.conv2d(x, P[ck + ".weight"], P[ck + ".bias"], 2, 1)
        x = _leaky(x, signs, trace)
        if train:
            x = x * masks[i].to(x.dtype)[:, :, None, None]
        if bk is not None:
            x = _bn(x, P, Bf, bk, train)
    out = x.reshape(x.shape[0], -1)
    return F.linear(out, P["adv_layer.weight"], P["adv_layer.bias"])


MIX_TRUNK_SPEC = [("model.0.0", "linear", (128 * 8 * 8, 100)), ("model.3", "conv", (128, 128)), ("model.4", "bn", 128),
                  ("model.7", "conv", (64, 128))]


def mix_head_spec(h):
    """One head of model/lsgan.py:53-60: BatchNorm2d(64, 0.8), LeakyReLU, Conv2d(64, 1), Tanh."""
    return [(f"paths.{h}.0", "bn", 64), (f"paths.{h}.2", "conv", (1, 64))]


def mixg_forward(P, Bf, z, n_heads, train=True):
    """MixGenerator.forward as model/lsgan.py:63-70 intends it (the reference's own forward raises at
    :68, ``self.img_shape`` unset -- parity unpinned by the reference): trunk once, every head on the
    same hidden tensor, heads concatenated on the batch dimension."""
    out = F.linear(z, P["model.0.0.weight"], P["model.0.0.bias"])
    x = out.view(out.shape[0], 128, 8, 8)
    x = F.interpolate(x, scale_factor=2, mode="nearest")
    x = F.conv2d(x, P["model.3.weight"], P["model.3.bias"], 1, 1)
    x = F.leaky_relu(_bn(x, P, Bf, "model.4", train), SLOPE)
    x = F.interpolate(x, scale_factor=2, mode="nearest")
    hidden = F.conv2d(x, P["model.7.weight"], P["model.7.bias"], 1, 1)
    imgs = []
    for h in range(n_heads):
        y = F.leaky_relu(_bn(hidden, P, Bf, f"paths.{h}.0", train), SLOPE)
        imgs.append(torch.tanh(F.conv2d(y, P[f"paths.{h}.2.weight"], P[f"paths.{h}.2.bias"], 1, 1)))
    return torch.cat(imgs, dim=0)


def adv_loss(v, target, kind):
    """LSGAN MSELoss (kind "mse") or nn.Sigmoid + nn.BCELoss (kind "bce") on the D logit."""
    t = torch.full_like(v, float(target))
    if kind == "mse":
        return F.mse_loss(v, t)
    return F.binary_cross_entropy(torch.sigmoid(v), t)


class ConvGan:
    """One CAPGAN worker + its server on the conv GAN (N = 1: alpha = 1, capgan.py:247-249)."""

    def __init__(self, gp, gb, dp, db, loss="mse", dtype=torch.float64):
        cv = lambda d: OrderedDict((k, v.detach().clone().to(dtype if v.is_floating_point() else v.dtype))
                                   for k, v in d.items())
        self.gp, self.gb, self.dp, self.db = cv(gp), cv(gb), cv(dp), cv(db)
        for p in list(self.gp.values()) + list(self.dp.values()):
            p.requires_grad_(True)
        self.loss = loss
        self.opt_g = Adam(list(self.gp.values()), LR, (B1, B2), ADAM_EPS)
        self.opt_d = Adam(list(self.dp.values()), LR, (B1, B2), ADAM_EPS)
        self.lam = 0.0
        self.dtype = dtype

    CALLS = ("g1", "g2", "dr", "df", "dg")   # forward calls of a round: G(z1), G(z2), D(real), D(Xd), D(Xg)

    def round(self, z1, z2, real, masks_real, masks_fake, masks_g, signs=None, trace=None):
        """capgan.py:215-260 with one worker (capgan.py:324-347), explicit inputs and masks.
        ``signs`` / ``trace``: optional dicts keyed by CALLS -- the LeakyReLU branch decisions to follow
        in each forward call and the lists that collect its LeakyReLU inputs (see ``_leaky``)."""
        dt = self.dtype
        z1, z2, real = z1.to(dt), z2.to(dt), real.to(dt)
        sg = lambda k: list(signs[k]) if signs else None
        tr = lambda k: trace.setdefault(k, []) if trace is not None else None
        with torch.no_grad():
            Xd = g_forward(self.gp, self.gb, z1, signs=sg("g1"), trace=tr("g1"))
        Xg = g_forward(self.gp, self.gb, z2, signs=sg("g2"), trace=tr("g2"))
        half = 0.5 if self.loss == "mse" else 1.0
        for p in self.dp.values():
            p.grad = None
        real_loss = adv_loss(d_forward(self.dp, self.db, real, masks_real, signs=sg("dr"), trace=tr("dr")), 1,
                             self.loss)
        fake_loss = adv_loss(d_forward(self.dp, self.db, Xd.detach(), masks_fake, signs=sg("df"), trace=tr("df")), 0,
                             self.loss)
        d_loss = (real_loss + fake_loss) * half
        d_loss.backward()
        d_grads = OrderedDict((k, p.grad.detach().clone()) for k, p in self.dp.items())
        self.opt_d.step()
        for p in self.gp.values():
            p.grad = None
        g_loss = adv_loss(d_forward(self.dp, self.db, Xg, masks_g, signs=sg("dg"), trace=tr("dg")), 1, self.loss)
        F_max = g_loss - LAMBDA_REG * self.lam
        F_max.backward()
        g_grads = OrderedDict((k, p.grad.detach().clone()) for k, p in self.gp.items())
        self.lam = self.lam + LAMBDA_LR * LAMBDA_REG   # SGD on Lambda: dF/dLambda = -0.001
        self.opt_g.step()
        return dict(Xd=Xd.detach(), Xg=Xg.detach(), d_loss=float(d_loss.detach()), d_real=float(real_loss.detach()),
                    d_fake=float(fake_loss.detach()), g_loss=float(g_loss.detach()), d_grads=d_grads, g_grads=g_grads)


class ConvCapgan:
    """N CAPGAN workers + their server on the conv GAN: capgan.py:211-262 (Server.train: Xd / Xg once,
    the N worker losses gathered, alpha = softmax(softmax(lambda l) * beta), F = sum alpha l - 0.001 lambda,
    F.backward() through every worker's D into the shared G, SGD on lambda, Adam G) with each worker's
    Worker.train (:316-349) on its own D and real batch.  ``weighting="mean"``: MDGAN/MNIST/mdgan.py:203-205
    (F = mean l, no lambda term)."""

    def __init__(self, gp, gb, dps, dbs, beta, loss="mse", weighting="capgan", dtype=torch.float64):
        from .gan_oracle import capgan_alpha
        self._alpha = capgan_alpha
        cv = lambda d: OrderedDict((k, v.detach().clone().to(dtype if v.is_floating_point() else v.dtype))
                                   for k, v in d.items())
        self.gp, self.gb = cv(gp), cv(gb)
        self.dps, self.dbs = [cv(d) for d in dps], [cv(d) for d in dbs]
        for p in list(self.gp.values()) + [p for d in self.dps for p in d.values()]:
            p.requires_grad_(True)
        self.loss, self.weighting, self.dtype = loss, weighting, dtype
        self.beta = torch.tensor([float(b) for b in beta], dtype=dtype)
        self.opt_g = Adam(list(self.gp.values()), LR, (B1, B2), ADAM_EPS)
        self.opt_d = [Adam(list(d.values()), LR, (B1, B2), ADAM_EPS) for d in self.dps]
        self.lam = 0.0

    def round(self, z1, z2, reals, masks):
        """``reals[i]`` worker i's real batch, ``masks[i]`` = (real-call, fake-call, G-loss-call) Dropout2d scales."""
        dt = self.dtype
        z1, z2 = z1.to(dt), z2.to(dt)
        with torch.no_grad():
            Xd = g_forward(self.gp, self.gb, z1)
        Xg = g_forward(self.gp, self.gb, z2)
        half = 0.5 if self.loss == "mse" else 1.0
        losses, d_grads = [], []
        for i, (dp, db) in enumerate(zip(self.dps, self.dbs)):
            mr, mf, mg = masks[i]
            for p in dp.values():
                p.grad = None
            d_loss = (adv_loss(d_forward(dp, db, reals[i].to(dt), mr), 1, self.loss) +
                      adv_loss(d_forward(dp, db, Xd.detach(), mf), 0, self.loss)) * half
            d_loss.backward()
            d_grads.append(OrderedDict((k, p.grad.detach().clone()) for k, p in dp.items()))
            self.opt_d[i].step()
            losses.append(adv_loss(d_forward(dp, db, Xg, mg), 1, self.loss))
        l = torch.stack(losses)
        lam = torch.tensor(self.lam, dtype=dt)
        n = len(self.dps)
        if self.weighting == "capgan":
            alpha = self._alpha(lam, l.detach(), self.beta)
            F_max = (alpha * l).sum() - LAMBDA_REG * lam
        elif self.weighting == "mean":
            alpha = torch.full((n,), 1.0 / n, dtype=dt)
            F_max = l.mean()
        else:
            raise ValueError(self.weighting)
        for p in self.gp.values():
            p.grad = None
        F_max.backward()
        g_grads = OrderedDict((k, p.grad.detach().clone()) for k, p in self.gp.items())
        if self.weighting == "capgan":
            # optim.SGD step on the fp32 0-d Lambda: p + (-lr) * grad, grad = -0.001 (capgan.py:141,249,259)
            f32 = lambda x: torch.tensor(x, dtype=torch.float32)
            self.lam = float(f32(self.lam) + f32(-LAMBDA_LR) * f32(-LAMBDA_REG))
        self.opt_g.step()
        return dict(Xd=Xd.detach(), Xg=Xg.detach(), losses=l.detach(), alpha=alpha.detach(), g_grads=g_grads,
                    d_grads=d_grads)
