"""Generate the golden fixtures that pin ``oracle/`` (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (NetworkCommunication/CGL-GAN) has no tests and no golden vectors
(SURVEY.md section 4), and its drivers cannot be imported here (torchvision/fedlab missing,
network download at module scope, hard-coded CUDA: SURVEY F6/F7).  Its *model*
modules are plain torch and import fine, so this script loads them from
``/root/reference`` and drives them with a line-by-line restatement of the
drivers' training step written against ``nn.Module`` + ``torch.optim`` -- an
implementation independent of ``oracle/gan_oracle.py`` (functional specs +
hand-written Adam).  Outputs are data only (losses, hashes, slices, norms and,
for the tiny 2-D ring models, full tensors); no reference source is copied.

Everything runs on CPU with one thread so the fixtures are bit-reproducible.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys

sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference tree

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn, optim

REF = os.environ.get("CGL_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 20211212
torch.set_num_threads(1)


def _load(relpath, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


mnist_model = _load("model/mnist_model.py", "ref_mnist_model")
md_model = _load("MDGAN/MNIST/mnist_model.py", "ref_mdgan_model")
ring_model = _load("CGLGAN/2DMG/model.py", "ref_ring_model")

IMS = (1, 28, 28)
lsgan_model = _load("model/lsgan.py", "ref_lsgan_model")


def sha(t):
    return hashlib.sha256(t.detach().contiguous().float().numpy().tobytes()).hexdigest()


def summarize(sd, full=False):
    """Per-tensor sha256 (bitwise pin at 1 thread), L2 norm (float64), first 16 values."""
    out = {}
    for k, v in sd.items():
        if v.dtype == torch.long:
            out[k] = {"int": int(v.item())}
            continue
        ent = {"sha256": sha(v), "norm": float(v.double().norm().item()),
               "head": [float(x) for x in v.flatten()[:16].tolist()], "shape": list(v.shape)}
        if full:
            ent["full"] = [float(x) for x in v.flatten().tolist()]
        out[k] = ent
    return out


def inputs(B, n_workers, epoch, seed, img_dim=784, z_dim=100, B_real=None):
    """Same recipe as oracle.synthetic_inputs (seeded torch.Generator)."""
    g = torch.Generator().manual_seed(seed)
    z1 = torch.randn(B, z_dim, generator=g)
    z2 = torch.randn(B, z_dim, generator=g)
    br = B if B_real is None else B_real
    reals = [[torch.rand(br, img_dim, generator=g) * 2 - 1 for _ in range(epoch)] for _ in range(n_workers)]
    return z1, z2, reals


def weights_init(m):  # mixed-gan.py:68-77 (restated)
    cn = m.__class__.__name__
    if cn.find("Conv") != -1:
        nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif cn.find("BatchNorm") != -1:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        nn.init.constant_(m.bias.data, 0)
    elif cn.find("Linear") != -1:
        nn.init.normal_(m.weight.data, 0.0, 0.02)
        nn.init.constant_(m.bias.data, 0)


# --------------------------------------------------------------------------------------------
# CAPGAN: Server.train capgan.py:211-262, Worker.train capgan.py:316-349 (driver restated)
# --------------------------------------------------------------------------------------------
def capgan_run(B, n_workers, steps, epoch=1, beta_sizes=None, loss_kind="ce", weighting="capgan",
               B_real=None, record_grads=True):
    torch.manual_seed(SEED)
    net_g = mnist_model.Generator(IMS)
    if loss_kind == "ce":
        nets_d = [mnist_model.Discriminator(IMS) for _ in range(n_workers)]
        lossf = nn.CrossEntropyLoss()
    else:
        nets_d = [md_model.Discriminator(IMS) for _ in range(n_workers)]
        lossf = nn.BCELoss()
    opti_g = optim.Adam(net_g.parameters(), lr=0.0002, betas=(0.5, 0.999))
    optis_d = [optim.Adam(d.parameters(), lr=0.0002, betas=(0.5, 0.999)) for d in nets_d]
    Lambda = torch.tensor(0., requires_grad=True)
    opti_L = optim.SGD([Lambda], lr=0.1)
    sizes = beta_sizes or [1] * n_workers
    beta = torch.tensor([float(s) for s in sizes])
    beta = beta / beta.sum()

    def tgt(n, v):
        if loss_kind == "ce":
            return torch.full((n,), v, dtype=torch.long)
        return torch.full((n, 1), float(v))

    rec = {"d_loss": [], "g_loss": [], "F": [], "lambda": [], "alpha": []}
    first = {}
    for step in range(steps):
        z1, z2, reals = inputs(B, n_workers, epoch, seed=1000 + step, B_real=B_real)
        with torch.no_grad():
            Xd = net_g(z1)
        z2.requires_grad_(True)
        Xg = net_g(z2)
        dls = []
        for i in range(n_workers):
            for e in range(epoch):
                real = reals[i][e].view(-1, *IMS)
                optis_d[i].zero_grad()
                real_loss = lossf(nets_d[i](real), tgt(real.shape[0], 1))
                fake_loss = lossf(nets_d[i](Xd.detach()), tgt(B, 0))
                D_loss = (real_loss + fake_loss) * 0.5 if loss_kind == "ce" else real_loss + fake_loss
                D_loss.backward()
                optis_d[i].step()
                dls.append(float(D_loss.item()))
        opti_g.zero_grad()
        loss = torch.zeros(n_workers)
        for i in range(n_workers):
            g_loss = lossf(nets_d[i](Xg.clone()), tgt(B, 1))
            loss[i] = g_loss.clone()
        opti_L.zero_grad()
        if weighting == "capgan":
            alpha = F.softmax(Lambda.detach() * loss.detach(), dim=0)
            alpha = F.softmax(alpha * beta, dim=0)
            F_max = (alpha * loss).sum() - 0.001 * Lambda
        else:  # MDGAN/MNIST/mdgan.py:203
            alpha = torch.full((n_workers,), 1.0 / n_workers)
            F_max = loss.mean()
        F_max.backward()
        if step == 0:
            first["Xd"] = summarize({"Xd": Xd.detach()})["Xd"]
            first["Xg"] = summarize({"Xg": Xg.detach()})["Xg"]
            if record_grads:
                first["g_grads"] = summarize({k: p.grad for k, p in net_g.named_parameters()})
        opti_L.step()
        opti_g.step()
        rec["d_loss"].append(dls)
        rec["g_loss"].append([float(x) for x in loss.detach().tolist()])
        rec["F"].append(float(F_max.item()))
        rec["lambda"].append(float(Lambda.item()))
        rec["alpha"].append([float(x) for x in alpha.detach().tolist()])
    return {"config": dict(B=B, n_workers=n_workers, steps=steps, epoch=epoch, beta_sizes=sizes,
                           loss=loss_kind, weighting=weighting, B_real=B_real, input_seed0=1000),
            "trajectory": rec, "step1": first,
            "final_G": summarize(net_g.state_dict()),
            "final_D": [summarize(d.state_dict()) for d in nets_d]}


# --------------------------------------------------------------------------------------------
# Mix-G: Server.train mixed-gan.py:238-292, Worker.train mixed-gan.py:355-392 (restated)
# --------------------------------------------------------------------------------------------
def mixg_run(B, n_heads, steps, beta_sizes=None, double_softmax=False):
    torch.manual_seed(SEED)
    net_g = mnist_model.MixGenerator(IMS, n_heads)
    net_g.apply(weights_init)
    nets_d = []
    for _ in range(n_heads):
        d = mnist_model.Discriminator(IMS)
        d.apply(weights_init)
        nets_d.append(d)
    lossf = nn.CrossEntropyLoss()
    opti_g = optim.Adam(net_g.parameters(), lr=0.0002, betas=(0.5, 0.999))
    optis_d = [optim.Adam(d.parameters(), lr=0.0002, betas=(0.5, 0.999)) for d in nets_d]
    Lambda = torch.tensor(0., requires_grad=True)
    opti_L = optim.SGD([Lambda], lr=0.1)
    sizes = beta_sizes or [1] * n_heads
    beta = torch.tensor([float(s) for s in sizes])
    beta = beta / beta.sum()
    rec = {"d_loss": [], "g_loss": [], "F": [], "lambda": []}
    first = {}
    for step in range(steps):
        z1, z2, reals = inputs(B, n_heads, 1, seed=2000 + step)
        with torch.no_grad():
            Xd = torch.chunk(net_g(z1), n_heads, dim=0)
        z2.requires_grad_(True)
        Xg = torch.chunk(net_g(z2), n_heads, dim=0)
        dls = []
        for i in range(n_heads):
            real = reals[i][0].view(-1, *IMS)
            optis_d[i].zero_grad()
            real_loss = lossf(nets_d[i](real), torch.ones(real.shape[0], dtype=torch.long))
            fake_loss = lossf(nets_d[i](Xd[i].clone()), torch.zeros(B, dtype=torch.long))
            D_loss = (real_loss + fake_loss) * 0.5
            D_loss.backward()
            optis_d[i].step()
            dls.append(float(D_loss.item()))
        opti_g.zero_grad()
        loss = torch.zeros(n_heads)
        for i in range(n_heads):
            loss[i] = lossf(nets_d[i](Xg[i].clone()), torch.ones(B, dtype=torch.long)).clone()
        losses = loss.sum()
        net_g.model.requires_grad_(False)
        losses.backward(retain_graph=True)
        net_g.model.requires_grad_(True)
        opti_L.zero_grad()
        if double_softmax:
            alpha = F.softmax(beta * F.softmax(Lambda.detach() * loss.detach(), dim=0), dim=0)
        else:
            alpha = F.softmax(beta * Lambda.detach() * loss.detach(), dim=0)
        F_max = (alpha * loss).sum() - 0.001 * Lambda
        net_g.paths.requires_grad_(False)
        F_max.backward()
        net_g.paths.requires_grad_(True)
        if step == 0:
            first["g_grads"] = summarize({k: p.grad for k, p in net_g.named_parameters()})
        opti_L.step()
        opti_g.step()
        rec["d_loss"].append(dls)
        rec["g_loss"].append([float(x) for x in loss.detach().tolist()])
        rec["F"].append(float(F_max.item()))
        rec["lambda"].append(float(Lambda.item()))
    return {"config": dict(B=B, n_heads=n_heads, steps=steps, beta_sizes=sizes, double_softmax=double_softmax,
                           input_seed0=2000),
            "trajectory": rec, "step1": first, "final_G": summarize(net_g.state_dict()),
            "final_D": [summarize(d.state_dict()) for d in nets_d]}


# --------------------------------------------------------------------------------------------
# CGLGAN 2-D ring: Server.train CGLGAN/2DMG/main.py:225-278, Worker.train :344-375 (restated)
# --------------------------------------------------------------------------------------------
def ring_run(B, steps, n_points_per_class=2000):
    torch.manual_seed(SEED)
    data_mod = _load("CGLGAN/2DMG/data.py", "ref_ring_data")  # seeds np.random at import (data.py:4)
    ds = data_mod.gmm(8, n_points_per_class)
    data = ds.data.clone()
    torch.manual_seed(SEED)
    net_g = ring_model.Generator(0, 1)
    net_d = ring_model.Discriminator()
    init_g = {k: v.clone() for k, v in net_g.state_dict().items()}
    init_d = {k: v.clone() for k, v in net_d.state_dict().items()}
    lossf = nn.BCELoss()
    opti_g = optim.Adam(net_g.parameters(), lr=0.0002, betas=(0.5, 0.999))
    opti_d = optim.Adam(net_d.parameters(), lr=0.0002, betas=(0.5, 0.999))
    Lambda = torch.tensor(0.)
    beta = torch.tensor([1.0])
    rec = {"d_loss": [], "g_loss": [], "F": [], "lambda": []}
    for step in range(steps):
        g = torch.Generator().manual_seed(3000 + step)
        z1 = torch.randn(B, 100, generator=g)
        z2 = torch.randn(B, 100, generator=g)
        idx = torch.randperm(data.shape[0], generator=g)[:B]
        real = data[idx]
        with torch.no_grad():
            Xd = net_g(z1)
        z2.requires_grad_(True)
        Xg = net_g(z2)
        opti_d.zero_grad()
        real_loss = lossf(net_d(real), torch.ones(real.shape[0], 1))
        fake_loss = lossf(net_d(Xd.clone()), torch.zeros(B, 1))
        D_loss = real_loss + fake_loss
        D_loss.backward()
        opti_d.step()
        opti_g.zero_grad()
        loss = torch.zeros(1)
        loss[0] = lossf(net_d(Xg.clone()), torch.ones(B, 1)).clone()
        gamma = F.softmax(Lambda * loss, dim=0).detach()
        F_beta = (beta * loss).sum()
        F_gamma = (gamma * loss).sum()
        F_max = (F_beta + F_gamma) / 2
        F_max.backward()
        grad = (loss * loss * gamma).sum() - (loss * gamma * F_gamma).sum()
        Lambda = (Lambda + 10 * grad).detach()
        opti_g.step()
        rec["d_loss"].append([float(D_loss.item())])
        rec["g_loss"].append([float(loss[0].item())])
        rec["F"].append(float(F_max.item()))
        rec["lambda"].append(float(Lambda.item()))
    return {"config": dict(B=B, steps=steps, n_points_per_class=n_points_per_class, input_seed0=3000),
            "data_sha256": sha(data), "data_head": [float(x) for x in data.flatten()[:16].tolist()],
            "init_G": summarize(init_g, full=True), "init_D": summarize(init_d, full=True),
            "trajectory": rec, "final_G": summarize(net_g.state_dict(), full=True),
            "final_D": summarize(net_d.state_dict(), full=True)}


# --------------------------------------------------------------------------------------------
# model/lsgan.py conv GAN: module structure, forward / backward, and a CAPGAN-shaped round
# (capgan.py:211-262 + 316-349 restated with the conv models and an LSGAN MSE or Sigmoid+BCE
# objective; the reference never trains these models).  Dropout2d draws from the
# global torch RNG exactly as in the reference module (torch.manual_seed before the round).
# --------------------------------------------------------------------------------------------
def lsgan_fixtures():
    out = {}
    torch.manual_seed(SEED)
    g = lsgan_model.Generator(None)
    d = lsgan_model.Discriminator(None)
    out["keys_G"] = [[k, list(v.shape)] for k, v in g.state_dict().items()]
    out["keys_D"] = [[k, list(v.shape)] for k, v in d.state_dict().items()]
    out["init_G"] = summarize(g.state_dict())
    out["init_D"] = summarize(d.state_dict())
    # forward / backward at B=4 (train mode), full tensors
    gen = torch.Generator().manual_seed(77)
    z = torch.randn(4, 100, generator=gen)
    img = g(z)
    dy = torch.randn(img.shape, generator=gen)
    (img * dy).sum().backward()
    out["g_fwd"] = {"z_seed": 77, "img": summarize({"img": img.detach()}, full=True)["img"],
                    "grads": summarize({k: p.grad for k, p in g.named_parameters()}),
                    "running": summarize({k: v for k, v in g.state_dict().items() if "running" in k}, full=True)}
    torch.manual_seed(1234)
    real = torch.rand(4, 1, 32, 32, generator=gen) * 2 - 1
    v = d(real)
    (v.sum()).backward()
    out["d_fwd"] = {"rng_seed": 1234, "v": [float(x) for x in v.detach().flatten().tolist()],
                    "grads": summarize({k: p.grad for k, p in d.named_parameters()})}
    g.eval()
    with torch.no_grad():
        out["g_eval"] = summarize({"img": g(z)}, full=True)["img"]
    # 3 CAPGAN rounds (N = 1), B = 8, per objective
    for kind in ("mse", "bce"):
        torch.manual_seed(SEED)
        net_g = lsgan_model.Generator(None)
        net_d = lsgan_model.Discriminator(None)
        opti_g = optim.Adam(net_g.parameters(), lr=0.0002, betas=(0.5, 0.999))
        opti_d = optim.Adam(net_d.parameters(), lr=0.0002, betas=(0.5, 0.999))
        Lambda = torch.tensor(0., requires_grad=True)
        opti_L = optim.SGD([Lambda], lr=0.1)
        crit = nn.MSELoss() if kind == "mse" else nn.BCELoss()
        post = (lambda x: x) if kind == "mse" else torch.sigmoid
        half = 0.5 if kind == "mse" else 1.0
        rec = {"d_loss": [], "g_loss": [], "lambda": []}
        for step in range(3):
            gg = torch.Generator().manual_seed(4000 + step)
            z1 = torch.randn(8, 100, generator=gg)
            z2 = torch.randn(8, 100, generator=gg)
            real = torch.rand(8, 1, 32, 32, generator=gg) * 2 - 1
            torch.manual_seed(5000 + step)    # Dropout2d stream of this round's three D calls
            with torch.no_grad():
                Xd = net_g(z1)
            z2.requires_grad_(True)
            Xg = net_g(z2)
            opti_d.zero_grad()
            real_loss = crit(post(net_d(real)), torch.ones(8, 1))
            fake_loss = crit(post(net_d(Xd.detach())), torch.zeros(8, 1))
            D_loss = (real_loss + fake_loss) * half
            D_loss.backward()
            opti_d.step()
            opti_g.zero_grad()
            loss = torch.zeros(1)
            loss[0] = crit(post(net_d(Xg.clone())), torch.ones(8, 1)).clone()
            opti_L.zero_grad()
            alpha = F.softmax(Lambda.detach() * loss.detach(), dim=0)
            alpha = F.softmax(alpha * torch.tensor([1.0]), dim=0)
            F_max = (alpha * loss).sum() - 0.001 * Lambda
            F_max.backward()
            opti_L.step()
            opti_g.step()
            rec["d_loss"].append(float(D_loss.item()))
            rec["g_loss"].append(float(loss[0].item()))
            rec["lambda"].append(float(Lambda.item()))
        out[f"round_{kind}"] = {"trajectory": rec, "final_G": summarize(net_g.state_dict()),
                                "final_D": summarize(net_d.state_dict()),
                                "config": {"B": 8, "steps": 3, "input_seed0": 4000, "rng_seed0": 5000}}
    return out


def init_hashes():
    """Initial-parameter recipe pins (torch.manual_seed(SEED); Generator; Discriminator)."""
    torch.manual_seed(SEED)
    g = mnist_model.Generator(IMS)
    d = mnist_model.Discriminator(IMS)
    out = {"capgan_G": summarize(g.state_dict()), "capgan_D": summarize(d.state_dict())}
    torch.manual_seed(SEED)
    mg = mnist_model.MixGenerator(IMS, 2)
    mg.apply(weights_init)
    out["mixg2_G"] = summarize(mg.state_dict())
    return out


def main():
    fixtures = {
        "init": init_hashes(),
        "capgan_b64_n1": capgan_run(64, 1, 10),
        "capgan_b256_n1": capgan_run(256, 1, 3),
        "capgan_b64_n3": capgan_run(64, 3, 3, beta_sizes=[100, 200, 300]),
        "capgan_b64_n1_ep2_partial": capgan_run(64, 1, 2, epoch=2, B_real=40, record_grads=False),
        "mdgan_b64_n2": capgan_run(64, 2, 3, loss_kind="bce", weighting="mean"),
        "mixg_b64_n2": mixg_run(64, 2, 3, beta_sizes=[300, 100]),
        "mixg_b64_n2_double": mixg_run(64, 2, 2, beta_sizes=[300, 100], double_softmax=True),
        "ring_b64": ring_run(64, 10),
        "lsgan": lsgan_fixtures(),
    }
    meta = {"torch": torch.__version__, "threads": torch.get_num_threads(), "seed": SEED,
            "generator": "tests/golden/make_golden.py"}
    fixtures["meta"] = meta
    path = os.path.join(OUT, "golden_steps.json")
    with open(path, "w") as f:
        json.dump(fixtures, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
