"""Replays of the golden-fixture configurations through ``oracle/`` (test helper).

Each function rebuilds the exact run that ``tests/golden/make_golden.py`` performed
with the reference's model modules, but through the oracle's functional
restatement, and returns comparable records.
"""
import hashlib
import json
import os

import torch

from oracle import gan_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_steps.json")


def load_golden():
    with open(GOLDEN) as f:
        return json.load(f)


def sha(t):
    return hashlib.sha256(t.detach().contiguous().float().numpy().tobytes()).hexdigest()


def capgan_replay(cfg, with_state=False):
    n = cfg["n_workers"]
    G, workers = O.build_capgan(n, loss=cfg["loss"])
    beta = torch.tensor([float(s) for s in cfg["beta_sizes"]])
    beta = beta / beta.sum()
    srv = O.CapganServer(G, beta)
    traj = {"d_loss": [], "g_loss": [], "F": [], "lambda": [], "alpha": []}
    first = None
    for step in range(cfg["steps"]):
        z1, z2, reals = O.synthetic_inputs(cfg["B"], n, cfg["epoch"], seed=cfg["input_seed0"] + step,
                                           B_real=cfg["B_real"])
        grads_cb = {}
        r = srv.round(workers, z1, z2, reals, weighting=cfg["weighting"])
        if step == 0:
            first = {"Xd": r["Xd"], "Xg": r["Xg"],
                     "g_grads": {k: p.grad.clone() for k, p in G.params.items()}}
        traj["d_loss"].append([float(x) for x in r["d_losses"].tolist()])
        traj["g_loss"].append([float(x) for x in r["g_losses"].tolist()])
        traj["F"].append(float(r["F"].item()))
        traj["lambda"].append(float(r["lam"].item()))
        traj["alpha"].append([float(x) for x in r["alpha"].tolist()])
    return traj, first, G, workers


def mixg_replay(cfg):
    n = cfg["n_heads"]
    G, workers = O.build_mixg(n)
    beta = torch.tensor([float(s) for s in cfg["beta_sizes"]])
    beta = beta / beta.sum()
    srv = O.MixgServer(G, beta, weighting="mix_double" if cfg["double_softmax"] else "mix_single")
    traj = {"d_loss": [], "g_loss": [], "F": [], "lambda": []}
    first = None
    for step in range(cfg["steps"]):
        z1, z2, reals = O.synthetic_inputs(cfg["B"], n, 1, seed=cfg["input_seed0"] + step)
        r = srv.round(workers, z1, z2, reals)
        if step == 0:
            first = {"g_grads": {k: p.grad.clone() for k, p in
                                 list(G.trunk.params.items()) + [kv for h in G.heads for kv in h.params.items()]}}
        traj["d_loss"].append([float(x) for x in r["d_losses"].tolist()])
        traj["g_loss"].append([float(x) for x in r["g_losses"].tolist()])
        traj["F"].append(float(r["F"].item()))
        traj["lambda"].append(float(r["lam"].item()))
    return traj, first, G, workers


def ring_replay(cfg):
    torch.manual_seed(O.SEED)
    data, _ = O.gmm_ring(8, cfg["n_points_per_class"])
    G, workers = O.build_ring(1, 1)
    init = (dict(G.state_dict()), dict(workers[0].D.state_dict()))
    init = ({k: v.clone() for k, v in init[0].items()}, {k: v.clone() for k, v in init[1].items()})
    srv = O.CglganServer(G, torch.tensor([1.0]))
    traj = {"d_loss": [], "g_loss": [], "F": [], "lambda": []}
    for step in range(cfg["steps"]):
        g = torch.Generator().manual_seed(cfg["input_seed0"] + step)
        z1 = torch.randn(cfg["B"], 100, generator=g)
        z2 = torch.randn(cfg["B"], 100, generator=g)
        idx = torch.randperm(data.shape[0], generator=g)[:cfg["B"]]
        r = srv.round(workers, z1, z2, [[data[idx]]])
        traj["d_loss"].append([float(x) for x in r["d_losses"].tolist()])
        traj["g_loss"].append([float(x) for x in r["g_losses"].tolist()])
        traj["F"].append(float(r["F"].item()))
        traj["lambda"].append(float(r["lam"].item()))
    return data, init, traj, G, workers
