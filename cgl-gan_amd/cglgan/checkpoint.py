"""Checkpoint files in the reference drivers' format.

Server.run writes, every 5000 rounds and at the end (capgan.py:185-200; mixed-gan.py likewise;
MDGAN/MNIST/mdgan.py:168-170 with its own 3-tuple):

  ``torch.save(net_g.state_dict(), "<dir>/<name>.pt")``   -- the generator state dict under the
      reference's keys (model.0.weight, model.3.running_var, paths.i.4.bias ...), CPU tensors
  ``pkl.dump((client_list, beta, lambda_list, [], gen_data, betas, gammas), f)`` -- "config<name>.pkl"

``save_server`` writes both from a fused step (cglgan.GanStep / ConvGanStep, whose state dicts carry
the reference's keys) or any module; ``load_generator`` reads a .pt back with torch.load(weights_only=
True), so reference checkpoints load into cglgan.model modules and vice versa.

Resume (new; the reference cannot resume): ``save_resume`` / ``load_resume`` write and read one file
per worker with the step's whole training state (``resume_state()``: both models, both Adams, the
round counter that drives z, the sampler and the Dropout counters, lambda) plus caller metadata --
tensors, ints, floats and strings only, so it loads with ``weights_only=True``.  A run resumed from
round r continues bitwise as the uninterrupted run would (tests/test_gpu_resume.py).
"""
from __future__ import annotations

import os
import pickle

import torch


def _cpu_state(sd):
    return {k: (v.detach().cpu().clone() if torch.is_tensor(v) else v) for k, v in sd.items()}


def generator_state(obj):
    """The reference-keyed generator state dict of a GanStep (g_state_dict), ConvGanStep (G) or module."""
    if hasattr(obj, "g_state_dict"):
        return obj.g_state_dict()
    if hasattr(obj, "G") and hasattr(obj.G, "state_dict"):
        return obj.G.state_dict()
    return obj.state_dict()


def save_server(obj, directory: str, name: str, client_list, beta, lambda_list=(), gen_data=(), betas=(),
                gammas=()):
    """capgan.py:198-200: ``<name>.pt`` (generator state dict) + ``config<name>.pkl`` (7-tuple)."""
    os.makedirs(directory, exist_ok=True)
    pt = os.path.join(directory, f"{name}.pt")
    torch.save(_cpu_state(generator_state(obj)), pt)
    cfg = os.path.join(directory, f"config{name}.pkl")
    beta_t = beta.detach().cpu() if torch.is_tensor(beta) else torch.tensor([float(b) for b in beta])
    tup = (list(client_list), beta_t, list(lambda_list), [], [g.detach().cpu() if torch.is_tensor(g) else g
                                                             for g in gen_data], list(betas), list(gammas))
    with open(cfg, "wb") as f:
        pickle.dump(tup, f)
    return pt, cfg


def save_resume(obj, path: str, **meta):
    """One worker's resume file: ``obj.resume_state()`` under "state" + ``meta`` (round, config ...)."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save({"state": dict(obj.resume_state()), "meta": dict(meta)}, tmp)
    os.replace(tmp, path)            # a crash mid-write never leaves a truncated resume file
    return path


def load_resume(obj, path: str):
    """Restore ``obj`` from a save_resume file; returns its metadata."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    obj.load_resume_state(ck["state"])
    return ck["meta"]


def load_generator(path: str):
    """A generator checkpoint (``torch.save(state_dict)``) -- tensors only, loaded without unpickling code."""
    return torch.load(path, map_location="cpu", weights_only=True)
