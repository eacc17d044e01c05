"""nn.Module drop-ins for CGLGAN/2DMG/model.py (the 2-D Gaussian-mixture ring GAN), computed by
libcglgan_hip.

``Generator(img_shape, num_client)``: trunk ``model`` = Linear(100, 32), LeakyReLU(0.2); one head per
client in ``paths`` = Linear(32, 2), Tanh; the heads' points concatenated on the batch dimension
(CGLGAN/2DMG/model.py:26-48; ``img_shape`` is stored and not used by forward, as in the reference).
``Discriminator(ns=1)``: Linear(2, 128), LeakyReLU, Linear(128, 256), LeakyReLU, Linear(256, 1),
Sigmoid (:52-71).  Same trees, attributes and state-dict keys as the reference; every layer runs
through the HIP ops of ``cglgan.model`` (asynchronous, graph-capturable), no CPU fallback.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .model import run_sequential


class Generator(nn.Module):
    """CGLGAN/2DMG/model.py:26-48: z[B,100] -> [num_client * B, 2]."""

    def __init__(self, img_shape, num_client):
        super().__init__()
        self.img_shape = img_shape
        self.model = nn.Sequential(nn.Linear(100, 32), nn.LeakyReLU(0.2))
        modules = nn.ModuleList()
        for _ in range(num_client):
            modules.append(nn.Sequential(nn.Linear(32, 2), nn.Tanh()))
        self.paths = modules

    def forward(self, z):
        hidden_space = run_sequential(self.model, z)
        return torch.cat([run_sequential(path, hidden_space) for path in self.paths], dim=0)


class Discriminator(nn.Module):
    """CGLGAN/2DMG/model.py:52-71: point[B,2] -> validity in (0, 1)."""

    def __init__(self, ns=1):
        super().__init__()
        self.model = nn.Sequential(nn.Linear(2, 128), nn.LeakyReLU(0.2), nn.Linear(128, 256), nn.LeakyReLU(0.2),
                                   nn.Linear(256, 1), nn.Sigmoid())

    def forward(self, img):
        return run_sequential(self.model, img.reshape(img.shape[0], -1))
