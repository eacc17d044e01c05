"""nn.Module drop-ins for CGLGAN/MNIST/mnist_model.py, computed by libcglgan_hip.

The reference's CGLGAN MNIST driver builds ``Generator(img_shape, num_client)`` -- a shared trunk
``model`` (block(100, 128, normalize=False), block(128, 256), block(256, 512)) and ``num_client``
heads ``paths`` (block(512, 1024), Linear(1024, prod(img_shape)), Tanh), the heads' images
concatenated on the batch dimension (CGLGAN/MNIST/mnist_model.py:30-64) -- and
``Discriminator(img_shape, ns=1)``: Linear(prod, 512), LeakyReLU, Linear(512, 256), LeakyReLU,
Linear(256, 1), Sigmoid (:69-86; ``ns`` is accepted and unused, as in the reference).

Same module trees, attribute names (``.model`` / ``.paths``, which the driver toggles with
``requires_grad_``) and state-dict keys as the reference; every layer runs through the HIP ops of
``cglgan.model`` (asynchronous, graph-capturable single ops), with no PyTorch-op or CPU fallback.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .model import _block, run_sequential


class Generator(nn.Module):
    """CGLGAN/MNIST/mnist_model.py:30-64: z[B,100] -> [num_client * B, *img_shape]."""

    def __init__(self, img_shape, num_client):
        super().__init__()
        self.img_shape = tuple(img_shape)
        self.model = nn.Sequential(*_block(100, 128, normalize=False), *_block(128, 256), *_block(256, 512))
        modules = nn.ModuleList()
        for _ in range(num_client):
            modules.append(nn.Sequential(*_block(512, 1024), nn.Linear(1024, int(np.prod(self.img_shape))), nn.Tanh()))
        self.paths = modules

    def forward(self, z):
        img = []
        hidden = run_sequential(self.model, z)
        for path in self.paths:
            out = run_sequential(path, hidden)
            img.append(out.view((out.shape[0], *self.img_shape)))
        return torch.cat(img, dim=0)


class Discriminator(nn.Module):
    """CGLGAN/MNIST/mnist_model.py:69-86: img -> validity in (0, 1) (BCELoss in the driver)."""

    def __init__(self, img_shape, ns=1):
        super().__init__()
        self.img_shape = tuple(img_shape)
        self.model = nn.Sequential(nn.Linear(int(np.prod(self.img_shape)), 512), nn.LeakyReLU(0.2), nn.Linear(512, 256),
                                   nn.LeakyReLU(0.2), nn.Linear(256, 1), nn.Sigmoid())

    def forward(self, img):
        return run_sequential(self.model, img.reshape(img.shape[0], -1))
