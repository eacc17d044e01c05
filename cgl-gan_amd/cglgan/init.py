"""Parameter initialisation matching the reference modules.

``default_init`` reproduces ``nn.Linear``'s default (kaiming_uniform_(a=sqrt(5)) weight, U(+-1/sqrt(fan_in))
bias) and BatchNorm1d's (weight 1, bias 0) in construction order, drawing from the torch CPU RNG,
so ``torch.manual_seed(s); default_init(...)`` yields the same tensors as
``torch.manual_seed(s); Generator(ims)`` in the reference (capgan.py:28,156).
``weights_init`` is mixed-gan.py:68-77 (Linear W ~ N(0, .02), b = 0; BN weight ~ N(1, .02), b = 0).
"""
from __future__ import annotations

import math

import torch

from .specs import MlpModel


@torch.no_grad()
def default_init(model: MlpModel, views, generator=None):
    for l in range(model.n_layers):
        fo, fi = model.dims[l + 1], model.dims[l]
        w = torch.empty(fo, fi)
        b = torch.empty(fo)
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5), generator=generator)
        bound = 1.0 / math.sqrt(fi)
        torch.nn.init.uniform_(b, -bound, bound, generator=generator)
        views[model.linear_keys[l] + ".weight"].copy_(w)
        views[model.linear_keys[l] + ".bias"].copy_(b)
        if model.bn[l]:
            views[model.bn_keys[l] + ".weight"].fill_(1.0)
            views[model.bn_keys[l] + ".bias"].fill_(0.0)


@torch.no_grad()
def weights_init(model: MlpModel, views, generator=None):
    for l in range(model.n_layers):
        fo, fi = model.dims[l + 1], model.dims[l]
        w = torch.empty(fo, fi)
        torch.nn.init.normal_(w, 0.0, 0.02, generator=generator)
        views[model.linear_keys[l] + ".weight"].copy_(w)
        views[model.linear_keys[l] + ".bias"].fill_(0.0)
        if model.bn[l]:
            g = torch.empty(fo)
            torch.nn.init.normal_(g, 1.0, 0.02, generator=generator)
            views[model.bn_keys[l] + ".weight"].copy_(g)
            views[model.bn_keys[l] + ".bias"].fill_(0.0)
