"""nn.Module drop-ins for model/mnist_model.py (and the Sigmoid discriminator of
MDGAN/MNIST/mnist_model.py:31-50), computed by libcglgan_hip.

The module structure is the reference's own layout -- ``self.model`` / ``self.paths`` built as
``nn.Sequential`` of nn.Linear / nn.BatchNorm1d(F, 0.8) / nn.LeakyReLU(0.2) / nn.Tanh -- so the
state-dict keys (``model.0.weight``, ``model.3.running_var``, ``paths.1.3.bias`` ...), the
``.model`` / ``.paths`` attributes that mixed-gan.py toggles with ``requires_grad_``
(mixed-gan.py:264-281), ``train()`` / ``eval()`` (capgan.py:204-208), ``torch.save(
state_dict())`` checkpoints and optimizers all behave as with the reference.  ``forward``
runs every layer through the library's HIP kernels (custom autograd Functions over the C ABI:
fused Linear + activation GEMMs, BatchNorm1d(+LeakyReLU) forward/backward); there is no
PyTorch-op or CPU fallback -- the modules require CUDA (ROCm) tensors and raise otherwise.

The training hot path of a worker round is ``cglgan.GanStep`` (one fused graph); these modules
are the drop-in surface for code that drives the reference models directly (sampling with a
fixed z, evaluation, custom loops).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.nn as nn

from . import _lib as C

ACT_NONE, ACT_LEAKY, ACT_TANH, ACT_SIGMOID = 0, 1, 2, 3


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


_WS = {}


def _ws(dev):
    """Op workspace (descriptor upload area) owned by the caching allocator, one per (device, stream):
    stream-ordered ops share it, ops on another stream never race on it."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(idx).cuda_stream)
    w = _WS.get(key)
    if w is None:
        w = torch.empty(C.lib.cgl_op_workspace_bytes(), dtype=torch.uint8, device=dev)
        _WS[key] = w
    return w


def _check_cuda(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or t.dtype != torch.float32):
            raise RuntimeError("cglgan.model computes on the GPU only: expected float32 CUDA (ROCm) tensors")


class _LinearAct(torch.autograd.Function):
    """y = act(x W^T + b) (nn.Linear + the activation module that follows it)."""

    @staticmethod
    def forward(ctx, x, w, b, act, slope):
        _check_cuda(x, w, b)
        x = x.contiguous()
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty(M, N, device=x.device, dtype=torch.float32)
        ws = _ws(x.device)
        C.check(C.lib.cgl_linear_fwd(_p(x), _p(w.contiguous()), _p(b), _p(y), M, N, K, act, float(slope), _p(ws),
                                     ws.numel(), _s()), "cgl_linear_fwd")
        ctx.save_for_backward(x, w, y)
        ctx.act, ctx.slope, ctx.has_b = act, slope, b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        gy = gy.contiguous()
        M, K = x.shape
        N = w.shape[0]
        ws = _ws(x.device)
        if ctx.act != ACT_NONE:
            g = torch.empty_like(gy)
            C.check(C.lib.cgl_act_bwd(_p(gy), _p(y), gy.numel(), ctx.act, float(ctx.slope), _p(g), _s()),
                    "cgl_act_bwd")
        else:
            g = gy
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty(M, K, device=x.device, dtype=torch.float32)
            C.check(C.lib.cgl_linear_bwd_data(_p(g), _p(w.contiguous()), _p(gx), M, N, K, _p(ws), ws.numel(), _s()),
                    "cgl_linear_bwd_data")
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            gw = torch.empty(N, K, device=x.device, dtype=torch.float32)
            gb = torch.empty(N, device=x.device, dtype=torch.float32) if ctx.has_b else None
            C.check(C.lib.cgl_linear_bwd_weight(_p(g), _p(x), _p(gw), _p(gb), M, N, K, _p(ws), ws.numel(), _s()),
                    "cgl_linear_bwd_weight")
            if not ctx.needs_input_grad[1]:
                gw = None
        return gx, gw, gb, None, None


class _Act(torch.autograd.Function):
    """A standalone activation module (LeakyReLU / Tanh / Sigmoid not preceded by a Linear)."""

    @staticmethod
    def forward(ctx, x, act, slope):
        _check_cuda(x)
        x = x.contiguous()
        y = torch.empty_like(x)
        C.check(C.lib.cgl_act_fwd(_p(x), x.numel(), act, float(slope), _p(y), _s()), "cgl_act_fwd")
        ctx.save_for_backward(y)
        ctx.act, ctx.slope = act, slope
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        gy = gy.contiguous()
        g = torch.empty_like(gy)
        C.check(C.lib.cgl_act_bwd(_p(gy), _p(y), gy.numel(), ctx.act, float(ctx.slope), _p(g), _s()), "cgl_act_bwd")
        return g, None, None


class _BatchNormAct(torch.autograd.Function):
    """nn.BatchNorm1d (train: batch statistics + running-stat update; eval: running statistics)
    fused with the LeakyReLU that follows it in block() (model/mnist_model.py:10-15)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, training, momentum, eps, act, slope):
        _check_cuda(x, gamma, beta, running_mean, running_var)
        x = x.contiguous()
        M, F = x.shape
        y = torch.empty_like(x)
        ws = _ws(x.device)
        save_mean = torch.empty(F, device=x.device, dtype=torch.float32) if training else None
        save_invstd = torch.empty(F, device=x.device, dtype=torch.float32) if training else None
        C.check(C.lib.cgl_bn1d_fwd(_p(x), M, F, F, _p(gamma), _p(beta), float(eps), float(momentum),
                                   _p(running_mean), _p(running_var), int(training), act, float(slope), _p(y),
                                   _p(save_mean), _p(save_invstd), _p(ws), ws.numel(), _s()), "cgl_bn1d_fwd")
        ctx.training, ctx.act, ctx.slope = training, act, slope
        if training:
            ctx.save_for_backward(x, y, gamma, save_mean, save_invstd)
        return y

    @staticmethod
    def backward(ctx, gy):
        gy = gy.contiguous()
        if not ctx.training:
            raise NotImplementedError("backward through eval-mode BatchNorm is not part of the reference "
                                      "workflow (eval is only used for sampling under no_grad)")
        x, y, gamma, save_mean, save_invstd = ctx.saved_tensors
        M, F = x.shape
        ws = _ws(x.device)
        gx = torch.empty_like(x)
        ggamma = torch.empty(F, device=x.device, dtype=torch.float32)
        gbeta = torch.empty(F, device=x.device, dtype=torch.float32)
        C.check(C.lib.cgl_bn1d_bwd(_p(gy), _p(y), _p(x), M, F, _p(save_mean), _p(save_invstd), _p(gamma), ctx.act,
                                   float(ctx.slope), _p(gx), _p(ggamma), _p(gbeta), _p(ws), ws.numel(), _s()),
                "cgl_bn1d_bwd")
        return gx, ggamma, gbeta, None, None, None, None, None, None, None


def run_sequential(seq: nn.Sequential, x):
    """Forward of an nn.Sequential of Linear / BatchNorm1d / LeakyReLU / Tanh / Sigmoid through
    the library, fusing each activation into the Linear or BatchNorm1d before it."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        nxt = mods[i + 1] if i + 1 < len(mods) else None
        act, slope = ACT_NONE, 0.0
        if isinstance(nxt, nn.LeakyReLU):
            act, slope = ACT_LEAKY, nxt.negative_slope
        elif isinstance(nxt, nn.Tanh):
            act = ACT_TANH
        elif isinstance(nxt, nn.Sigmoid):
            act = ACT_SIGMOID
        if isinstance(m, nn.Linear):
            x = _LinearAct.apply(x, m.weight, m.bias, act, slope)
            i += 2 if act != ACT_NONE else 1
        elif isinstance(m, nn.BatchNorm1d):
            if act not in (ACT_NONE, ACT_LEAKY):
                raise NotImplementedError("BatchNorm1d followed by " + type(nxt).__name__)
            train = m.training or not m.track_running_stats
            if m.training and m.track_running_stats:
                m.num_batches_tracked.add_(1)
            mom = m.momentum if m.momentum is not None else 0.0
            x = _BatchNormAct.apply(x, m.weight, m.bias, m.running_mean, m.running_var, train, mom, m.eps, act,
                                    slope)
            i += 2 if act != ACT_NONE else 1
        elif isinstance(m, nn.LeakyReLU):
            x = _Act.apply(x, ACT_LEAKY, m.negative_slope)
            i += 1
        elif isinstance(m, nn.Tanh):
            x = _Act.apply(x, ACT_TANH, 0.0)
            i += 1
        elif isinstance(m, nn.Sigmoid):
            x = _Act.apply(x, ACT_SIGMOID, 0.0)
            i += 1
        else:
            raise NotImplementedError(f"module {type(m).__name__} is not on the hot path of the reference models")
    return x


def _block(in_feat, out_feat, normalize=True):
    """block() of model/mnist_model.py:10-15."""
    layers = [nn.Linear(in_feat, out_feat)]
    if normalize:
        layers.append(nn.BatchNorm1d(out_feat, 0.8))
    layers.append(nn.LeakyReLU(0.2, inplace=True))
    return layers


class Generator(nn.Module):
    """model/mnist_model.py:5-29: z[B,100] -> img[B,*img_shape]."""

    def __init__(self, img_shape, latent_dim=100):
        super().__init__()
        self.img_shape = tuple(img_shape)
        self.model = nn.Sequential(*_block(latent_dim, 128, normalize=False), *_block(128, 256), *_block(256, 512),
                                   *_block(512, 1024), nn.Linear(1024, int(np.prod(self.img_shape))), nn.Tanh())

    def forward(self, z):
        img = run_sequential(self.model, z)
        return img.view((img.shape[0], *self.img_shape))


class MixGenerator(nn.Module):
    """model/mnist_model.py:32-66: shared trunk ``model`` + ``num_client`` heads ``paths``;
    the output is every head's batch concatenated on the batch dimension."""

    def __init__(self, img_shape, num_client, latent_dim=100):
        super().__init__()
        self.img_shape = tuple(img_shape)
        self.model = nn.Sequential(*_block(latent_dim, 128, normalize=False), *_block(128, 256), *_block(256, 512))
        self.paths = nn.ModuleList(
            nn.Sequential(*_block(512, 1024), nn.Linear(1024, int(np.prod(self.img_shape))), nn.Tanh())
            for _ in range(num_client))

    def forward(self, z):
        hidden = run_sequential(self.model, z)
        imgs = []
        for path in self.paths:
            out = run_sequential(path, hidden)
            imgs.append(out.view((out.shape[0], *self.img_shape)))
        return torch.cat(imgs, dim=0)


class Discriminator(nn.Module):
    """model/mnist_model.py:71-88 (2 logits, CrossEntropyLoss), or with ``sigmoid=True`` the
    Sigmoid/BCE discriminator of MDGAN/MNIST/mnist_model.py:31-50."""

    def __init__(self, img_shape, sigmoid=False):
        super().__init__()
        self.img_shape = tuple(img_shape)
        layers = [nn.Linear(int(np.prod(self.img_shape)), 512), nn.LeakyReLU(0.2), nn.Linear(512, 256),
                  nn.LeakyReLU(0.2)]
        layers += [nn.Linear(256, 1), nn.Sigmoid()] if sigmoid else [nn.Linear(256, 2)]
        self.model = nn.Sequential(*layers)

    def forward(self, img):
        return run_sequential(self.model, img.reshape(img.shape[0], -1))
