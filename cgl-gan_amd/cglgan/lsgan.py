"""nn.Module drop-ins for model/lsgan.py, computed by libcglgan_hip (no PyTorch-op or CPU fallback).

``Generator(ims)``, ``Discriminator(ims)`` and ``MixGenerator(ims, N)`` build the reference's own
module trees (model/lsgan.py:3-27, 73-99, 37-70) -- ``l1`` / ``conv_blocks`` / ``model`` / ``paths``
/ ``adv_layer`` of nn.Linear, nn.Upsample, nn.Conv2d, nn.BatchNorm2d(c, 0.8), nn.LeakyReLU(0.2),
nn.Dropout2d(0.25), nn.Tanh -- so state-dict keys (``conv_blocks.2.running_var``,
``model.14.weight``, ``adv_layer.bias`` ...), ``train()`` / ``eval()``, optimizers and checkpoints
behave as with the reference.  ``forward`` interprets the Sequentials through custom autograd
Functions over the C ABI, fusing Upsample into the following Conv2d (phase-form convolution) and
the LeakyReLU / Dropout2d / Tanh that follow a Conv2d into its epilogue.

Tensors: inputs and outputs have the reference's NCHW shapes; activations live in NHWC memory
(``channels_last``), so a returned image batch is a channels_last view (identical memory to NCHW
for the 1-channel images).  ``Discriminator.last_masks`` holds the Dropout2d scales of the last
train-mode forward ([B, C] per block), for inspection and for replaying the same step elsewhere.

Reference defect fixed: model/lsgan.py:68 reads ``self.img_shape``, which MixGenerator never sets
(its forward raises AttributeError); here ``img_shape`` is taken from ``ims`` (default (1, 32, 32)).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import conv_ops as O

_COUNTER = [0]


def _chk(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or t.dtype != torch.float32):
            raise RuntimeError("cglgan.lsgan computes on the GPU only: expected float32 CUDA (ROCm) tensors")


class _Dense(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        _chk(x, w, b)
        x = x.contiguous()
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty(M, N, device=x.device)
        O.dense_fwd(x, w.contiguous(), b, y, M, K, N)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        M, K = x.shape
        N = w.shape[0]
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty(M, K, device=x.device)
            O.dense_bwd_data(gy, w.contiguous(), gx, M, K, N)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            gw = torch.empty(N, K, device=x.device)
            gb = torch.empty(N, device=x.device)
            O.dense_bwd_weight(gy, x, gw, gb, M, K, N)
        return gx, gw, gb


class _ToNHWC(torch.autograd.Function):
    """[B, C, H, W] (NCHW memory, e.g. the Linear output viewed as in model/lsgan.py:25) -> NHWC."""

    @staticmethod
    def forward(ctx, x, c, hw):
        x = x.contiguous()
        n = x.shape[0]
        y = torch.empty(n, hw, c, device=x.device)
        O.nchw_to_nhwc(x, y, n, c, hw)
        ctx.c, ctx.hw, ctx.shape = c, hw, x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        gy = gy.contiguous()
        n = gy.shape[0]
        gx = torch.empty(ctx.shape, device=gy.device)
        O.nhwc_to_nchw(gy, gx, n, ctx.c, ctx.hw)
        return gx, None, None


class _ToNCHWFlat(torch.autograd.Function):
    """NHWC [B, H, W, C] -> [B, C*H*W] in NCHW order (out.view(B, -1), model/lsgan.py:96)."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        n, h, w, c = x.shape
        y = torch.empty(n, c * h * w, device=x.device)
        O.nhwc_to_nchw(x, y, n, c, h * w)
        ctx.dims = (n, h, w, c)
        return y

    @staticmethod
    def backward(ctx, gy):
        n, h, w, c = ctx.dims
        gx = torch.empty(n, h, w, c, device=gy.device)
        O.nchw_to_nhwc(gy.contiguous(), gx, n, c, h * w)
        return gx


class _Conv(torch.autograd.Function):
    """[Upsample(2)] -> Conv2d(k3, p1) -> [LeakyReLU [-> Dropout2d] | Tanh] on NHWC tensors."""

    @staticmethod
    def forward(ctx, x, w, b, stride, up, act, slope, drop):
        _chk(x, w, b, drop)
        x = x.contiguous()
        n, h, wd, cin = x.shape
        cout = w.shape[0]
        ho, wo = O.conv_out_hw(h, wd, stride, up)
        y = torch.empty(n, ho, wo, cout, device=x.device)
        O.conv3x3_fwd(x, w.contiguous(), b, y, n, h, wd, cin, cout, stride, up, act, slope, drop)
        ctx.save_for_backward(x, w, y, drop)
        ctx.cfg = (n, h, wd, cin, cout, stride, up, act, slope)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y, drop = ctx.saved_tensors
        n, h, wd, cin, cout, stride, up, act, slope = ctx.cfg
        ho, wo = y.shape[1], y.shape[2]
        gy = gy.contiguous()
        if act == O.ACT_TANH:
            g = torch.empty_like(gy)
            O.act_drop_bwd(gy, y, None, n, ho * wo, cout, g, tanh_y=True)
        elif act == O.ACT_LEAKY or drop is not None:
            g = torch.empty_like(gy)
            O.act_drop_bwd(gy, y if act == O.ACT_LEAKY else None, drop, n, ho * wo, cout, g, slope=slope)
        elif act == O.ACT_NONE:
            g = gy
        else:
            raise NotImplementedError("activation backward")
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            O.conv3x3_bwd_data(g, w.contiguous(), gx, n, h, wd, cin, cout, stride, up)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            gw = torch.empty_like(w)
            gb = torch.empty(cout, device=x.device)
            O.conv3x3_bwd_weight(g, x, gw, gb, n, h, wd, cin, cout, stride, up)
        return gx, gw, gb, None, None, None, None, None


class _BN2d(torch.autograd.Function):
    """nn.BatchNorm2d (train: batch statistics + running update; eval: running statistics) [+ LeakyReLU]."""

    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, training, momentum, eps, act, slope):
        _chk(x, gamma, beta, rm, rv)
        x = x.contiguous()
        n, h, w, c = x.shape
        y = torch.empty_like(x)
        sm = torch.empty(1, c, device=x.device) if training else None
        si = torch.empty(1, c, device=x.device) if training else None
        O.bn2d_fwd(x, n, h * w, c, gamma, beta, y, groups=1, eps=eps, momentum=momentum, running_mean=rm,
                   running_var=rv, train=training, act=act, slope=slope, save_mean=sm, save_invstd=si)
        ctx.training, ctx.act, ctx.slope = training, act, slope
        if training:
            ctx.save_for_backward(x, y, gamma, sm, si)
        return y

    @staticmethod
    def backward(ctx, gy):
        if not ctx.training:
            raise NotImplementedError("backward through eval-mode BatchNorm2d is not part of the reference workflow")
        x, y, gamma, sm, si = ctx.saved_tensors
        n, h, w, c = x.shape
        gx = torch.empty_like(x)
        gg = torch.empty(c, device=x.device)
        gbt = torch.empty(c, device=x.device)
        O.bn2d_bwd(gy.contiguous(), x, n, h * w, c, sm, si, gamma, gx, post=y if ctx.act == O.ACT_LEAKY else None,
                   dgamma=gg, dbeta=gbt, slope=ctx.slope)
        return gx, gg, gbt, None, None, None, None, None, None, None


def _mask(n, c, p, device):
    m = torch.empty(n, c, device=device)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())   # torch CPU RNG: torch.manual_seed reproducible
    _COUNTER[0] += 1
    O.dropout2d_mask(m, n, c, p, seed, _COUNTER[0])
    return m


def run_conv_seq(seq, x, masks_out=None):
    """Forward of an nn.Sequential of the model/lsgan.py vocabulary on an NHWC tensor."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.Upsample) or isinstance(m, nn.Conv2d):
            up = 0
            if isinstance(m, nn.Upsample):
                if not (m.scale_factor in (2, 2.0, (2.0, 2.0)) and m.mode == "nearest"):
                    raise NotImplementedError("only nn.Upsample(scale_factor=2) (nearest) is on the reference path")
                up, i = 1, i + 1
                m = mods[i]
                if not isinstance(m, nn.Conv2d):
                    raise NotImplementedError("Upsample must be followed by Conv2d (model/lsgan.py:11-12)")
            if m.kernel_size != (3, 3) or m.padding != (1, 1) or m.stride[0] != m.stride[1] or m.groups != 1:
                raise NotImplementedError("only Conv2d(k=3, padding=1) is on the reference path")
            i += 1
            act, slope, drop = O.ACT_NONE, 0.2, None
            if i < len(mods) and isinstance(mods[i], nn.LeakyReLU):
                act, slope, i = O.ACT_LEAKY, mods[i].negative_slope, i + 1
                if i < len(mods) and isinstance(mods[i], nn.Dropout2d):
                    d = mods[i]
                    if d.training and d.p > 0:
                        drop = _mask(x.shape[0], m.out_channels, d.p, x.device)
                        if masks_out is not None:
                            masks_out.append(drop)
                    i += 1
            elif i < len(mods) and isinstance(mods[i], nn.Tanh):
                act, i = O.ACT_TANH, i + 1
            x = _Conv.apply(x, m.weight, m.bias, m.stride[0], up, act, slope, drop)
        elif isinstance(m, nn.BatchNorm2d):
            i += 1
            act, slope = O.ACT_NONE, 0.2
            if i < len(mods) and isinstance(mods[i], nn.LeakyReLU):
                act, slope, i = O.ACT_LEAKY, mods[i].negative_slope, i + 1
            train = m.training or not m.track_running_stats
            if m.training and m.track_running_stats:
                m.num_batches_tracked.add_(1)
            mom = m.momentum if m.momentum is not None else 0.0
            x = _BN2d.apply(x, m.weight, m.bias, m.running_mean, m.running_var, train, mom, m.eps, act, slope)
        elif isinstance(m, nn.Dropout2d):
            if m.training and m.p > 0:
                raise NotImplementedError("Dropout2d is fused after Conv2d -> LeakyReLU (model/lsgan.py:78)")
            i += 1
        elif isinstance(m, (nn.Sequential, Reshape)):
            raise NotImplementedError("nested Sequential handled by the module forward")
        else:
            raise NotImplementedError(f"module {type(m).__name__} is not on the hot path of model/lsgan.py")
    return x


def _nchw_view(x_nhwc):
    """NHWC memory as the reference's NCHW-shaped tensor (channels_last strides, no copy)."""
    return x_nhwc.permute(0, 3, 1, 2)


def _to_nhwc_input(img):
    """An NCHW image batch as an NHWC tensor (a free view for 1-channel images)."""
    n, c, h, w = img.shape
    if c == 1:
        return img.reshape(n, h, w, 1)
    return _ToNHWC.apply(img.reshape(n, c, h * w), c, h * w).view(n, h, w, c)


class Reshape(nn.Module):
    """model/lsgan.py:29-35."""

    def __init__(self, init_size):
        super().__init__()
        self.init_size = init_size

    def forward(self, input):
        return input.view(input.shape[0], 128, self.init_size, self.init_size)


class Generator(nn.Module):
    """model/lsgan.py:3-27: z [B,100] -> img [B,1,32,32]."""

    def __init__(self, ims=(1, 32, 32)):
        super().__init__()
        self.init_size = 32 // 4
        self.l1 = nn.Sequential(nn.Linear(100, 128 * self.init_size ** 2))
        self.conv_blocks = nn.Sequential(
            nn.Upsample(scale_factor=2), nn.Conv2d(128, 128, 3, stride=1, padding=1), nn.BatchNorm2d(128, 0.8),
            nn.LeakyReLU(0.2, inplace=True), nn.Upsample(scale_factor=2), nn.Conv2d(128, 64, 3, stride=1, padding=1),
            nn.BatchNorm2d(64, 0.8), nn.LeakyReLU(0.2, inplace=True), nn.Conv2d(64, 1, 3, stride=1, padding=1), nn.Tanh())

    def forward(self, z):
        lin = self.l1[0]
        out = _Dense.apply(z, lin.weight, lin.bias)
        s = self.init_size
        x = _ToNHWC.apply(out, 128, s * s).view(out.shape[0], s, s, 128)
        return _nchw_view(run_conv_seq(self.conv_blocks, x))


class MixGenerator(nn.Module):
    """model/lsgan.py:37-70: shared trunk ``model`` (Linear, Reshape, Upsample, Conv 128->128, BN,
    LeakyReLU, Upsample, Conv 128->64) and N heads ``paths`` (BN(64), LeakyReLU, Conv 64->1, Tanh);
    the output is every head's images concatenated on the batch dimension."""

    def __init__(self, ims=(1, 32, 32), N=1):
        super().__init__()
        self.img_shape = tuple(ims) if isinstance(ims, (tuple, list)) else (1, 32, 32)
        self.init_size = 32 // 4
        self.model = nn.Sequential(
            nn.Sequential(nn.Linear(100, 128 * self.init_size ** 2)), Reshape(init_size=self.init_size),
            nn.Upsample(scale_factor=2), nn.Conv2d(128, 128, 3, stride=1, padding=1), nn.BatchNorm2d(128, 0.8),
            nn.LeakyReLU(0.2, inplace=True), nn.Upsample(scale_factor=2), nn.Conv2d(128, 64, 3, stride=1, padding=1))
        self.paths = nn.ModuleList(
            nn.Sequential(nn.BatchNorm2d(64, 0.8), nn.LeakyReLU(0.2, inplace=True), nn.Conv2d(64, 1, 3, stride=1, padding=1),
                          nn.Tanh()) for _ in range(N))

    def trunk(self, z):
        lin = self.model[0][0]
        out = _Dense.apply(z, lin.weight, lin.bias)
        s = self.init_size
        x = _ToNHWC.apply(out, 128, s * s).view(out.shape[0], s, s, 128)
        return run_conv_seq(list(self.model)[2:], x)

    def forward(self, z):
        hidden = self.trunk(z)
        imgs = [_nchw_view(run_conv_seq(path, hidden)).reshape(hidden.shape[0], *self.img_shape)
                for path in self.paths]
        return torch.cat(imgs, dim=0)


class Discriminator(nn.Module):
    """model/lsgan.py:73-99: img [B,1,32,32] (or 28x28) -> validity logit [B,1]."""

    def __init__(self, ims=(1, 32, 32)):
        super().__init__()

        def discriminator_block(in_filters, out_filters, bn=True):
            block = [nn.Conv2d(in_filters, out_filters, 3, 2, 1), nn.LeakyReLU(0.2, inplace=True), nn.Dropout2d(0.25)]
            if bn:
                block.append(nn.BatchNorm2d(out_filters, 0.8))
            return block

        self.model = nn.Sequential(*discriminator_block(1, 16, bn=False), *discriminator_block(16, 32),
                                   *discriminator_block(32, 64), *discriminator_block(64, 128))
        ds_size = 32 // 2 ** 4
        self.adv_layer = nn.Linear(128 * ds_size ** 2, 1)
        self.last_masks = []

    def forward(self, img):
        masks = []
        x = run_conv_seq(self.model, _to_nhwc_input(img.contiguous()), masks)
        self.last_masks = masks
        flat = _ToNCHWFlat.apply(x)
        return _Dense.apply(flat, self.adv_layer.weight, self.adv_layer.bias)
