"""Checked Python wrappers of the conv-path C ABI (include/cglgan.h, "conv GAN ops").

Tensors are float32 CUDA (ROCm) tensors; activations are NHWC -- a logically NCHW tensor in
``torch.channels_last`` memory, or a plain contiguous [n, h, w, c] tensor -- and weights keep the
reference nn.Conv2d layout [cout][cin][3][3].  Every call is stream-ordered on the current torch
stream (no host synchronisation) and raises on a non-zero return code; there is no fallback.
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
import os

import torch

from . import _lib as C

ACT_NONE, ACT_LEAKY, ACT_TANH, ACT_SIGMOID = 0, 1, 2, 3
LOSS = {"ce": C.LOSS_OP_CE2, "bce_prob": C.LOSS_OP_BCE, "mse": C.LOSS_OP_MSE, "bce": C.LOSS_OP_BCE_LOGIT}

_WS = {}
_CUR = None     # (device index, stream handle, ctypes handle) inside a stream_cache() block
_NO_CACHE = os.environ.get("CGL_STREAM_CACHE", "1") == "0"


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _s():
    if _CUR is not None:
        return _CUR[2]
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


@contextlib.contextmanager
def launch_batch(enabled=True):
    """cgl_conv_batch_begin / _end around the round start's pack / masks / z draw / sampler calls: one launch
    instead of four (same results).  The block must stay on the current stream."""
    if not enabled:
        yield
        return
    s = _s()
    C.check(C.lib.cgl_conv_batch_begin(s), "cgl_conv_batch_begin")
    ok = False
    try:
        yield
        ok = True
    finally:
        rc = C.lib.cgl_conv_batch_end(s)
        if ok:
            C.check(rc, "cgl_conv_batch_end")


_WDEFER = False     # a wgrad_defer block is open (its weight gradients need workspaces of their own)


@contextlib.contextmanager
def wgrad_defer(enabled=True):
    """cgl_conv_wgrad_defer_begin / _end around a backward pass: the weight gradients' split reductions (and the
    single-input-channel kernel's finish) run as ONE launch at the end of the block, on the current stream
    (bitwise the separate launches).  Every conv3x3_bwd_weight inside must get its own ``ws``."""
    global _WDEFER
    if not enabled:
        yield
        return
    C.check(C.lib.cgl_conv_wgrad_defer_begin(), "cgl_conv_wgrad_defer_begin")
    _WDEFER = True
    ok = False
    try:
        yield
        ok = True
    finally:
        _WDEFER = False
        rc = C.lib.cgl_conv_wgrad_defer_end(_s())
        if ok:
            C.check(rc, "cgl_conv_wgrad_defer_end")


@contextlib.contextmanager
def stream_cache():
    """Resolve the current torch stream once for a block of ops that all run on it (the fused conv
    round issues ~100 ops per round; looking the stream up per op was a visible share of the host
    time that leaves the GPU idle between the small discriminator kernels).  The block must not
    switch streams."""
    global _CUR
    if _NO_CACHE:
        yield
        return
    prev = _CUR
    s = torch.cuda.current_stream()
    _CUR = (s.device.index, s.cuda_stream, ctypes.c_void_p(s.cuda_stream))
    try:
        yield
    finally:
        _CUR = prev


def workspace(nbytes: int, device) -> torch.Tensor:
    """Scratch owned by the caching allocator, one buffer per (device, stream): ops issued on one
    stream are ordered, so they share it; ops on another stream (a side-stream round beside the
    drop-in modules, two-stream overlap) get their own and never race on it.  Grown on demand."""
    if _CUR is not None and (getattr(device, "index", None) in (None, _CUR[0])):
        key = (_CUR[0], _CUR[1])
        w = _WS.get(key)
        if w is not None and w.numel() >= nbytes:
            return w
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(idx).cuda_stream)
    w = _WS.get(key)
    if w is None or w.numel() < nbytes:
        w = torch.empty(max(int(nbytes), 1 << 20), dtype=torch.uint8, device=dev)
        _WS[key] = w
    return w


def _chk(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or t.dtype != torch.float32):
            raise RuntimeError("cglgan conv ops compute on the GPU only: expected float32 CUDA (ROCm) tensors")


def conv_out_hw(h, w, stride, up):
    return ((h << up) - 1) // stride + 1, ((w << up) - 1) // stride + 1


@functools.lru_cache(maxsize=512)
def conv_ws_bytes(n, h, w, cin, cout, stride, up):
    b = C.lib.cgl_conv3x3_workspace_bytes(n, h, w, cin, cout, stride, up)
    if b < 0:
        raise RuntimeError(f"conv3x3: bad geometry (rc={b})")
    return b


def stat_chunks(n, h, wd, cin, cout, stride=1, up=0, groups=1, bwd=False):
    """32-row statistic chunks of a forward's output, or (bwd) of an input gradient's output
    (0: epilogue statistics unsupported)."""
    fn = C.lib.cgl_conv3x3_bwd_stat_chunks if bwd else C.lib.cgl_conv3x3_stat_chunks
    return int(fn(n, h, wd, cin, cout, stride, up, groups))


def conv3x3_fwd(x, w, b, y, n, h, wd, cin, cout, stride=1, up=0, act=ACT_NONE, slope=0.2, drop=None, wp=None,
                stats=None, bn_in=None, nvalid=None):
    """``wp``: the weights pre-packed by a PackSet (no per-call pack launch); ``w`` is then unused.
    ``stats`` = (part, groups): also write the next BatchNorm2d's {sum, M2} partials per 32-row chunk
    (float64 tensor of stat_chunks(...) * cout * 2) -- consumed by bn2d_fwd_stats.
    ``bn_in`` = (coef, groups, act, slope): ``x`` is the PRE-BatchNorm map; the BatchNorm (+ LeakyReLU)
    whose scale / shift bn2d_fwd_stats(coef=...) wrote is applied as the operands are loaded (needs ``wp``).
    ``nvalid`` (device int32, with ``stats``): the first forward call is a short batch of *nvalid images (the
    rest padding, left out of the statistics; see bn2d_fwd)."""
    _chk(x, w, b, y, drop, wp)
    ws = workspace(conv_ws_bytes(n, h, wd, cin, cout, stride, up), x.device)
    if nvalid is not None and stats is None:
        raise RuntimeError("conv3x3_fwd(nvalid=...): only with stats=")
    if bn_in is not None:
        coef, groups_in, act_in, slope_in = bn_in
        _chk(coef)
        part, groups = stats if stats is not None else (None, 1)
        if wp is None:
            raise RuntimeError("conv3x3_fwd(bn_in=...): needs packed weights")
        C.check(C.lib.cgl_conv3x3_fwd_packed_bnin(_p(x), _p(wp), _p(b), _p(y), n, h, wd, cin, cout, stride, up, act,
                                                  float(slope), _p(drop), int(groups), _p(part), _p(coef),
                                                  int(groups_in), int(act_in), float(slope_in), _p(nvalid), _p(ws),
                                                  ws.numel(), _s()), "cgl_conv3x3_fwd_packed_bnin")
        return y
    if stats is not None:
        part, groups = stats
        if wp is None or not part.is_cuda or part.dtype != torch.float64:
            raise RuntimeError("conv3x3_fwd(stats=...): needs packed weights and a float64 CUDA partial buffer")
        C.check(C.lib.cgl_conv3x3_fwd_packed_stats(_p(x), _p(wp), _p(b), _p(y), n, h, wd, cin, cout, stride, up, act,
                                                   float(slope), _p(drop), int(groups), _p(part), _p(nvalid), _p(ws),
                                                   ws.numel(), _s()), "cgl_conv3x3_fwd_packed_stats")
        return y
    if wp is not None:
        C.check(C.lib.cgl_conv3x3_fwd_packed(_p(x), _p(wp), _p(b), _p(y), n, h, wd, cin, cout, stride, up, act,
                                             float(slope), _p(drop), _p(ws), ws.numel(), _s()), "cgl_conv3x3_fwd_packed")
        return y
    C.check(C.lib.cgl_conv3x3_fwd(_p(x), _p(w), _p(b), _p(y), n, h, wd, cin, cout, stride, up, act, float(slope),
                                  _p(drop), _p(ws), ws.numel(), _s()), "cgl_conv3x3_fwd")
    return y


def conv3x3_bwd_data(dy, w, dx, n, h, wd, cin, cout, stride=1, up=0, wp=None, stats=None):
    """``stats`` = (part, groups, x, post, mean, slope[, post_coef]): also write the previous BatchNorm2d's
    backward partials {sum g, sum g (x - mean)} per 32-row chunk of dx (g = dx * leaky'(post) if post; with
    post_coef = (coef, group, groups) and post None: leaky' from the forward's scale / shift, bn2d_bwd's
    post_coef) -- consumed by bn2d_bwd_stats (R = 32); with ``wp`` None only the one-output-channel 3x3
    geometry, per 128-row chunk (bn2d_bwd_stats R = 128, bitwise bn2d_bwd)."""
    _chk(dy, w, dx, wp)
    ws = workspace(conv_ws_bytes(n, h, wd, cin, cout, stride, up), dy.device)
    if stats is not None:
        part, groups, x, post, mean, slope = stats[:6]
        pc, pld = _post_coef(stats[6] if len(stats) > 6 else None, cin)
        _chk(x, post, mean)
        if not part.is_cuda or part.dtype != torch.float64:
            raise RuntimeError("conv3x3_bwd_data(stats=...): needs a float64 CUDA partial buffer")
        if wp is None:      # the vector one-output-channel kernel: partials per 128-row chunk
            C.check(C.lib.cgl_conv3x3_bwd_data_stats(_p(dy), _p(w), _p(dx), n, h, wd, cin, cout, stride, up,
                                                     int(groups), _p(part), _p(x), _p(post), _p(pc), int(pld),
                                                     _p(mean), float(slope), _p(ws), ws.numel(), _s()),
                    "cgl_conv3x3_bwd_data_stats")
            return dx
        C.check(C.lib.cgl_conv3x3_bwd_data_packed_stats(_p(dy), _p(wp), _p(dx), n, h, wd, cin, cout, stride, up,
                                                        int(groups), _p(part), _p(x), _p(post), _p(pc), int(pld),
                                                        _p(mean), float(slope), _p(ws), ws.numel(), _s()),
                "cgl_conv3x3_bwd_data_packed_stats")
        return dx
    if wp is not None:
        C.check(C.lib.cgl_conv3x3_bwd_data_packed(_p(dy), _p(w), _p(wp), _p(dx), n, h, wd, cin, cout, stride, up,
                                                  _p(ws), ws.numel(), _s()), "cgl_conv3x3_bwd_data_packed")
        return dx
    C.check(C.lib.cgl_conv3x3_bwd_data(_p(dy), _p(w), _p(dx), n, h, wd, cin, cout, stride, up, _p(ws), ws.numel(),
                                       _s()), "cgl_conv3x3_bwd_data")
    return dx


def conv3x3_bwd_weight(dy, x, dw, db, n, h, wd, cin, cout, stride=1, up=0, bn_in=None, act_drop=None, ws=None):
    """``bn_in`` = (coef, group, groups, act, slope): ``x`` is the PRE-BatchNorm map of forward call ``group``
    (-1: ``groups`` stacked calls of n / groups images); the BatchNorm (+ LeakyReLU) is applied in the operand
    loads (cgl_conv3x3_bwd_weight_bnin).  ``act_drop`` = (post, drop, slope), cin == 1 only: ``dy`` is the
    gradient at the block's output, the LeakyReLU + Dropout2d backward applied per loaded value
    (cgl_conv3x3_bwd_weight_actdrop, bitwise act_drop_bwd + this).  ``ws``: a uint8 workspace of its own
    (inside wgrad_defer: the deferred reduction reads its partials from it), else the stream's shared one."""
    if ws is None and _WDEFER:
        raise RuntimeError("conv3x3_bwd_weight inside wgrad_defer: pass a workspace of its own (ws=)")
    _chk(dy, x, dw, db)
    need = conv_ws_bytes(n, h, wd, cin, cout, stride, up)
    if ws is None:
        ws = workspace(need, dy.device)
    elif ws.numel() < need or ws.dtype != torch.uint8:
        raise RuntimeError(f"conv3x3_bwd_weight: workspace of {need} bytes (uint8) needed")
    if act_drop is not None:
        post, drop, slope = act_drop
        _chk(post, drop)
        C.check(C.lib.cgl_conv3x3_bwd_weight_actdrop(_p(dy), _p(post), _p(drop), float(slope), _p(x), _p(dw), _p(db),
                                                     n, h, wd, cin, cout, stride, up, _p(ws), ws.numel(), _s()),
                "cgl_conv3x3_bwd_weight_actdrop")
        return dw
    if bn_in is not None:
        coef, group, groups, act, slope = bn_in
        _chk(coef)
        C.check(C.lib.cgl_conv3x3_bwd_weight_bnin(_p(dy), _p(x), _p(dw), _p(db), n, h, wd, cin, cout, stride, up,
                                                  _p(coef), int(groups), int(group), int(act), float(slope), _p(ws),
                                                  ws.numel(), _s()), "cgl_conv3x3_bwd_weight_bnin")
        return dw
    C.check(C.lib.cgl_conv3x3_bwd_weight(_p(dy), _p(x), _p(dw), _p(db), n, h, wd, cin, cout, stride, up, _p(ws),
                                         ws.numel(), _s()), "cgl_conv3x3_bwd_weight")
    return dw


def dense_ws_bytes(M, K, N):
    b = C.lib.cgl_dense_workspace_bytes(M, K, N)
    if b < 0:
        raise RuntimeError(f"dense: bad geometry (rc={b})")
    return b


def dense_fwd(x, w, b, y, M, K, N, act=ACT_NONE, slope=0.2, wp=None):
    _chk(x, w, b, y, wp)
    ws = workspace(dense_ws_bytes(M, K, N), x.device)
    if wp is not None:
        C.check(C.lib.cgl_dense_fwd_packed(_p(x), _p(wp), _p(b), _p(y), M, K, N, act, float(slope), _p(ws), ws.numel(),
                                           _s()), "cgl_dense_fwd_packed")
        return y
    C.check(C.lib.cgl_dense_fwd(_p(x), _p(w), _p(b), _p(y), M, K, N, act, float(slope), _p(ws), ws.numel(), _s()),
            "cgl_dense_fwd")
    return y


def dense_bwd_data(dy, w, dx, M, K, N, wp=None):
    _chk(dy, w, dx, wp)
    ws = workspace(dense_ws_bytes(M, K, N), dy.device)
    if wp is not None:
        C.check(C.lib.cgl_dense_bwd_data_packed(_p(dy), _p(wp), _p(dx), M, K, N, _p(ws), ws.numel(), _s()),
                "cgl_dense_bwd_data_packed")
        return dx
    C.check(C.lib.cgl_dense_bwd_data(_p(dy), _p(w), _p(dx), M, K, N, _p(ws), ws.numel(), _s()), "cgl_dense_bwd_data")
    return dx


def dense_bwd_weight(dy, x, dw, db, M, K, N):
    _chk(dy, x, dw, db)
    ws = workspace(dense_ws_bytes(M, K, N), dy.device)
    C.check(C.lib.cgl_dense_bwd_weight(_p(dy), _p(x), _p(dw), _p(db), M, K, N, _p(ws), ws.numel(), _s()),
            "cgl_dense_bwd_weight")
    return dw


class PreparedLinear:
    """A Linear GEMM (op 0 forward, 1 input gradient, 2 weight + bias gradient) prepared once on the
    fused-MLP GEMM kernel (cgl_linear_prepare) and launched stream-ordered, capturable, without a
    descriptor upload: the operand tensors given here are the ones every launch reads."""

    def __init__(self, op, a, b, bias, c, db, M, N, K, act=ACT_NONE, slope=0.2, b_rows=None, nhwc=None):
        _chk(a, b, bias, c, db)
        self._keep = (a, b, bias, c, db, b_rows)
        self.desc = torch.zeros(int(C.lib.cgl_linear_desc_bytes()), dtype=torch.uint8, device=a.device)
        self.launch = C.LinearLaunch()
        if nhwc is not None:     # op 2 with A an NHWC [M][HW][C] gradient (cgl_linear_prepare_wgrad_nhwc)
            ch, hw = nhwc
            if op != 2 or bias is not None or ch * hw != N or act != ACT_NONE or b_rows is not None:
                raise ValueError("PreparedLinear: nhwc=(C, HW) is for op 2 with N = C * HW")
            C.check(C.lib.cgl_linear_prepare_wgrad_nhwc(_p(a), _p(b), _p(c), _p(db), M, ch, hw, K, _p(self.desc),
                                                        ctypes.byref(self.launch)), "cgl_linear_prepare_wgrad_nhwc")
            return
        if b_rows is not None:   # op 0 with gathered B rows (cgl_linear_prepare_gather)
            if op != 0 or db is not None:
                raise ValueError("PreparedLinear: b_rows is for op 0 only")
            if b_rows.dtype != torch.int32 or b_rows.numel() != N or not b_rows.is_contiguous():
                raise ValueError("PreparedLinear: b_rows must be a contiguous int32 tensor of N row indices")
            if int(b_rows.min()) < 0 or int(b_rows.max()) >= b.numel() // K:
                raise ValueError("PreparedLinear: b_rows index outside B's rows")
            C.check(C.lib.cgl_linear_prepare_gather(_p(a), _p(b), _p(b_rows), _p(bias), _p(c), M, N, K, act,
                                                    float(slope), _p(self.desc), ctypes.byref(self.launch)),
                    "cgl_linear_prepare_gather")
            return
        C.check(C.lib.cgl_linear_prepare(int(op), _p(a), _p(b), _p(bias), _p(c), _p(db), M, N, K, act, float(slope),
                                         _p(self.desc), ctypes.byref(self.launch)), "cgl_linear_prepare")

    def __call__(self):
        C.check(C.lib.cgl_linear_launch(_p(self.desc), ctypes.byref(self.launch), _s()), "cgl_linear_launch")


class PackSet:
    """The packed MFMA weight operands of several layers, refreshed by ONE cgl_conv_pack_multi launch.

    ``add(group, key, w, h, w_, cin, cout, stride, up, ks, dir)`` registers a (layer, direction)
    pair; ``finalize(device)`` allocates one flat buffer (views ``self[key]``); ``run(group)`` packs
    every operand of that group (None: all groups) from the current weights (stream-ordered,
    capturable)."""

    def __init__(self):
        self._jobs, self._views, self._arrs = [], {}, {}

    def add(self, group, key, w, h, wd, cin, cout, stride=1, up=0, ks=3, dir=0):
        n = C.lib.cgl_conv_packed_floats(h, wd, cin, cout, stride, up, ks, dir)
        if n < 0:
            raise RuntimeError(f"PackSet: bad geometry for {key} (rc={n})")
        self._jobs.append((group, key, w, int(n), (h, wd, cin, cout, stride, up, ks, dir)))

    def finalize(self, device):
        tot = sum((n + 63) // 64 * 64 for _, _, _, n, _ in self._jobs)
        self.buf = torch.zeros(max(tot, 64), dtype=torch.float32, device=device)
        recs, off = [], 0
        for group, key, w, n, geo in self._jobs:
            _chk(w)
            self._views[key] = self.buf[off:off + n]
            recs.append((group, C.ConvPackJob(w.data_ptr(), self.buf[off:].data_ptr(), *geo)))
            off += (n + 63) // 64 * 64
        for g in [None] + sorted({r[0] for r in recs}):
            sel = [j for grp, j in recs if g is None or grp == g]
            self._arrs[g] = (len(sel), (C.ConvPackJob * len(sel))(*sel))
        return self

    def __getitem__(self, key):
        return self._views[key]

    def run(self, group=None):
        n, arr = self._arrs[group]
        C.check(C.lib.cgl_conv_pack_multi(n, arr, _s()), "cgl_conv_pack_multi")


def gather_rows(src, idx, row0, nrows, row_floats, dst):
    _chk(src, dst)
    if idx is not None and (not idx.is_cuda or idx.dtype != torch.int32):
        raise RuntimeError("gather_rows: idx must be an int32 CUDA tensor")
    C.check(C.lib.cgl_gather_rows(_p(src), _p(idx), int(row0), nrows, row_floats, _p(dst), _s()), "cgl_gather_rows")
    return dst


def bn2d_ws_bytes(n, hw, c, groups):
    b = C.lib.cgl_bn2d_workspace_bytes(n, hw, c, groups)
    if b < 0:
        raise RuntimeError(f"bn2d: bad geometry (rc={b})")
    return b


def bn2d_fwd(x, n, hw, c, gamma, beta, y, groups=1, eps=0.8, momentum=0.1, running_mean=None, running_var=None,
             train=True, act=ACT_NONE, slope=0.2, save_mean=None, save_invstd=None, nvalid=None):
    """``nvalid`` (device int32, may be None): the first of the ``groups`` forward calls is a short batch --
    only its first *nvalid images are data (the D step's real call on DataLoader's short final batch,
    capgan.py:282,326-331); its other images are padding, left out of the statistics."""
    _chk(x, gamma, beta, y, running_mean, running_var, save_mean, save_invstd)
    ws = workspace(bn2d_ws_bytes(n, hw, c, groups), x.device)
    C.check(C.lib.cgl_bn2d_fwd(_p(x), n, hw, c, groups, _p(gamma), _p(beta), float(eps), float(momentum),
                               _p(running_mean), _p(running_var), int(train), act, float(slope), _p(y), _p(save_mean),
                               _p(save_invstd), _p(nvalid), _p(ws), ws.numel(), _s()), "cgl_bn2d_fwd")
    return y


def bn2d_stats_scratch(c, groups, device):
    """The zeroed per-BatchNorm scratch of bn2d_fwd_stats (sliced finalize tickets + slice results)."""
    n = C.lib.cgl_bn2d_stats_scratch_bytes(c, groups)
    if n < 0:
        raise RuntimeError(f"bn2d_stats_scratch: bad shape (rc={n})")
    return torch.zeros(int(n), dtype=torch.uint8, device=device)


def bn2d_fwd_stats(part, x, n, hw, c, gamma, beta, y, groups=1, eps=0.8, momentum=0.1, running_mean=None,
                   running_var=None, act=ACT_NONE, slope=0.2, save_mean=None, save_invstd=None, R=32, scratch=None,
                   coef=None, apply_from=0, nvalid=None):
    """bn2d_fwd (train) from the partials a conv3x3_fwd(stats=...) wrote: finalize + apply.
    ``scratch``: bn2d_stats_scratch(c, max groups) kept with the layer (parallel finalize).
    ``coef`` ([2 * groups * c] float32): also keep the scale / shift (for a consumer's bn_in);
    ``apply_from``: apply (write ``y``) to images [apply_from, n) only."""
    _chk(x, gamma, beta, y, running_mean, running_var, save_mean, save_invstd, coef)
    ws = workspace(bn2d_ws_bytes(n, hw, c, groups), x.device)
    if coef is not None or apply_from:
        C.check(C.lib.cgl_bn2d_fwd_stats_coef(_p(part), int(R), _p(x), n, hw, c, groups, _p(gamma), _p(beta),
                                              float(eps), float(momentum), _p(running_mean), _p(running_var), act,
                                              float(slope), _p(y), _p(save_mean), _p(save_invstd), _p(scratch),
                                              _p(coef), int(apply_from), _p(nvalid), _p(ws), ws.numel(), _s()),
                "cgl_bn2d_fwd_stats_coef")
        return y
    C.check(C.lib.cgl_bn2d_fwd_stats(_p(part), int(R), _p(x), n, hw, c, groups, _p(gamma), _p(beta), float(eps),
                                     float(momentum), _p(running_mean), _p(running_var), act, float(slope), _p(y),
                                     _p(save_mean), _p(save_invstd), _p(scratch), _p(nvalid), _p(ws), ws.numel(),
                                     _s()), "cgl_bn2d_fwd_stats")
    return y


def _post_coef(post_coef, c):
    """post_coef = (coef, group, groups): the [2][groups][c] scale / shift a bn2d_fwd_stats(coef=) call kept,
    the forward call (group) whose rows this backward covers -> (pointer, ld) of cgl_bn2d_bwd."""
    if post_coef is None:
        return None, 0
    coef, g, groups = post_coef
    _chk(coef)
    return coef[g * c:], groups * c


def bn2d_bwd(dy, x, n, hw, c, save_mean, save_invstd, gamma, dx, groups=1, post=None, post_out=None, drop=None,
             dgamma=None, dbeta=None, slope=0.2, nvalid=None, post_coef=None):
    """``post_coef`` = (coef, group, groups): LeakyReLU'(post) from the forward's own scale / shift (post unread)."""
    _chk(dy, x, save_mean, save_invstd, gamma, dx, post, post_out, drop, dgamma, dbeta)
    ws = workspace(bn2d_ws_bytes(n, hw, c, groups), dy.device)
    pc, pld = _post_coef(post_coef, c)
    C.check(C.lib.cgl_bn2d_bwd(_p(dy), _p(post), _p(x), n, hw, c, groups, _p(save_mean), _p(save_invstd), _p(gamma),
                               float(slope), _p(post_out), _p(drop), _p(dx), _p(dgamma), _p(dbeta), _p(pc), int(pld),
                               _p(nvalid), _p(ws), ws.numel(), _s()), "cgl_bn2d_bwd")
    return dx


def bn2d_bwd_stats(part, dy, x, n, hw, c, save_mean, save_invstd, gamma, dx, groups=1, post=None, post_out=None,
                   drop=None, dgamma=None, dbeta=None, slope=0.2, R=32, nvalid=None, post_coef=None, colsum=None):
    """bn2d_bwd from the partials a conv3x3_bwd_data(stats=...) wrote: finalize + apply.  ``colsum``: float64
    [n hw / 256, c, 2] -- also dx's column sums per 256-row chunk (colsum_finalize(colsum, n hw // 256, c, db):
    bitwise the bias gradient conv3x3_bwd_weight computes from dx)."""
    if colsum is not None and (not colsum.is_cuda or colsum.dtype != torch.float64 or
                               colsum.numel() < (n * hw // 256) * c * 2):
        raise RuntimeError("bn2d_bwd_stats(colsum=...): float64 CUDA buffer of [n hw / 256][c][2]")
    _chk(dy, x, save_mean, save_invstd, gamma, dx, post, post_out, drop, dgamma, dbeta)
    ws = workspace(bn2d_ws_bytes(n, hw, c, groups), dy.device)
    pc, pld = _post_coef(post_coef, c)
    C.check(C.lib.cgl_bn2d_bwd_stats(_p(part), int(R), _p(dy), _p(post), _p(x), n, hw, c, groups, _p(save_mean),
                                     _p(save_invstd), _p(gamma), float(slope), _p(post_out), _p(drop), _p(dx),
                                     _p(dgamma), _p(dbeta), _p(pc), int(pld), _p(nvalid), _p(colsum), _p(ws),
                                     ws.numel(), _s()), "cgl_bn2d_bwd_stats")
    return dx


def act_drop_bwd(dy, post, drop, n, hw, c, dx, slope=0.2, tanh_y=False, colsum=None):
    """``colsum`` (c == 1): float64 [(n hw + 255) // 256, 2] -- also the column-sum partials of dx per 256-row
    chunk (cgl_act_drop_bwd_colsum; colsum_finalize turns them into the bias gradient)."""
    _chk(dy, post, drop, dx)
    if colsum is not None:
        if not colsum.is_cuda or colsum.dtype != torch.float64 or colsum.numel() < 2 * ((n * hw + 255) // 256):
            raise RuntimeError("act_drop_bwd(colsum=...): float64 CUDA buffer of 2 per 256 rows")
        C.check(C.lib.cgl_act_drop_bwd_colsum(_p(dy), _p(post), _p(drop), n, hw, c, float(slope), int(tanh_y), _p(dx),
                                              _p(colsum), _s()), "cgl_act_drop_bwd_colsum")
        return dx
    C.check(C.lib.cgl_act_drop_bwd(_p(dy), _p(post), _p(drop), n, hw, c, float(slope), int(tanh_y), _p(dx), _s()),
            "cgl_act_drop_bwd")
    return dx


def colsum_finalize(part, nch, c, out):
    _chk(out)
    C.check(C.lib.cgl_colsum_finalize(_p(part), int(nch), int(c), _p(out), _s()), "cgl_colsum_finalize")
    return out


def dropout2d_mask(mask, n, c, p, seed, counter):
    _chk(mask)
    C.check(C.lib.cgl_dropout2d_mask(_p(mask), n, c, float(p), int(seed) & (2 ** 64 - 1), int(counter) & (2 ** 64 - 1),
                                     _s()), "cgl_dropout2d_mask")
    return mask


def dropout2d_masks(masks, ns, cs, p, seed, counters):
    """Several dropout2d_mask calls in one launch (same p and seed)."""
    _chk(*masks)
    k = len(masks)
    C.check(C.lib.cgl_dropout2d_masks(k, (ctypes.c_void_p * k)(*[m.data_ptr() for m in masks]),
                                      (ctypes.c_int * k)(*ns), (ctypes.c_int * k)(*cs), float(p),
                                      int(seed) & (2 ** 64 - 1),
                                      (ctypes.c_ulonglong * k)(*[int(c) & (2 ** 64 - 1) for c in counters]), _s()),
            "cgl_dropout2d_masks")


def dropout2d_masks_dev(masks, ns, cs, p, seed, counters, round_dev, round_stride):
    """dropout2d_masks with counter j = counters[j] + round_stride * round_dev[0] (device int32)."""
    _chk(*masks)
    k = len(masks)
    C.check(C.lib.cgl_dropout2d_masks_dev(k, (ctypes.c_void_p * k)(*[m.data_ptr() for m in masks]),
                                          (ctypes.c_int * k)(*ns), (ctypes.c_int * k)(*cs), float(p),
                                          int(seed) & (2 ** 64 - 1),
                                          (ctypes.c_ulonglong * k)(*[int(c) & (2 ** 64 - 1) for c in counters]),
                                          _p(round_dev), int(round_stride), _s()), "cgl_dropout2d_masks_dev")


def normal_fill_dev(out, seed, round_dev, stream_id=0):
    """N(0,1) fill of the z stream with round = round_dev[0] (device int32)."""
    _chk(out)
    C.check(C.lib.cgl_normal_fill_dev(_p(out), out.numel(), int(seed) & (2 ** 64 - 1), _p(round_dev), stream_id, _s()),
            "cgl_normal_fill_dev")


def sample_rows_dev(src, nrows, seed, round_dev, dst, nv_out=None):
    """Real batch of round round_dev[0] from a device-resident [n, f] shard (keyed per-pass permutation).
    ``nv_out`` (device int32): DataLoader semantics, each pass ending with its short batch, whose real rows
    land in nv_out[0]; None: whole batches only (drop_last)."""
    _chk(src, dst)
    C.check(C.lib.cgl_sample_rows_dev(_p(src), src.shape[0], nrows, src.shape[1], int(seed) & (2 ** 64 - 1),
                                      _p(round_dev), _p(dst), _p(nv_out), _s()), "cgl_sample_rows_dev")
    return dst


def defer_counters(counters, snap, snap_index, v=1):
    """Inside wgrad_defer: the deferred launch also snapshots counters[snap_index] into snap and adds v to every
    counter (cgl_conv_wgrad_defer_counters) -- counters_add without a launch of its own."""
    if not _WDEFER:
        raise RuntimeError("defer_counters outside wgrad_defer")
    if not (counters.is_cuda and snap.is_cuda and counters.dtype == torch.int32 and snap.dtype == torch.int32):
        raise ValueError("defer_counters: int32 device tensors")
    C.check(C.lib.cgl_conv_wgrad_defer_counters(_p(counters), counters.numel(), int(v), _p(snap), int(snap_index)),
            "cgl_conv_wgrad_defer_counters")


def counters_add(counters, v=1):
    """counters (device int32) += v, stream-ordered."""
    C.check(C.lib.cgl_counters_add(_p(counters), counters.numel(), int(v), _s()), "cgl_counters_add")


def nchw_to_nhwc(x, y, n, c, hw):
    _chk(x, y)
    C.check(C.lib.cgl_nchw_to_nhwc(_p(x), _p(y), n, c, hw, _s()), "cgl_nchw_to_nhwc")
    return y


def dense1_fwd_nhwc(x, w, b, y, n, c, hw, flat=None):
    """Linear(c*hw, 1) over the NCHW flattening of an [n, hw, c] NHWC map (model/lsgan.py:96-97), read
    from the NHWC map -- bitwise nhwc_to_nchw + dense_fwd(N=1); ``flat`` (optional) receives the NCHW view."""
    _chk(x, w, b, y, flat)
    if x.numel() < n * c * hw or w.numel() < c * hw or y.numel() < n or (flat is not None and flat.numel() < n * c * hw):
        raise ValueError("dense1_fwd_nhwc: tensor too small for the geometry")
    C.check(C.lib.cgl_dense1_fwd_nhwc(_p(x), _p(w), _p(b), _p(y), _p(flat), n, c, hw, _s()), "cgl_dense1_fwd_nhwc")
    return y


def dense1_bwd_data_nhwc(dy, w, dx, n, c, hw):
    """d/dx of Linear(c*hw, 1) over an NCHW-flattened [n, hw, c] NHWC map, stored NHWC
    (model/lsgan.py:96-97; replaces dense_bwd_data(K=1) + nchw_to_nhwc)."""
    _chk(dy, w, dx)
    if dy.numel() < n or w.numel() < c * hw or dx.numel() < n * c * hw:
        raise ValueError("dense1_bwd_data_nhwc: tensor too small for the geometry")
    C.check(C.lib.cgl_dense1_bwd_data_nhwc(_p(dy), _p(w), _p(dx), n, c, hw, _s()), "cgl_dense1_bwd_data_nhwc")
    return dx


def nhwc_to_nchw(x, y, n, c, hw):
    _chk(x, y)
    C.check(C.lib.cgl_nhwc_to_nchw(_p(x), _p(y), n, c, hw, _s()), "cgl_nhwc_to_nchw")
    return y


def dense1_head_nhwc(x, w, b, y, dy, dx, n, c, hw, kind, calls, scratch, flat=None, bn_in=None):
    """adv_layer forward + loss + input gradient in one launch (cgl_dense1_head_nhwc).  ``calls``: [(rows, target,
    weight, loss_out, nvalid)] -- one or two calls over consecutive rows (nvalid: the first call only).
    ``scratch``: >= n + 16 floats, zeroed once before its first use (a monotonic ticket + the loss terms).
    ``bn_in`` = (coef, groups): ``x`` is the pre-BatchNorm map, its BatchNorm (bn2d_fwd_stats(coef=)'s scale /
    shift, act none) applied in the loads."""
    coef, groups = bn_in if bn_in is not None else (None, 1)
    _chk(x, w, b, y, dy, dx, flat, scratch, coef)
    if coef is not None and coef.numel() < 2 * groups * c:
        raise ValueError("dense1_head_nhwc: bn_in coefficients [2][groups][c] expected")
    if len(calls) not in (1, 2) or sum(cl[0] for cl in calls) != n:
        raise ValueError("dense1_head_nhwc: one or two calls covering the n rows")
    if (x.numel() < n * c * hw or w.numel() < c * hw or y.numel() < n or dy.numel() < n or dx.numel() < n * c * hw or
            scratch.numel() < n + 16 or (flat is not None and flat.numel() < n * c * hw)):
        raise ValueError("dense1_head_nhwc: tensor too small for the geometry")
    (n0, t0, w0, l0, nv0) = calls[0]
    (t1, w1, l1) = (calls[1][1], calls[1][2], calls[1][3]) if len(calls) > 1 else (0, 0.0, None)
    C.check(C.lib.cgl_dense1_head_nhwc(_p(x), _p(w), _p(b), _p(y), _p(flat), _p(dy), _p(dx), n, c, hw, LOSS[kind],
                                       n0, int(t0), float(w0), _p(l0), _p(nv0), int(t1), float(w1), _p(l1),
                                       _p(coef), int(groups), _p(scratch), _s()), "cgl_dense1_head_nhwc")


def adv_loss(x, M, Cc, kind, target, weight, loss_out=None, grad=None, nvalid=None):
    """``nvalid`` (device int32, may be None): only the first *nvalid rows form the batch (mean over them,
    zero gradient on the rest)."""
    _chk(x, loss_out, grad)
    C.check(C.lib.cgl_adv_loss(_p(x), M, Cc, LOSS[kind], int(target), float(weight), _p(loss_out), _p(grad),
                               _p(nvalid), _s()), "cgl_adv_loss")


def adam_multi(params, grads, ms, vs, step, lr=2e-4, betas=(0.5, 0.999), eps=1e-8, step_dev=None):
    """One optim.Adam step over up to 32 tensors per launch (chunks larger lists).  ``step_dev``
    (device int32, completed steps): the step is step_dev[0] + 1, read on the device (graph replay)."""
    for i in range(0, len(params), 32):
        ps, gs, mm, vv = params[i:i + 32], grads[i:i + 32], ms[i:i + 32], vs[i:i + 32]
        _chk(*ps, *gs, *mm, *vv)
        nt = len(ps)
        arr = lambda ts: (ctypes.c_void_p * nt)(*[t.data_ptr() for t in ts])
        ns = (ctypes.c_int64 * nt)(*[t.numel() for t in ps])
        if step_dev is not None:
            C.check(C.lib.cgl_adam_multi_dev(nt, arr(ps), arr(gs), arr(mm), arr(vv), ns, _p(step_dev), float(lr),
                                             float(betas[0]), float(betas[1]), float(eps), _s()), "cgl_adam_multi_dev")
            continue
        C.check(C.lib.cgl_adam_multi(nt, arr(ps), arr(gs), arr(mm), arr(vv), ns, int(step), float(lr), float(betas[0]),
                                     float(betas[1]), float(eps), _s()), "cgl_adam_multi")


WEIGHTING = {"capgan": 0, "mean": 1, "mix_single": 2, "mix_double": 3, "cglgan": 4}


def weights_scale(weighting, lam, beta, losses, rank, x=None, alpha_out=None):
    """alpha = the reference's lambda-weighting of the gathered losses; x *= alpha[rank] in place."""
    _chk(losses, x, alpha_out)
    n = losses.numel()
    arr = (ctypes.c_float * n)(*[float(b) for b in beta])
    C.check(C.lib.cgl_weights_scale(WEIGHTING[weighting], n, rank, float(lam), arr, _p(losses), _p(x),
                                    x.numel() if x is not None else 0, _p(alpha_out), _s()), "cgl_weights_scale")
