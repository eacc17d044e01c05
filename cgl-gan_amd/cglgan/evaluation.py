"""Sampling and evaluation of the 2-D Gaussian-mixture GAN.

* ``sample_fixed``: Server.plot_2d -- ``net.eval(); X = net(fixed_z); net.train()`` (capgan.py:203-209,
  CGLGAN/2DMG/main.py Server.plot_2d) on the drop-in modules of cglgan.model (HIP kernels, BatchNorm
  from running statistics in eval mode).
* ``kl_score``: the KL score of CGLGAN/2DMG/main.py:63-101 -- np.histogram2d of the strided real test
  subsample (``test_set[::len // num_sample]``, :68) and of the servers' generated points
  (``X[::len // (num_sample // S)]``, :78) over 16 x 16 bins of [-1, 1]^2, scipy.stats.entropy(gen,
  real) over the bins with a non-zero real count -- computed on the GPU by ``cgl_kl_score``
  (include/cglgan.h); the histograms stay on the device, only the score is read back.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as C


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def kl_score(real: torch.Tensor, gen, num_sample: int | None = None, num_servers: int | None = None,
             bins: int = 16, range_=((-1.0, 1.0), (-1.0, 1.0)), return_counts: bool = False):
    """``real``: the real test points [n, 2]; ``gen``: the generated points -- one [m, 2] tensor, or the
    list of every server's X as plot_2d receives them (CGLGAN/2DMG/main.py:75-80).  With
    ``num_sample`` the reference's strided subsamples are taken: real stride n // num_sample (:68) and,
    PER SERVER, stride len(X_s) // (num_sample // S) before the servers' samples are concatenated
    (:78-80); ``num_servers`` defaults to the number of tensors given.  Without ``num_sample`` every
    point is binned.  Float32 CUDA tensors."""
    gens = list(gen) if isinstance(gen, (list, tuple)) else [gen]
    for t in [real] + gens:
        if not t.is_cuda or t.dtype != torch.float32 or t.dim() != 2 or t.shape[1] != 2:
            raise RuntimeError("kl_score: expected float32 CUDA tensors of shape [n, 2]")
    S = num_servers if num_servers is not None else len(gens)
    if num_sample is not None and S != len(gens):
        # the subsample is strided per server (:78), so a concatenation of several servers' X cannot be
        # subsampled correctly: pass one tensor per server
        raise ValueError("num_servers must match the number of per-server tensors given")
    real = real.contiguous()
    nr = real.shape[0]
    sr = sg = 1
    if num_sample is not None:
        sr = max(1, nr // num_sample)
        if len(gens) > 1:
            # each server's X strided on its own, then concatenated (:78-80): one gathered copy
            gens = [x[::max(1, x.shape[0] // (num_sample // S))] for x in gens]
        else:
            sg = max(1, gens[0].shape[0] // (num_sample // S))
    g = gens[0].contiguous() if len(gens) == 1 else torch.cat(gens, 0)
    ng = g.shape[0]
    cnt_r, cnt_g = (nr + sr - 1) // sr, (ng + sg - 1) // sg
    counts = torch.empty(2, bins, bins, dtype=torch.int32, device=real.device)
    kl = torch.empty(1, dtype=torch.float64, device=real.device)
    (lo0, hi0), (lo1, hi1) = range_
    C.check(C.lib.cgl_kl_score(_p(real), cnt_r, sr, _p(g), cnt_g, sg, bins, float(lo0), float(hi0), float(lo1),
                               float(hi1), _p(counts), _p(kl),
                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "cgl_kl_score")
    out = float(kl.item())
    return (out, counts) if return_counts else out


@torch.no_grad()
def sample_fixed(net: torch.nn.Module, fixed_z: torch.Tensor) -> torch.Tensor:
    """Server.plot_2d: generate from the server's fixed noise in eval mode, restoring train mode."""
    was = net.training
    net.eval()
    try:
        return net(fixed_z)
    finally:
        net.train(was)
