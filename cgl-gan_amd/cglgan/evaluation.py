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


def kl_score(real: torch.Tensor, gen: torch.Tensor, num_sample: int | None = None, num_servers: int = 1,
             bins: int = 16, range_=((-1.0, 1.0), (-1.0, 1.0)), return_counts: bool = False):
    """``real``: the real test points [n, 2]; ``gen``: the generated points [m, 2] (one server's, or
    the servers' concatenated X, as plot_2d receives them).  With ``num_sample`` the reference's
    strided subsamples are taken (real stride n // num_sample, generated stride
    m // (num_sample // num_servers)); otherwise every point is binned.  Float32 CUDA tensors."""
    for t in (real, gen):
        if not t.is_cuda or t.dtype != torch.float32 or t.dim() != 2 or t.shape[1] != 2:
            raise RuntimeError("kl_score: expected float32 CUDA tensors of shape [n, 2]")
    real, gen = real.contiguous(), gen.contiguous()
    nr, ng = real.shape[0], gen.shape[0]
    sr = sg = 1
    if num_sample is not None:
        sr = max(1, nr // num_sample)
        sg = max(1, ng // (num_sample // num_servers))
    cnt_r, cnt_g = (nr + sr - 1) // sr, (ng + sg - 1) // sg
    counts = torch.empty(2, bins, bins, dtype=torch.int32, device=real.device)
    kl = torch.empty(1, dtype=torch.float64, device=real.device)
    (lo0, hi0), (lo1, hi1) = range_
    C.check(C.lib.cgl_kl_score(_p(real), cnt_r, sr, _p(gen), cnt_g, sg, bins, float(lo0), float(hi0), float(lo1),
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
