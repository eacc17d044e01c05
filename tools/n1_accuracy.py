"""Accuracy of the G's Conv2d(64, 1) + Tanh forward (model/lsgan.py:19-20) on the GPU: tap-partial
kernel (cgl_conv_n1_part) vs the LDS-halo kernel (CGL_N1_TILE=1), both against float64, plus the
conv-round parity error of the G's last conv bias gradient under either kernel (test_gpu_conv_step)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cgl-gan_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from cglgan import conv_ops as O  # noqa: E402


def fwd_err(n=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 32, 32, 64, generator=g, dtype=torch.float64)
    w = torch.randn(1, 64, 3, 3, generator=g, dtype=torch.float64) / 24
    b = torch.randn(1, generator=g, dtype=torch.float64) * 0.1
    ref = torch.tanh(torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, b, padding=1)).permute(0, 2, 3, 1)
    r32 = torch.tanh(torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b.float(), padding=1))
    y = torch.empty(n, 32, 32, 1, device="cuda")
    O.conv3x3_fwd(x.float().cuda(), w.float().cuda(), b.float().cuda(), y, n, 32, 32, 64, 1, 1, 0, O.ACT_TANH)
    torch.cuda.synchronize()
    e = lambda a: float((a.double().cpu() - ref).norm() / ref.norm())
    return e(y), e(r32.permute(0, 2, 3, 1))


if __name__ == "__main__":
    from tests import test_gpu_conv_step as T
    for mode in ("part", "tile"):
        if mode == "tile":
            os.environ["CGL_N1_TILE"] = "1"
        else:
            os.environ.pop("CGL_N1_TILE", None)
        eh, e32 = fwd_err()
        line = f"{mode}: fwd rel err {eh:.3e} (torch fp32 CPU {e32:.3e})"
        for loss in ("mse", "bce"):
            st, o64, o32, outs = T._run(8, loss)
            gg = outs[0][3]
            k = "conv_blocks.8.bias"
            v = outs[0][1]["g_grads"][k]
            line += f"; {loss} {k} err {T._err(gg[k], v):.3e} (fp32 oracle {T._err(outs[0][2]['g_grads'][k], v):.3e}," \
                    f" norm {float(v.double().norm()):.3e})"
        print(line, flush=True)
