"""The LDS-staged operand panels of the 2 x 2-wave conv tiling (cgl_conv_fwd_body LDSM, CGL_CONV_LDSM): the
fragment values and the MFMA order are the direct-load path's, so the input gradient of the G up-convolution
(model/lsgan.py:15-16, its phase-form 4 x 4-tap stride-2 problem at the benchmarked 256 images, 512 tiles of
128 x 128) and the same call with its BatchNorm backward statistics in the epilogue are bitwise equal with and
without it; a fp64 check of a smaller case that still takes the tiling is in test_gpu_conv_ops."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(ldsm, dy, w, n, stats):
    from cglgan import conv_ops as O
    os.environ["CGL_CONV_LDSM"] = "1" if ldsm else "0"
    try:
        pk = O.PackSet()
        pk.add("G", "c5b", w, 16, 16, 128, 64, 1, 1, dir=1)
        pk.finalize(w.device)
        pk.run()
        dx = torch.empty(n, 16, 16, 128, device="cuda")
        if stats:
            x = torch.randn(n, 16, 16, 128, device="cuda", generator=torch.Generator("cuda").manual_seed(2))
            mean = x.mean(dim=(0, 1, 2)).contiguous()
            nch = O.stat_chunks(n, 16, 16, 128, 64, 1, 1, 1, bwd=True)
            assert nch > 0
            part = torch.zeros(nch * 128 * 2, dtype=torch.float64, device="cuda")
            O.conv3x3_bwd_data(dy, w, dx, n, 16, 16, 128, 64, 1, 1, wp=pk["c5b"], stats=(part, 1, x, None, mean, 0.2))
            torch.cuda.synchronize()
            return dx, part
        O.conv3x3_bwd_data(dy, w, dx, n, 16, 16, 128, 64, 1, 1, wp=pk["c5b"])
        torch.cuda.synchronize()
        return dx, None
    finally:
        os.environ.pop("CGL_CONV_LDSM", None)


@pytest.mark.parametrize("stats", [False, True])
def test_conv_ldsm_bitwise(stats):
    n = 256
    g = torch.Generator("cuda").manual_seed(1)
    dy = torch.randn(n, 32, 32, 64, device="cuda", generator=g)
    w = torch.randn(64, 128, 3, 3, device="cuda", generator=g) / 30
    a, pa = _run(True, dy, w, n, stats)
    b, pb = _run(False, dy, w, n, stats)
    assert torch.equal(a, b)
    if stats:
        assert torch.equal(pa, pb)
