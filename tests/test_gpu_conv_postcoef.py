"""The G BatchNorm2d backward takes LeakyReLU'(a) from the sign of the forward's own fmaf(y, scale, shift)
(cgl_bn2d_bwd / cgl_bn2d_bwd_stats post_coef, ConvGanStep: the coef the forward finalize kept) instead of
reading the activation a: the forward wrote a = LeakyReLU(that value), so the mask -- and every tensor of the
round -- is bitwise the one read from a (CGL_CONV_POSTCOEF=0), eager and graph-replayed, at B = 8 and the
benchmarked B = 256, with the default fold mask and with no fold (model/lsgan.py:13-22)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(B, graph, data, post_coef, fold):
    from cglgan.conv_step import ConvGanStep
    os.environ["CGL_CONV_POSTCOEF"] = "1" if post_coef else "0"
    os.environ["CGL_CONV_BNFOLD"] = str(fold)
    try:
        st = ConvGanStep(B, seed=21, data=data, graph=graph)
    finally:
        os.environ.pop("CGL_CONV_POSTCOEF", None)
        os.environ.pop("CGL_CONV_BNFOLD", None)
    st.init_default(5, 6)
    return st


@pytest.mark.parametrize("B,graph,fold", [(8, False, 2), (256, False, 0), (256, True, 2)])
def test_conv_post_coef_bitwise(B, graph, fold):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        data = torch.rand(4 * B + 3, 1024, device="cuda", generator=torch.Generator("cuda").manual_seed(3)) * 2 - 1
        a, b = _step(B, graph, data, True, fold), _step(B, graph, data, False, fold)
        for _ in range(3):
            a.run()
            b.run()
        torch.cuda.synchronize()
    assert a.post_coef_on and not b.post_coef_on
    assert {"conv_blocks.2", "conv_blocks.6"} <= a.coef_kept
    for name in ("p", "g", "m", "v"):
        assert torch.equal(getattr(a.G, name), getattr(b.G, name)), ("G", name)
        assert torch.equal(getattr(a.D, name), getattr(b.D, name)), ("D", name)
    assert torch.equal(a.x3, b.x3) and torch.equal(a.lbuf, b.lbuf)
    assert torch.equal(a.dy1, b.dy1) and torch.equal(a.dy2, b.dy2)
