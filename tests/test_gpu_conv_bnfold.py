"""The G BatchNorm2d + LeakyReLU folded into the next conv's operand load (ConvGanStep.bn_fold,
cgl_conv3x3_fwd_packed_bnin / cgl_bn2d_fwd_stats_coef; model/lsgan.py:15-22): the consumer applies the
finalize's scale / shift with cgl_eltwise's arithmetic as it loads, so a round with the fold equals the
round with the separate apply passes (CGL_CONV_BNFOLD=0) bitwise -- eager and graph-replayed, at B = 8 and
the benchmarked B = 256, both layers folded (mask 3) and the default (mask 2: conv_blocks.6 into
conv_blocks.8 only); the Xd half the fold no longer writes is recomputable (g_act_xd)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(B, graph, data, mask):
    from cglgan.conv_step import ConvGanStep
    steps = []
    for fold in (mask, 0):
        os.environ["CGL_CONV_BNFOLD"] = str(fold)
        os.environ["CGL_CONV_ELIDE"] = "0"      # (the elision is tests/test_gpu_conv_fusions.py's)
        try:
            st = ConvGanStep(B, seed=21, data=data, graph=graph)
        finally:
            os.environ.pop("CGL_CONV_BNFOLD", None)
            os.environ.pop("CGL_CONV_ELIDE", None)
        st.init_default(5, 6)
        steps.append(st)
    assert steps[0].bn_fold == mask and not steps[1].bn_fold
    return steps


@pytest.mark.parametrize("B,graph,mask", [(8, False, 3), (256, False, 3), (256, True, 3), (256, True, 2)])
def test_conv_bn_fold_bitwise(B, graph, mask):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        data = torch.rand(4 * B + 3, 1024, device="cuda", generator=torch.Generator("cuda").manual_seed(3)) * 2 - 1
        a, b = _pair(B, graph, data, mask)
        for _ in range(3):
            a.run()
            b.run()
        torch.cuda.synchronize()
    for name in ("p", "g", "m", "v"):
        assert torch.equal(getattr(a.G, name), getattr(b.G, name)), ("G", name)
        assert torch.equal(getattr(a.D, name), getattr(b.D, name)), ("D", name)
    assert torch.equal(a.x3, b.x3) and torch.equal(a.lbuf, b.lbuf)
    for k in a.G.running:
        assert torch.equal(a.G.running[k], b.G.running[k]), k
    # the Xg half of the activations is still written (the G backward reads it), the Xd half recomputes
    assert torch.equal(a.a1[B:], b.a1[B:]) and torch.equal(a.a2[B:], b.a2[B:])
    for k in ("a1", "a2"):
        assert torch.allclose(a.g_act_xd(k), b.g_act_xd(k), rtol=1e-6, atol=1e-6), k
