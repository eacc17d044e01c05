"""The phase-form upsampling convs (model/lsgan.py:14-18: Upsample(2) -> Conv2d(128, 128) and Upsample(2) ->
Conv2d(128, 64)) with the input window staged in LDS once per 64-row tile and shared by the 4 output-parity waves
(cgl_conv.hip HALO path, conv_halo_ok): the same chunk order and MFMA sequence as the direct path's
one-wave-per-K tiling, so bitwise equal to it (CGL_CONV_HALO=0) whenever the direct path picks that tiling
(>= 512 workgroups: n >= 128 images for the 64-channel conv, n >= 512 for the 128-channel one; the bench runs
n = 512) -- as a single op and over whole eager rounds (with and without the folded input BatchNorm).
Smaller batches make the direct path split K over the waves of a workgroup (conv_tiling_for), a different
summation order: there the two agree to fp32 accumulation tolerance."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _with(env, fn):
    os.environ["CGL_CONV_HALO"] = env
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        os.environ.pop("CGL_CONV_HALO", None)


# (input side, output channels): conv_blocks.5 (Upsample 16 -> 32, Conv2d(128, 64)) and conv_blocks.1
# (Upsample 8 -> 16, Conv2d(128, 128): two 64-channel workgroups per row tile)
GEOMS = [(16, 64), (8, 128)]


def _upconv_pair(n, hw, cout):
    from cglgan import conv_ops as O
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(n, hw, hw, 128, device="cuda", generator=g)
    w = torch.randn(cout, 128, 3, 3, device="cuda", generator=g) * 0.05
    b = torch.randn(cout, device="cuda", generator=g)
    outs = []
    for env in ("1", "0"):
        y = torch.empty(n, 2 * hw, 2 * hw, cout, device="cuda")
        outs.append(_with(env, lambda: O.conv3x3_fwd(x, w, b, y, n, hw, hw, 128, cout, 1, 1, O.ACT_LEAKY,
                                                     0.2).clone()))
    return outs


@pytest.mark.parametrize("n,geom", [(128, GEOMS[0]), (512, GEOMS[0]), (512, GEOMS[1])])
def test_upconv_halo_op_bitwise(n, geom):
    a, b = _upconv_pair(n, *geom)
    assert torch.equal(a, b)


@pytest.mark.parametrize("n,geom", [(2, GEOMS[0]), (64, GEOMS[0]), (2, GEOMS[1]), (64, GEOMS[1]), (128, GEOMS[1])])
def test_upconv_halo_op_small_batch(n, geom):
    a, b = _upconv_pair(n, *geom)
    # K = 1152 products of |x| ~ 1, |w| ~ 0.05 per output: fp32 reassociation error well below 1e-4
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("fold", [0, 3])
def test_conv_round_halo_bitwise(fold):
    from cglgan.conv_step import ConvGanStep
    B = 256   # G's up-convs over n = 2B = 512 images: the direct path's one-wave-per-K tiling for both
    data = torch.rand(4 * B + 3, 1024, device="cuda", generator=torch.Generator("cuda").manual_seed(3)) * 2 - 1
    steps = []
    for env in ("1", "0"):
        os.environ["CGL_CONV_BNFOLD"] = str(fold)
        try:
            st = ConvGanStep(B, seed=21, data=data, graph=False)
        finally:
            os.environ.pop("CGL_CONV_BNFOLD", None)
        st.init_default(5, 6)
        for _ in range(2):
            _with(env, lambda: st.run(eager=True))
        steps.append(st)
    a, b = steps
    for name in ("p", "g", "m", "v"):
        assert torch.equal(getattr(a.G, name), getattr(b.G, name)), ("G", name)
        assert torch.equal(getattr(a.D, name), getattr(b.D, name)), ("D", name)
    assert torch.equal(a.x3, b.x3) and torch.equal(a.y2, b.y2)
