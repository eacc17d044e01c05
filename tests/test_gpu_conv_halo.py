"""The phase-form upsampling conv (model/lsgan.py:17-18: Upsample(2) -> Conv2d(128, 64)) with its input window
staged in LDS once per 64-row tile and shared by the 4 output-parity waves (cgl_conv.hip HALO path,
conv_halo_ok): the same chunk order and MFMA sequence as the direct path's one-wave-per-K tiling, so bitwise equal
to it (CGL_CONV_HALO=0) whenever the direct path picks that tiling (>= 512 workgroups: n >= 128 images, which the
bench's n = 512 meets) -- as a single op and over whole eager rounds (with and without the folded input BatchNorm).
Smaller batches make the direct path split K over the waves of a workgroup (conv_tiling_for), a different summation
order: there the two agree to fp32 accumulation tolerance."""
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


def _upconv_pair(n):
    from cglgan import conv_ops as O
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(n, 16, 16, 128, device="cuda", generator=g)
    w = torch.randn(64, 128, 3, 3, device="cuda", generator=g) * 0.05
    b = torch.randn(64, device="cuda", generator=g)
    outs = []
    for env in ("1", "0"):
        y = torch.empty(n, 32, 32, 64, device="cuda")
        outs.append(_with(env, lambda: O.conv3x3_fwd(x, w, b, y, n, 16, 16, 128, 64, 1, 1, O.ACT_LEAKY, 0.2).clone()))
    return outs


@pytest.mark.parametrize("n", [128, 512])
def test_upconv_halo_op_bitwise(n):
    a, b = _upconv_pair(n)
    assert torch.equal(a, b)


@pytest.mark.parametrize("n", [2, 64])
def test_upconv_halo_op_small_batch(n):
    a, b = _upconv_pair(n)
    # K = 1152 products of |x| ~ 1, |w| ~ 0.05 per output: fp32 reassociation error well below 1e-4
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("fold", [0, 3])
def test_conv_round_halo_bitwise(fold):
    from cglgan.conv_step import ConvGanStep
    B = 64   # G's up-conv over n = 2B = 128 images: the direct path's one-wave-per-K tiling
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
