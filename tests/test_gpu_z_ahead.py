"""z drawn one round ahead (round 5, cgl_runtime.hip plan z_ahead, CGL_Z_AHEAD=0 off): the G Adam launch that ends
round r draws round r + 1's z into the workspace (Philox stream 0, counter r + 1), and G's first GEMM reads it
there, copying the rows out to GanStep.z -- bitwise the rounds (and the z) of the in-round draw.  Also: a resumed
step (device round state loaded from a resume file) draws the z that follows the loaded round counter."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

NAMES = ("g_params", "g_grads", "g_m", "g_v", "d_params", "d_m", "d_v", "g_running", "z")


def _step(on, B=256, **kw):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    os.environ["CGL_Z_AHEAD"] = "1" if on else "0"
    try:
        gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
        g = torch.Generator().manual_seed(3)
        real = (torch.rand(4 * B + 17, 784, generator=g) * 2 - 1).cuda()
        st = GanStep(gm, dm, batch=B, loss="ce", weighting="capgan", gen_z=True, real=real, sample_n=real.shape[0],
                     seed=99, **kw)
    finally:
        os.environ.pop("CGL_Z_AHEAD", None)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(4242)
    default_init(dm, st.d_views)
    st.reset()
    return st


def _same(a, b, tag):
    torch.cuda.synchronize()
    for name in NAMES:
        x, y = getattr(a, name), getattr(b, name)
        assert torch.equal(x, y), (tag, name, (x - y).abs().max().item())
    sa, sb = a.stats(), b.stats()
    for k in ("round", "g_loss", "F", "lambda", "d_loss"):
        assert sa[k] == sb[k], (tag, k, sa[k], sb[k])


@pytest.mark.parametrize("B", [64, 256])
def test_z_ahead_bitwise(B):
    a, b = _step(True, B), _step(False, B)
    ka, kb = a.launches(), b.launches()
    assert [k for k, _, _ in ka] == [k for k, _, _ in kb]
    assert ka[-1][2] > kb[-1][2]          # the G Adam launch carries the z blocks
    for r in range(6):
        a.run(graph=r >= 2)
        b.run(graph=r >= 2)
        _same(a, b, f"B={B} round {r + 1}")


def test_z_ahead_resume():
    a, b = _step(True, 64), _step(True, 64)
    for _ in range(3):
        a.run()
    sd = a.resume_state()
    b.load_resume_state(sd)              # b's own z buffer still holds round 1's: the load must redraw it
    for r in range(2):
        a.run(graph=r >= 1)
        b.run(graph=r >= 1)
    _same(a, b, "resumed")
