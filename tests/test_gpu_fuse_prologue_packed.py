"""The round prologue rides in G's first GEMM (fuse_prologue, CGL_FUSE_PRO) only when that GEMM does not read
operands the prologue writes: with z_dim >= 256 the planner gives G's layer 0 fragment-packed weights, which the
prologue's pack blocks rewrite every round -- fused, the GEMM tiles of the same launch could read them half
written.  The plan keeps two launches then, and the rounds are bitwise those of the unfused plan
(ADVICE r3).  z_dim = 100 (the reference's) still fuses."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(z_dim, fuse):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    os.environ["CGL_FUSE_PRO"] = "1" if fuse else "0"
    try:
        gm, dm = specs.mnist_generator(z_dim=z_dim), specs.mnist_discriminator()
        g = torch.Generator(device="cuda").manual_seed(3)
        real = torch.rand(512, 784, device="cuda", generator=g) * 2 - 1
        st = GanStep(gm, dm, batch=64, loss="ce", weighting="capgan", gen_z=True, real=real, sample_n=512, seed=9)
    finally:
        os.environ.pop("CGL_FUSE_PRO", None)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(7)
    default_init(dm, st.d_views)
    st.reset()
    return st


@pytest.mark.parametrize("z_dim", [100, 256])
def test_fused_prologue_bitwise_and_packed_layer0_unfused(z_dim):
    a, b = _step(z_dim, True), _step(z_dim, False)
    kinds = [k for k, _, _ in a.launches()]
    if z_dim >= 256:
        assert "prologue" in kinds and "gemm_prologue" not in kinds, kinds
    else:
        assert "gemm_prologue" in kinds, kinds
    for r in range(4):
        a.run(graph=(r % 2 == 1))
        b.run(graph=(r % 2 == 1))
    torch.cuda.synchronize()
    for name in ("g_params", "d_params", "g_running", "g_m", "g_v"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
