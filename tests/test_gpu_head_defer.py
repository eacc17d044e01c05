"""Deferred head-loss reduction (cgl_runtime.hip defer_heads, off with CGL_HEAD_DEFER=0): a head launch followed by
a GEMM launch stores only its per-workgroup loss partials, and one extra workgroup of that GEMM launch reduces them
(cgl_head_finish) in the ticket path's fixed order -- so the rounds are bitwise those of the last-arriver path,
including a pass's short real batch (the head's device-sized real segment)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(defer, B):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    os.environ["CGL_HEAD_DEFER"] = "1" if defer else "0"
    try:
        gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
        g = torch.Generator().manual_seed(5)
        real = (torch.rand(4 * B + 17, 784, generator=g) * 2 - 1).cuda()   # 4 full batches + a short one per pass
        st = GanStep(gm, dm, batch=B, loss="ce", weighting="capgan", gen_z=True, real=real, sample_n=real.shape[0],
                     seed=77)
    finally:
        os.environ.pop("CGL_HEAD_DEFER", None)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(4242)
    default_init(dm, st.d_views)
    st.reset()
    return st


@pytest.mark.parametrize("B", [64, 256])
def test_deferred_head_bitwise(B):
    a, b = _step(True, B), _step(False, B)
    ka = [k for k, _, _ in a.launches()]
    kb = [k for k, _, _ in b.launches()]
    assert ka == kb, (ka, kb)           # same launches: the finisher is one more workgroup, not a launch
    for r in range(7):                  # rounds 4 and 5 straddle the pass's short batch
        a.run(graph=r >= 2)
        b.run(graph=r >= 2)
        torch.cuda.synchronize()
        sa, sb = a.stats(), b.stats()
        for k in ("round", "g_loss", "F", "lambda", "d_loss"):
            assert sa[k] == sb[k], (r, k, sa[k], sb[k])
    for name in ("g_params", "g_m", "g_v", "d_params", "d_m", "d_v", "g_running", "z"):
        x, y = getattr(a, name), getattr(b, name)
        assert torch.equal(x, y), (name, (x - y).abs().max().item())
