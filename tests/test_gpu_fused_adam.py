"""Launch fusions of the MLP round, each bitwise the same rounds as the separate launches:
  * K_GEMM_ADAM (cgl_runtime.hip fuse_wgrad_adam, off with CGL_FUSE_GADAM=0 / CGL_FUSE_DADAM=0): a model's
    first-layer weight gradient with its Adam -- the fused tiles apply cgl_adam_update to the gradient values
    they store, the companion workgroups run cgl_adam over every other parameter of the model, and the G
    Adam's scalar tail (lambda, F, round) runs once;
  * K_GEMM_PRO (fuse_prologue, off with CGL_FUSE_PRO=0): the round prologue with G's first GEMM -- each GEMM
    workgroup draws its own rows of z (the same Philox stream), the prologue's other blocks ride along."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(fuse, B=256, var="CGL_FUSE_GADAM"):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    os.environ[var] = "1" if fuse else "0"
    if var == "CGL_FUSE_DADAM":     # (the fused D Adam turns D's packed weights off: compare against that plan)
        os.environ["CGL_DPACK"] = "0"
    try:
        gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
        g = torch.Generator().manual_seed(3)
        real = (torch.rand(4 * B + 17, 784, generator=g) * 2 - 1).cuda()
        st = GanStep(gm, dm, batch=B, loss="ce", weighting="capgan", gen_z=True, real=real, sample_n=real.shape[0],
                     seed=99)
    finally:
        os.environ.pop(var, None)
        os.environ.pop("CGL_DPACK", None)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(4242)
    default_init(dm, st.d_views)
    st.reset()
    return st


@pytest.mark.parametrize("var,kind,pos", [("CGL_FUSE_GADAM", "gemm_adam", -1), ("CGL_FUSE_DADAM", "gemm_adam", None),
                                          ("CGL_FUSE_PRO", "gemm_prologue", 0)])
@pytest.mark.parametrize("B", [64, 256])
def test_fused_launch_bitwise(B, var, kind, pos):
    a, b = _step(True, B, var), _step(False, B, var)
    ka = [k for k, _, _ in a.launches()]
    kb = [k for k, _, _ in b.launches()]
    assert ka.count(kind) == kb.count(kind) + 1 and len(ka) == len(kb) - 1, (ka, kb)
    if pos is not None:
        assert ka[pos] == kind and kb[pos] != kind, (ka, kb)
    for r in range(6):
        a.run(graph=r >= 2)
        b.run(graph=r >= 2)
    torch.cuda.synchronize()
    for name in ("g_params", "g_grads", "g_m", "g_v", "d_params", "d_m", "d_v", "g_running", "z"):
        x, y = getattr(a, name), getattr(b, name)
        assert torch.equal(x, y), (name, (x - y).abs().max().item())
    sa, sb = a.stats(), b.stats()
    for k in ("round", "g_loss", "F", "lambda", "d_loss"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])


def test_adam4_bitwise():
    """cgl_adam4 (four elements per thread, 16-byte accesses; default) vs cgl_adam (CGL_ADAM4=0): the same
    pinned per-element arithmetic, so the same rounds bit for bit."""
    os.environ["CGL_ADAM4"] = "0"
    try:
        b = _step(False, 256, "CGL_FUSE_GADAM")
    finally:
        os.environ.pop("CGL_ADAM4", None)
    a = _step(False, 256, "CGL_FUSE_GADAM")
    assert [g for k, _, g in a.launches() if k == "adam"] != [g for k, _, g in b.launches() if k == "adam"]
    for r in range(5):
        a.run(graph=r >= 2)
        b.run(graph=r >= 2)
    torch.cuda.synchronize()
    for name in ("g_params", "g_grads", "g_m", "g_v", "d_params", "d_m", "d_v", "g_running", "z"):
        x, y = getattr(a, name), getattr(b, name)
        assert torch.equal(x, y), (name, (x - y).abs().max().item())
    assert a.stats()["lambda"] == b.stats()["lambda"] and a.stats()["F"] == b.stats()["F"]
