"""cglgan.lsgan nn.Module drop-ins (model/lsgan.py Generator / Discriminator / MixGenerator) on the
GPU vs the float64 conv oracle from the same state: forward, backward (parameter and input grads),
BatchNorm2d running statistics, Dropout2d (masks read back from the module), eval-mode sampling.
Tolerance: the survey's 1e-5 relative to each tensor's max magnitude (fp32 vs fp64) for forwards, every
gradient and the running statistics (largest observed 1.0e-6, `dz`, profiles/r05_lsgan_module_errors.txt;
CGL_PRINT_ERR=1 prints each ratio); gradients of conv biases that feed BatchNorm2d excluded (analytically
zero, rounding noise)."""
import os

import pytest
import torch

from oracle import conv_oracle as CV

pytestmark = pytest.mark.gpu
NOISE = {"conv_blocks.1.bias", "conv_blocks.5.bias", "model.3.bias"}


def close(got, ref, rel=1e-5, what=""):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = max(float(ref.abs().max()), 1e-12)
    err = float((got - ref).abs().max())
    if os.environ.get("CGL_PRINT_ERR"):
        print(f"ERR {what}: {err / scale:.3e} (bound {rel:.0e})")
    assert err <= rel * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def _oracle_state(mod):
    sd = mod.state_dict()
    P = {k: v.detach().double().cpu().clone().requires_grad_(True) for k, v in sd.items()
         if "running" not in k and "num_batches" not in k}
    Bf = {k: (v.double().cpu().clone() if v.is_floating_point() else v.cpu().clone()) for k, v in sd.items()
          if "running" in k or "num_batches" in k}
    return P, Bf


def test_generator_forward_backward_eval():
    from cglgan import lsgan
    torch.manual_seed(3)
    g = lsgan.Generator((1, 32, 32)).cuda()
    P, Bf = _oracle_state(g)
    z = torch.randn(6, 100)
    zc = z.cuda().requires_grad_(True)
    img = g(zc)
    assert img.shape == (6, 1, 32, 32)
    z64 = z.double().requires_grad_(True)
    ref = CV.g_forward(P, Bf, z64)
    close(img, ref, what="G fwd")
    dy = torch.randn(6, 1, 32, 32)
    (img * dy.cuda()).sum().backward()
    (ref * dy.double()).sum().backward()
    for k, p in g.named_parameters():
        if k not in NOISE:
            close(p.grad, P[k].grad, rel=1e-5, what="G grad " + k)
    close(zc.grad, z64.grad, rel=1e-5, what="dz")
    for k, v in g.state_dict().items():
        if "running" in k:
            close(v, Bf[k], what=k)
    assert int(g.conv_blocks[2].num_batches_tracked) == 1
    g.eval()
    with torch.no_grad():
        ev = g(z.cuda())
        ref_ev = CV.g_forward(P, Bf, z.double(), train=False)
    close(ev, ref_ev, what="G eval")


@pytest.mark.parametrize("hw", [32, 28])
def test_discriminator_forward_backward(hw):
    from cglgan import lsgan
    torch.manual_seed(4)
    d = lsgan.Discriminator((1, hw, hw)).cuda()
    P, Bf = _oracle_state(d)
    x = torch.rand(5, 1, hw, hw) * 2 - 1
    xc = x.cuda().requires_grad_(True)
    v = d(xc)
    masks = [m.cpu() for m in d.last_masks]
    assert len(masks) == 4 and all(set(torch.unique(m).tolist()) <= {0.0, float(torch.tensor(1.0) / 0.75)}
                                   for m in masks)
    x64 = x.double().requires_grad_(True)
    ref = CV.d_forward(P, Bf, x64, masks)
    close(v, ref, what="D fwd")
    v.sum().backward()
    ref.sum().backward()
    for k, p in d.named_parameters():
        if k not in NOISE:
            close(p.grad, P[k].grad, rel=1e-5, what="D grad " + k)
    close(xc.grad, x64.grad, rel=1e-5, what="d img")
    d.eval()
    with torch.no_grad():
        close(d(x.cuda()), CV.d_forward(P, Bf, x.double(), None, train=False), what="D eval")


def test_mixgenerator_heads():
    from cglgan import lsgan
    torch.manual_seed(5)
    m = lsgan.MixGenerator((1, 32, 32), 3).cuda()
    P, Bf = _oracle_state(m)
    z = torch.randn(4, 100)
    out = m(z.cuda())
    assert out.shape == (12, 1, 32, 32)
    ref = CV.mixg_forward(P, Bf, z.double(), 3)
    close(out, ref, what="MixG fwd")
    dy = torch.randn(12, 1, 32, 32)
    (out * dy.cuda()).sum().backward()
    (ref * dy.double()).sum().backward()
    for k, p in m.named_parameters():
        if k not in ("model.3.bias", "model.7.bias"):   # feed BatchNorm2d: gradient is rounding noise
            close(p.grad, P[k].grad, rel=1e-5, what="MixG grad " + k)
