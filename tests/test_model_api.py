"""nn.Module drop-ins (cglgan.model) for model/mnist_model.py: structure and state-dict keys of
the reference modules (CPU), and HIP forward / backward / running statistics / eval sampling
against the oracle's fp64 restatement of the same modules (GPU).

Tolerances: outputs <= 1e-5 relative to fp64 (fp32 GEMM + BatchNorm); parameter gradients
<= 1e-4 relative per tensor, plus 1e-6 of the largest gradient norm of the model for tensors
whose true gradient is analytically zero (Linear biases feeding BatchNorm).
"""
import pytest
import torch

from cglgan import model as CM
from oracle import gan_oracle as O

IMG = (1, 28, 28)


def _oracle_for(mod, kind):
    if kind == "G":
        net = O.SeqNet(O.mnist_generator_spec())
    elif kind == "D":
        net = O.SeqNet(O.mnist_discriminator_spec())
    elif kind == "Ds":
        net = O.SeqNet(O.mnist_discriminator_spec(sigmoid=True))
    else:
        net = O.MixNet(O.mnist_mixgen_trunk_spec(), [O.mnist_mixgen_head_spec(h) for h in range(2)])
    return net


def test_state_dict_keys_match_reference_layout():
    for mod, kind in ((CM.Generator(IMG), "G"), (CM.Discriminator(IMG), "D"),
                      (CM.Discriminator(IMG, sigmoid=True), "Ds"), (CM.MixGenerator(IMG, 2), "MixG")):
        keys = list(mod.state_dict().keys())
        ref = list(_oracle_for(mod, kind).state_dict().keys())
        assert keys == ref, (kind, keys, ref)
    g = CM.MixGenerator(IMG, 3)
    assert hasattr(g, "model") and len(g.paths) == 3   # mixed-gan.py toggles .model / .paths


def test_cpu_tensors_are_refused():
    g = CM.Generator(IMG)
    with pytest.raises(RuntimeError):
        g(torch.randn(4, 100))


def _load64(net, mod):
    sd = mod.state_dict()
    nets = [net.trunk] + list(net.heads) if hasattr(net, "trunk") else [net]
    for n in nets:
        for k in list(n.params):
            n.params[k] = sd[k].detach().double().cpu().clone().requires_grad_(True)
        for k in list(n.buffers):
            n.buffers[k] = sd[k].detach().cpu().clone().double() if sd[k].dtype == torch.float32 else sd[k].clone()


def _rel(a, b):
    return float((a.detach().double().cpu() - b.detach().double().cpu()).norm() / max(float(b.detach().norm()), 1e-30))


def _grads(net):
    nets = [net.trunk] + list(net.heads) if hasattr(net, "trunk") else [net]
    out = {}
    for n in nets:
        for k, v in n.params.items():
            out[k] = v.grad
    return out


def _margin_ok(net, x, margin=1e-6):
    tr = []
    with torch.no_grad():
        if hasattr(net, "trunk"):
            h = net.trunk.forward(x.clone(), train=True, trace=tr)
            for hd in net.heads:
                hd.forward(h, train=True, trace=tr)
        else:
            net.forward(x.clone(), train=True, trace=tr)
    return min(float(t.abs().min() / (t.std() + 1e-30)) for t in tr) >= margin


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["G", "MixG", "D", "Ds"])
def test_forward_backward_vs_oracle(kind):
    torch.manual_seed(20211212)
    mod = {"G": lambda: CM.Generator(IMG), "MixG": lambda: CM.MixGenerator(IMG, 2),
           "D": lambda: CM.Discriminator(IMG), "Ds": lambda: CM.Discriminator(IMG, sigmoid=True)}[kind]().cuda()
    net = _oracle_for(mod, kind)
    _load64(net, mod)
    B = 64
    in_dim = 100 if kind in ("G", "MixG") else 784
    for seed in range(100, 164):   # LeakyReLU inputs away from the kink (see parity_helpers)
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(B, in_dim, generator=g) if in_dim == 100 else torch.rand(B, in_dim, generator=g) * 2 - 1
        probe = _oracle_for(mod, kind)
        _load64(probe, mod)
        if _margin_ok(probe, x.double()):
            break
    y = mod(x.cuda())
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        y64 = net.forward(x.double(), train=True) if not hasattr(net, "trunk") else net.forward(x.double())
    finally:
        torch.set_default_dtype(prev)
    y64 = y64.reshape(y.shape[0], -1)
    assert _rel(y.reshape(y.shape[0], -1), y64) <= 1e-5
    w = torch.randn(y64.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
    (y.reshape(y.shape[0], -1) * w.float().cuda()).sum().backward()
    (y64 * w).sum().backward()
    ref = _grads(net)
    gmax = max(float(v.norm()) for v in ref.values())
    for k, p in mod.named_parameters():
        err = float((p.grad.double().cpu() - ref[k]).norm())
        assert err <= 1e-4 * float(ref[k].norm()) + 1e-6 * gmax, (k, err, float(ref[k].norm()))
    # running statistics of the train-mode BatchNorm calls
    sd = mod.state_dict()
    nets = [net.trunk] + list(net.heads) if hasattr(net, "trunk") else [net]
    for n in nets:
        for k, v in n.buffers.items():
            if k.endswith("running_mean") or k.endswith("running_var"):
                assert _rel(sd[k], v) <= 1e-5, k
            elif k.endswith("num_batches_tracked"):
                assert int(sd[k]) == int(v), k


@pytest.mark.gpu
def test_eval_sampling_uses_running_stats():
    """capgan.py:203-209: net_g.eval(); gen = net_g(fixed_z) -- BatchNorm on running statistics."""
    torch.manual_seed(3)
    mod = CM.Generator(IMG).cuda()
    with torch.no_grad():
        for m in mod.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.running_mean.uniform_(-0.5, 0.5)
                m.running_var.uniform_(0.5, 2.0)
    net = _oracle_for(mod, "G")
    _load64(net, mod)
    z = torch.randn(200, 100, generator=torch.Generator().manual_seed(11))
    mod.eval()
    with torch.no_grad():
        y = mod(z.cuda())
    assert y.shape == (200, 1, 28, 28)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        with torch.no_grad():
            y64 = net.forward(z.double(), train=False)
    finally:
        torch.set_default_dtype(prev)
    assert _rel(y.reshape(200, -1), y64) <= 1e-5
