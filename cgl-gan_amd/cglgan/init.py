"""Parameter initialisation matching the reference modules.

``default_init`` reproduces ``nn.Linear``'s default (kaiming_uniform_(a=sqrt(5)) weight, U(+-1/sqrt(fan_in))
bias) and BatchNorm1d's (weight 1, bias 0) in construction order, drawing from the torch CPU RNG,
so ``torch.manual_seed(s); default_init(...)`` yields the same tensors as
``torch.manual_seed(s); Generator(ims)`` in the reference (capgan.py:28,156).
``weights_init`` is mixed-gan.py:68-77 (Linear W ~ N(0, .02), b = 0; BN weight ~ N(1, .02), b = 0).
"""
from __future__ import annotations

import math

import torch

from .specs import MlpModel


@torch.no_grad()
def default_init(model: MlpModel, views, generator=None):
    for l in range(model.n_layers):
        fo, fi = model.dims[l + 1], model.dims[l]
        w = torch.empty(fo, fi)
        b = torch.empty(fo)
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5), generator=generator)
        bound = 1.0 / math.sqrt(fi)
        torch.nn.init.uniform_(b, -bound, bound, generator=generator)
        views[model.linear_keys[l] + ".weight"].copy_(w)
        views[model.linear_keys[l] + ".bias"].copy_(b)
        if model.bn[l]:
            views[model.bn_keys[l] + ".weight"].fill_(1.0)
            views[model.bn_keys[l] + ".bias"].fill_(0.0)


@torch.no_grad()
def weights_init(model: MlpModel, views, generator=None):
    for l in range(model.n_layers):
        fo, fi = model.dims[l + 1], model.dims[l]
        w = torch.empty(fo, fi)
        torch.nn.init.normal_(w, 0.0, 0.02, generator=generator)
        views[model.linear_keys[l] + ".weight"].copy_(w)
        views[model.linear_keys[l] + ".bias"].fill_(0.0)
        if model.bn[l]:
            g = torch.empty(fo)
            torch.nn.init.normal_(g, 1.0, 0.02, generator=generator)
            views[model.bn_keys[l] + ".weight"].copy_(g)
            views[model.bn_keys[l] + ".bias"].fill_(0.0)


def _views_of(model: MlpModel, out=None):
    """CPU tensors, one per state-dict key of ``model`` (shapes of cgl_gan_param_tensor)."""
    out = {} if out is None else out
    for l in range(model.n_layers):
        fo, fi = model.dims[l + 1], model.dims[l]
        out.setdefault(model.linear_keys[l] + ".weight", torch.zeros(fo, fi))
        out.setdefault(model.linear_keys[l] + ".bias", torch.zeros(fo))
        if model.bn[l]:
            out.setdefault(model.bn_keys[l] + ".weight", torch.zeros(fo))
            out.setdefault(model.bn_keys[l] + ".bias", torch.zeros(fo))
    return out


def _trunk_and_heads(n_heads, img_dim, z_dim):
    from .specs import MIXGEN_HEAD_LAYER, mixgen_worker
    trunk = mixgen_worker(0, img_dim, z_dim)
    cut = MIXGEN_HEAD_LAYER
    t = MlpModel("mixgen_trunk", trunk.dims[:cut + 1], trunk.bn[:cut], trunk.linear_keys[:cut], trunk.bn_keys[:cut])
    heads = []
    for h in range(n_heads):
        w = mixgen_worker(h, img_dim, z_dim)
        heads.append(MlpModel(f"mixgen_head{h}", w.dims[cut:], w.bn[cut:], w.linear_keys[cut:], w.bn_keys[cut:]))
    return t, heads


def _draw_default(model: MlpModel):
    v = _views_of(model)
    default_init(model, v)
    return v


def _draw_mixgen(n_heads, img_dim, z_dim):
    trunk, heads = _trunk_and_heads(n_heads, img_dim, z_dim)
    g = _views_of(trunk)
    for h in heads:
        _views_of(h, g)
    default_init(trunk, g)
    for h in heads:
        default_init(h, g)
    weights_init(trunk, g)
    for h in heads:
        weights_init(h, g)
    return g


def _draw_d(img_dim, sigmoid=False, reinit=False):
    from .specs import mnist_discriminator
    dm = mnist_discriminator(img_dim, sigmoid)
    d = _views_of(dm)
    default_init(dm, d)
    if reinit:
        weights_init(dm, d)
    return d


def topology_state(algo: str, num_servers: int, num_workers: int, seed: int = 20211212, img_dim: int = 784,
                   z_dim: int = 100):
    """Initial parameters of a whole driver topology, drawn once from ``torch.manual_seed(seed)``: every
    server's generator (capgan.py:156 ``Generator(ims)`` / mixed-gan.py:180-181 ``MixGenerator(ims, H)
    .apply(weights_init)`` with H = num_workers // num_servers heads), servers in rank order, then every
    worker's discriminator (capgan.py:309 default init; mixed-gan.py:347-348 ``.apply(weights_init)``;
    the Sigmoid D for MD-GAN).  The reference constructs these inside its Server / Worker threads, servers
    started first (capgan.py:521-525), so this is its order with the thread interleaving fixed; with one
    server it equals ``capgan_state`` / ``mixgen_state``.  Returns ``([G params per server], [D params per
    worker])`` keyed by the reference's state-dict keys."""
    from .specs import mnist_generator
    if algo not in ("capgan", "mixg", "mdgan"):
        raise ValueError(algo)
    if num_workers % num_servers:
        raise ValueError("num_workers must be a multiple of num_servers")
    torch.manual_seed(seed)
    heads = num_workers // num_servers
    if algo == "mixg":
        gs = [_draw_mixgen(heads, img_dim, z_dim) for _ in range(num_servers)]
    else:
        gs = [_draw_default(mnist_generator(img_dim, z_dim)) for _ in range(num_servers)]
    ds = [_draw_d(img_dim, sigmoid=(algo == "mdgan"), reinit=(algo == "mixg")) for _ in range(num_workers)]
    return gs, ds


def capgan_state(n_workers: int = 1, seed: int = 20211212, sigmoid: bool = False, img_dim: int = 784,
                 z_dim: int = 100):
    """``torch.manual_seed(seed); net_g = Generator(ims)`` then one ``Discriminator(ims)`` per worker
    with torch's default init (capgan.py:28,156,309; MDGAN/MNIST/mdgan.py for ``sigmoid``), drawn from
    the global CPU generator in construction order.  Returns ``(G params, [D params])`` keyed by the
    reference's state-dict keys (BatchNorm buffers start at 0 / 1, which ``GanStep.reset`` sets)."""
    from .specs import mnist_discriminator, mnist_generator
    torch.manual_seed(seed)
    gm = mnist_generator(img_dim, z_dim)
    g = _views_of(gm)
    default_init(gm, g)
    ds = []
    for _ in range(n_workers):
        dm = mnist_discriminator(img_dim, sigmoid)
        d = _views_of(dm)
        default_init(dm, d)
        ds.append(d)
    return g, ds


def mixgen_state(n_heads: int, seed: int = 20211212, img_dim: int = 784, z_dim: int = 100,
                 n_discriminators: int = 0):
    """``torch.manual_seed(seed); net_g = MixGenerator(ims, N); net_g.apply(weights_init)``
    (mixed-gan.py:34,180-181; model/mnist_model.py:32-56): the full generator (trunk ``model.*`` +
    every head ``paths.h.*``) with the reference's draw order -- nn.Linear's default draws at
    construction (trunk layers, then head 0, 1, ...), then weights_init's draws in Module.apply's
    post-order, which visits the same layers in the same order.  With ``n_discriminators`` > 0 the
    workers' ``Discriminator(ims).apply(weights_init)`` (mixed-gan.py:347-348) follow, each default-
    constructed then re-initialised.  Returns ``(G params, [D params])``; a worker's ``mixgen_worker(h)``
    step loads the trunk and its own head from the G dict."""
    from .specs import mnist_discriminator
    torch.manual_seed(seed)
    trunk, heads = _trunk_and_heads(n_heads, img_dim, z_dim)
    g = _views_of(trunk)
    for h in heads:
        _views_of(h, g)
    default_init(trunk, g)
    for h in heads:
        default_init(h, g)
    weights_init(trunk, g)
    for h in heads:
        weights_init(h, g)
    ds = []
    for _ in range(n_discriminators):
        dm = mnist_discriminator(img_dim)
        d = _views_of(dm)
        default_init(dm, d)
        weights_init(dm, d)
        ds.append(d)
    return g, ds
