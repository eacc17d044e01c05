"""Product initialisation pinned bit-for-bit against the reference's own modules (CPU).

tests/golden/golden_steps.json ``init`` holds the sha256 of every tensor of
  * ``capgan_G`` / ``capgan_D``: ``torch.manual_seed(20211212); Generator(ims); Discriminator(ims)``
    (capgan.py:28,156,309 -- torch's default nn.Linear init), made by make_golden.py with the
    reference's model/mnist_model.py;
  * ``mixg2_G``: ``torch.manual_seed(20211212); MixGenerator(ims, 2).apply(weights_init)``
    (mixed-gan.py:68-77,180-181).
The draws are RNG streams, not reductions, so the match must be exact on every host.
"""
import torch

from cglgan import specs
from cglgan.init import capgan_state, default_init, mixgen_state, _views_of
from golden_replay import load_golden, sha


def _same(summary, params):
    checked = 0
    for k, ent in summary.items():
        if "sha256" not in ent or k not in params:
            assert k.endswith(("running_mean", "running_var", "num_batches_tracked")) or k in params, k
            continue
        v = params[k]
        assert list(v.shape) == ent["shape"], k
        assert sha(v) == ent["sha256"], k
        checked += 1
    return checked


def test_default_init_is_the_reference_generator_and_discriminator():
    g = load_golden()["init"]
    torch.manual_seed(20211212)                       # capgan.py:28
    gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
    gv, dv = _views_of(gm), _views_of(dm)
    default_init(gm, gv)                              # Server: Generator(ims)      (:156)
    default_init(dm, dv)                              # Worker: Discriminator(ims)  (:309)
    assert _same(g["capgan_G"], gv) == 16
    assert _same(g["capgan_D"], dv) == 6
    G, Ds = capgan_state(1)
    assert _same(g["capgan_G"], G) == 16 and _same(g["capgan_D"], Ds[0]) == 6


def test_mixgen_weights_init_draw_order():
    g = load_golden()["init"]["mixg2_G"]
    G, _ = mixgen_state(2)
    assert _same(g, G) == len([k for k in g if "sha256" in g[k] and not k.endswith(("running_mean", "running_var"))])
    # every worker's slice (trunk + its own head) is a view of the same draw
    for h in range(2):
        keys = specs.mixgen_worker(h).tensor_keys()
        assert all(k in G for k in keys)
