"""Constructor API of the CGLGAN drop-in modules (CPU: construction only, no compute).

INTEGRATION.md's CGLGAN section: `cglgan.cglgan_2dmg.Discriminator` keeps the reference's signature
`__init__(self, ns=1)` (/root/reference/CGLGAN/2DMG/model.py:56), so the reference driver's own call
`Discriminator(ims, N)` (CGLGAN/2DMG/main.py:335) raises TypeError exactly as it does against the
reference class; `Discriminator(N)` / `Discriminator()` are the working calls.  The MNIST variant takes
`(img_shape, ns=1)` (CGLGAN/MNIST/mnist_model.py:69)."""
import pytest

from cglgan import cglgan_2dmg, cglgan_mnist


def test_2dmg_discriminator_signature():
    with pytest.raises(TypeError):
        cglgan_2dmg.Discriminator((2,), 4)
    for d in (cglgan_2dmg.Discriminator(4), cglgan_2dmg.Discriminator()):
        assert [k for k in d.state_dict()] == ["model.0.weight", "model.0.bias", "model.2.weight", "model.2.bias",
                                               "model.4.weight", "model.4.bias"]


def test_mnist_discriminator_signature():
    d = cglgan_mnist.Discriminator((1, 28, 28), 4)
    assert d.model[0].weight.shape == (512, 784)
    assert cglgan_mnist.Discriminator((1, 28, 28)).model[4].weight.shape == (1, 256)
