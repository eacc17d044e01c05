"""Model specifications of the reference's MLP GANs, with their state-dict key names.

Each spec is an MLP as the C ABI sees it (``cgl_mlp_spec``: Linear dims + BatchNorm flags) plus
the reference's ``nn.Sequential`` key of every tensor, in the order the flat parameter buffer
stores them (``cgl_gan_param_tensor``).  Keys are identical to the reference modules so a
state dict saved by the reference (``torch.save(net_g.state_dict())`` capgan.py:186) loads
as-is, and vice versa.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class MlpModel:
    name: str
    dims: List[int]
    bn: List[int]
    linear_keys: List[str]                       # prefix of each Linear ("model.0")
    bn_keys: List[Optional[str]] = field(default_factory=list)   # prefix of each layer's BatchNorm

    @property
    def n_layers(self):
        return len(self.dims) - 1

    def tensor_keys(self):
        """Keys in flat-buffer order: per layer W, b, then BN weight, bias (cgl_gan_param_tensor)."""
        out = []
        for l in range(self.n_layers):
            out += [self.linear_keys[l] + ".weight", self.linear_keys[l] + ".bias"]
            if self.bn[l]:
                out += [self.bn_keys[l] + ".weight", self.bn_keys[l] + ".bias"]
        return out

    def bn_layers(self):
        return [l for l in range(self.n_layers) if self.bn[l]]


def mnist_generator(img_dim=784, z_dim=100):
    """``Generator`` model/mnist_model.py:5-29: Sequential indices 0,2(3),5(6),8(9),11."""
    return MlpModel("mnist_generator", [z_dim, 128, 256, 512, 1024, img_dim], [0, 1, 1, 1, 0],
                    ["model.0", "model.2", "model.5", "model.8", "model.11"],
                    [None, "model.3", "model.6", "model.9", None])


def mixgen_worker(head, img_dim=784, z_dim=100):
    """One worker's slice of ``MixGenerator`` model/mnist_model.py:32-66: the shared trunk
    (``model.*``) + its own head ``paths.<head>.*``.  Layers >= 3 are the head."""
    h = f"paths.{head}"
    return MlpModel(f"mixgen_worker{head}", [z_dim, 128, 256, 512, 1024, img_dim], [0, 1, 1, 1, 0],
                    ["model.0", "model.2", "model.5", f"{h}.0", f"{h}.3"],
                    [None, "model.3", "model.6", f"{h}.1", None])


MIXGEN_HEAD_LAYER = 3   # first layer of a Mix-G head (exchange point of the trunk gradient)


def mnist_discriminator(img_dim=784, sigmoid=False):
    """``Discriminator`` model/mnist_model.py:71-88 (2 logits), or the Sigmoid/BCE variant of
    MDGAN/MNIST/mnist_model.py:31-50 and CGLGAN/MNIST/mnist_model.py:69-86."""
    return MlpModel("mnist_discriminator" + ("_sigmoid" if sigmoid else ""), [img_dim, 512, 256, 1 if sigmoid else 2],
                    [0, 0, 0], ["model.0", "model.2", "model.4"], [None, None, None])


def ring_generator(head=0):
    """CGLGAN/2DMG/model.py:26-50 worker slice: trunk Linear(100,32)+LReLU, head Linear(32,2)+Tanh."""
    return MlpModel(f"ring_generator{head}", [100, 32, 2], [0, 0], ["model.0", f"paths.{head}.0"], [None, None])


RING_HEAD_LAYER = 1


def ring_discriminator():
    """CGLGAN/2DMG/model.py:54-71: 2->128->256->1, Sigmoid."""
    return MlpModel("ring_discriminator", [2, 128, 256, 1], [0, 0, 0], ["model.0", "model.2", "model.4"],
                    [None, None, None])
