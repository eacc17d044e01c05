"""cglgan.checkpoint: the drivers' checkpoint files (capgan.py:185-200) -- a generator state dict under
the reference's keys that round-trips into the drop-in modules, and the 7-tuple config pickle."""
import pickle

import torch

from cglgan import checkpoint as CK
from cglgan import specs
from cglgan.conv_step import LSGAN_G, tensor_shapes


class _Step:
    """A fused step's surface: g_state_dict() with reference keys (values as a round would leave them)."""

    def __init__(self, keys_shapes):
        g = torch.Generator().manual_seed(0)
        self.sd = {k: torch.randn(*s, generator=g) for k, s in keys_shapes}

    def g_state_dict(self):
        return self.sd


def test_generator_pt_roundtrip(tmp_path):
    from cglgan.model import Generator
    ref = Generator((1, 28, 28))
    step = _Step([(k, v.shape) for k, v in ref.state_dict().items() if v.dim() > 0])
    step.sd = {k: (step.sd[k] if v.dim() > 0 else v) for k, v in ref.state_dict().items()}
    pt, cfg = CK.save_server(step, str(tmp_path), "Server1", [0, 1], torch.tensor([0.25, 0.75]), [0.0001],
                             [torch.zeros(3, 2)], [0], [0])
    sd = CK.load_generator(pt)
    assert list(sd) == list(ref.state_dict())
    g2 = Generator((1, 28, 28))
    g2.load_state_dict(sd, strict=True)
    for k, v in g2.state_dict().items():
        assert torch.equal(v, step.sd[k])
    with open(cfg, "rb") as f:     # our own file
        tup = pickle.load(f)
    assert len(tup) == 7 and tup[0] == [0, 1] and torch.equal(tup[1], torch.tensor([0.25, 0.75])) and tup[3] == []


def test_conv_generator_keys(tmp_path):
    keys = [(k, s) for k, s, _ in tensor_shapes(LSGAN_G)]
    step = _Step(keys)
    pt, _ = CK.save_server(step, str(tmp_path), "Server1", [0], [1.0])
    assert [k for k, _ in keys] == list(CK.load_generator(pt))
