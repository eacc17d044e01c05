"""The N > 1 conv round (model/lsgan.py workers through ConvLocalComm: phase A, G-loss gather, lambda
weighting, image-gradient sum, phase B) with phase A and phase B replayed as hipGraphs
(ConvGanStep(graph=True).round_a / round_b) is bitwise the same rounds issued op by op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _steps(N, B, weighting, graph=True):
    from cglgan.conv_step import ConvGanStep
    out = []
    for r in range(N):
        g = torch.Generator().manual_seed(40 + r)
        data = (torch.rand(3 * B + 5, 1024, generator=g) * 2 - 1).cuda()
        s = ConvGanStep(B, loss="mse", seed=11, n_workers=N, rank=r, weighting=weighting, data=data, graph=graph)
        s.init_default(20211212, 20211213 + r)
        out.append(s)
    return out


@pytest.mark.parametrize("weighting", ["capgan", "mean"])
@pytest.mark.parametrize("B", [8, 64])
def test_split_round_graph_equals_eager(weighting, B):
    from cglgan.exchange import ConvLocalComm
    N, rounds = 2, 5
    sg, se = _steps(N, B, weighting), _steps(N, B, weighting)
    cg, ce = ConvLocalComm(sg), ConvLocalComm(se)
    for r in range(rounds):
        cg.round(r, share_every=2)
        ce.round(r, share_every=2, eager=True)
    torch.cuda.synchronize()
    assert sg[0]._phase_graphs is not None, "phase graphs never captured"
    for a, b in zip(sg, se):
        assert a.round == b.round == rounds and a.G.step == b.G.step and a.D.step == b.D.step
        assert a.lam == b.lam
        assert torch.equal(a.G.p, b.G.p) and torch.equal(a.D.p, b.D.p)
        assert torch.equal(a.G.m, b.G.m) and torch.equal(a.D.v, b.D.v)
        assert torch.equal(a.lbuf, b.lbuf) and torch.equal(a.dimg, b.dimg)
        assert all(torch.equal(x, y) for x, y in zip(a.D.running.values(), b.D.running.values()))
        assert all(torch.equal(x, y) for x, y in zip(a.G.running.values(), b.G.running.values()))
    assert torch.equal(sg[0].G.p, sg[1].G.p)      # replicated G
