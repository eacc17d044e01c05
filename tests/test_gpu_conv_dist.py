"""ConvWorkerExchange over a real process group: two processes, one conv-GAN worker each
(cglgan.conv_step.ConvGanStep on cuda:0), gloo collectives on host-staged copies of the device
tensors (the box has one GPU; RCCL needs one GPU per rank), run through every exchange step the
multi-GPU bench uses -- the G-loss all-gather, the alpha weighting on device, the image-gradient
all-reduce, the E-share of D's parameters and BatchNorm running statistics, and the D-swap of both
-- and compared BITWISE with the same two workers in one process through ConvLocalComm (sums in rank
order; with two ranks a + b == b + a exactly)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
B = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reals(rank, r):
    g = torch.Generator().manual_seed(1000 * rank + r)
    return torch.rand(B, 1, 32, 32, generator=g) * 2 - 1


def _data(rank):
    g = torch.Generator().manual_seed(500 + rank)
    return (torch.rand(4 * B + 3, 1024, generator=g) * 2 - 1).cuda()


def _make(rank, world, graph=False):
    """graph=True: the worker draws its real batches on the device from its own shard, so rounds after the
    first replay phase A / phase B as hipGraphs (ConvGanStep.round_a / round_b)."""
    from cglgan.conv_step import ConvGanStep
    st = ConvGanStep(B, loss="mse", seed=77, n_workers=world, rank=rank, data=_data(rank) if graph else None,
                     graph=graph)
    st.init_default(20211212, 20211213 + rank)
    return st


class HostComm:
    """DistComm's collectives over gloo on host copies of the device tensors."""

    def __init__(self):
        from cglgan.exchange import DistComm
        self.inner = DistComm()
        self.rank, self.size = self.inner.rank, self.inner.size

    def _do(self, fn, *ts):
        hs = [t.detach().cpu() for t in ts]
        fn(*hs)
        ts[0].copy_(hs[0].to(ts[0].device))

    def all_gather(self, out, inp):
        h = [torch.empty_like(inp.cpu()) for _ in range(self.size)]
        dist.all_gather(h, inp.detach().cpu())
        out.copy_(torch.cat(h).to(out.device))

    def all_reduce_sum(self, t):
        self._do(self.inner.all_reduce_sum, t)

    def all_reduce_mean(self, t, weights=None):
        self._do(lambda x: self.inner.all_reduce_mean(x, weights), t)

    def swap(self, tensors, perm):
        hs = [t.detach().cpu() for t in tensors]
        self.inner.swap(hs, perm)
        for t, h in zip(tensors, hs):
            t.copy_(h.to(t.device))


def _proc(rank, world, port, outdir, rounds, graph=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cglgan.exchange import ConvWorkerExchange
        torch.cuda.set_device(0)
        st = _make(rank, world, graph)
        ex = ConvWorkerExchange(st, HostComm(), share_every=1, swap_every=2)
        for r in range(rounds):
            ex.round(r, real=None if graph else _reals(rank, r).cuda())
        torch.cuda.synchronize()
        torch.save({"g": st.G.p.cpu(), "d": st.D.p.cpu(), "run": [v.cpu() for v in st.D.running.values()],
                    "grun": [v.cpu() for v in st.G.running.values()], "lbuf": st.lbuf.cpu()},
                   os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("graph", [False, True])
def test_conv_worker_exchange_distcomm_matches_local(graph):
    """graph=True: the two processes replay phase A / phase B as hipGraphs (rounds 1..3) around the eager
    collectives and the side-stream D exchange; the in-process reference issues every round op by op."""
    world, rounds = 2, (4 if graph else 2)
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_proc, args=(world, _free_port(), td, rounds, graph), nprocs=world, join=True)
        res = [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(world)]
    from cglgan.exchange import ConvLocalComm, DSwap
    steps = [_make(r, world, graph) for r in range(world)]
    comm, dsw = ConvLocalComm(steps), DSwap(world)
    for r in range(rounds):
        comm.round(r, reals=None if graph else [_reals(i, r).cuda() for i in range(world)], share_every=1,
                   eager=True)
        if (r + 1) % 2 == 0:           # ConvWorkerExchange's D-swap: parameters + running statistics
            perm = dsw.next_perm()
            old = [[s.D.p.clone()] + [v.clone() for v in s.D.running.values()] for s in steps]
            for i, s in enumerate(steps):
                for t, src in zip([s.D.p] + list(s.D.running.values()), old[perm[i]]):
                    t.copy_(src)
    torch.cuda.synchronize()
    for i, s in enumerate(steps):
        assert torch.equal(res[i]["g"], s.G.p.cpu()), i
        assert torch.equal(res[i]["d"], s.D.p.cpu()), i
        assert all(torch.equal(a, b.cpu()) for a, b in zip(res[i]["run"], s.D.running.values())), i
        assert all(torch.equal(a, b.cpu()) for a, b in zip(res[i]["grun"], s.G.running.values())), i
        assert torch.equal(res[i]["lbuf"], s.lbuf.cpu()), i
    assert torch.equal(res[0]["g"], res[1]["g"])     # replicated G
