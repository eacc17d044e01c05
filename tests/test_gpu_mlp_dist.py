"""WorkerExchange (the MLP round's cross-worker exchange) over a real process group with its E-share
all-reduce and D-swap on a side stream, concurrent with phase B: two processes on the box's GPU,
one CAPGAN worker (cglgan.GanStep, B=64) each, both exchange forms (gathered / reduce), gloo on host-staged
copies of the device tensors
(one GPU: RCCL needs one per rank), E-share every round and a D-swap every second round; compared
BITWISE with the same two workers in one process through LocalComm (with two ranks a + b == b + a
exactly, and the side stream must change nothing but the overlap)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
B, ROUNDS = 64, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(rank, world):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
    g = torch.Generator().manual_seed(100 + rank)
    real = (torch.rand(8 * B, 784, generator=g) * 2 - 1).cuda()
    st = GanStep(gm, dm, batch=B, loss="ce", weighting="capgan", n_workers=world, rank=rank, gen_z=True,
                 real=real, sample_n=real.shape[0], seed=77)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(555 + rank)
    default_init(dm, st.d_views)
    st.reset()
    return st


class HostComm:
    """DistComm's collectives over gloo on host copies of the device tensors (current stream)."""

    def __init__(self):
        from cglgan.exchange import DistComm
        self.inner = DistComm()
        self.rank, self.size = self.inner.rank, self.inner.size

    def all_gather(self, out, inp):
        h = [torch.empty_like(inp.cpu()) for _ in range(self.size)]
        dist.all_gather(h, inp.detach().cpu())
        out.copy_(torch.cat(h).to(out.device))

    def all_reduce_sum(self, t):
        h = t.detach().cpu()
        self.inner.all_reduce_sum(h)
        t.copy_(h.to(t.device))

    def all_reduce_mean(self, t, weights=None):
        h = t.detach().cpu()
        self.inner.all_reduce_mean(h, weights)
        t.copy_(h.to(t.device))

    def swap(self, tensors, perm):
        hs = [t.detach().cpu() for t in tensors]
        self.inner.swap(hs, perm)
        for t, h in zip(tensors, hs):
            t.copy_(h.to(t.device))


def _proc(rank, world, port, outdir, exchange, side):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cglgan.exchange import WorkerExchange
        torch.cuda.set_device(0)
        st = _make(rank, world)
        ex = WorkerExchange(st, HostComm(), share_every=1, swap_every=2, exchange=exchange)
        ex.d_side = side
        for r in range(ROUNDS):
            ex.round(r, graph=True)
        torch.cuda.synchronize()
        torch.save({"g": st.g_params.cpu(), "d": st.d_params.cpu(), "side": getattr(ex, "_side", None) is not None},
                   os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


# "gather": one all_gather of [gradient | loss] slots, alpha + the rank-ordered sum at phase B's head (on
# device); "reduce": loss all_gather, alpha_scale, gradient all_reduce.  Both bitwise LocalComm's round.
# side: D's exchange on a side stream beside phase B (CGL_DX_SIDE=1) or after it on the main stream (default)
@pytest.mark.parametrize("exchange,side", [("gather", False), ("reduce", False), ("gather", True)])
def test_worker_exchange_side_stream_matches_local(exchange, side):
    world = 2
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_proc, args=(world, _free_port(), td, exchange, side), nprocs=world, join=True)
        res = [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(world)]
    from cglgan.exchange import LocalComm
    steps = [_make(r, world) for r in range(world)]
    comm = LocalComm(steps, share_every=1, swap_every=2)
    for r in range(ROUNDS):
        comm.round(r, graph=True)
    torch.cuda.synchronize()
    for i, s in enumerate(steps):
        assert res[i]["side"] == side
        assert torch.equal(res[i]["g"], s.g_params.cpu()), i
        assert torch.equal(res[i]["d"], s.d_params.cpu()), i
    assert torch.equal(res[0]["g"], res[1]["g"])     # replicated G
