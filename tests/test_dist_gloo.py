"""Multi-process exchange (world_size 2, gloo, CPU): cglgan.exchange.WorkerExchange drives one
worker per process through phase A -> all_gather(losses) -> alpha -> all_reduce(gradient) ->
phase B (+ E-share of D), and must reproduce the single-process oracle round in which the
reference's Server backpropagates F_max through every worker's D (capgan.py:211-262, 316-349).

The per-worker compute is the oracle stand-in (tests/dist_oracle_step.py); what is under test
is the host-side exchange logic and its collectives, SURVEY 8e.  Both sides run in float64 so
that the only difference -- the order in which the N gradient contributions are summed -- stays
at 1e-12 relative (in fp32 the analytically-zero gradients of the Linear biases that feed
BatchNorm are pure rounding noise, which Adam amplifies to ~lr per step).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gan_oracle as O

N, B, ROUNDS = 2, 32, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(r):
    z1, z2, reals = O.synthetic_inputs(B, N, 1, seed=300 + r)
    return z1, z2, [rs[0] for rs in reals]


def _worker(rank, port, outdir, kind, share_every, exchange):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    torch.set_default_dtype(torch.float64)
    dist.init_process_group("gloo", rank=rank, world_size=N)
    try:
        from cglgan.exchange import DistComm, WorkerExchange
        from dist_oracle_step import OracleWorkerStep
        loss, weighting = ("ce", "capgan") if kind == "capgan" else ("bce", "mean")
        step = OracleWorkerStep(N, rank, loss=loss, weighting=weighting)
        ex = WorkerExchange(step, DistComm(), share_every=share_every, exchange=exchange)
        Fs = []
        for r in range(ROUNDS):
            z1, z2, reals = _inputs(r)
            step.set_inputs(z1, z2, reals[rank])
            ex.round(r)
            Fs.append(step.F)
        torch.save({"g": step.g_params(), "d": step.d_params, "F": Fs, "losses": step.losses_all.clone()},
                   os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _reference(kind, share_every):
    """Single process: all workers on one 'device', F_max backpropagated through every D."""
    torch.set_num_threads(1)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return _reference64(kind, share_every)
    finally:
        torch.set_default_dtype(prev)


def _reference64(kind, share_every):
    loss = "ce" if kind == "capgan" else "bce"
    G, workers = O.build_capgan(N, loss=loss)
    srv = O.CapganServer(G, torch.full((N,), 1.0 / N))
    Fs = []
    for r in range(ROUNDS):
        z1, z2, reals = _inputs(r)
        out = srv.round(workers, z1, z2, [[x] for x in reals], weighting="capgan" if kind == "capgan" else "mean")
        Fs.append(float(out["F"]))
        if share_every > 0 and (r + 1) % share_every == 0:   # E-share: D <- mean over workers (a19)
            with torch.no_grad():
                for k in workers[0].D.params:
                    m = sum(w.D.params[k] for w in workers) / N
                    for w in workers:
                        w.D.params[k].copy_(m)
    return G, workers, Fs


def _rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


# exchange: "reduce" = loss all_gather, alpha, gradient all_reduce; "gather" = one all_gather of [gradient | loss]
# slots, alpha and the rank-ordered weighted sum at the start of phase B (cglgan.exchange module docstring)
@pytest.mark.parametrize("kind,share_every,exchange", [("capgan", 0, "reduce"), ("capgan", 0, "gather"),
                                                       ("capgan", 1, "gather"), ("mdgan", 2, "reduce"),
                                                       ("mdgan", 2, "gather")])
def test_two_worker_exchange_matches_oracle(kind, share_every, exchange):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(port, d, kind, share_every, exchange), nprocs=N, join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(N)]
    G, workers, Fs = _reference(kind, share_every)
    # replicated G: bitwise identical on both ranks
    for k in res[0]["g"]:
        assert torch.equal(res[0]["g"][k], res[1]["g"][k]), k
    # and equal to the single-process round up to the summation order of the contributions
    for k, v in G.params.items():
        assert _rel(res[0]["g"][k], v.detach()) < 1e-10, k
    for r in range(N):
        ref = torch.cat([workers[r].D.params[k].detach().flatten() for k in workers[r].D.params])
        assert _rel(res[r]["d"], ref) < 1e-10
    for a, b in zip(res[0]["F"], Fs):
        assert abs(a - b) <= 1e-10 * max(abs(b), 1e-3)
    if share_every == 1:
        assert torch.equal(res[0]["d"], res[1]["d"])
