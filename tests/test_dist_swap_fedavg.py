"""Multi-process (gloo, CPU) tests of the remaining exchange collectives of cglgan.exchange:

* D-swap (MD-GAN, MDGAN/MNIST/mdgan.py:122-123,158-164, commented out in the reference -- parity
  unpinned): every rank ends with the discriminator of rank perm[rank], perm drawn by the
  server's Random(server + 100).shuffle, identical on every rank without communication;
* Cloud FedAvg across server groups (mixed-gan.py:104-124, 193-200): the trunk (parameters and
  BatchNorm running statistics) becomes sum_s A_s p_s, A_s = data_len_s / sum -- compared with the
  oracle's restatement oracle.gan_oracle.fedavg; with fedavg_compat_noop the reference's actual
  behaviour (its load_state_dict ignores every key) leaves the trunk untouched.
"""
import os
import random
import socket
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gan_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _swap_worker(rank, world, port, outdir):
    _init(rank, world, port)
    try:
        from cglgan.exchange import DistComm, DSwap
        comm, ds = DistComm(), DSwap(world)
        d = torch.full((1000,), float(rank))
        run = torch.full((7,), 10.0 + rank)
        perms = []
        for _ in range(3):
            p = ds.next_perm()
            perms.append(p)
            comm.swap([d, run], p)
        torch.save({"d": d, "run": run, "perms": perms}, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_d_swap_three_ranks():
    world = 3
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_swap_worker, args=(world, _free_port(), td), nprocs=world, join=True)
        res = [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(world)]
    rd = random.Random()
    rd.seed(100)            # the single server's generator, mdgan.py:122-123
    owner = list(range(world))
    for it in range(3):
        p = list(range(world))
        rd.shuffle(p)
        assert all(r["perms"][it] == p for r in res)
        owner = [owner[p[i]] for i in range(world)]   # worker i continues with D_{perm[i]}
    for r in range(world):
        assert torch.equal(res[r]["d"], torch.full((1000,), float(owner[r])))
        assert torch.equal(res[r]["run"], torch.full((7,), 10.0 + owner[r]))


class _TrunkStep:
    """The surface WorkerExchange.cloud_average uses: g_params / g_running with trunk prefixes."""

    def __init__(self, sd, trunk_keys, running_keys):
        self.g_params = torch.cat([sd[k].flatten() for k in trunk_keys]).clone()
        self.g_running = torch.cat([sd[k].flatten() for k in running_keys]).clone()
        self.n_workers = 1

    def trunk_slices(self):
        return self.g_params, self.g_running

    def run(self, *a, **k):
        pass


def _fedavg_worker(rank, world, port, outdir, sizes, noop):
    _init(rank, world, port)
    try:
        from cglgan.exchange import DistComm, WorkerExchange
        G, _ = O.build_mixg(2, seed=100 + rank)     # each server: its own Mix-G (different init)
        sd = G.state_dict()
        tk = [k for k in sd if k.startswith("model.") and ("weight" in k or "bias" in k)]
        rk = [k for k in sd if k.startswith("model.") and "running" in k]
        step = _TrunkStep(sd, tk, rk)
        A = [s / sum(sizes) for s in sizes]
        ex = WorkerExchange(step, None, cloud=DistComm(), cloud_every=1, cloud_weights=A, fedavg_compat_noop=noop)
        ex.round(0)
        torch.save({"p": step.g_params, "r": step.g_running, "sd": {k: sd[k].detach() for k in tk + rk}},
                   os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _run_fedavg(noop):
    world, sizes = 2, [300, 100]
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_fedavg_worker, args=(world, _free_port(), td, sizes, noop), nprocs=world, join=True)
        return [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(world)], sizes


def test_cloud_fedavg_weighted_trunk():
    res, sizes = _run_fedavg(False)
    ref = O.fedavg([r["sd"] for r in res], sizes)
    keys = list(res[0]["sd"])
    tk = [k for k in keys if "running" not in k]
    rk = [k for k in keys if "running" in k]
    exp_p = torch.cat([ref[k].flatten() for k in tk])
    exp_r = torch.cat([ref[k].flatten() for k in rk])
    for r in res:
        assert torch.allclose(r["p"], exp_p, rtol=1e-6, atol=1e-7)
        assert torch.allclose(r["r"], exp_r, rtol=1e-6, atol=1e-7)
    assert torch.equal(res[0]["p"], res[1]["p"])


def test_cloud_fedavg_compat_noop():
    res, _ = _run_fedavg(True)
    for r in res:
        tk = [k for k in r["sd"] if "running" not in k]
        assert torch.equal(r["p"], torch.cat([r["sd"][k].flatten() for k in tk]))


class _GStep:
    """CAPGAN server surface: every G parameter in one flat buffer (fedlab serialize_model order)."""

    def __init__(self, G):
        self.g_params = torch.cat([p.detach().flatten() for p in G.parameters()]).clone()
        self.n_workers = 1

    def run(self, *a, **k):
        pass


def _capgan_cloud_worker(rank, world, port, outdir, sizes, segema):
    _init(rank, world, port)
    try:
        from cglgan.exchange import DistComm, WorkerExchange, capgan_cloud_due
        G, _ = O.build_capgan(1, seed=300 + rank)
        step = _GStep(G)
        own = step.g_params.clone()
        A = [s / sum(sizes) for s in sizes]
        due = capgan_cloud_due(20, 400.0, 1, 100)    # period 4 rounds: fires before r = 0, 4, 8, ...
        ex = WorkerExchange(step, None, cloud=DistComm(), cloud_weights=A, cloud_scope="all", segema=segema,
                            cloud_due=due)
        fired = []
        for r in range(3):
            before = step.g_params.clone()
            ex.round(r)
            fired.append(not torch.equal(before, step.g_params))
        torch.save({"p": step.g_params, "own": own, "fired": fired}, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_capgan_cloud_fedavg_all_params_segema():
    """capgan.py:169-175: fedavg_aggregate of every G parameter (data-size weights), mixed with segema,
    before the rounds where t % (data_len * cloud_epoch / batch_size) == 0."""
    world, sizes, segema = 2, [300, 100], 0.25
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_capgan_cloud_worker, args=(world, _free_port(), td, sizes, segema), nprocs=world, join=True)
        res = [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(world)]
    w = torch.tensor(sizes, dtype=torch.float32)
    w = w / w.sum()
    avg = res[0]["own"] * w[0] + res[1]["own"] * w[1]
    for r in res:
        assert r["fired"] == [True, False, False]
        exp = segema * r["own"] + (1 - segema) * avg
        assert torch.allclose(r["p"], exp, rtol=1e-6, atol=1e-7)
