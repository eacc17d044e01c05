"""The driver layer (cglgan.driver) run multi-process over gloo on CPU, one process
per worker, with the oracle stand-in for the fused round (tests/dist_oracle_step.py), against a
single-process run of the reference's roles (oracle MixgServer / CapganServer + Workers + Cloud FedAvg).

* Mix-G, num_workers=4, num_servers=2 (BASELINE config 4's topology at world size 4): two server groups
  built with dist.new_group (capgan.py:509-516 block assignment), the trunk gradient all-reduced inside
  each group, the Cloud's A_s-weighted trunk FedAvg (parameters + BatchNorm running statistics) over
  the world before every round (mixed-gan.py:104-124, 193-200, cloud_epoch = 1), and the D-swap inside
  each group every 2 rounds (server s's Random(s + 100), MDGAN/MNIST/mdgan.py:122-123,158-164) --
  cloud_due and swap_every together in one WorkerExchange.
* CAPGAN, num_workers=2, one server, E-share of D every round.
"""
import os
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


def _cfg(**kw):
    from cglgan.driver import DriverConfig
    base = dict(batch_size=16, dataset_rows=1500, num_sample=100, num_class=10, num_communication=3, iid=1,
                graph=False)
    base.update(kw)
    return DriverConfig(**base)


def _proc(rank, world, port, outdir, kw, rounds):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cglgan.driver import Driver
        from dist_oracle_step import oracle_step_factory
        drv = Driver(_cfg(**kw), step_factory=oracle_step_factory, device="cpu")
        drv.run(rounds, log=None)
        s = drv.step
        torch.save({"g": s.g_params, "r": s.g_running, "d": s.d_params, "server": drv.topo.server,
                    "local": drv.topo.local, "members": drv.topo.members(), "stats": s.stats()},
                   os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _spawn(world, kw, rounds):
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_proc, args=(world, _free_port(), td, kw, rounds), nprocs=world, join=True)
        return [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(world)]


def _reference(kw, rounds):
    """The single-process reference: every server's role with its workers, the Cloud before each due
    round, D-swap / E-share after the round, on the same inputs as the stand-in."""
    from cglgan.data import beta_weights, cloud_weights
    from cglgan.driver import Topology, make_shards
    from cglgan.exchange import DSwap, mixg_cloud_due
    from cglgan.init import topology_state
    from dist_oracle_step import driver_inputs
    cfg = _cfg(**kw).validate()
    x, shards = make_shards(cfg)
    lens = [len(s) for s in shards]
    H, S = cfg.heads, cfg.num_servers
    gs, ds = topology_state(cfg.algo, S, cfg.num_workers, cfg.seed)
    servers, groups = [], []
    for s in range(S):
        members = Topology(cfg.num_workers, S, s * H).members()
        beta = beta_weights([lens[i] for i in members])[0]
        if cfg.algo == "mixg":
            G = O.MixNet(O.mnist_mixgen_trunk_spec(), [O.mnist_mixgen_head_spec(h) for h in range(H)])
            srv = O.MixgServer(G, beta, weighting=cfg.weighting_)
            nets = [G.trunk] + G.heads
        else:
            G = O.SeqNet(O.mnist_generator_spec())
            srv = O.CapganServer(G, beta)
            nets = [G]
        with torch.no_grad():
            for n in nets:
                for k, v in n.params.items():
                    v.copy_(gs[s][k])
        ws = []
        for i in members:
            w = O.Worker(O.SeqNet(O.mnist_discriminator_spec()), "ce")
            with torch.no_grad():
                for k, v in w.D.params.items():
                    v.copy_(ds[i][k])
            ws.append(w)
        servers.append(srv)
        groups.append((members, ws, DSwap(H, s)))
    A = cloud_weights([sum(lens[i] for i in Topology(cfg.num_workers, S, s * H).members()) for s in range(S)])
    due = mixg_cloud_due(cfg.num_communication, cfg.cloud_epoch)
    for r in range(rounds):
        if S > 1 and due(r):
            avg = O.fedavg([srv.G.trunk.state_dict() for srv in servers], A.tolist())
            with torch.no_grad():
                for srv in servers:
                    for k, v in avg.items():
                        (srv.G.trunk.params if k in srv.G.trunk.params else srv.G.trunk.buffers)[k].copy_(v)
        for s, srv in enumerate(servers):
            members, ws, dsw = groups[s]
            ins = [driver_inputs(cfg, s, i, x[torch.as_tensor(shards[i])], r) for i in members]
            z1, z2 = ins[0][0], ins[0][1]
            if cfg.algo == "mixg":
                srv.round(ws, z1, z2, [i[2] for i in ins])
            else:
                srv.round(ws, z1, z2, [i[2] for i in ins], weighting=cfg.weighting_)
            if cfg.share_every and (r + 1) % cfg.share_every == 0:
                O.eshare_mean(ws)
            if cfg.swap_every and (r + 1) % cfg.swap_every == 0:
                O.dswap(ws, dsw.next_perm())
    return servers, groups


def _flat(ts):
    return torch.cat([t.detach().flatten() for t in ts])


def _close(a, b, what):
    """SURVEY F8 form: the group all-reduce sums the trunk / image gradient in another order than the
    reference's autograd, and Adam turns rounding-level gradient differences of near-zero gradients
    into up to ~lr per step -- so 1e-5 relative in norm, and no element off by half an Adam step."""
    d = (a - b).abs()
    assert float(d.norm()) <= 1e-5 * float(b.norm()) and float(d.max()) <= 1e-4, \
        (what, float(d.norm() / b.norm()), float(d.max()))


def test_driver_mixg_two_servers_cloud_fedavg_dswap_world4():
    kw = dict(algo="mixg", num_workers=4, num_servers=2, cloud_epoch=1, swap_every=2)
    rounds = 3
    res = _spawn(4, kw, rounds)
    servers, groups = _reference(kw, rounds)
    for r in res:
        assert r["members"] == [2 * r["server"], 2 * r["server"] + 1]
    for s, srv in enumerate(servers):
        members, ws, _ = groups[s]
        for h, rank in enumerate(members):
            got = res[rank]
            trunk, head = srv.G.trunk, srv.G.heads[h]
            _close(got["g"], _flat(list(trunk.params.values()) + list(head.params.values())), ("G", rank))
            run = [b for k, b in list(trunk.buffers.items()) + list(head.buffers.items()) if "running" in k]
            _close(got["r"], _flat(run), ("running", rank))
            _close(got["d"], _flat(ws[h].D.params.values()), ("D", rank))
    # one trunk everywhere after the Cloud (every round here); replicas of a server's trunk identical
    ntr = sum(p.numel() for p in servers[0].G.trunk.params.values())
    assert torch.equal(res[0]["g"][:ntr], res[1]["g"][:ntr]) and torch.equal(res[2]["g"][:ntr], res[3]["g"][:ntr])


def test_driver_capgan_eshare_world2():
    kw = dict(algo="capgan", num_workers=2, num_servers=1, share_every=1, iid=0)
    rounds = 2
    res = _spawn(2, kw, rounds)
    servers, groups = _reference(kw, rounds)
    srv, (members, ws, _) = servers[0], groups[0]
    for rank in members:
        _close(res[rank]["g"], _flat(srv.G.params.values()), ("G", rank))
        _close(res[rank]["d"], _flat(ws[rank].D.params.values()), ("D", rank))
    assert torch.equal(res[0]["d"], res[1]["d"])          # E-share: one D
    assert torch.equal(res[0]["g"], res[1]["g"])          # replicated G


def test_driver_config_knobs_and_cli():
    """The reference's module-level knobs (names, defaults) and -c / -s flags."""
    import cglgan.driver as D
    cfg = D.DriverConfig.from_module()
    assert (cfg.num_workers, cfg.num_servers, cfg.epoch, cfg.batch_size, cfg.num_communication) == (10, 1, 1, 100, 20000)
    assert (cfg.cloud_epoch, cfg.segema, cfg.iid, cfg.num_class, cfg.num_sample) == (1, 0.0, 0, 10, 1000)
    assert (cfg.b1, cfg.b2, cfg.seed) == (0.5, 0.999, 20211212)
    old = D.num_workers
    try:
        D.num_workers = 8
        assert D.DriverConfig.from_module().num_workers == 8
    finally:
        D.num_workers = old
    a = D.parse_args(["-c", "3", "-s", "0.5", "--algo", "mixg", "--num_workers", "8", "--num_servers", "2"])
    assert (a.cloud_epoch, a.segema, a.algo, a.num_workers, a.num_servers) == (3, 0.5, "mixg", 8, 2)
    t = D.Topology(8, 2, 5)
    assert (t.server, t.local, t.members()) == (1, 1, [4, 5, 6, 7])
    import pytest
    with pytest.raises(ValueError):
        D.DriverConfig(num_workers=10, num_servers=3).validate()


def test_capgan_multi_server_cloud_schedule():
    """capgan servers with different shard totals sync on different rounds (capgan.py:169);
    the world all-reduce Cloud refuses such a run instead of pairing mismatched rounds (or hanging)."""
    import pytest

    from cglgan.driver import capgan_cloud_schedule
    cfg = _cfg(algo="capgan", num_workers=4, num_servers=2, num_communication=40, batch_size=10, cloud_epoch=1)
    due = capgan_cloud_schedule(cfg, [100.0, 100.0], 1)        # period 10: rounds with t % 10 == 0
    assert [r for r in range(40) if due(r)] == [0, 10, 20, 30]
    with pytest.raises(ValueError, match="periods"):
        capgan_cloud_schedule(cfg, [100.0, 150.0], 0)
    # different totals whose schedules coincide over the run are accepted (both never fire)
    due = capgan_cloud_schedule(cfg, [1001.0, 1003.0], 0)
    assert not any(due(r) for r in range(40))
