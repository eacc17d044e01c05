"""BASELINE.json configs 3, 4 and 5 at their stated shape, rehearsed on ONE GPU: every worker of the
configuration is its own HIP worker context (cglgan.GanStep) and the exchange runs through the
in-process lockstep collectives (cglgan.exchange.LocalComm / local_cloud_average -- the same phase A
-> all-gather -> alpha -> sum -> phase B sequence, E-share, D-swap and Cloud FedAvg that
WorkerExchange runs over RCCL), against the oracle in which the reference's Server backpropagates
F_max through every worker's D:

  config 3  CAPGAN num_workers=8, E=1 D all-reduce, bs256      capgan.py:211-262,316-349 (+ E-share, a19)
  config 4  Mix-G num_workers=8 num_servers=2, Cloud FedAvg     mixed-gan.py:104-124,193-200,238-292,355-392
  config 5  MD-GAN num_workers=8 non-IID shards, D-swap, bs512  MDGAN/MNIST/mdgan.py:158-164,180-207,266-297
  + the CAPGAN/MNIST/mixed-gan.py:276-278 double-softmax weighting (mix_double)

Shards are cut by cglgan.data.allocate_dataset from a labelled synthetic MNIST-shaped set (no MNIST
here), beta / A are the reference's data-size weights.  Config 5's fp16 is parity-unpinned and not here.

Tolerances (parity_helpers): round 1 from identical state -- updated parameters (after the
exchange) <= max(1e-5 rel, 2x the fp32 oracle's own error) vs the fp64 oracle; round 2 free-running --
losses <= 1e-4 rel.  At 8 workers x 256-512 rows a round has 6-11 million LeakyReLU inputs, so some lie
within fp32 rounding of the kink; the oracle runs therefore follow the GPU's own branch decisions there
and those decisions are checked against the fp64 signs separately (parity_helpers.MaskedRun).
"""
import copy

import pytest
import torch

from cglgan import GanStep, specs
from cglgan.data import allocate_dataset, beta_weights, cloud_weights, sample_batches, synthetic_mnist
from cglgan.exchange import DSwap, LocalComm, local_cloud_average
from cglgan.init import capgan_state, mixgen_state
from oracle import gan_oracle as O
from parity_helpers import (TRAJ_TOL, MaskedRun, g_params, gpu_masks, masked_pair, rel_scalar, to_double,
                            within)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _threads():
    n = torch.get_num_threads()
    torch.set_num_threads(8)
    yield
    torch.set_num_threads(n)


@pytest.fixture(scope="module")
def shards():
    """60,000 labelled rows (MNIST's train size), non-IID iid=1 shards for 8 workers
    (capgan.py:378-411), and the IID split (iid=0) for the CAPGAN config."""
    x, y = synthetic_mnist(60000, seed=11)
    _, nonid, _ = allocate_dataset(y, iid=1, num_workers=8, num_sample=1000)
    _, iid, _ = allocate_dataset(y, iid=0, num_workers=8, num_sample=1000)
    return x, [x[torch.as_tensor(s)] for s in nonid], [x[torch.as_tensor(s)] for s in iid]


def _round64(srv64, workers64, z1, z2, reals):
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return srv64.round(workers64, z1.double(), z2.double(), [[r.double() for r in rs] for rs in reals])
    finally:
        torch.set_default_dtype(prev)


def _oracle_round(srv, workers, z1, z2, reals, weighting=None):
    if weighting is not None:
        return srv.round(workers, z1, z2, reals, weighting=weighting)
    return srv.round(workers, z1, z2, reals)


def _round64w(srv64, workers64, z1, z2, reals, weighting=None):
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return _oracle_round(srv64, workers64, z1.double(), z2.double(), [[r.double() for r in rs] for rs in reals],
                             weighting)
    finally:
        torch.set_default_dtype(prev)


def _load(steps, g_sd, d_sds, beta):
    for s, d in zip(steps, d_sds):
        s.load_state_dicts(g_sd, d)
        s.reset(beta=beta)


def _feed(steps, z1, z2, reals):
    for s, r in zip(steps, reals):
        B = s.B
        s.z[:B].copy_(z1)
        s.z[B:].copy_(z2)
        s.real.copy_(r.reshape(r.shape[0], -1))


def _check_g(step, G32, G64, names):
    p32, p64 = g_params(G32), g_params(G64)
    fails = []
    for k in names:
        g64 = p64[k].grad.detach().double().flatten()
        dg = (step.g_grad_views[k].detach().double().cpu().flatten() - g64).abs()
        extra = 1.5 * float((2e-4 * dg / (g64.abs() + 1e-8)).norm())   # Adam step-1 sensitivity
        ok, e, a = within(step.g_views[k], p32[k], p64[k], extra)
        if not ok:
            fails.append((k, e, a))
    return fails


def _check_d(steps, workers32, workers64):
    fails = []
    for r, s in enumerate(steps):
        for k, v in s.d_views.items():
            ok, e, a = within(v, workers32[r].D.params[k], workers64[r].D.params[k])
            if not ok:
                fails.append((r, k, e, a))
    return fails


def _traj(steps, out, tag):
    for r, s in enumerate(steps):
        st = s.stats()
        assert rel_scalar(st["d_loss"][0], out["d_losses"][r]) <= TRAJ_TOL, (tag, r, st["d_loss"], out["d_losses"])
        assert rel_scalar(st["g_loss"], out["g_losses"][r]) <= TRAJ_TOL, (tag, r, st["g_loss"], out["g_losses"])


# ------------------------------------------------------------------------------------------------
def _oracles(srv, workers):
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    return srv64, workers64


def test_config3_capgan_8_workers_eshare(shards):
    """CAPGAN num_workers=8, S=1, bs256, E=1: after the round every worker's D is the mean of the 8."""
    N, B = 8, 256
    _, _, iid = shards
    beta = beta_weights([len(s) for s in iid])[0].tolist()
    g_sd, d_sds = capgan_state(N)
    G, workers = O.build_capgan(N)
    for k, v in G.params.items():                       # product init == the oracle's reference init
        assert torch.equal(v.detach(), g_sd[k])
    steps = [GanStep(specs.mnist_generator(), specs.mnist_discriminator(), batch=B, n_workers=N, rank=r)
             for r in range(N)]
    _load(steps, g_sd, d_sds, beta)

    def inputs(seed):
        g = torch.Generator().manual_seed(seed)
        z1, z2 = torch.randn(B, 100, generator=g), torch.randn(B, 100, generator=g)
        return z1, z2, [sample_batches(s, B, 1, seed * 16 + r)[0] for r, s in enumerate(iid)]

    z1, z2, reals = inputs(101)
    _feed(steps, z1, z2, reals)
    comm = LocalComm(steps, share_every=1)
    comm.round(0)
    torch.cuda.synchronize()
    srv = O.CapganServer(G, torch.tensor(beta))
    srv64, workers64 = _oracles(srv, workers)
    masks = [gpu_masks(s) for s in steps]
    _, m64 = masked_pair(srv.G, workers, srv64.G, workers64, masks)
    r32 = srv.round(workers, z1, z2, [[x] for x in reals])
    r64 = _round64(srv64, workers64, z1, z2, [[x] for x in reals])
    m64.check_signs()
    O.eshare_mean(workers)
    O.eshare_mean(workers64)
    for s in steps[1:]:
        assert torch.equal(s.g_params, steps[0].g_params)       # replicated G stays bitwise identical
        assert torch.equal(s.d_params, steps[0].d_params)       # E-share: one D everywhere
    st = steps[0].stats()
    assert abs(st["F"] - float(r64["F"])) <= max(1e-5 * abs(float(r64["F"])), 2 * abs(float(r32["F"] - r64["F"])))
    assert abs(st["lambda"] - float(r32["lam"])) <= 1e-7
    assert not _check_g(steps[0], srv.G, srv64.G, list(steps[0].g_views))
    assert not _check_d(steps, workers, workers64)
    # round 2 from the shared D, free running
    z1, z2, reals = inputs(7919)
    _feed(steps, z1, z2, reals)
    comm.round(1)
    torch.cuda.synchronize()
    # the fp32 and fp64 oracles both follow the round's LeakyReLU decisions, and the decisions are checked against
    # the fp64 run's own signs (as in round 1)
    m32, m64 = masked_pair(srv.G, workers, srv64.G, workers64, [gpu_masks(s) for s in steps])
    out = srv.round(workers, z1, z2, [[x] for x in reals])
    _round64(srv64, workers64, z1, z2, [[x] for x in reals])
    m64.check_signs()
    m32.check_signs()
    _traj(steps, out, "round 2")


def test_config4_mixg_8_workers_2_servers_cloud_fedavg(shards):
    """Mix-G num_workers=8 num_servers=2 (4 heads per server group), bs256 per head, Cloud FedAvg of
    the trunk (parameters + BatchNorm running statistics) with A_s weights after round 1."""
    S, H, B = 2, 4, 256
    XL = specs.MIXGEN_HEAD_LAYER
    _, nonid, _ = shards
    lens = [len(s) for s in nonid]
    betas = [beta_weights(lens[H * s:H * (s + 1)])[0].tolist() for s in range(S)]
    A = cloud_weights([sum(lens[H * s:H * (s + 1)]) for s in range(S)]).tolist()
    srvs, wss, groups = [], [], []
    for s in range(S):
        g_sd, d_sds = mixgen_state(H, seed=20211212 + s, n_discriminators=H)
        G, workers = O.build_mixg(H, seed=20211212 + s)
        for k, v in G.state_dict().items():                # product init == the oracle's reference init
            if k in g_sd:
                assert torch.equal(v.detach(), g_sd[k]), k
        srvs.append(O.MixgServer(G, torch.tensor(betas[s])))
        wss.append(workers)
        groups.append([GanStep(specs.mixgen_worker(h), specs.mnist_discriminator(), batch=B, n_workers=H, rank=h,
                               weighting="mix_single", exchange_layer=XL) for h in range(H)])
        _load(groups[s], g_sd, d_sds, betas[s])

    def inputs(seed):
        out = []
        for s in range(S):
            g = torch.Generator().manual_seed(seed * 8 + s)
            z1, z2 = torch.randn(B, 100, generator=g), torch.randn(B, 100, generator=g)
            out.append((z1, z2, [sample_batches(nonid[H * s + h], B, 1, seed * 16 + H * s + h)[0] for h in range(H)]))
        return out

    ins = inputs(201)
    for steps, (z1, z2, reals) in zip(groups, ins):
        _feed(steps, z1, z2, reals)
        LocalComm(steps).round(0)
    torch.cuda.synchronize()
    masks = [[gpu_masks(st) for st in steps] for steps in groups]
    everyone = [st for steps in groups for st in steps]
    local_cloud_average(everyone, [A[s] / H for s in range(S) for _ in range(H)], cloud_scope="trunk")
    torch.cuda.synchronize()
    o64 = [_oracles(srv, ws) for srv, ws in zip(srvs, wss)]
    for s in range(S):
        z1, z2, reals = ins[s]
        _, m64 = masked_pair(srvs[s].G, wss[s], o64[s][0].G, o64[s][1], masks[s], head_layer=XL)
        srvs[s].round(wss[s], z1, z2, [[x] for x in reals])
        _round64w(o64[s][0], o64[s][1], z1, z2, [[x] for x in reals])
        m64.check_signs()
    for ss in ([srv.G for srv in srvs], [o[0].G for o in o64]):      # Cloud: trunk <- sum_s A_s trunk_s
        avg = O.fedavg([g.trunk.state_dict() for g in ss], [A[0], A[1]])
        with torch.no_grad():
            for g in ss:
                for k, v in avg.items():
                    (g.trunk.params if k in g.trunk.params else g.trunk.buffers)[k].copy_(v)
    p0 = groups[0][0].trunk_slices()
    for st in everyone[1:]:                        # one trunk (and its running statistics) everywhere
        p = st.trunk_slices()
        assert torch.equal(p[0], p0[0]) and torch.equal(p[1], p0[1])
    for s in range(S):
        G32, G64 = srvs[s].G, o64[s][0].G
        for h, st in enumerate(groups[s]):
            names = [k for k in st.g_views if k.startswith("model.") or k.startswith(f"paths.{h}.")]
            assert not _check_g(st, G32, G64, names), (s, h)
            for k in ("model.3.running_mean", "model.3.running_var", "model.6.running_mean", "model.6.running_var"):
                ok, e, a = within(st.running[k], G32.trunk.buffers[k], G64.trunk.buffers[k])
                assert ok, (k, e, a)
        assert not _check_d(groups[s], wss[s], o64[s][1]), s
    # round 2 from the averaged trunk, free running
    ins2 = inputs(7919)
    for s in range(S):
        z1, z2, reals = ins2[s]
        _feed(groups[s], z1, z2, reals)
        LocalComm(groups[s]).round(1)
        torch.cuda.synchronize()
        m32, m64 = masked_pair(srvs[s].G, wss[s], o64[s][0].G, o64[s][1], [gpu_masks(st) for st in groups[s]],
                               head_layer=XL)
        out = srvs[s].round(wss[s], z1, z2, [[x] for x in reals])
        _round64w(o64[s][0], o64[s][1], z1, z2, [[x] for x in reals])
        m64.check_signs()
        m32.check_signs()
        _traj(groups[s], out, f"round 2 server {s}")


def test_config5_mdgan_8_workers_noniid_dswap_bs512(shards):
    """MD-GAN num_workers=8, non-IID (iid=1) shards, bs512, fp32: G on mean(l_i) with the Sigmoid/BCE
    D, then the server's D-swap (Random(server + 100).shuffle; worker i continues with D_perm[i])."""
    N, B = 8, 512
    _, nonid, _ = shards
    g_sd, d_sds = capgan_state(N, sigmoid=True)
    G, workers = O.build_capgan(N, loss="bce")
    for r in range(N):
        for k, v in workers[r].D.params.items():
            assert torch.equal(v.detach(), d_sds[r][k])
    steps = [GanStep(specs.mnist_generator(), specs.mnist_discriminator(sigmoid=True), batch=B, loss="bce",
                     weighting="mean", n_workers=N, rank=r) for r in range(N)]
    beta = [1.0 / N] * N
    _load(steps, g_sd, d_sds, beta)

    def inputs(seed):
        g = torch.Generator().manual_seed(seed)
        z1, z2 = torch.randn(B, 100, generator=g), torch.randn(B, 100, generator=g)
        return z1, z2, [sample_batches(s, B, 1, seed * 16 + r)[0] for r, s in enumerate(nonid)]

    z1, z2, reals = inputs(301)
    _feed(steps, z1, z2, reals)
    comm = LocalComm(steps, swap_every=1)
    perm = comm.round(0)
    torch.cuda.synchronize()
    assert perm == DSwap(N).next_perm()          # Random(0 + 100).shuffle, MDGAN/MNIST/mdgan.py:122-123
    srv = O.CapganServer(G, torch.tensor(beta))
    srv64, workers64 = _oracles(srv, workers)
    _, m64 = masked_pair(srv.G, workers, srv64.G, workers64, [gpu_masks(s) for s in steps])
    srv.round(workers, z1, z2, [[x] for x in reals], weighting="mean")
    _round64w(srv64, workers64, z1, z2, [[x] for x in reals], weighting="mean")
    m64.check_signs()
    O.dswap(workers, perm)
    O.dswap(workers64, perm)
    for s in steps[1:]:
        assert torch.equal(s.g_params, steps[0].g_params)
    assert not _check_g(steps[0], srv.G, srv64.G, list(steps[0].g_views))
    assert not _check_d(steps, workers, workers64)
    z1, z2, reals = inputs(7919)
    _feed(steps, z1, z2, reals)
    comm.round(1)
    torch.cuda.synchronize()
    m32, m64 = masked_pair(srv.G, workers, srv64.G, workers64, [gpu_masks(s) for s in steps])
    out = srv.round(workers, z1, z2, [[x] for x in reals], weighting="mean")
    _round64w(srv64, workers64, z1, z2, [[x] for x in reals], weighting="mean")
    m64.check_signs()
    m32.check_signs()
    _traj(steps, out, "round 2")


def test_mixg_double_softmax_weighting():
    """CAPGAN/MNIST/mixed-gan.py:276-278: alpha = softmax(beta * softmax(lambda l)) (mix_double), 2 heads."""
    N, B = 2, 64
    XL = specs.MIXGEN_HEAD_LAYER
    beta = [0.3, 0.7]
    g_sd, d_sds = mixgen_state(N, n_discriminators=N)
    G, workers = O.build_mixg(N)
    srv = O.MixgServer(G, torch.tensor(beta), weighting="mix_double")
    steps = [GanStep(specs.mixgen_worker(h), specs.mnist_discriminator(), batch=B, n_workers=N, rank=h,
                     weighting="mix_double", exchange_layer=XL) for h in range(N)]
    _load(steps, g_sd, d_sds, beta)

    def inputs(seed):
        z1, z2, reals = O.synthetic_inputs(B, N, 1, seed=seed)
        return z1, z2, [rs[0] for rs in reals]

    z1, z2, reals = inputs(61)
    _feed(steps, z1, z2, reals)
    LocalComm(steps).round(0)
    torch.cuda.synchronize()
    srv64, workers64 = _oracles(srv, workers)
    _, m64 = masked_pair(srv.G, workers, srv64.G, workers64, [gpu_masks(s) for s in steps], head_layer=XL)
    srv.round(workers, z1, z2, [[x] for x in reals])
    _round64w(srv64, workers64, z1, z2, [[x] for x in reals])
    m64.check_signs()
    for h, st in enumerate(steps):
        names = [k for k in st.g_views if k.startswith("model.") or k.startswith(f"paths.{h}.")]
        assert not _check_g(st, srv.G, srv64.G, names), h
    assert not _check_d(steps, workers, workers64)
    # a second round with lambda > 0 makes the inner softmax non-uniform
    z1, z2, reals = inputs(1061)
    _feed(steps, z1, z2, reals)
    LocalComm(steps).round(1)
    torch.cuda.synchronize()
    m32, m64 = masked_pair(srv.G, workers, srv64.G, workers64, [gpu_masks(s) for s in steps], head_layer=XL)
    out = srv.round(workers, z1, z2, [[x] for x in reals])
    _round64w(srv64, workers64, z1, z2, [[x] for x in reals])
    m64.check_signs()
    m32.check_signs()
    _traj(steps, out, "round 2")
    st = steps[0].stats()
    assert rel_scalar(st["F"], out["F"]) <= TRAJ_TOL and abs(st["lambda"] - float(out["lam"])) <= 1e-7
