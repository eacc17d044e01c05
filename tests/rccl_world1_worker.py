"""Worker of tests/test_gpu_rccl_world1.py (run under torch.distributed.run, one process, one nccl = RCCL rank).

Every collective of the exchange layer is issued over RCCL with the N > 1 code path forced, and the result is
compared bitwise with the same rounds run without a group (a one-rank all_gather / all_reduce is exact, alpha = 1):
  * MLP CAPGAN round (WorkerExchange, force_split): phase A, loss all_gather_into_tensor, on-device alpha,
    gradient all_reduce, side-stream E-share all_reduce of D, phase B -- eager and graph-replayed alternating;
  * Cloud FedAvg (WorkerExchange.cloud_average, mixed-gan.py:104-124,193-200 / capgan.py:169-175): scope
    "all" on a CAPGAN step and scope "trunk" (parameters + BatchNorm running statistics) on a Mix-G step, both
    with segema = 0.3, against cglgan.exchange.local_cloud_average;
  * conv round (ConvWorkerExchange, force_split, ConvGanStep(graph=True): phase A / phase B replayed as two
    hipGraphs around the collectives from the second round on) with the side-stream E-share of D's parameters
    AND BatchNorm running statistics, against the same rounds run unsplit (ConvGanStep.run).
The MD-GAN D-swap of a one-rank group is the identity permutation (DistComm.swap returns before any
send / recv), so it has no RCCL coverage here; its semantics are tested over gloo (tests/test_dist_swap_fedavg.py).
  * the whole-round graph of WorkerExchange (phase A + the collective(s) + phase B captured as one torch CUDA
    graph), both exchange forms, against the unsplit rounds.
Also times the MLP B = 256 round with the forced split against the unsplit round (the fixed cost of the N > 1
structure) in both exchange forms, with and without the whole-round graph.
Prints "RCCL-WORLD1 OK ..." on success."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cgl-gan_amd"), ROOT]


def mlp_step(B=64, kind="capgan", rows=None):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    if kind == "mixg":
        gm, xl, wt = specs.mixgen_worker(0), specs.MIXGEN_HEAD_LAYER, "mix_single"
    else:
        gm, xl, wt = specs.mnist_generator(), -1, "capgan"
    dm = specs.mnist_discriminator()
    g = torch.Generator().manual_seed(5)
    real = (torch.rand(rows or 8 * B, 784, generator=g) * 2 - 1).cuda()
    st = GanStep(gm, dm, batch=B, loss="ce", weighting=wt, n_workers=1, rank=0, gen_z=True, real=real,
                 sample_n=real.shape[0], seed=77, exchange_layer=xl)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(555)
    default_init(dm, st.d_views)
    st.reset()
    return st


def same(a, b, names):
    for name in names:
        x, y = getattr(a, name), getattr(b, name)
        assert torch.equal(x, y), (name, (x - y).abs().max().item())


def check_mlp_round(exchange="gather"):
    from cglgan.exchange import DistComm, WorkerExchange
    a, b = mlp_step(), mlp_step()
    ex = WorkerExchange(a, DistComm(), share_every=1, force_split=True, exchange=exchange)
    ref = WorkerExchange(b, None)
    for r in range(4):
        ex.round(r, graph=(r % 2 == 1))
        ref.round(r, graph=(r % 2 == 1))
    torch.cuda.synchronize()
    same(a, b, ("g_params", "g_m", "g_v", "d_params", "d_m", "d_v", "g_running"))
    sa, sb = a.stats(), b.stats()
    assert sa["round"] == sb["round"] == 4 and sa["g_loss"] == sb["g_loss"] and sa["alpha"] == 1.0, (sa, sb)
    return sa


def check_cloud(kind, scope):
    from cglgan.exchange import DistComm, WorkerExchange, local_cloud_average
    a, b = mlp_step(kind=kind), mlp_step(kind=kind)
    ex = WorkerExchange(a, None, cloud=DistComm(None), cloud_every=1, cloud_weights=[1.0], cloud_scope=scope,
                        segema=0.3)
    ref = WorkerExchange(b, None)
    for r in range(3):
        ex.round(r, graph=(r % 2 == 1))         # the Cloud step after every round, over RCCL
        ref.round(r, graph=(r % 2 == 1))
        local_cloud_average([b], [1.0], cloud_scope=scope, segema=0.3)
    torch.cuda.synchronize()
    same(a, b, ("g_params", "g_m", "g_v", "d_params", "g_running"))
    if scope == "trunk":
        pa, ra = a.trunk_slices()
        assert ra is not None and ra.numel() > 0         # the trunk's BatchNorm running statistics travel too
    return a.stats()["g_loss"]


def conv_step(B=8):
    from cglgan.conv_step import ConvGanStep
    g = torch.Generator(device="cuda").manual_seed(9)
    data = torch.rand(6 * B, 1024, device="cuda", generator=g) * 2 - 1
    st = ConvGanStep(B, loss="mse", data=data, seed=4242, n_workers=1, rank=0, graph=True)
    st.init_default(20211212, 31)
    return st


def check_conv_round():
    from cglgan.exchange import ConvWorkerExchange, DistComm
    a, b = conv_step(), conv_step()
    ex = ConvWorkerExchange(a, DistComm(), share_every=1, force_split=True)
    ref = ConvWorkerExchange(b, None)
    for r in range(4):
        ex.round(r)
        ref.round(r)
    torch.cuda.synchronize()
    assert a._phase_graphs is not None, "the split round did not replay as phase graphs"
    for x, y, n in ((a.G.p, b.G.p, "G"), (a.D.p, b.D.p, "D")):
        assert torch.equal(x, y), (n, (x - y).abs().max().item())
    for k in a.D.running:
        assert torch.equal(a.D.running[k], b.D.running[k]), k
    for k in a.G.running:
        assert torch.equal(a.G.running[k], b.G.running[k]), k
    sa, sb = a.stats(), b.stats()
    assert sa["g_loss"] == sb["g_loss"] and sa["round"] == sb["round"] == 4, (sa, sb)
    return sa["g_loss"]


def _ex(s, exchange, round_graph, share_every=0):
    from cglgan.exchange import DistComm, WorkerExchange
    ex = WorkerExchange(s, DistComm(), force_split=True, exchange=exchange, share_every=share_every)
    assert ex.round_graph        # (RCCL: capturable)
    ex.round_graph = round_graph
    return ex


def _side(ex):
    ex.d_side = True       # D's exchange on a side stream beside phase B (CGL_DX_SIDE=1)
    return ex


def check_round_graph(exchange, share_every=0):
    """WorkerExchange's whole-round graph (phase A + collective(s) + phase B as one torch CUDA graph, captured
    after the first split round; with share_every, the E-share of D and D's packed-copy refresh on a side stream
    inside it): bitwise the unsplit rounds, graph and eager rounds interleaved."""
    from cglgan.exchange import WorkerExchange
    a, b = mlp_step(), mlp_step()
    ex, ref = _ex(a, exchange, True, share_every), WorkerExchange(b, None)
    for r in range(6):
        ex.round(r, graph=(r != 3))
        ref.round(r, graph=(r != 3))
    torch.cuda.synchronize()
    assert ex._rgraph and ex.round_graph
    # every captured form's first replay was verified against the split round (bitwise, group verdict)
    assert ex.round_graph_checks and all(ok and ok_all for _, ok, ok_all in ex.round_graph_checks), \
        ex.round_graph_checks
    same(a, b, ("g_params", "g_m", "g_v", "d_params", "d_m", "d_v", "g_running"))
    assert a.stats()["round"] == b.stats()["round"] == 6


def time_split(rounds=200):
    """Device + host time per B = 256 round, all graph-replayed: the unsplit round vs the forced split over RCCL
    in the reduce form (loss all_gather, alpha, gradient all_reduce) and the gathered form (one all_gather,
    alpha + sum at phase B's head), each as two library graphs around the collective calls and as
    WorkerExchange's whole-round graph.  Each form's state after the rounds is compared bitwise with the
    unsplit one's."""
    from cglgan.exchange import WorkerExchange
    out, states = {}, {}
    for name, mk in (("unsplit", lambda s: WorkerExchange(s, None)),
                     ("split_reduce", lambda s: _ex(s, "reduce", False)),
                     ("split_gather", lambda s: _ex(s, "gather", False)),
                     ("round_graph_reduce", lambda s: _ex(s, "reduce", True)),
                     ("round_graph_gather", lambda s: _ex(s, "gather", True)),
                     ("split_gather_eshare1", lambda s: _ex(s, "gather", False, 1)),
                     ("round_graph_gather_eshare1", lambda s: _ex(s, "gather", True, 1)),
                     ("round_graph_gather_eshare1_side", lambda s: _side(_ex(s, "gather", True, 1)))):
        s = mlp_step(B=256, rows=60000)
        ex = mk(s)
        for r in range(20):
            ex.round(r, graph=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(rounds):
            ex.round(20 + r, graph=True)
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) / rounds * 1e6
        states[name] = (s.g_params.clone(), s.d_params.clone(), s.stats()["round"])
    for name in list(states):
        if name != "unsplit":
            out["delta_" + name + "_us"] = out[name] - out["unsplit"]
            gp, dp, rd = states[name]
            out["bitwise_" + name] = bool(torch.equal(gp, states["unsplit"][0]) and
                                          torch.equal(dp, states["unsplit"][1]) and rd == states["unsplit"][2])
    return {k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        sa = check_mlp_round("gather")
        check_mlp_round("reduce")
        check_round_graph("gather")
        check_round_graph("reduce")
        check_round_graph("gather", share_every=1)
        check_round_graph("reduce", share_every=2)
        ga = check_cloud("capgan", "all")
        gt = check_cloud("mixg", "trunk")
        gc = check_conv_round()
        tm = time_split() if "--time" in sys.argv else None
    dist.destroy_process_group()
    print(f"RCCL-WORLD1 OK mlp_rounds=4 g_loss={sa['g_loss']:.6f} lambda={sa['lambda']:.6f} cloud_all={ga:.6f} "
          f"cloud_trunk={gt:.6f} conv_g_loss={gc:.6f}", flush=True)
    if tm is not None:
        print("RCCL-WORLD1 TIMING " + json.dumps(tm), flush=True)


if __name__ == "__main__":
    main()
