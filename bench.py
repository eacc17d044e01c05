#!/usr/bin/env python3
"""Benchmark: images/s of the CGL-GAN worker round (G+D step) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE.json configs[1] at N=1, configs[2] at N>1):
  * model/mnist_model.py MLP GAN (G 100-128-256-512-1024-784 with BatchNorm1d(eps .8), D 784-512-256-2),
    fp32, batch 256, CAPGAN worker round: two train-mode G forwards (Xd, Xg), one local D step on a
    real batch (CE, Adam), the G loss through the updated D, G backward, lambda SGD and Adam G
    (capgan.py:211-262 + :316-349), captured as hipGraph(s) and replayed.
  * inputs: z drawn on device each round (Philox); the real batch gathered each round from a
    synthetic 28x28 dataset resident in HBM (60,000 rows, uniform(-1,1)) through the in-graph
    per-pass shuffle sampler (234 full batches, then the pass's short batch of 96 real rows).
  * N > 1: one worker per GPU (CAPGAN N workers, S=1, G replicated with a shared z stream): per
    round all_gather(G losses) -> lambda-weighting -> all_reduce(sum) of the weighted G-output
    gradient -> replicated G update, plus the E-share all_reduce(avg) of D every --E rounds (RCCL).
A "step" is one round; value = images/s over all ranks = N * 256 * K / max-over-ranks time.
At N = 1 the line also carries "conv_round": the model/lsgan.py conv GAN round (B=256) timed in its own
graph-replayed region (--conv-steps rounds, default 60) with its own conv-family roofline -- a second,
labelled workload of the same run, never part of `value`.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cgl-gan_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec (G+D step) MNIST bs256 at 1/2/4/8 MI355X; D-loss match vs CPU"
PEAK_F32_MFMA = 157.3    # TFLOP/s, MI355X dense fp32 matrix (MI355X_MICROARCH.md)
PEAK_HBM = 8000.0        # GB/s
# algorithmic work per image (BASELINE.md / SURVEY 8d): FLOPs excluding the D weight-gradient of
# the G-loss path that the reference computes and discards
FLOP_PER_IMAGE_MIN = 18.95e6


def default_batch(model):
    return {"mdgan": 512, "ring": 64}.get(model, 256)


def args_():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--batch", type=int, default=None, help="per-worker batch (default 256; 512 for mdgan, 64 for ring)")
    p.add_argument("--rows", type=int, default=60000,
                   help="synthetic dataset rows per worker (MNIST train size: 234 full batches + one of 96)")
    p.add_argument("--E", type=int, default=1, help="D-share all-reduce period (N > 1)")
    p.add_argument("--eager", action="store_true", help="launch without hipGraph")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--profile-rounds", type=int, default=10,
                   help="rounds issued launch by launch with per-dispatch events (in-round launch durations)")
    p.add_argument("--model", choices=["mlp", "lsgan", "mixg", "mdgan", "ring"], default="mlp",
                   help="mlp: model/mnist_model.py CAPGAN round (BASELINE configs[1] at N=1, configs[2] at N>1, "
                        "the default workload); mixg: configs[3], Mix-G through cglgan.driver (num_servers=2 when N "
                        "is even, Cloud FedAvg every round); mdgan: configs[4] (non-IID shards, D-swap every --E "
                        "rounds, bs512, fp32); ring: configs[0], the CGLGAN 2-D Gaussian-mixture round (B=64); "
                        "lsgan: the model/lsgan.py conv GAN round (32x32, MSE/LSGAN loss)")
    p.add_argument("--loss", choices=["mse", "bce"], default="mse", help="conv GAN objective (--model lsgan)")
    p.add_argument("--conv-steps", type=int, default=60,
                   help="--model mlp at N = 1: also time this many graph-replayed conv GAN rounds (model/lsgan.py, "
                        "same batch) and report them as 'conv_round' beside the line (0: skip)")
    p.add_argument("--conv-warmup", type=int, default=5)
    p.add_argument("--lowp", choices=["none", "f16", "bf16"], default="f16",
                   help="--model mdgan: also time the same round with 16-bit GEMM operands (BASELINE configs[4]'s "
                        "fp16) and report it beside the fp32 line as 'lowp_variant' (parity unpinned)")
    p.add_argument("--ring-steps", type=int, default=400,
                   help="--model mlp at N = 1: also time this many graph-replayed CGLGAN 2-D Gaussian-mixture rounds "
                        "(configs[0], B=64) and report them as 'ring_round' beside the line (0: skip)")
    p.add_argument("--graph-rounds", type=int, default=int(os.environ.get("CGL_GRAPH_ROUNDS", "10")),
                   help="N = 1 fused rounds: this many complete rounds per hipGraph launch in the timed region "
                        "(cgl_gan_run_graph_rounds; 1 = one graph launch per round)")
    p.add_argument("--launch-selftest", choices=["ok", "fail"], default=None, help=argparse.SUPPRESS)
    a = p.parse_args()
    if a.batch is None:
        a.batch = default_batch(a.model)
    return a


def build_step(a, rank, world):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)
    data = torch.rand(a.rows, 784, device="cuda", generator=g) * 2 - 1
    step = GanStep(gm, dm, batch=a.batch, batch_real=a.batch, epoch=1, loss="ce", weighting="capgan",
                   n_workers=world, rank=rank, seed=20211212, gen_z=True, real=data, sample_n=a.rows)
    torch.manual_seed(20211212)          # G identical on every replica (capgan.py:28,156)
    default_init(gm, step.g_views)
    torch.manual_seed(20211212 + 1 + rank)
    default_init(dm, step.d_views)
    step.reset(beta=[1.0 / world] * world)
    return step, data


def make_exchange(step, world, a):
    from cglgan.exchange import DistComm, WorkerExchange
    return WorkerExchange(step, DistComm() if world > 1 else None, share_every=a.E if world > 1 else 0)


def profile_inround(step, world, rounds, ex=None):
    """Device time per launch of the round's plan, measured IN the round: ``rounds`` extra rounds issued
    launch by launch, every dispatch carrying its own start / stop event pair (cgl_gan_profile: the
    dispatch's begin / end timestamps, the interval rocprofv3's kernel trace reports), each launch
    reading the operands its producer has just written -- the timed rounds' data state.  Returns the
    median over rounds per launch (this runs after the timed region; the rounds advance the state).
    N > 1: phase A and phase B around this rank's collectives, as WorkerExchange.round issues them."""
    from cglgan._lib import PHASE_A, PHASE_ALL, PHASE_B
    split = ex is not None and ex.comm is not None and ex.comm.size > 1
    phases = [PHASE_A, PHASE_B] if split else [PHASE_ALL]
    info = []
    for ph in phases:
        info += step.launches(ph)
    runs = []
    for _ in range(rounds):
        if not split:
            runs.append(step.profile_round(PHASE_ALL))
        else:
            a = step.profile_round(PHASE_A)
            ex.exchange_mid()
            runs.append(a + step.profile_round(PHASE_B))
    med = [sorted(col)[len(col) // 2] for col in zip(*runs)]
    per_kind = {}
    gemm_us, gemm_flops, gemm_n = [], 0.0, 0
    for (kind, flops, grid), us in zip(info, med):
        k = per_kind.setdefault(kind, [0.0, 0])
        k[0] += us
        k[1] += 1
        if kind == "gemm":
            gemm_us.append(us)
            gemm_flops += flops
            gemm_n += 1
    launches = [{"kind": kind, "grid": grid, "gflop": round(flops / 1e9, 4), "us": round(us, 2),
                 "tflops": round(flops / (us * 1e-6) / 1e12, 2) if flops else None}
                for (kind, flops, grid), us in zip(info, med)]
    return per_kind, gemm_us, gemm_flops, gemm_n, launches


def _latest_profile(names):
    for n in names:
        path = os.path.join(ROOT, "profiles", n)
        if os.path.exists(path):
            return n, json.load(open(path))
    return None, None


def traffic_per_gemm_launch():
    """HBM-side bytes per GEMM dispatch (every cgl_gemm_f32 instantiation, dispatch-weighted) from the
    newest committed FETCH_SIZE / WRITE_SIZE passes (tools/gpu_session.sh traffic -> tools/pmc_traffic.py).
    A static, labelled measurement: PMC passes cannot run inside the timed bench, so roofline.traffic
    names the profile file and the commit it was measured at (traffic_source).  None when absent."""
    name, d = _latest_profile(["r06_traffic.json", "r05_traffic.json", "r04_traffic.json", "r03_traffic.json", "r02_traffic.json"])
    if d is None:
        return None, None
    src = {"file": f"profiles/{name}", "commit": (d.get("_meta") or {}).get("commit"),
           "kind": "static PMC measurement (not measured in this run)"}
    fam = d.get("cgl_gemm_f32 (all instantiations)")
    if fam:
        return round(fam["bytes_per_dispatch"]), src
    for k, v in d.items():
        if "cgl_gemm_f32" in k:
            return round(v["bytes_per_dispatch"]), src
    return None, None


def traffic_per_launch():
    """Per-launch PMC traffic of the round's GEMM launches against each launch's own compulsory bytes
    (A + B + C of its descriptors, f32), from the newest committed per-launch pass (tools/pmc_traffic.py
    --plan): [{"i": position in the round, "bytes", "algorithmic", "ratio"}], plus the launch-summed ratio."""
    name, d = _latest_profile(["r06_traffic.json", "r05_traffic.json", "r04_traffic.json"])
    if not d or "per_launch" not in d:
        return {}
    rows = [{"i": e["i"], "kernel": e["kernel"].split("<")[0], "bytes": round(e["bytes"]),
             "algorithmic": e["algorithmic_bytes"], "ratio": e["ratio"]}
            for e in d["per_launch"] if "algorithmic_bytes" in e]
    # the ratio over the cgl_gemm_f32 launches (the fused prologue also moves the round's operand packing)
    g = [r for r in rows if r["kernel"] == "cgl_gemm_f32"]
    tb, ta = sum(r["bytes"] for r in g), sum(r["algorithmic"] for r in g)
    return {"traffic_per_launch": rows, "traffic_ratio_launch_sum": round(tb / ta, 3) if ta else None,
            "traffic_per_launch_source": f"profiles/{name} (static PMC measurement, commit "
                                         f"{(d.get('_meta') or {}).get('commit')})"}


def mlp_traffic_algorithmic(B, gemm_n):
    """Compulsory bytes per GEMM launch of the MLP round (SURVEY §8d byte model without its Adam
    term 28·(P_G+P_D): weight reads, gradient writes, inputs, images and saved activations), spread
    over the round's GEMM launches.  An upper bound on what the GEMMs must move (it includes the
    BatchNorm / head passes' share), so traffic / this is a lower bound on the over-fetch."""
    pg, pd = 1510032, 533762
    nbytes = (4 * (2 * pg + 4 * pd) + 4 * (pg + pd) + 4 * B * (784 + 2 * 100) + 8 * B * 784
              + 8 * B * (2 * 1920 + 3 * 768))
    per = nbytes / max(gemm_n, 1)
    t, _ = traffic_per_gemm_launch()
    return {"traffic_algorithmic": round(per), "traffic_ratio": round(t / per, 2) if t else None,
            "traffic_algorithmic_note": "SURVEY 8d compulsory bytes/round minus the Adam term, / GEMM launches"}


def host_info(threads):
    """the host the CPU baseline ran on -- CPU model, logical CPUs of the machine and of
    this process's affinity mask, the torch threads actually used, torch version."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"cpu_model": model, "host_logical_cpus": os.cpu_count(), "affinity_cpus": affinity,
            "threads": threads, "torch": torch.__version__}


def cpu_threads():
    """Torch threads of the CPU leg: the process's CPU share, at most 16 (the GPU box's per-GPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_variants(leg):
    """the CPU baseline at the process's CPU share (``value``; at most 16 threads -- the GPU
    pool's per-GPU CPU share, OMP_NUM_THREADS there) and at 1 thread (``single_thread``).  The machine's
    other logical CPUs (``host.host_logical_cpus``) belong to the other GPUs' jobs of a shared node, so a
    whole-host figure is not taken on this pool."""
    main = leg(None)
    if main["cores"] > 1:
        one = leg(1)
        main["single_thread"] = {k: one[k] for k in ("value", "unit", "cores", "sample")}
        main["speedup_vs_1_thread"] = round(main["value"] / one["value"], 2)
    main["threads_note"] = ("value at the process's CPU share (<= 16 threads, the GPU pool's per-GPU share); "
                            "single_thread at 1; the host's remaining logical CPUs serve other GPUs' jobs")
    return main


def cpu_baseline(a, threads=None):
    """The CPU oracle (torch-CPU restatement of the reference step) on this host's cores."""
    sys.path.insert(0, ROOT)
    from oracle import gan_oracle as O
    threads = threads or cpu_threads()
    torch.set_num_threads(threads)
    G, workers = O.build_capgan(1)
    srv = O.CapganServer(G, torch.tensor([1.0]))
    B = a.batch
    n, t_total = 0, 0.0
    warm = 3
    while True:
        z1, z2, reals = O.synthetic_inputs(B, 1, 1, seed=5000 + n)
        t0 = time.perf_counter()
        srv.round(workers, z1, z2, reals)
        dt = time.perf_counter() - t0
        n += 1
        if n > warm:
            t_total += dt
        if (n > warm and t_total >= a.cpu_seconds) or n >= 2000:
            break
    rounds = n - warm
    return {"value": round(B * rounds / t_total, 1), "unit": "images/s", "cores": threads, "kind": "port", "host": host_info(threads),
            "sample": f"{rounds} CAPGAN rounds (B={B}, N=1) of the torch-CPU oracle after {warm} warm-up "
                      f"rounds, {t_total:.1f} s, torch {torch.__version__}"}


# ------------------------------------------------------------------------------------------
# conv GAN (model/lsgan.py) round
def conv_flops(n, h, w, cin, cout, stride, up, which):
    """(executed, reference-formulation) FLOPs of one conv3x3 op of cglgan.conv_ops.
    Executed = the MFMA work of the tap tables (phase-form upsampling: 2x2 taps per output parity,
    4x4 taps at stride 2 for its input gradient; stride-2 input gradients by input parity);
    reference = the direct 9-tap convolution on the upsampled input that torch runs."""
    ho, wo = ((h << up) - 1) // stride + 1, ((w << up) - 1) // stride + 1
    ref = 2.0 * n * ho * wo * cout * 9 * cin
    if which in ("fwd", "wgrad"):
        exe = 2.0 * n * ho * wo * cout * 4 * cin if up else ref
    elif up:
        exe = 2.0 * n * h * w * cin * 16 * cout
    elif stride == 1:
        exe = ref
    else:
        t = lambda d: sum(((d - p + 1) // 2) * (1 if p == 0 else 2) for p in (0, 1))
        exe = 2.0 * n * cin * cout * t(h) * t(w)
    return exe, ref


def profile_conv_round(run_round):
    """One extra round with every conv op bracketed by HIP events on the launch stream: per-op
    device time (pack + MFMA kernel, + fixed-order reduction for weight gradients) and FLOPs."""
    from cglgan import conv_ops as CO
    s = torch.cuda.current_stream()
    recs = []
    orig = {k: getattr(CO, k) for k in ("conv3x3_fwd", "conv3x3_bwd_data", "conv3x3_bwd_weight")}
    kinds = {"conv3x3_fwd": "fwd", "conv3x3_bwd_data": "bwd_data", "conv3x3_bwd_weight": "wgrad"}

    def wrap(name):
        fn = orig[name]

        def f(*args, **kw):
            geo = args[4:11] if name == "conv3x3_bwd_weight" else (args[3:10] if name == "conv3x3_bwd_data"
                                                                     else args[4:11])
            n, h, w, cin, cout, stride, up = (list(geo) + [1, 0])[:7]
            if name == "conv3x3_fwd":
                stride = kw.get("stride", stride)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            out = fn(*args, **kw)
            e1.record(s)
            exe, ref = conv_flops(n, h, w, cin, cout, stride, up, kinds[name])
            recs.append((kinds[name], (n, h, w, cin, cout, stride, up), e0, e1, exe, ref))
            return out
        return f

    for k in orig:
        setattr(CO, k, wrap(k))
    try:
        run_round()
    finally:
        for k, f in orig.items():
            setattr(CO, k, f)
    torch.cuda.synchronize()
    out = []
    for kind, geo, e0, e1, exe, ref in recs:
        out.append({"op": kind, "geom": geo, "us": e0.elapsed_time(e1) * 1e3, "exec_flops": exe, "ref_flops": ref})
    return out


def conv_cpu_baseline(a, threads=None):
    """The conv oracle (torch-CPU restatement of the model/lsgan.py round) on this host's cores."""
    sys.path.insert(0, ROOT)
    from oracle import conv_oracle as CV
    threads = threads or cpu_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(20211212)
    gp, gb = CV.init_params(CV.G_SPEC)
    dp, db = CV.init_params(CV.D_SPEC)
    o = CV.ConvGan(gp, gb, dp, db, loss=a.loss, dtype=torch.float32)
    B = a.batch
    g = torch.Generator().manual_seed(5)
    n, t_total, warm = 0, 0.0, 1
    while True:
        z = torch.randn(2 * B, 100, generator=g)
        real = torch.rand(B, 1, 32, 32, generator=g) * 2 - 1
        m = [CV.draw_masks(B) for _ in range(3)]
        t0 = time.perf_counter()
        o.round(z[:B], z[B:], real, *m)
        dt = time.perf_counter() - t0
        n += 1
        if n > warm:
            t_total += dt
        if (n > warm and t_total >= a.cpu_seconds) or n >= 200:
            break
    rounds = n - warm
    return {"value": round(B * rounds / t_total, 2), "unit": "images/s", "cores": threads, "kind": "port", "host": host_info(threads),
            "sample": f"{rounds} conv-GAN CAPGAN rounds (model/lsgan.py, B={B}, N=1, {a.loss}) of the torch-CPU "
                      f"oracle after {warm} warm-up round, {t_total:.1f} s, torch {torch.__version__}"}


def conv_traffic():
    """HBM-side traffic of the dominant conv op per dispatch from the newest committed PMC passes
    (tools/conv_traffic.py: FETCH_SIZE x2 + WRITE_SIZE; None when absent), labelled with its source."""
    name, p = _latest_profile(["r06_conv_dominant_traffic.json", "r04_conv_dominant_traffic.json", "r03_conv_dominant_traffic.json",
                               "r02_conv_dominant_traffic.json"])
    if p is None:
        return {"traffic": None}
    return {"traffic": round(p["bytes"]), "traffic_unit": f"bytes per {p['kernel']} dispatch of the dominant op "
            f"{p['geom']} (PMC FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": {"file": f"profiles/{name}", "commit": p.get("commit"),
                               "kind": "static PMC measurement (not measured in this run)"},
            "traffic_algorithmic": p["algorithmic_bytes"], "traffic_ratio": round(p["ratio"], 2)}


def conv_round_measure(a, world, rank, steps, warmup, with_cpu):
    """The model/lsgan.py conv GAN round: W untimed + K timed graph-replayed rounds (barrier + synchronize on
    both sides, max over ranks), then one eager round with every conv op bracketed by HIP events for the
    conv-family roofline.  Returns (line, ms_step) on rank 0, (None, ms_step) elsewhere."""
    from cglgan.conv_step import ConvGanStep
    from cglgan.exchange import ConvWorkerExchange, DistComm
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        g = torch.Generator(device="cuda").manual_seed(1000 + rank)
        rows = a.rows                # every pass ends with its short batch (60,000 = 234 x 256 + 96)
        data = torch.rand(rows, 1024, device="cuda", generator=g) * 2 - 1
        # one worker per GPU: G replicated (same init and z stream), D and real shard per rank
        # the round replays as one hipGraph at N = 1 (device-side round state, cglgan.conv_step graph mode);
        # at N > 1 phase A and phase B replay as two graphs around the eager collectives (round_a / round_b)
        step = ConvGanStep(a.batch, loss=a.loss, data=data, seed=20211212, n_workers=world, rank=rank,
                           graph=not a.eager)
        step.init_default(20211212, 20211212 + 1 + rank)
        ex = ConvWorkerExchange(step, DistComm() if world > 1 else None, share_every=a.E if world > 1 else 0)
        torch.cuda.synchronize()
        r = 0
        for _ in range(warmup):
            ex.round(r)
            r += 1
        # N = 1 graph rounds: --graph-rounds whole rounds per graph replay (ConvGanStep.run_rounds), captured here
        chunks = (round_chunks(steps, a.graph_rounds) if world == 1 and not a.eager and a.graph_rounds > 1
                  else [1] * steps)
        for n in sorted(set(chunks)):
            if n > 1:
                step.prepare_rounds(n)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for n in chunks:
            if n == 1:
                ex.round(r)
            else:
                ex.rounds(r, n)
            r += n
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        st = step.stats()
        # per-op timing needs the ops issued one by one: an eager round (same device round state)
        ops = profile_conv_round(lambda: step.run(eager=True) if world == 1 else ex.round(r, eager=True))
    ms_step = el / steps * 1e3
    value = world * a.batch * steps / el
    if rank != 0:
        return None, ms_step
    mma_us = sum(o["us"] for o in ops)
    exe = sum(o["exec_flops"] for o in ops)
    ref = sum(o["ref_flops"] for o in ops)
    tf = exe / (mma_us * 1e-6) / 1e12
    dom = max(ops, key=lambda o: o["us"])
    out = {
        "metric": METRIC + " [conv GAN model/lsgan.py variant]", "value": round(value, 1), "unit": "images/s",
        "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"model/lsgan.py conv GAN, CAPGAN worker round (G fwd x2, D step, G loss, G bwd, "
                               f"Adam G/D), {a.loss} objective, 32x32x1, 1 worker per GPU"
                               + (f", {world} workers: loss all-gather, alpha-weighted image-gradient "
                                  f"all-reduce, E={a.E} D all-reduce over RCCL" if world > 1 else ""),
                   "global_batch": a.batch * world, "batch_per_worker": a.batch, "img": "32x32x1",
                   "parallelism": f"workers{world}", "dataset_rows_per_worker": rows,
                   "graph": not a.eager},
        "roofline": {"bound": "mfma", "kernel": "cgl_conv_fwd + cgl_conv_wgrad (+ pack / reduce), every conv op of "
                                                "one round", "achieved": round(tf, 3), "peak": PEAK_F32_MFMA,
                     "unit": "TFLOP/s", "frac": round(tf / PEAK_F32_MFMA, 4), **conv_traffic(),
                     "timing": "per conv op: HIP events on the launch stream around the op in one eager round "
                               "(pack + MFMA kernel, + fixed-order reduction for weight gradients)",
                     "conv_exec_gflop_per_round": round(exe / 1e9, 3),
                     "conv_ref_gflop_per_round": round(ref / 1e9, 3),
                     "conv_us_per_round": round(mma_us, 1),
                     "effective_ref_tflops": round(ref / (mma_us * 1e-6) / 1e12, 3),
                     "step_exec_tflops": round(exe / (ms_step * 1e-3) / 1e12, 3),
                     "dominant_op": {"op": dom["op"], "geom": dom["geom"], "us": round(dom["us"], 1),
                                     "tflops": round(dom["exec_flops"] / (dom["us"] * 1e-6) / 1e12, 2)},
                     "ops": [{"op": o["op"], "geom": o["geom"], "us": round(o["us"], 1),
                              "tflops": round(o["exec_flops"] / (o["us"] * 1e-6) / 1e12, 2)} for o in ops]},
        "losses": {"d_loss": st["d_loss"], "g_loss": st["g_loss"], "round": st["round"]},
    }
    if with_cpu and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_variants(lambda t: conv_cpu_baseline(a, t))
    return out, ms_step


def main_lsgan(a, world, rank, local):
    out, _ = conv_round_measure(a, world, rank, a.steps, a.warmup, with_cpu=True)
    if out is not None:
        print(json.dumps(out), flush=True)
    return out


def conv_extra(a, world, rank):
    """The conv GAN round (model/lsgan.py) timed beside the default C2 line at N = 1: its own graph-replayed
    timed region (--conv-steps rounds, default >= 50), its own conv-family roofline, no CPU leg (the conv
    oracle runs ~300 images/s; `bench.py --model lsgan` reports it).  A labelled extra key, never `value`."""
    if world != 1 or a.conv_steps <= 0:
        return None
    out, _ = conv_round_measure(a, world, rank, a.conv_steps, a.conv_warmup, with_cpu=False)
    if out is None:
        return None
    out["note"] = ("second workload of the same bench run (model/lsgan.py conv GAN, B=%d), timed in its own "
                   "region after the C2 line's; not part of `value`" % a.batch)
    return out


def parity_vs_cpu(kind, B, rounds=10):
    """The metric's "D-loss match vs CPU": ``rounds`` rounds of the fused HIP step and of the CPU oracle
    (the torch-fp32 restatement of the reference step, oracle/gan_oracle.py -- the checker, run only in
    this CPU leg) from the same initial state on identical explicit inputs (z, real batches); the
    largest per-round relative difference of D_loss and G_loss.  SURVEY F8: <= 1e-4 over 10 rounds."""
    sys.path.insert(0, ROOT)
    from cglgan import GanStep, specs
    from cglgan.data import gmm
    from oracle import gan_oracle as O
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    if kind == "capgan":
        G, ws = O.build_capgan(1)
        srv, kw = O.CapganServer(G, torch.tensor([1.0])), {"weighting": "capgan"}
        gm, dm, loss, wt, xl = specs.mnist_generator(), specs.mnist_discriminator(), "ce", "capgan", -1
    elif kind == "mdgan":
        G, ws = O.build_capgan(1, loss="bce")
        srv, kw = O.CapganServer(G, torch.tensor([1.0])), {"weighting": "mean"}
        gm, dm, loss, wt, xl = specs.mnist_generator(), specs.mnist_discriminator(sigmoid=True), "bce", "mean", -1
    elif kind == "mixg":
        G, ws = O.build_mixg(1)
        srv, kw = O.MixgServer(G, torch.tensor([1.0])), {}
        gm, dm, loss, wt, xl = specs.mixgen_worker(0), specs.mnist_discriminator(), "ce", "mix_single", \
            specs.MIXGEN_HEAD_LAYER
    else:
        G, ws = O.build_ring(1, 1)
        srv, kw = O.CglganServer(G, torch.tensor([1.0])), {}
        gm, dm, loss, wt, xl = specs.ring_generator(0), specs.ring_discriminator(), "bce", "cglgan", -1
    step = GanStep(gm, dm, batch=B, loss=loss, weighting=wt, exchange_layer=xl)
    step.load_state_dicts(G.state_dict(), ws[0].D.state_dict())
    step.reset()
    ring = gmm(8, 2000)[0] if kind == "ring" else None
    g = torch.Generator().manual_seed(4242)
    dmax = gmax = 0.0
    rows = []
    for r in range(rounds):
        z1, z2 = torch.randn(B, gm.dims[0], generator=g), torch.randn(B, gm.dims[0], generator=g)
        if ring is not None:
            real = ring[torch.randint(0, ring.shape[0], (B,), generator=g)]
        else:
            real = torch.rand(B, 784, generator=g) * 2 - 1
        step.z[:B].copy_(z1)
        step.z[B:].copy_(z2)
        step.real.copy_(real)
        step.run()
        st = step.stats()
        if kind in ("capgan", "mdgan"):
            out = srv.round(ws, z1, z2, [[real]], **kw)
        else:
            out = srv.round(ws, z1, z2, [[real]])
        dc, gc = float(out["d_losses"][0]), float(out["g_losses"][0])
        dr, gr = abs(st["d_loss"][0] - dc) / abs(dc), abs(st["g_loss"] - gc) / abs(gc)
        dmax, gmax = max(dmax, dr), max(gmax, gr)
        rows.append([round(st["d_loss"][0], 7), round(dc, 7)])
    return {"rounds": rounds, "batch": B, "kind": kind, "d_loss_max_rel": dmax, "g_loss_max_rel": gmax, "tol": 1e-4,
            "pass": bool(dmax <= 1e-4 and gmax <= 1e-4),
            "d_loss_gpu_cpu_per_round": rows,
            "reference": "CPU oracle: torch fp32 restatement of the reference step, same initial state, identical "
                         "z and real batches every round"}


def cpu_rounds(kind, B, seconds, threads=None):
    """The CPU oracle's round rate on this host (kind: ring / mdgan / mixg; N = 1)."""
    sys.path.insert(0, ROOT)
    from cglgan.data import gmm
    from oracle import gan_oracle as O
    threads = threads or cpu_threads()
    torch.set_num_threads(threads)
    if kind == "ring":
        G, ws = O.build_ring(1, 1)
        srv = O.CglganServer(G, torch.tensor([1.0]))
        ring = gmm(8, 2000)[0]
    elif kind == "mdgan":
        G, ws = O.build_capgan(1, loss="bce")
        srv = O.CapganServer(G, torch.tensor([1.0]))
    else:
        G, ws = O.build_mixg(1)
        srv = O.MixgServer(G, torch.tensor([1.0]))
    g = torch.Generator().manual_seed(5)
    n, t_total, warm = 0, 0.0, 3
    while True:
        z1, z2 = torch.randn(B, 100, generator=g), torch.randn(B, 100, generator=g)
        real = ring[torch.randint(0, ring.shape[0], (B,), generator=g)] if kind == "ring" else \
            torch.rand(B, 784, generator=g) * 2 - 1
        t0 = time.perf_counter()
        if kind == "mdgan":
            srv.round(ws, z1, z2, [[real]], weighting="mean")
        else:
            srv.round(ws, z1, z2, [[real]])
        dt = time.perf_counter() - t0
        n += 1
        if n > warm:
            t_total += dt
        if (n > warm and t_total >= seconds) or n >= 20000:
            break
    rounds = n - warm
    return {"value": round(B * rounds / t_total, 1), "unit": "images/s", "cores": threads, "kind": "port", "host": host_info(threads),
            "sample": f"{rounds} {kind} rounds (B={B}, N=1) of the torch-CPU oracle after {warm} warm-up rounds, "
                      f"{t_total:.1f} s, torch {torch.__version__}"}


def round_chunks(k, per):
    """k rounds as multi-round graph launches of `per` rounds plus one of the remainder."""
    out = [per] * (k // per)
    if k % per:
        out.append(k % per)
    return out


def timed_rounds(round_fn, a, world, ex=None):
    """W untimed rounds, then K rounds between barrier + synchronize; max over ranks.  With ``ex`` (an N = 1
    WorkerExchange, graph mode) the rounds run as multi-round graphs of --graph-rounds rounds (GanStep.run_rounds:
    every round complete, no graph-launch boundary inside a launch); their graphs are captured before the timed
    region."""
    chunks = None
    if ex is not None and world == 1 and not a.eager and a.graph_rounds > 1 and ex.comm is None:
        chunks = round_chunks(a.steps, a.graph_rounds)
        for n in sorted(set(chunks)):
            ex.step.prepare_rounds(n)
    torch.cuda.synchronize()
    for r in range(a.warmup):
        round_fn(r)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if chunks is not None:
        r = a.warmup
        for n in chunks:
            ex.rounds(r, n, graph=True)
            r += n
    else:
        for r in range(a.steps):
            round_fn(a.warmup + r)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def fused_report(a, world, rank, step, el, workload, config_extra, cpu_leg=None, parity_kind=None, extra=None,
                 ex=None, emit=True):
    """The bench line of a fused-round model (mlp / mixg / mdgan / ring): GEMM-family roofline from the
    in-round per-launch device durations (profile_inround), CPU baseline and CPU parity at N = 1."""
    st = step.stats()           # the timed rounds' end state (the profile rounds below advance it)
    per_kind, gemm_us, gemm_flops, gemm_n, launches = profile_inround(step, world, a.profile_rounds, ex)
    plan = step.plan_info()
    ms_step = el / a.steps * 1e3
    value = world * a.batch * a.steps / el
    if rank != 0:
        return None
    # The graph-replayed timed rounds run their launches back to back (the rocprofv3 graph-round timeline,
    # profiles/r04_final_graph_round_timeline.txt: 0.0 us between launches), so the timed period IS the sum of
    # the round's launch durations.  An eager dispatch's event interval differs from the same launch's duration in
    # a graph replay by about the same amount for every launch (rocprofv3 of both: 3.2-3.7 us on each of 27 of
    # the 28 launches, gpurun_out/r04q), so each launch's duration in the timed rounds = its eager in-round
    # duration + (timed period - eager sum) / launches: the roofline prices the same rounds `value` counts.
    # N > 1 (the period also holds the collectives) and --eager keep the eager durations.
    eager_us = sum(v[0] for v in per_kind.values())
    nl = sum(v[1] for v in per_kind.values())
    offset = ((ms_step * 1e3 - eager_us) / nl) if (world == 1 and not a.eager and nl > 0) else 0.0
    gemm_s = (sum(gemm_us) + offset * gemm_n) * 1e-6
    gemm_tf = gemm_flops / gemm_s / 1e12 if gemm_s > 0 else 0.0
    # the unmodelled figure beside it: the raw in-round eager GEMM durations, no offset
    gemm_raw_s = sum(gemm_us) * 1e-6
    gemm_raw_tf = gemm_flops / gemm_raw_s / 1e12 if gemm_raw_s > 0 else 0.0
    step_flops = plan["gemm_flops"]
    step_tf = step_flops / (ms_step * 1e-3) / 1e12
    cfg = {"workload": workload, "global_batch": a.batch * world, "batch_per_worker": a.batch,
           "parallelism": f"workers{world}", "graph": not a.eager}
    cfg.update(config_extra)
    if world > 1:
        cfg["dist"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic", "config": cfg,
        "roofline": {"bound": "mfma", "kernel": "cgl_gemm_f32 (the round's GEMM launches)",
                     "achieved": round(gemm_tf, 3), "peak": PEAK_F32_MFMA, "unit": "TFLOP/s",
                     "frac": round(gemm_tf / PEAK_F32_MFMA, 4),
                     "timing": (f"each launch's in-round device duration (median over {a.profile_rounds} rounds of "
                                "dispatch begin / end events on the launch stream, cgl_gan_profile) plus the timed "
                                "graph-replay period's per-launch offset (timed_offset_us = (ms_per_step - eager "
                                "device sum) / launches)"
                                if offset != 0.0 else
                                f"median over {a.profile_rounds} rounds of each launch's in-round device duration "
                                "(dispatch begin / end events on the launch stream, cgl_gan_profile)"),
                     "timed_offset_us": round(offset, 3),
                     "achieved_eager_raw": round(gemm_raw_tf, 3),
                     "frac_eager_raw": round(gemm_raw_tf / PEAK_F32_MFMA, 4),
                     "eager_raw_note": "GEMM FLOPs / the summed raw in-round eager GEMM durations (no offset model)",
                     "traffic": traffic_per_gemm_launch()[0] if a.model == "mlp" else None,
                     "traffic_unit": "bytes per GEMM launch, all cgl_gemm_f32 instantiations (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_source": traffic_per_gemm_launch()[1] if a.model == "mlp" else None,
                     **(mlp_traffic_algorithmic(a.batch, gemm_n) if a.model == "mlp" else {}),
                     **(traffic_per_launch() if a.model == "mlp" else {}),
                     "gemm_launches_per_round": gemm_n, "gemm_flops_per_round": gemm_flops,
                     "flops_per_gemm_launch": gemm_flops / max(gemm_n, 1),
                     "avg_gemm_launch_us": round(sum(gemm_us) / max(gemm_n, 1) + offset, 3),
                     "avg_gemm_launch_us_eager": round(sum(gemm_us) / max(gemm_n, 1), 3),
                     "gemm_launch_us": [round(u, 2) for u in gemm_us],
                     "step_achieved_tflops": round(step_tf, 3),
                     "step_frac_mfma": round(step_tf / PEAK_F32_MFMA, 4),
                     "per_kind_us_per_round": {k: round(v[0], 2) for k, v in per_kind.items()},
                     "device_us_per_round": round(eager_us, 2),
                     "launches_per_round": plan["launches"], "launches": launches},
        "losses": {"d_loss": st["d_loss"][0], "g_loss": st["g_loss"], "lambda": st["lambda"], "round": st["round"]},
    }
    if extra:
        out.update(extra)
    if world == 1 and not a.no_cpu_baseline:
        if cpu_leg is not None:
            out["cpu_baseline"] = cpu_leg()
        if parity_kind is not None:
            out["parity"] = parity_vs_cpu(parity_kind, a.batch)
    if emit:
        print(json.dumps(out), flush=True)
    return out


def main_mlp(a, world, rank):
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        step, _ = build_step(a, rank, world)
        ex = make_exchange(step, world, a)
        el = timed_rounds(lambda r: ex.round(r, graph=not a.eager), a, world, ex=ex)
        conv = conv_extra(a, world, rank)
    ring = ring_extra(a, world, rank)
    extra = {k: v for k, v in (("conv_round", conv), ("ring_round", ring)) if v}
    with torch.cuda.stream(stream):
        wl = ("C2: model/mnist_model.py MLP GAN, CAPGAN worker round (G fwd x2, D step, G loss, G bwd, Adam G/D), "
              "1 worker per GPU" if world == 1 else
              f"C3: CAPGAN {world} workers (1 per GPU), S=1, lambda-weighted G-gradient all-reduce + E={a.E} D "
              f"all-reduce over RCCL")
        return fused_report(a, world, rank, step, el, wl, {"img": "28x28x1", "dataset_rows_per_worker": a.rows},
                            cpu_leg=lambda: cpu_variants(lambda t: cpu_baseline(a, t)), parity_kind="capgan", ex=ex,
                            extra=extra or None)


def main_driver(a, world, rank, algo):
    """BASELINE configs[3] (mixg) / configs[4] (mdgan) through cglgan.driver: the reference's topology
    (server groups, Cloud), shards cut by allocate_dataset from a synthetic labelled dataset."""
    from cglgan.driver import Driver, DriverConfig
    S = 2 if (algo == "mixg" and world % 2 == 0) else 1
    cfg = DriverConfig(algo=algo, num_workers=world, num_servers=S, batch_size=a.batch,
                       num_communication=a.warmup + a.steps + a.profile_rounds + 8, cloud_epoch=1,
                       iid=1 if algo == "mdgan" else 0, swap_every=(a.E if (algo == "mdgan" and world > 1) else 0),
                       dataset_rows=max(60000, 8 * a.batch * world), graph=not a.eager)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        drv = Driver(cfg)
        el = timed_rounds(lambda r: drv.exchange.round(r, graph=cfg.graph), a, world)
        if algo == "mixg":
            wl = (f"C4: mixed-gan.py Mix-G, num_workers={world} num_servers={S} (one MixGenerator head per "
                  f"worker, trunk gradient all-reduced in each server group, Cloud trunk FedAvg every round)")
        else:
            wl = (f"C5: MD-GAN, num_workers={world}, non-IID (iid=1) shards, Sigmoid D + BCE, G on mean(l_i)"
                  + (f", D-swap every {a.E} rounds" if world > 1 else "") + " (fp32 GEMMs; the 16-bit GEMM "
                  "variant is 'lowp_variant')")
        lowp = None
        if algo == "mdgan" and a.lowp != "none":
            # the same workload with 16-bit GEMM operands (fp32 accumulation, fp32 master weights /
            # BatchNorm / losses / Adam): reported BESIDE the fp32 line, never as its value
            # f16 runs with dynamic loss scaling from torch's default initial scale (GradScaler semantics)
            scale16 = 65536.0 if a.lowp == "f16" else 0.0
            cfg16 = DriverConfig(**{**cfg.__dict__, "gemm_dtype": a.lowp, "loss_scale": scale16})
            drv16 = Driver(cfg16)
            el16 = timed_rounds(lambda r: drv16.exchange.round(r, graph=cfg16.graph), a, world)
            st16 = drv16.step.stats()
            lowp = {"gemm_dtype": a.lowp, "value": round(world * a.batch * a.steps / el16, 1), "unit": "images/s",
                    "ms_per_step": round(el16 / a.steps * 1e3, 4),
                    "losses": {"d_loss": st16["d_loss"][0], "g_loss": st16["g_loss"]},
                    "loss_scaling": ({"init": scale16, "scale_now": st16["loss_scale"], "skipped_steps": st16["skipped"]}
                                     if scale16 else None),
                    "parity": "unpinned (the reference has no 16-bit path); tests/test_gpu_lowp.py checks it "
                              "against an fp64 oracle restating the operand rounding (losses <= 1e-4; tensors "
                              "<= 0.1-0.35 of their distance to the exact fp64 round)"}
        return fused_report(a, world, rank, drv.step, el, wl,
                            {"img": "28x28x1", "num_servers": S, "shard_rows": int(drv.step.real.shape[0])},
                            cpu_leg=lambda: cpu_variants(lambda t: cpu_rounds(algo, a.batch, a.cpu_seconds, t)),
                            parity_kind=algo,
                            extra={"lowp_variant": lowp} if lowp else None, ex=drv.exchange)


def main_ring(a, world, rank, emit=True):
    """BASELINE configs[0]: CGLGAN/2DMG, one worker, the 2-D Gaussian-mixture ring (num_class=8), B=64."""
    from cglgan import GanStep, specs
    from cglgan.data import gmm
    from cglgan.init import default_init
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        torch.manual_seed(20211212 + rank)
        data, _ = gmm(8, 10000, device="cuda")       # CGLGAN/2DMG/main.py:456: num_sample = 10000 per mode
        gm, dm = specs.ring_generator(0), specs.ring_discriminator()
        step = GanStep(gm, dm, batch=a.batch, loss="bce", weighting="cglgan", n_workers=world, rank=rank,
                       gen_z=True, real=data, sample_n=data.shape[0])
        torch.manual_seed(20211212)
        default_init(gm, step.g_views)
        default_init(dm, step.d_views)
        step.reset()
        ex = make_exchange(step, world, a)
        el = timed_rounds(lambda r: ex.round(r, graph=not a.eager), a, world, ex=ex)
        wl = ("C1: CGLGAN/2DMG ring GAN (G 100-32-2, D 2-128-256-1 Sigmoid, BCE, closed-form lambda), 8-mode 2-D "
              "Gaussian mixture, 1 worker per GPU" + (f", {world} workers" if world > 1 else ""))
        return fused_report(a, world, rank, step, el, wl, {"data_points": int(data.shape[0])},
                            cpu_leg=lambda: cpu_variants(lambda t: cpu_rounds("ring", a.batch, a.cpu_seconds, t)),
                            parity_kind="ring", ex=ex, emit=emit)


def ring_extra(a, world, rank):
    """BASELINE configs[0] (the CGLGAN/2DMG 2-D Gaussian-mixture round, B=64) timed beside the default C2 line at
    N = 1: its own graph-replayed timed region (--ring-steps rounds), GEMM-family roofline, 10-round CPU parity and a
    short CPU-oracle sample.  A labelled extra key, never `value`."""
    if world != 1 or a.ring_steps <= 0:
        return None
    ra = argparse.Namespace(**vars(a))
    ra.model, ra.batch, ra.steps, ra.warmup = "ring", default_batch("ring"), a.ring_steps, 20
    ra.cpu_seconds = min(a.cpu_seconds, 3.0)
    out = main_ring(ra, world, rank, emit=False)
    if out is None:
        return None
    out["metric"] = METRIC + " [configs[0]: CGLGAN/2DMG 2-D Gaussian-mixture round]"
    out["note"] = ("third workload of the same bench run (BASELINE configs[0], B=%d), timed in its own region after "
                   "the C2 line's; not part of `value`; cpu_baseline is a %.0f s sample" % (ra.batch, ra.cpu_seconds))
    return out


# ------------------------------------------------------------------------------------------
# --gpus N > 1 without a launcher: this process spawns torch.distributed.run as a CHILD (never an exec) before
# anything touches the GPU, forwards the ranks' stdout (rank 0's JSON line) and exits with the launcher's status.
_RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
             "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
             "TORCHELASTIC_MAX_RESTARTS")


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(argv, n, port):
    """The child command: one rank per GPU on this node, rendezvous on 127.0.0.1 (the container's hostname may
    not resolve), this script with the caller's arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launcher_env(base=None):
    """The children's environment: the parent's, without any rank variables (the launcher sets its own), with
    dmabuf IPC for RCCL (HSA_ENABLE_IPC_MODE_LEGACY=0, the only IPC mode of this pool's host driver)."""
    env = dict(os.environ if base is None else base)
    for k in _RANK_ENV:
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONUNBUFFERED"] = "1"
    return env


def self_launch(n, argv):
    """Run this bench on n ranks through torch.distributed.run as a child process: every stdout line of the
    ranks is forwarded as it arrives; returns the launcher's exit status, or 1 when it succeeded without
    printing the JSON line."""
    import subprocess
    cmd = launcher_cmd(argv, n, free_port())
    print("bench: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, env=launcher_env(), stdout=subprocess.PIPE, text=True, bufsize=1)
    lines = 0
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
        if line.lstrip().startswith("{"):
            lines += 1
    rc = p.wait()
    if rc != 0:
        print(f"bench: torch.distributed.run exited with status {rc}", file=sys.stderr, flush=True)
        return rc
    if lines == 0:
        print("bench: no JSON line from rank 0", file=sys.stderr, flush=True)
        return 1
    return 0


def launch_selftest(mode):
    """The launcher plumbing on CPU (tests/test_bench_launcher.py): gloo group over the launcher's env, one
    all_reduce, rank 0 prints a JSON line with what each rank saw; mode "fail" makes rank 1 exit with status 3."""
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    if mode == "fail" and rank == 1:
        sys.exit(3)
    dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    seen = [None] * world
    dist.all_gather_object(seen, {"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"]),
                                  "master": f"{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}",
                                  "ipc_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")})
    if rank == 0:
        print(json.dumps({"selftest": True, "world": world, "sum": float(t.item()), "ranks": seen}), flush=True)
    dist.destroy_process_group()


def main():
    a = args_()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # (nothing has initialised the GPU yet: the child launcher owns the devices)
        sys.exit(self_launch(a.gpus, sys.argv[1:]))
    if a.launch_selftest:
        return launch_selftest(a.launch_selftest)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench: --gpus {a.gpus}, the launcher started {world} ranks: measuring {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
        if rank == 0:
            print(f"bench: {dist.get_world_size()} ranks, backend {dist.get_backend()}", file=sys.stderr, flush=True)
    try:
        if a.model == "lsgan":
            return main_lsgan(a, world, rank, local)
        if a.model in ("mixg", "mdgan"):
            return main_driver(a, world, rank, a.model)
        if a.model == "ring":
            return main_ring(a, world, rank)
        return main_mlp(a, world, rank)
    finally:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
