#!/usr/bin/env python3
"""Per-descriptor tile search of the MLP round's GEMMs, measured in the round (MI355X).

For every GEMM descriptor i of the B=256 CAPGAN plan and every wave arrangement WM x WN x WK of a
256-thread workgroup, the plan is rebuilt with only descriptor i forced (CGL_GEMM_TILE_AT) and timed:
  * round: graph-replayed rounds between two events (the bench's quantity), interleaved with baseline
    rounds so that drift cancels;
  * launches: cgl_gan_profile per-launch device durations (dispatch begin / end) of a few rounds.
Then every descriptor takes its best arrangement and the combination is A/B'd against the cost model.

    python tools/tile_search.py [--rounds 300] [--reps 3] [--out gpurun_out/tile_search.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cgl-gan_amd"))

import torch  # noqa: E402

OPTS = [(1, 1, 4), (2, 1, 2), (1, 2, 2), (2, 2, 1), (4, 1, 1), (1, 4, 1)]


def build(real, force):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    if force:
        os.environ["CGL_GEMM_TILE_AT"] = force
    else:
        os.environ.pop("CGL_GEMM_TILE_AT", None)
    gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
    step = GanStep(gm, dm, batch=256, batch_real=256, epoch=1, loss="ce", weighting="capgan", n_workers=1, rank=0,
                   seed=20211212, gen_z=True, real=real, sample_n=real.shape[0])
    torch.manual_seed(20211212)
    default_init(gm, step.g_views)
    torch.manual_seed(20211213)
    default_init(dm, step.d_views)
    step.reset(beta=[1.0])
    return step


def time_rounds(step, n):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        step.run(graph=True)
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def measure(real, force, rounds, prof_rounds=5):
    step = build(real, force)
    for _ in range(30):
        step.run(graph=True)
    torch.cuda.synchronize()
    us = time_rounds(step, rounds)
    prof = [step.profile_round() for _ in range(prof_rounds)]
    kinds = [k for k, _, _ in step.launches()]
    st = step.stats()
    ok = all(map(lambda v: v == v and abs(v) < 1e6, [st["d_loss"][0], st["g_loss"]]))
    step.close()
    per = [sorted(col)[len(col) // 2] for col in zip(*prof)]      # median per launch
    return {"round_us": us, "launch_us": per, "kinds": kinds, "finite": ok}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=300)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--ndesc", type=int, default=24)
    p.add_argument("--descs", default="", help="comma list of descriptor indices (default: all)")
    p.add_argument("--opts", default="", help="semicolon list WM,WN,WK[,T] (default: the 6 arrangements)")
    p.add_argument("--final", default="", help="only A/B this CGL_GEMM_TILE_AT string against the default")
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tile_search.json"))
    a = p.parse_args()
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    res = {"base": [], "trials": {}, "final": None}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with torch.cuda.stream(s):
        g = torch.Generator(device="cuda").manual_seed(1000)
        real = torch.rand(60000, 784, device="cuda", generator=g) * 2 - 1
        opts = [tuple(int(x) for x in o.split(",")) for o in a.opts.split(";")] if a.opts else OPTS
        descs = [int(x) for x in a.descs.split(",")] if a.descs else list(range(a.ndesc))
        if not a.final:
            t0 = time.time()
            for i in descs:
                for rep in range(a.reps):
                    b = measure(real, "", a.rounds)
                    res["base"].append(b["round_us"])
                    for o in opts:
                        f = f"{i}:" + ",".join(map(str, o))
                        m = measure(real, f, a.rounds)
                        res["trials"].setdefault(f, []).append({"round_us": m["round_us"], "base_us": b["round_us"],
                                                                "launch_us": m["launch_us"], "finite": m["finite"]})
                best = min(res["trials"].items() if False else
                           [(f, v) for f, v in res["trials"].items() if f.startswith(f"{i}:")],
                           key=lambda kv: sum(t["round_us"] - t["base_us"] for t in kv[1]) / len(kv[1]))
                d = sum(t["round_us"] - t["base_us"] for t in best[1]) / len(best[1])
                print(f"desc {i:2d}: best {best[0]:12s} {d:+7.2f} us vs cost model  ({time.time() - t0:.0f} s)",
                      flush=True)
                json.dump(res, open(a.out, "w"))
            picks = []
            for i in descs:
                cand = [(f, sum(t["round_us"] - t["base_us"] for t in v) / len(v))
                        for f, v in res["trials"].items() if f.startswith(f"{i}:")]
                f, d = min(cand, key=lambda x: x[1])
                if d < -0.3:
                    picks.append(f)
            a.final = ";".join(picks)
        print("final:", a.final, flush=True)
        ab = {"default": [], "forced": []}
        for rep in range(5):
            ab["default"].append(measure(real, "", a.rounds))
            ab["forced"].append(measure(real, a.final, a.rounds))
        res["final"] = {"force": a.final,
                        "default_round_us": [m["round_us"] for m in ab["default"]],
                        "forced_round_us": [m["round_us"] for m in ab["forced"]],
                        "default_launch_us": ab["default"][-1]["launch_us"],
                        "forced_launch_us": ab["forced"][-1]["launch_us"],
                        "kinds": ab["default"][-1]["kinds"]}
        print("default", [round(m["round_us"], 2) for m in ab["default"]], flush=True)
        print("forced ", [round(m["round_us"], 2) for m in ab["forced"]], flush=True)
        json.dump(res, open(a.out, "w"))


if __name__ == "__main__":
    main()
