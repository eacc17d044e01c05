#!/usr/bin/env python3
"""Traffic per dispatch of the conv round's dominant op (G Upsample(2) + Conv2d(128, 64) on the 2B
images of [z1; z2], model/lsgan.py:18-20) from the FETCH_SIZE / WRITE_SIZE passes of an eager conv
bench run.

    python tools/conv_traffic.py <fetch.csv> <write.csv> out.json [--commit SHA] [--command "..."]

The dominant op is the (kernel, grid) group of --kernel (default ``cgl_conv_fwd_halo``, the LDS-window
path the up-convolutions run since round 3; ``cgl_conv_fwd<2, 2, true>`` before) with the most bytes per
dispatch; read = FETCH_SIZE x 2 (gfx950 wide-read correction), write = WRITE_SIZE.  Algorithmic
bytes: the fp32 input [512, 16, 16, 128], the output [512, 32, 32, 64] and the weights, once each."""
import argparse
import collections
import csv
import json

KERNEL = "cgl_conv_fwd_halo"
GEOM = [512, 16, 16, 128, 64, 1, 1]
ALG = 4 * (512 * 16 * 16 * 128 + 512 * 32 * 32 * 64 + 64 * 128 * 9)


def load(path, name, kernel):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name and kernel in r["Kernel_Name"]:
            per[int(r["Grid_Size"])].append(float(r["Counter_Value"]) * 1024)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--commit", default=None)
    ap.add_argument("--command", default=None)
    ap.add_argument("--kernel", default=KERNEL)
    a = ap.parse_args()
    f, w = load(a.fetch, "FETCH_SIZE", a.kernel), load(a.write, "WRITE_SIZE", a.kernel)
    best = None
    for g, v in f.items():
        rb = 2.0 * sum(v) / len(v)
        wb = sum(w.get(g, [0.0])) / max(len(w.get(g, [])), 1)
        print(f"{a.kernel} grid {g:9d} n={len(v):4d} read {rb / 1e6:9.3f} MB write {wb / 1e6:9.3f} MB")
        if best is None or rb + wb > best[1] + best[2]:
            best = (g, rb, wb, len(v))
    if best is None:
        raise SystemExit(f"no {a.kernel} dispatches in {a.fetch}")
    g, rb, wb, n = best
    out = {"kernel": a.kernel, "op": "fwd", "geom": GEOM, "grid_threads": g, "dispatches": n,
           "read_bytes": rb, "write_bytes": wb, "bytes": rb + wb, "algorithmic_bytes": ALG, "ratio": (rb + wb) / ALG,
           "commit": a.commit, "command": a.command,
           "note": "G Upsample(2)+Conv2d(128, 64) on [z1; z2] (2B = 512 images), phase form; PMC FETCH_SIZE x2 "
                   "(gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE per dispatch, separate rocprofv3 --pmc "
                   "passes over bench.py --model lsgan (graph-replayed rounds)"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(f"dominant: grid {g}, {(rb + wb) / 1e6:.1f} MB per dispatch, {out['ratio']:.2f}x algorithmic")


if __name__ == "__main__":
    main()
