#!/usr/bin/env python3
"""Per-kernel HBM traffic per dispatch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json]
                                [--commit SHA] [--command "..."] [--plan PLAN_DEBUG_LOG]

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters from TCC_EA0_RDREQ/WRREQ).  Per
MI355X_MICROARCH.md (HBM section) gfx950's FETCH_SIZE reports half the bytes of a wide (16 B per
lane) read, so the read bytes are FETCH_SIZE x 2; WRITE_SIZE is taken as is.  Infinity-Cache
hits are counted (not excluded), so this is memory-side fabric traffic, an upper bound on HBM.
Every template instantiation of a kernel is also summed into one "<family> (all instantiations)"
entry (dispatch-weighted), which is what bench.py's roofline.traffic reads for the GEMM family.

Per launch: the dispatches are cut into rounds at the fused prologue GEMM (cgl_gemm_pro) and, per position
in the round, the median bytes are reported ("per_launch").  With --plan (the stderr of the same run under
CGL_PLAN_DEBUG=1) every GEMM launch also gets its algorithmic bytes -- each descriptor's compulsory
A (M x K) + B (N x K) reads and C (M x N) write in f32 -- and the measured / algorithmic ratio.
"""
import argparse
import collections
import csv
import json
import re
import statistics


def load(path, name):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            per[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def load_rows(path, name):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            rows.append((int(r["Dispatch_Id"]), kname(r["Kernel_Name"]), float(r["Counter_Value"])))
    rows.sort()
    return rows


def kname(k):
    """Kernel name without its argument list ('(anonymous namespace)::' prefixes dropped first)."""
    return k.replace("(anonymous namespace)::", "").split("(")[0]


def rounds_of(rows, marker="cgl_gemm_pro"):
    starts = [i for i, r in enumerate(rows) if marker in r[1]]
    if len(starts) < 2:
        return []
    n = statistics.mode(starts[k + 1] - starts[k] for k in range(len(starts) - 1))
    return [rows[s:s + n] for k, s in enumerate(starts[:-1]) if starts[k + 1] - s == n]


def plan_gemm_bytes(path):
    """Algorithmic f32 bytes per GEMM launch, in round order, from CGL_PLAN_DEBUG lines."""
    launches, key, phase, last = [], None, 0, -1
    for line in open(path):
        m = re.match(r"gemm launch (\d+): desc \d+ layout (\d) M (\d+) N (\d+) K (\d+)", line)
        if not m:
            continue
        li, lay, M, N, K = (int(x) for x in m.groups())
        if li < last:
            phase += 1
        last = li
        if key != (phase, li):
            launches.append(0)
            key = (phase, li)
        launches[-1] += 4 * (M * K + N * K + M * N)
    return launches


def family(k):
    m = re.match(r"(?:void )?(\w+)<", k)
    return m.group(1) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--commit", default=None)
    ap.add_argument("--command", default=None)
    ap.add_argument("--plan", default=None)
    ap.add_argument("--marker", default="cgl_gemm_pro", help="first kernel of a round")
    a = ap.parse_args()
    f = load(a.fetch, "FETCH_SIZE")
    w = load(a.write, "WRITE_SIZE")
    out, fam = {}, collections.defaultdict(lambda: [0, 0.0, 0.0])
    for k in sorted(set(f) | set(w)):
        if "cgl" not in k:
            continue
        n = len(f.get(k, []))
        fb = 2.0 * 1024 * sum(f.get(k, [0])) / max(n, 1)
        wb = 1024 * sum(w.get(k, [0])) / max(len(w.get(k, [1])), 1)
        out[k] = {"dispatches": n, "read_bytes_per_dispatch": fb, "write_bytes_per_dispatch": wb,
                  "bytes_per_dispatch": fb + wb}
        print(f"{k:48s} n={n:5d} read {fb / 1e6:8.3f} MB  write {wb / 1e6:8.3f} MB per dispatch")
        fk = family(k)
        if fk:
            fam[fk][0] += n
            fam[fk][1] += fb * n
            fam[fk][2] += wb * n
    for fk, (n, fbs, wbs) in fam.items():
        if n:
            key = f"{fk} (all instantiations)"
            out[key] = {"dispatches": n, "read_bytes_per_dispatch": fbs / n, "write_bytes_per_dispatch": wbs / n,
                        "bytes_per_dispatch": (fbs + wbs) / n}
            print(f"{key:48s} n={n:5d} read {fbs / n / 1e6:8.3f} MB  write {wbs / n / 1e6:8.3f} MB per dispatch")
    rf, rw = (rounds_of(load_rows(a.fetch, "FETCH_SIZE"), a.marker),
              rounds_of(load_rows(a.write, "WRITE_SIZE"), a.marker))
    per_launch = []
    if rf and rw and len(rf[0]) == len(rw[0]):
        alg = plan_gemm_bytes(a.plan) if a.plan else []
        gi = 0
        for j in range(len(rf[0])):
            name = rf[0][j][1].replace("void ", "")
            fb = 2.0 * 1024 * statistics.median(r[j][2] for r in rf)
            wb = 1024 * statistics.median(r[j][2] for r in rw)
            e = {"i": j, "kernel": name, "read_bytes": fb, "write_bytes": wb, "bytes": fb + wb}
            if name.startswith("cgl_gemm_f32<") or name.startswith("cgl_gemm_pro<"):
                if gi < len(alg):
                    e["algorithmic_bytes"] = alg[gi]
                    e["ratio"] = round((fb + wb) / alg[gi], 3)
                gi += 1
            per_launch.append(e)
            print(f"{j:3d} {name[:36]:36s} read {fb / 1e6:7.3f} MB write {wb / 1e6:7.3f} MB"
                  + (f"  alg {e['algorithmic_bytes'] / 1e6:7.3f} MB ratio {e['ratio']:.2f}" if "ratio" in e else ""))
        out["per_launch"] = per_launch
        out["rounds"] = min(len(rf), len(rw))
    if a.out:
        meta = {"commit": a.commit, "command": a.command,
                "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; read = FETCH_SIZE x 2 "
                          "(gfx950 wide-read correction), write = WRITE_SIZE; memory-side fabric bytes incl. "
                          "Infinity-Cache hits"}
        json.dump({"_meta": meta, **out}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
