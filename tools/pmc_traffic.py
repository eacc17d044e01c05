#!/usr/bin/env python3
"""Per-kernel HBM traffic per dispatch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json]
                                [--commit SHA] [--command "..."]

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters from TCC_EA0_RDREQ/WRREQ).  Per
MI355X_MICROARCH.md (HBM section) gfx950's FETCH_SIZE reports half the bytes of a wide (16 B per
lane) read, so the read bytes are FETCH_SIZE x 2; WRITE_SIZE is taken as is.  Infinity-Cache
hits are counted (not excluded), so this is memory-side fabric traffic, an upper bound on HBM.
Every template instantiation of a kernel is also summed into one "<family> (all instantiations)"
entry (dispatch-weighted), which is what bench.py's roofline.traffic reads for the GEMM family.
"""
import argparse
import collections
import csv
import json
import re


def load(path, name):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            per[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return per


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
    if a.out:
        meta = {"commit": a.commit, "command": a.command,
                "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; read = FETCH_SIZE x 2 "
                          "(gfx950 wide-read correction), write = WRITE_SIZE; memory-side fabric bytes incl. "
                          "Infinity-Cache hits"}
        json.dump({"_meta": meta, **out}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
