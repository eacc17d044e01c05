#!/usr/bin/env python3
"""Per-kernel HBM traffic per dispatch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json]

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters from TCC_EA0_RDREQ/WRREQ).  Per
MI355X_MICROARCH.md (HBM section) gfx950's FETCH_SIZE reports half the bytes of a wide (16 B per
lane) read, so the read bytes are FETCH_SIZE x 2; WRITE_SIZE is taken as is.  Infinity-Cache
hits are counted (not excluded), so this is memory-side fabric traffic, an upper bound on HBM.
"""
import collections
import csv
import json
import sys


def load(path, name):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            per[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return per


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(f) | set(w)):
        if "cgl" not in k:
            continue
        fb = 2.0 * 1024 * sum(f.get(k, [0])) / max(len(f.get(k, [1])), 1)
        wb = 1024 * sum(w.get(k, [0])) / max(len(w.get(k, [1])), 1)
        out[k] = {"dispatches": len(f.get(k, [])), "read_bytes_per_dispatch": fb, "write_bytes_per_dispatch": wb,
                  "bytes_per_dispatch": fb + wb}
        print(f"{k:40s} n={len(f.get(k, [])):5d} read {fb / 1e6:8.3f} MB  write {wb / 1e6:8.3f} MB per dispatch")
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
