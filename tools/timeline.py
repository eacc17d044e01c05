#!/usr/bin/env python3
"""Per-round kernel timeline of a rocprofv3 kernel trace (tuning aid).

    python tools/timeline.py <kernel_trace.csv | results.db> [--round-start cgl_step_begin]

Splits the trace into rounds at each launch of the round's first kernel and prints, for the
median round, every kernel's duration and the idle gap before it, plus round totals.
"""
import csv
import sqlite3
import statistics
import sys


def load(path):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e in c.execute("select name, start, end from kernels order by start"):
            rows.append((name, int(s), int(e)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        rows.sort(key=lambda x: x[1])
    return rows


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "cgl_step_begin"
    rows = [r for r in load(path) if r[0].startswith("cgl_") or "cgl_" in r[0]]
    starts = [i for i, r in enumerate(rows) if first in r[0]]
    rounds = [rows[a:b] for a, b in zip(starts, starts[1:])]
    if not rounds:
        print("no rounds found")
        return
    spans = [r[-1][2] - r[0][1] for r in rounds]
    med = sorted(range(len(rounds)), key=lambda i: spans[i])[len(rounds) // 2]
    rd = rounds[med]
    t0 = rd[0][1]
    busy = 0
    prev_end = None
    print(f"{len(rounds)} rounds; span median {statistics.median(spans) / 1e3:.1f} us, min {min(spans) / 1e3:.1f} us")
    print(f"{'#':>3} {'kernel':40s} {'start':>8s} {'dur':>8s} {'gap':>7s}")
    for i, (n, s, e) in enumerate(rd):
        gap = (s - prev_end) if prev_end is not None else 0
        busy += e - s
        print(f"{i:3d} {n.split('(')[0][:40]:40s} {(s - t0) / 1e3:8.2f} {(e - s) / 1e3:8.2f} {gap / 1e3:7.2f}")
        prev_end = e
    span = rd[-1][2] - rd[0][1]
    print(f"round span {span / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, gaps {(span - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
