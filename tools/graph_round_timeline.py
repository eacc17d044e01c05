#!/usr/bin/env python3
"""Per-launch durations and gaps of the graph-replayed MLP rounds from a rocprofv3 kernel trace.

    python tools/graph_round_timeline.py KERNEL_TRACE.csv [--json OUT] [--bench LOG]

Rounds start at the fused prologue GEMM (cgl_gemm_pro).  Only rounds with the plan's full launch count and
no host gap (graph replays back to back: the timed region) are used; per launch position the median of
its duration, of the gap before it (previous end -> its start) and of the round period are reported, and
the GEMM family's in-round average duration (cgl_gemm_f32 dispatches) -- the figure bench.py's
roofline.avg_gemm_launch_us is checked against.  --bench LOG (a bench.py JSON line: use the same commit's
UNPROFILED run -- under the kernel trace every eager launch's event timing grows ~4 us, which skews the line's
eager sum and its per-launch offset; r04y: 13.7 vs 9.7 us eager average, -8.3% against the trace instead of
-2.1%) recomputes the GEMM family's roofline fraction from the trace's timed rounds -- the line's
gemm_flops_per_round over the summed in-round cgl_gemm_f32 durations -- and compares it with roofline.frac."""
import argparse
import csv
import json
import statistics as S


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--json", default=None)
    p.add_argument("--marker", default="cgl_gemm_pro")
    p.add_argument("--bench", default=None)
    p.add_argument("--launches", type=int, default=None, help="launches per round (default: the most frequent count)")
    a = p.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lens = [starts[k + 1] - starts[k] for k in range(len(starts) - 1)]
    n = a.launches or S.mode(lens)
    rounds = []
    for k in range(len(starts) - 1):
        i0 = starts[k]
        if starts[k + 1] - i0 != n:
            continue
        rr = rows[i0:i0 + n]
        gaps = [0.0] + [(int(rr[j]["Start_Timestamp"]) - int(rr[j - 1]["End_Timestamp"])) / 1e3 for j in range(1, n)]
        if max(gaps) > 20.0:          # a host gap: not a back-to-back replay
            continue
        period = (int(rows[starts[k + 1]]["Start_Timestamp"]) - int(rr[0]["Start_Timestamp"])) / 1e3
        rounds.append((rr, gaps, period))
    if not rounds:
        raise SystemExit("no back-to-back rounds found")
    out = {"rounds": len(rounds), "launches": n, "period_us": S.median(r[2] for r in rounds), "per_launch": []}
    gemm = []
    for j in range(n):
        name = rounds[0][0][j]["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        du = [(int(r[0][j]["End_Timestamp"]) - int(r[0][j]["Start_Timestamp"])) / 1e3 for r in rounds]
        ga = [r[1][j] for r in rounds]
        wg = int(rounds[0][0][j]["Grid_Size_X"]) // int(rounds[0][0][j]["Workgroup_Size_X"])
        out["per_launch"].append({"i": j, "kernel": name, "wg": wg, "us": round(S.median(du), 2),
                                  "gap_us": round(S.median(ga), 2)})
        if name.startswith("cgl_gemm_f32<"):
            gemm += du
    out["busy_us"] = round(sum(x["us"] for x in out["per_launch"]), 2)
    out["gaps_us"] = round(sum(x["gap_us"] for x in out["per_launch"]), 2)
    out["gemm_f32_avg_us"] = round(S.mean(gemm), 3) if gemm else None
    out["gemm_f32_dispatches"] = len(gemm)
    for x in out["per_launch"]:
        print(f"{x['i']:3d} {x['us']:7.2f} gap {x['gap_us']:5.2f} wg {x['wg']:6d} {x['kernel'][:60]}")
    print(f"rounds {out['rounds']} launches {n} period {out['period_us']:.2f} us busy {out['busy_us']} gaps "
          f"{out['gaps_us']} gemm_f32 avg {out['gemm_f32_avg_us']} us over {len(gemm)} dispatches")
    if a.bench:
        line = [l for l in open(a.bench) if l.startswith('{"metric"')][-1]
        rl = json.loads(line)["roofline"]
        gus = sum(x["us"] for x in out["per_launch"] if x["kernel"].startswith("cgl_gemm_f32<"))
        frac = rl["gemm_flops_per_round"] / (gus * 1e-6) / 1e12 / rl["peak"]
        out["check"] = {"frac_trace": round(frac, 4), "frac_line": rl["frac"],
                        "rel_diff": round(rl["frac"] / frac - 1.0, 4),
                        "avg_gemm_us_trace": round(gus / max(1, rl["gemm_launches_per_round"]), 3),
                        "avg_gemm_us_line": rl["avg_gemm_launch_us"]}
        print("roofline check:", out["check"])
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
