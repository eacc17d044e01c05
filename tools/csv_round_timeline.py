"""One round's kernel timeline from a rocprofv3 kernel-trace CSV (--output-format csv), with a
per-kernel summary of that round.  usage: python tools/csv_round_timeline.py TRACE.csv [marker]"""
import collections
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "cgl_normal"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]          # the last full round before the bench's per-op profiling round
tot = collections.defaultdict(lambda: [0, 0.0])
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    wg = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    print(f"{d:8.2f} {wg:7d} vgpr={r['VGPR_Count']:>3s} scratch={r['Scratch_Size']:>4s} {r['Kernel_Name'][:64]}")
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    tot[k][0] += 1
    tot[k][1] += d
span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1000
print(f"launches {b - a}  span {span:.1f} us  busy {sum(v[1] for v in tot.values()):.1f} us")
for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f"{d:9.1f} {n:4d} {k}")
