"""Print one round's kernel timeline from a rocprofv3 rocpd database (kernel trace), with a
per-kernel-name summary of that round.  usage: python tools/round_timeline.py DB [marker]"""
import collections
import sqlite3
import sys

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "cgl_normal"
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, grid_x, grid_y, workgroup_x from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[0].startswith(marker)]
a, b = idx[-2], idx[-1]
tot = collections.defaultdict(lambda: [0, 0.0])
for r in rows[a:b]:
    d = (r[2] - r[1]) / 1000
    print(f"{d:8.2f} {r[3] // r[5]:7d}x{r[4]:<4d} {r[0][:70]}")
    k = r[0].split("(")[0].replace("void ", "")
    tot[k][0] += 1
    tot[k][1] += d
print(f"launches {b - a}  span {(rows[b][1] - rows[a][1]) / 1000:.1f} us  busy {sum(v[1] for v in tot.values()):.1f} us")
for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f"{d:9.1f} {n:4d} {k}")
