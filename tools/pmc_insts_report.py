"""Per-dispatch instruction mix of the MLP round's kernels from tools/pmc_insts.sh (one line per kernel shape of
the last profiled round, per-wave means): python tools/pmc_insts_report.py OUTDIR"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
order = []
for f in sorted(glob.glob(f"{d}/i*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "cgl_" not in n:
            continue
        key = (n.split("(")[0].replace("void ", "")[:34], int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
        if key not in acc:
            order.append(key)
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = ["SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
        "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_IFETCH", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
        "SQ_ACTIVE_INST_ANY", "SQC_ICACHE_MISSES", "SQC_ICACHE_HITS"]
short = {c: c.replace("SQ_INSTS_", "").replace("SQ_", "").replace("SQC_ICACHE_", "ic_").lower() for c in cols}
print(f"{'kernel':34s} {'wg':>5s} " + " ".join(f"{short[c]:>9s}" for c in cols) + "   (per wave; cycles in SQ units)")
for key in order:
    m = {k: sum(v) / len(v) for k, v in acc[key].items()}
    wv = m.get("SQ_WAVES", 1) or 1
    print(f"{key[0]:34s} {key[1]:5d} " + " ".join(f"{m.get(c, 0) / wv:9.1f}" for c in cols))
