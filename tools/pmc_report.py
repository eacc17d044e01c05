"""Per-launch PMC summary of a tools/pmc_passes.sh run: for every cgl_* kernel dispatch shape
(kernel, grid), the mean of each counter over its dispatches and derived ratios."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
vgpr = {}
for f in glob.glob(f"{d}/*/runc/*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "cgl_" not in n:
            continue
        short = n.split("(")[0].replace("void ", "")
        key = (short, int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        vgpr[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"])
for key, cs in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0])) / max(1, len(kv[1].get("SQ_WAVE_CYCLES", [1])))):
    m = {k: sum(v) / len(v) for k, v in cs.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    out = [f"{key[0]:28s} wg={key[1]:5d} vgpr={vgpr[key]}"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in m:
            out.append(f"{k[3:]}={m[k] / wc:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
        out.append(f"mfma_busy/busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / max(m['SQ_BUSY_CYCLES'], 1):.3f}")
    if "TCP_TCC_READ_REQ_LATENCY" in m and "TCP_TCC_READ_REQ" in m:
        out.append(f"l2_lat={m['TCP_TCC_READ_REQ_LATENCY'] / max(m['TCP_TCC_READ_REQ'], 1):.0f}cyc")
    for k in ("TA_TA_BUSY", "TCP_PENDING_STALL_CYCLES", "TA_ADDR_STALLED_BY_TC_CYCLES", "SQ_LDS_BANK_CONFLICT",
              "SQ_INSTS_MFMA", "SQ_INSTS_VMEM_RD", "SQ_INST_LEVEL_VMEM", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES"):
        if k in m:
            out.append(f"{k}={m[k]:.3g}")
    print(" ".join(out))
