"""Per-dispatch-shape means of the I-cache / wait counters of an I-cache counter pass (tools/pmc_icache.sh)."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    order = []
    for f in glob.glob(f"{d}/*/*_counter_collection.csv") + glob.glob(f"{d}/*_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "cgl_" not in n:
                continue
            short = n.split("(")[0].replace("void ", "")[:40]
            key = (short, int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
            if key not in acc:
                order.append(key)
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d)
    for key in order:
        m = {k: sum(v) / len(v) for k, v in acc[key].items()}
        wv = m.get("SQ_WAVES", 1) or 1
        print(f"  {key[0]:40s} wg={key[1]:5d} waves={wv:7.0f} icmiss={m.get('SQC_ICACHE_MISSES', 0):8.0f} "
              f"ichit={m.get('SQC_ICACHE_HITS', 0):9.0f} ifetch={m.get('SQ_IFETCH', 0):9.0f} "
              f"cyc/wave={m.get('SQ_WAVE_CYCLES', 0) / wv:7.0f} waitinst/wave={m.get('SQ_WAIT_INST_ANY', 0) / wv:6.0f} "
              f"wait/wave={m.get('SQ_WAIT_ANY', 0) / wv:7.0f}")
