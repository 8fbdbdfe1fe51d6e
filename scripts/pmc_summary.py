"""Aggregate rocprofv3 --pmc CSVs per kernel name (sum over dispatches)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(set)
for f in sorted(glob.glob(f"{root}/pmc*/*_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"][:70]
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        cnt[k].add((f, row["Dispatch_Id"]))
for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:int(sys.argv[2]) if len(sys.argv) > 2 else 8]:
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:18.4g}")
    if d.get("SQ_WAVE_CYCLES"):
        w = d["SQ_WAVE_CYCLES"]
        print("   wait_any %.3f wait_inst %.3f active %.3f" % (d.get("SQ_WAIT_ANY", 0) / w, d.get("SQ_WAIT_INST_ANY", 0) / w,
                                                         d.get("SQ_ACTIVE_INST_ANY", 0) / w))
