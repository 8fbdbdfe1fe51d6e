"""Aggregate rocprofv3 CSVs per kernel (sum + per-dispatch mean) and emit the roofline traffic
record bench.py reports.

usage: python scripts/pmc_summary.py <prof_dir> [--json out.json] [--top N]
HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB; on
gfx950 FETCH_SIZE reads exactly half the bytes of a 16-B-per-lane coalesced stream, so the
read side is doubled (the conv kernel's weight tiles are 16-B LDS-DMA pieces; its im2col
gather is 4-B per lane and uncalibrated — see DESIGN.md)."""
import argparse
import csv
import glob
import json
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--json")
ap.add_argument("--top", type=int, default=6)
args = ap.parse_args()

agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for f in sorted(glob.glob(f"{args.root}/pmc*/*_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k][row["Counter_Name"]].add((f, row["Dispatch_Id"]))
trace = {}
for f in glob.glob(f"{args.root}/trace/*_kernel_stats.csv"):
    for row in csv.DictReader(open(f)):
        trace[row["Name"]] = row

out = {}
for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:args.top]:
    rec = {c: v / max(1, len(disp[k][c])) for c, v in d.items()}
    if "FETCH_SIZE" in rec and "WRITE_SIZE" in rec:
        rec["hbm_bytes_per_launch"] = (2 * rec["FETCH_SIZE"] + rec["WRITE_SIZE"]) * 1024
    if d.get("SQ_WAVE_CYCLES"):
        w = d["SQ_WAVE_CYCLES"]
        rec["wait_any_frac"] = d.get("SQ_WAIT_ANY", 0) / w
        rec["wait_inst_frac"] = d.get("SQ_WAIT_INST_ANY", 0) / w
        rec["active_frac"] = d.get("SQ_ACTIVE_INST_ANY", 0) / w
    if k in trace:
        rec["trace_calls"] = int(trace[k]["Calls"])
        rec["trace_avg_ns"] = float(trace[k]["AverageNs"])
    out[k] = rec
    print(k[:100])
    for c, v in sorted(rec.items()):
        print(f"   {c:28s} {v:18.6g}")
if args.json:
    # provenance: the library these counters were collected from (bench.py compares it with the
    # library it runs, so a stale summary is reported as such)
    import hashlib
    import os
    lib = os.environ.get("OPOSE_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                      "pytorch-openpose_amd", "lib", "libopose.so")
    out["_meta"] = {"libopose_md5": hashlib.md5(open(lib, "rb").read()).hexdigest()}
    json.dump(out, open(args.json, "w"), indent=1)
