#!/bin/bash
# Bound on what a conflict-free 7x7 tap order could gain: pytorch-openpose_amd/lib/ab_bank.so is a
# timing-only build (wrong outputs) whose four k-groups of a chunk all read the same tap, so the
# B-fragment reads conflict only where a 16-pixel run crosses a row end.  Same box: bench.py
# --steps 20 (frames/s, serial 7x7 class ms) alternated with the default library, then one PMC
# pass (bank conflicts / LDS cycles) of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/bank && export TMPDIR=/tmp
for round in 1 2; do
for L in pytorch-openpose_amd/lib/ab_bank.so ""; do
  if [ -n "$L" ]; then export OPOSE_LIB=$L; else unset OPOSE_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --latency-iters 0 > gpurun_out/ab_bench.json 2>/dev/null || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/ab_bench.json').read().strip().splitlines()[-1])
print('lib %s: %.1f frames/s  serial conv7x7 %.4f ms  event mean 7x7 launch %.4f ms' % ('${L:-default}', d['value'], d['stage_ms_per_step']['conv7x7'], d['roofline']['mean_launch_ms']))"
done
done
for L in pytorch-openpose_amd/lib/ab_bank.so ""; do
  if [ -n "$L" ]; then export OPOSE_LIB=$L; else unset OPOSE_LIB; fi
  n=$([ -n "$L" ] && echo bank || echo base)
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES -d gpurun_out/bank/$n -o $n --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --latency-iters 0 > gpurun_out/bank/$n.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for n in ("bank", "base"):
    f = glob.glob(f"gpurun_out/bank/{n}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for row in csv.DictReader(open(f[0])):
        k = row["Kernel_Name"]
        if "conv_win_x6<128, 256, 7" not in k: continue
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    for k, v in acc.items():
        print(n, k[:60], {c: "%.4g" % x for c, x in v.items()}, "conflict/active %.3f" % (v["SQ_LDS_BANK_CONFLICT"] / v["SQ_LDS_IDX_ACTIVE"]))
PY
