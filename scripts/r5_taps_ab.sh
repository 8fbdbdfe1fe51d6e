#!/bin/bash
# Same-box A/B of the 7x7 tap order (tap7_of) and of computing the fragment offsets in block 4 MFMA
# gaps: ab_r5.so (committed: row-major taps, offsets at the chunk top), ab_place.so (row-major taps,
# offsets in block 4), the default library (tap7_of order, offsets in block 4). bench.py --steps 20
# alternated, then one PMC pass (bank conflicts / LDS cycles) of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/taps && export TMPDIR=/tmp
for round in 1 2; do
for L in pytorch-openpose_amd/lib/ab_r5.so pytorch-openpose_amd/lib/ab_place.so ""; do
  if [ -n "$L" ]; then export OPOSE_LIB=$L; else unset OPOSE_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --latency-iters 0 > gpurun_out/ab_bench.json 2>/dev/null || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/ab_bench.json').read().strip().splitlines()[-1])
print('lib %s: %.1f frames/s  serial conv7x7 %.4f ms  event mean 7x7 launch %.4f ms' % ('${L:-default}', d['value'], d['stage_ms_per_step']['conv7x7'], d['roofline']['mean_launch_ms']))"
done
done
for L in pytorch-openpose_amd/lib/ab_r5.so pytorch-openpose_amd/lib/ab_place.so ""; do
  if [ -n "$L" ]; then export OPOSE_LIB=$L; else unset OPOSE_LIB; fi
  n=$(case "$L" in *ab_r5*) echo base;; *ab_place*) echo place;; *) echo taps;; esac)
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES -d gpurun_out/taps/$n -o $n --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --latency-iters 0 > gpurun_out/taps/$n.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for n in ("base", "place", "taps"):
    f = glob.glob(f"gpurun_out/taps/{n}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for row in csv.DictReader(open(f[0])):
        k = row["Kernel_Name"]
        if "conv_win_x6<128, 256, 7" not in k: continue
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    for k, v in acc.items():
        print(n, k[:60], {c: "%.4g" % x for c, x in v.items()}, "conflict/active %.3f" % (v["SQ_LDS_BANK_CONFLICT"] / v["SQ_LDS_IDX_ACTIVE"]))
PY
