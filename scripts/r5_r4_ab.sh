#!/bin/bash
# Same-box A/B of the round-4 library (pytorch-openpose_amd/lib/ab_base.so, built from 1949b92 by
# scripts/build_alt.sh) against the current one: C5 4-frame batch (scripts/c5_ab.py) and the bench
# line (frames/s, C2 latency, Hand), two alternations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for L in pytorch-openpose_amd/lib/ab_base.so "" pytorch-openpose_amd/lib/ab_base.so ""; do
  echo "== lib ${L:-default}"
  if [ -n "$L" ]; then export OPOSE_LIB=$L; else unset OPOSE_LIB; fi
  timeout -k 10 200 python scripts/c5_ab.py || exit 1
  BENCH_NO_PROF=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab_bench.json || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/ab_bench.json').read().strip().splitlines()[-1])
print('bench %.1f frames/s  C2 %.3f ms  hand %.3f ms  7x7 %.4f' % (d['value'], d['latency_ms_single_frame'], d['c3_hand']['latency_ms'], (d.get('roofline') or {}).get('mean_launch_ms') or 0))"
done 2>&1 | grep -v amdgpu.ids
