#!/bin/bash
# Same-box bench.py --steps 20 over several libraries, alternated twice: arguments are library
# paths (OPOSE_LIB), "default" for the in-tree build.  No output comparison (see ab_bench.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2; do
for L in "$@"; do
  if [ "$L" != default ]; then export OPOSE_LIB=$L; else unset OPOSE_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab_bench.json 2>/dev/null || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/ab_bench.json').read().strip().splitlines()[-1])
s = d['stage_ms_per_step']
print('lib %s: %.1f frames/s  C2 %.3f ms  hand %.3f ms  serial 3x3 %.4f 7x7 %.4f 1x1 %.4f | 7x7 launch %.4f ms' % ('$L', d['value'], d['latency_ms_single_frame'], d['c3_hand']['latency_ms'], s['conv3x3'], s['conv7x7'], s['conv1x1'], d['roofline']['mean_launch_ms']))"
done
done
