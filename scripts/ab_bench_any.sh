#!/bin/bash
# Same-box A/B of pytorch-openpose_amd/lib/ab_base.so (the previous build) against the default
# library when the two may sum in different orders: raw outputs compared (printed, not required
# to be bit-identical), then bench.py --steps 20 alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OPOSE_LIB=pytorch-openpose_amd/lib/ab_base.so timeout -k 10 200 python scripts/ab_outputs.py save gpurun_out/ab_a.npz > /dev/null 2>&1 || exit 1
timeout -k 10 200 python scripts/ab_outputs.py save gpurun_out/ab_b.npz > /dev/null 2>&1 || exit 1
python scripts/ab_outputs.py compare gpurun_out/ab_a.npz gpurun_out/ab_b.npz > gpurun_out/ab_cmp.txt 2>&1; grep -v "^saved" gpurun_out/ab_cmp.txt | cut -c1-100 || true
for round in 1 2; do
for L in pytorch-openpose_amd/lib/ab_base.so ""; do
  if [ -n "$L" ]; then export OPOSE_LIB=$L; else unset OPOSE_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab_bench.json 2>/dev/null || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/ab_bench.json').read().strip().splitlines()[-1])
s = d['stage_ms_per_step']
print('lib %s: %.1f frames/s  C2 %.3f ms  hand %.3f ms  serial 3x3 %.4f 7x7 %.4f 1x1 %.4f assemble %.4f gauss %.4f | pipelined assemble %.4f gauss %.4f' % ('base' if '$L' else 'new', d['value'], d['latency_ms_single_frame'], d['c3_hand']['latency_ms'], s['conv3x3'], s['conv7x7'], s['conv1x1'], s['assemble'], s['gauss_nms_resize'], d['stage_ms_per_step_pipelined']['assemble'], d['stage_ms_per_step_pipelined']['gauss_nms_resize']))"
done
done
