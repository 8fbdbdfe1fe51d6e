#!/bin/bash
# Same-box A/B: ab_r5.so (the committed round-5 library) against the default library (+ the
# row-staged preprocess, upsample8 block maxima with
# gauss_nms_resize's coarse cold-tile test, and the register-resident person assembly);
# bench.py --steps 20: frames/s, C2 latency and the serial stage times of the changed kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for round in 1 2; do
for L in pytorch-openpose_amd/lib/ab_r5.so ""; do
  if [ -n "$L" ]; then export OPOSE_LIB=$L; else unset OPOSE_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab_bench.json 2>/dev/null || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/ab_bench.json').read().strip().splitlines()[-1])
s, q = d['stage_ms_per_step'], d['stage_ms_per_step_pipelined']
print('lib %s: %.1f frames/s  C2 %.3f ms  hand %.3f ms  serial preprocess %.4f upsample8 %.4f gauss %.4f assemble %.4f | pipelined gauss %.4f assemble %.4f conv3x3 %.3f' % ('${L:-default}', d['value'], d['latency_ms_single_frame'], d['c3_hand']['latency_ms'], s['preprocess'], s['upsample8'], s['gauss_nms_resize'], s['assemble'], q['gauss_nms_resize'], q['assemble'], q['conv3x3']))"
done
done
