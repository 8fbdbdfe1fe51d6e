#!/bin/bash
# The whole GPU test suite (as the driver runs it), then the Winograd serial A/B (opt-in kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r6_gpu_tests.log | tail -3
grep -E "keypoints across" gpurun_out/r6_gpu_tests.log | head
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r6_gpu_tests.log | head; exit $rc; }
for wv in 1 0; do
  OPOSE_WINO=$wv BENCH_PIPELINE=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --latency-iters 0 --detail > gpurun_out/r6_wino_serial_$wv.log 2>&1 || exit 1
  grep '^{' gpurun_out/r6_wino_serial_$wv.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('WINO=$wv', round(d['value'],1), d['stage_ms_per_step'].get('conv3x3'))"
done
