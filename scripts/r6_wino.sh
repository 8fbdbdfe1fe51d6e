#!/bin/bash
# Round-6 Winograd check: accuracy + network tests, then the serial per-layer bench with and
# without conv_wino_x6 (OPOSE_WINO=0).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py -x -v --timeout 120 --timeout-method thread -k "wino" > gpurun_out/r6_wino_tests.log 2>&1 || { tail -40 gpurun_out/r6_wino_tests.log; exit 1; }
grep -E "passed|failed|wino mean" gpurun_out/r6_wino_tests.log | tail -12
for wv in 1 0; do
  OPOSE_WINO=$wv BENCH_PIPELINE=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --latency-iters 0 --detail > gpurun_out/r6_wino_serial_$wv.log 2>&1 || { tail -20 gpurun_out/r6_wino_serial_$wv.log; exit 1; }
  grep '^{' gpurun_out/r6_wino_serial_$wv.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('WINO=$wv', round(d['value'],1), d['stage_ms_per_step'].get('conv3x3'), d['stage_ms_per_step'].get('conv7x7'))"
  grep -E "conv3|conv4|conv5_[123]" gpurun_out/r6_wino_serial_$wv.log | head -14
done
