#!/bin/bash
# Round-6 evidence on the final library: the default bench line (with the CPU baseline), a serial
# per-layer breakdown, the Hand per-layer breakdown, the C2 trace over graph replays, then
# rocprofv3 kernel stats + PMC passes (scripts/gpu_profile.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 > gpurun_out/r6_bench.log 2>&1 || { tail -5 gpurun_out/r6_bench.log; exit 1; }
grep '^{' gpurun_out/r6_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['value_host_to_host'], d['value_host_to_host_ratio'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['mean_launch_ms'], d['cpu_baseline']['value'], d['c3_hand']['latency_ms'], d['latency_ms_single_frame'], d['host_to_host'])"
BENCH_PIPELINE=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --latency-iters 0 --detail > gpurun_out/r6_bench_serial.log 2>&1 || exit 1
timeout -k 10 200 python scripts/hand_profile_layers.py > gpurun_out/r6_hand_layers.log 2>&1 || exit 1
bash scripts/gpu_profile.sh
