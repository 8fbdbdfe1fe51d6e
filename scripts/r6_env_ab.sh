#!/bin/bash
# Same box, alternated: runtime knobs for the bench process -- kernel arguments in device memory
# (HIP_FORCE_DEV_KERNARG=1) and more hardware queues per process (GPU_MAX_HW_QUEUES=8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
A="bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 3 --host-steps 20"
for r in 1 2; do
  for f in base kernarg hwq8; do
    unset HIP_FORCE_DEV_KERNARG GPU_MAX_HW_QUEUES
    [ $f = kernarg ] && export HIP_FORCE_DEV_KERNARG=1
    [ $f = hwq8 ] && export GPU_MAX_HW_QUEUES=8
    timeout -k 10 200 python $A > gpurun_out/ev_${f}_$r.log 2>&1 || exit 1
    grep '^{' gpurun_out/ev_${f}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', $r, round(d['value'],1), round(d['ms_per_step'],3), 'h2h', round(d['value_host_to_host'],1), 'frac', round(d['roofline']['frac'],4), 'c2', round(d['latency_ms_single_frame'],3), 'hand', round(d['c3_hand']['latency_ms'],3))"
  done
done
