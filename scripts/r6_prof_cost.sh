#!/bin/bash
# Same box: the bench's timed steps with and without the 7x7 events (BENCH_NO_PROF), and the
# one- / two-handle loop of scripts/two_handles_ab.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
A="bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 --host-steps 2"
for r in 1 2; do
  timeout -k 10 200 python $A > gpurun_out/pc_prof_$r.log 2>&1 || exit 1
  BENCH_NO_PROF=1 timeout -k 10 200 python $A > gpurun_out/pc_noprof_$r.log 2>&1 || exit 1
  for f in prof noprof; do grep '^{' gpurun_out/pc_${f}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', $r, round(d['value'],1), round(d['ms_per_step'],3))"; done
done
timeout -k 10 300 python scripts/two_handles_ab.py --rounds 2 2>&1 | grep -v amdgpu.ids
