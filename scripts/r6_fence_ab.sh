#!/bin/bash
# Same box, alternated: the bench (pipelined calls without a torch-stream marker) on the library
# whose 7x7 timing events fence system scope (alt_lib/base.so) and on the one whose events do not,
# plus BENCH_NO_PROF=1 (no events) as the floor.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
A="bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 --host-steps 4"
for r in 1 2; do
  OPOSE_LIB=alt_lib/base.so timeout -k 10 200 python $A > gpurun_out/fe_base_$r.log 2>&1 || exit 1
  timeout -k 10 200 python $A > gpurun_out/fe_new_$r.log 2>&1 || exit 1
  BENCH_NO_PROF=1 timeout -k 10 200 python $A > gpurun_out/fe_noprof_$r.log 2>&1 || exit 1
  for f in base new noprof; do grep '^{' gpurun_out/fe_${f}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', $r, round(d['value'],1), round(d['ms_per_step'],3), 'h2h', round(d['value_host_to_host'],1), 'frac', round(r['frac'],4), 'launch_ms', round(r['mean_launch_ms'],4), 'c7', d['stage_ms_per_step']['conv7x7'], 'c3', d['stage_ms_per_step']['conv3x3'])"; done
done
