#!/bin/bash
# Same box, alternated: the bench's 7x7 timing events per launch (alt_lib/base.so) vs one event
# pair per CPM stage's five 7x7 launches, and no events (BENCH_NO_PROF=1) as the floor.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
A="bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 --host-steps 10"
for r in 1 2 3; do
  for f in base new noprof; do
    unset OPOSE_LIB BENCH_NO_PROF
    [ $f = base ] && export OPOSE_LIB=alt_lib/base.so
    [ $f = noprof ] && export BENCH_NO_PROF=1
    timeout -k 10 200 python $A > gpurun_out/gr_${f}_$r.log 2>&1 || exit 1
    grep '^{' gpurun_out/gr_${f}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', $r, round(d['value'],1), round(d['ms_per_step'],3), 'h2h', round(d['value_host_to_host'],1), 'frac', round(r['frac'],4), 'launch_ms', round(r['mean_launch_ms'],4), 'c7', d['stage_ms_per_step']['conv7x7'])"
  done
done
