#!/bin/bash
# Same box, alternated: the pipelined bench on alt_lib/base.so (network <-> post events with the
# default system-scope fence) and on the library whose internal pipeline events skip it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
A="bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 --host-steps 10"
timeout -k 10 300 python -m pytest tests/test_gpu_records.py tests/test_gpu_c4_shard.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/se_tests.log 2>&1 || { tail -5 gpurun_out/se_tests.log; exit 1; }
tail -1 gpurun_out/se_tests.log
for r in 1 2 3; do
  for f in base new; do
    if [ $f = base ]; then export OPOSE_LIB=alt_lib/base.so; else unset OPOSE_LIB; fi
    timeout -k 10 200 python $A > gpurun_out/se_${f}_$r.log 2>&1 || exit 1
    grep '^{' gpurun_out/se_${f}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', $r, round(d['value'],1), round(d['ms_per_step'],3), 'h2h', round(d['value_host_to_host'],1), 'frac', round(r['frac'],4))"
  done
done
