#!/bin/bash
# Round-6 host-to-host A/B: sync / stream / round-5 passes alternated, then one kernel + copy trace
# per mode, with the per-step network gaps (scripts/h2h_trace_gaps.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u scripts/h2h_ab.py --steps 10 --rounds 3 > gpurun_out/r6_h2h_ab.log 2>&1 || { tail -20 gpurun_out/r6_h2h_ab.log; exit 1; }
grep leg gpurun_out/r6_h2h_ab.log | python -c "import sys,json; [print(d['leg'], d['round'], round(d['value'],1), round(d['ms'],3)) for d in map(json.loads, sys.stdin)]"
for m in sync old; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/h2h_trace_$m -o run -- python3 scripts/h2h_ab.py --steps 8 --rounds 1 --only $m > gpurun_out/r6_h2h_trace_$m.log 2>&1 || { tail -20 gpurun_out/r6_h2h_trace_$m.log; exit 1; }
  python scripts/h2h_trace_gaps.py gpurun_out/h2h_trace_$m/run > gpurun_out/r6_h2h_gaps_$m.txt && tail -12 gpurun_out/r6_h2h_gaps_$m.txt
done
