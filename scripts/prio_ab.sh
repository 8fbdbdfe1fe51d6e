# Screened-NMS peak loss vs the network stream's priority; then the pipelined records test and
# the bench at both priorities (exact NMS)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for pr in 1 0; do
  OPOSE_NET_PRIORITY=$pr OPOSE_GAUSS_SCREEN=1 timeout -k 10 300 python scripts/pipeline_check.py > gpurun_out/prio_$pr.log 2>&1 || exit 1
  echo "priority=$pr screen=1: $(grep -c frame gpurun_out/prio_$pr.log) bad frames"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_records.py > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for pr in 1 0; do
  OPOSE_NET_PRIORITY=$pr timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/bp_$pr.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/bp_$pr.log') if l.startswith('{')][-1]); print('priority=$pr', round(d['value'],1), round(d['ms_per_step'],3))"
done
