# Which stream should win the CUs in a pipelined step: network (default) or post-network
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
OPOSE_POST_PRIORITY=1 OPOSE_NET_PRIORITY=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_records.py > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1 0" "0 1" "1 0" "0 1" "0 0"; do
  set -- $cfg
  OPOSE_NET_PRIORITY=$1 OPOSE_POST_PRIORITY=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/p2_$1$2.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/p2_$1$2.log') if l.startswith('{')][-1]); print('net=$1 post=$2', round(d['value'],1), round(d['ms_per_step'],3))"
done
