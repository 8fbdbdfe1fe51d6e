cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_hand.py tests/test_gpu_pipeline.py > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 3 > gpurun_out/b.log 2>&1; python -c "
import json; d=json.loads([l for l in open('gpurun_out/b.log') if l.startswith('{')][-1]); print(d['value'], d['latency_ms_single_frame'], d['stage_ms_per_step'])"
