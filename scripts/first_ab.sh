# conv1_1 direct kernel check: x6 + parity tests, then per-layer times
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6.py tests/test_gpu_parity.py tests/test_gpu_records.py > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 --detail > gpurun_out/first.log 2>&1 || exit 1
grep -E "conv1_1|conv1_2/" gpurun_out/first.log
python -c "
import json; d=json.loads([l for l in open('gpurun_out/first.log') if l.startswith('{')][-1]); print(round(d['value'],1), round(d['ms_per_step'],3), d['stage_ms_per_step']['conv3x3'])"
