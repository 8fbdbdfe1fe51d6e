# Row-staged resize with LDS vertical taps: parity tests, then stage times
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_batch_model.py tests/test_gpu_hand.py tests/test_gpu_scale_shard.py tests/test_gpu_pipeline.py > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/pt.log | head; exit $rc; }
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/rs.log 2>&1 || exit 1
python -c "
import json; d=json.loads([l for l in open('gpurun_out/rs.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; print(round(d['value'],1), round(d['ms_per_step'],3), 'heat_full', s['heat_full'], 'upsample8', s['upsample8'])"
done
