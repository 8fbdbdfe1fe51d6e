# Staged cubic resize: resize / NMS / hand parity tests, then pipelined and serial bench lines
# (stage times of upsample8 and heat_full).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_gauss_screen.py tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_scale_shard.py tests/test_gpu_hand.py tests/test_gpu_batch_model.py > gpurun_out/pt_r.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_r.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pt_r.log | head; exit $rc; }
for pl in 1 0 1 0; do
  BENCH_PIPELINE=$pl timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/b_$pl.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$pl.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']
print('pipeline$pl', round(d['value'],1), round(d['ms_per_step'],3), {k: s[k] for k in ('upsample8','heat_full','gauss_nms','conv3x3') if k in s})"
done
