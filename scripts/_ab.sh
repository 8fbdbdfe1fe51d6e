cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_records.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_scale_shard.py > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  BENCH_PIPELINE=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 5 > gpurun_out/b_$v.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$v.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; print('pipe$v', round(d['value'],1), d['ms_per_step'], d['latency_ms_single_frame'], s['assemble'], s['gauss_nms'], s['conv7x7'])"
done
