cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for sc in 1 0; do
  OPOSE_GAUSS_SCREEN=$sc timeout -k 10 300 python scripts/pipeline_check.py > gpurun_out/dbg_$sc.log 2>&1 || exit 1
  echo "screen=$sc: $(grep -c frame gpurun_out/dbg_$sc.log) bad frames; $(tail -1 gpurun_out/dbg_$sc.log)"
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_gauss_screen.py tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_scale_shard.py tests/test_gpu_pipeline.py > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for sc in 1 0; do
  for p in 1 0; do
  OPOSE_GAUSS_SCREEN=$sc BENCH_PIPELINE=$p timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/b_$sc$p.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$sc$p.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; print('screen$sc pipe$p', round(d['value'],1), round(d['ms_per_step'],3), s['gauss_nms'])"
  done
done
