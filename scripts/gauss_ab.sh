# Wide-tile vs 64x32 float64 Gaussian NMS (OPOSE_GAUSS_OLD=1): stress-map + parity tests, bench lines.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_gauss_screen.py tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_scale_shard.py > gpurun_out/pt_g.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_g.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pt_g.log | head; exit $rc; }
for old in 0 1 0 1; do
  env $( [ $old = 1 ] && echo OPOSE_GAUSS_OLD=1 ) timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/b_$old.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$old.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; print('old$old', round(d['value'],1), round(d['ms_per_step'],3), 'gauss', s['gauss_nms'], d['stage_roofline']['gauss_nms']['frac'])"
done
