# Fused heat-map resize + Gaussian NMS (gauss_nms_resize, OPOSE_FUSE_HEAT=1) vs heat_full_f32 + gauss_nms_wide
# (default): NMS / parity tests, then bench lines. Round 2: 1,860 vs 1,890 frames/s (fused 1.10 ms vs 0.90).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_gauss_screen.py tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_scale_shard.py > gpurun_out/pt_g.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_g.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pt_g.log | head; exit $rc; }
for f in 1 0; do
  OPOSE_FUSE_HEAT=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/b_$f.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$f.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; r=d['stage_roofline']
print('fuse$f', round(d['value'],1), round(d['ms_per_step'],3), {k: s[k] for k in ('heat_full','gauss_nms','gauss_nms_resize') if k in s}, {k: r[k]['frac'] for k in ('gauss_nms','gauss_nms_resize') if k in r})"
done
