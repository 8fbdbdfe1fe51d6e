# Post-network latency kernels (peaks_finalize per (frame, part), limb_greedy register cache,
# paf_score per (pair, sample)): post parity tests, C2 breakdown, bench line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_gauss_screen.py tests/test_gpu_batch_model.py tests/test_gpu_scale_shard.py tests/test_gpu_pipeline.py > gpurun_out/pt_p.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_p.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_p.log | head; exit $rc; }
timeout -k 10 200 python scripts/c2_profile.py > gpurun_out/c2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/c2.log | head -3
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/bp.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/bp.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']
print('bench', round(d['value'],1), round(d['ms_per_step'],3), {k: s[k] for k in ('peaks_finalize','paf_score','limb_greedy','assemble') if k in s})"
done
