# conv1_2 + pool with the input window in LDS (conv3_pool_win_x6, default) vs conv_x6's pooled
# launch over the im2col stream (OPOSE_CONV12_WIN=0): bit-identity tests, bench lines, per-layer
# times (pipelined and serial).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6.py -k "conv12" > gpurun_out/pt_w.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_w.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_w.log | head; exit $rc; }
for f in 1 0 1; do
  OPOSE_CONV12_WIN=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 --detail > gpurun_out/b_$f.log 2> gpurun_out/d_$f.log || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$f.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']
print('win$f', round(d['value'],1), round(d['ms_per_step'],3), {k: s[k] for k in ('conv3x3','conv7x7','gauss_nms','heat_full') if k in s})"
  grep -E "conv1_2|conv1_1" gpurun_out/d_$f.log || true
done
for f in 1 0; do
  BENCH_PIPELINE=0 OPOSE_CONV12_WIN=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 --detail > gpurun_out/bs_$f.log 2> gpurun_out/ds_$f.log || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/bs_$f.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']
print('serial win$f', round(d['value'],1), round(d['ms_per_step'],3), {k: s[k] for k in ('conv3x3',) if k in s})"
  grep -E "conv1_2|conv1_1" gpurun_out/ds_$f.log || true
done
