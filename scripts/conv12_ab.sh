# Fused conv1_1+conv1_2+pool vs the separate launches: x6 / parity tests, then bench lines.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6.py tests/test_gpu_parity.py tests/test_gpu_records.py > gpurun_out/pt_c12.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_c12.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_c12.log | head -20; exit $rc; }
for f in 1 0 1 0; do  # pipelined
  OPOSE_CONV12_FUSED=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 --detail > gpurun_out/b_$f.log 2>gpurun_out/bd_$f.log || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$f.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; print('fused$f', round(d['value'],1), round(d['ms_per_step'],3), 'conv3x3', s['conv3x3'])"
  grep "conv1_" gpurun_out/bd_$f.log | head -3
done
for f in 1 0; do
  BENCH_PIPELINE=0 OPOSE_CONV12_FUSED=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 --detail > gpurun_out/bs_$f.log 2>gpurun_out/bds_$f.log || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/bs_$f.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; print('serial fused$f', round(d['value'],1), round(d['ms_per_step'],3), 'conv3x3', s['conv3x3'])"
  grep "conv1_" gpurun_out/bds_$f.log | head -3
done
