# 64x256 tile A/B: x6 accuracy tests, network variants, then per-layer times with / without it
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6.py tests/test_gpu_records.py tests/test_gpu_parity.py > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for t in 1 0; do
  OPOSE_X6_T64X256=$t timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 --detail > gpurun_out/t64_$t.log 2>&1 || exit 1
  grep -E "conv1_2|conv5_5|Mconv7_stage2" gpurun_out/t64_$t.log
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/t64_$t.log') if l.startswith('{')][-1]); print('t64=$t', round(d['value'],1), round(d['ms_per_step'],3), d['stage_ms_per_step']['conv3x3'])"
done
