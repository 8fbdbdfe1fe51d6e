# Deferred post-processing (OPOSE_PIPELINE_DEFER) check and same-box bench A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_records.py tests/test_gpu_c4_shard.py > gpurun_out/df_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/df_tests.log | head; tail -3 gpurun_out/df_tests.log; exit 1; }
tail -1 gpurun_out/df_tests.log
for r in 1 2; do for d in 0 1; do
  BENCH_DEFER=$d timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/df_$d_$r.log 2>&1 || { echo fail; tail -3 gpurun_out/df_$d_$r.log; exit 1; }
  echo "defer=$d: $(grep '^{' gpurun_out/df_$d_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['mean_launch_ms'], d['roofline']['frac'])")"
done; done
BENCH_DEFER=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --latency-iters 0 --detail > gpurun_out/df_detail.log 2>&1 && grep -E "conv1_2|conv2_|conv3_1|conv4_1" gpurun_out/df_detail.log
