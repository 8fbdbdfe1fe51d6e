# Hand scales concurrent (default) vs sequential (OPOSE_SCALE_STREAMS=0): hand/pipeline tests, C3 numbers.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_hand.py tests/test_gpu_pipeline.py tests/test_gpu_batch_model.py tests/test_gpu_x6.py > gpurun_out/pt_h.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_h.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_h.log | head -20; exit $rc; }
for c in 1 0 1 0; do
  OPOSE_SCALE_STREAMS=$c timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bhh_$c.log 2>&1 || exit 1
  grep '^{' gpurun_out/bhh_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['c3_hand']; print('streams$c', round(d['value'],1), 'hand ms', round(c['latency_ms'],3), 'frac', round(c['conv_roofline']['frac'],3))"
done
