# Round-4 planner check: targeted GPU tests, then the secondary configs (C2/C3/C5/f2) and the
# Hand per-layer table.  Each GPU step has its own time limit; stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${TESTS:-tests/test_gpu_x6.py tests/test_gpu_band.py tests/test_gpu_scale_shard.py tests/test_gpu_pipeline.py}
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu $T > gpurun_out/r4_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r4_tests.log | head -20; tail -3 gpurun_out/r4_tests.log; exit 1; }
tail -1 gpurun_out/r4_tests.log
timeout -k 10 600 python scripts/bench_configs.py > gpurun_out/r4_configs.log 2>&1 || { tail -5 gpurun_out/r4_configs.log; exit 1; }
grep '^{' gpurun_out/r4_configs.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); [print(k, v) for k, v in d.items() if k.startswith(('C2', 'C3_hand_lat', 'C5'))]"
timeout -k 10 200 python scripts/hand_profile_layers.py > gpurun_out/r4_hand_layers.log 2>&1 && head -1 gpurun_out/r4_hand_layers.log
