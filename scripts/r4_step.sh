# Round-4 step check: the multi-handle graph repro, targeted GPU tests, a short bench line.
# Steps chained: the first failure ends the call.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 200 python -u scripts/r4_c5three.py c2,hand,l0 > gpurun_out/rs_repro.log 2>&1 || { echo "repro failed rc=$?"; grep -v amdgpu.ids gpurun_out/rs_repro.log | tail -8; exit 1; }
echo repro ok
T=${TESTS:-tests/test_gpu_x6.py tests/test_gpu_band.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_scale_shard.py tests/test_gpu_streams.py tests/test_gpu_pipeline.py}
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu $T > gpurun_out/rs_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/rs_tests.log | head -20; tail -3 gpurun_out/rs_tests.log; exit 1; }
tail -1 gpurun_out/rs_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --detail > gpurun_out/rs_bench.log 2>&1 || { tail -20 gpurun_out/rs_bench.log; exit 1; }
grep '^{' gpurun_out/rs_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['mean_launch_ms'], d.get('latency_ms_single_frame'), d.get('c3_hand', {}).get('latency_ms'))"
timeout -k 10 120 python scripts/c2_profile.py > gpurun_out/rs_c2.log 2>&1 && head -4 gpurun_out/rs_c2.log
