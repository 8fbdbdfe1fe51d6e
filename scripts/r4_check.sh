# Round-4 check: targeted GPU tests, a short bench line with the per-layer table, and the Hand
# per-layer breakdown.  Each GPU step has its own time limit; stops at the first hard failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${TESTS:-tests/test_gpu_x6.py tests/test_gpu_band.py tests/test_gpu_parity.py}
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $T > gpurun_out/r4_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r4_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --detail > gpurun_out/r4_bench.log 2>&1 || { tail -20 gpurun_out/r4_bench.log; exit 1; }
grep '^{' gpurun_out/r4_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('latency_ms_single_frame'), d.get('c3_hand', {}).get('latency_ms'))"
timeout -k 10 200 python scripts/hand_profile_layers.py > gpurun_out/r4_hand_layers.log 2>&1 || exit 1
head -3 gpurun_out/r4_hand_layers.log
exit $rc
