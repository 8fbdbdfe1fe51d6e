# Stream-ordering / records / pipeline GPU tests, then one bench line (host-to-host + CPU legs).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_streams.py tests/test_gpu_records.py tests/test_gpu_scale_shard.py > gpurun_out/pt_streams.log 2>&1; rc=$?; tail -3 gpurun_out/pt_streams.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_streams.log | head -20; exit $rc; }
timeout -k 10 400 python -X faulthandler bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['value_host_to_host'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['cpu_baseline']))"
