cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T="tests/test_gpu_x6.py tests/test_gpu_band.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_scale_shard.py tests/test_gpu_streams.py tests/test_gpu_pipeline.py"
OPOSE_LEAK_GRAPHS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $T > gpurun_out/g_leak2.log 2>&1; rc=$?; echo "leak rc=$rc"; grep -v "^Extension" gpurun_out/g_leak2.log | grep -E "passed|failed|Fatal|Segm|File .*(test_|src/)" | head -20
[ $rc -eq 0 ] || exit 1
OPOSE_SCALE_STREAMS=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $T > gpurun_out/g_serial2.log 2>&1; rc=$?; echo "serial rc=$rc"; grep -v "^Extension" gpurun_out/g_serial2.log | grep -E "passed|failed|Fatal|Segm|File .*(test_|src/)" | head -20
