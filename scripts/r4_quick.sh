cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 120 python scripts/c2_profile.py > gpurun_out/q_c2.log 2>&1 && grep -v amdgpu gpurun_out/q_c2.log | head -14 | cut -c1-150 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_x6.py tests/test_gpu_parity.py tests/test_gpu_scale_shard.py tests/test_gpu_records.py > gpurun_out/q_tests.log 2>&1; rc=$?; tail -1 gpurun_out/q_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/q_tests.log | head; exit 1; }
