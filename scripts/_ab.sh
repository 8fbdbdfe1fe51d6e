cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6.py > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
OPOSE_X6_MODE=2 AB_TAG=m2 timeout -k 10 120 python scripts/x6_ab.py > gpurun_out/ab.log 2>&1 &&
OPOSE_X6_MODE=1 AB_TAG=m1 timeout -k 10 120 python scripts/x6_ab.py >> gpurun_out/ab.log 2>&1 &&
OPOSE_X6_MODE=2 AB_TAG=m2 timeout -k 10 120 python scripts/x6_ab.py >> gpurun_out/ab.log 2>&1; cat gpurun_out/ab.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py > gpurun_out/pt2.log 2>&1; tail -3 gpurun_out/pt2.log
