#!/bin/bash
# The driver's GPU test list in one process, under a time limit; log in gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 ${2:-900} python -u -m pytest tests -x -v -s --timeout 200 --timeout-method thread -m gpu ${1:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error|Fatal|Segm" gpurun_out/gpu_tests.log | tail -5
exit $rc
