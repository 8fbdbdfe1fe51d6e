# Round-2 quick check: GPU tests, then one default bench line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_all.log 2>&1; rc=$?; tail -2 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | cut -c1-400
