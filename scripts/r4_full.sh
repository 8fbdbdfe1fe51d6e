# Full GPU test suite + smoke on the current tree (stops at the first failure)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pt_all.log 2>&1; rc=$?; tail -2 gpurun_out/r4_pt_all.log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "FAIL|Error|Fatal" gpurun_out/r4_pt_all.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -5 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
