# All GPU tests, smoke, then the secondary-config measurements (C2/C3/C5/f2/fast mode).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pt_all.log 2>&1; rc=$?; tail -2 gpurun_out/r4_pt_all.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r4_pt_all.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -5 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
timeout -k 10 600 python scripts/bench_configs.py > gpurun_out/r4_configs.log 2>&1 || { tail -5 gpurun_out/r4_configs.log; exit 1; }
grep '^{' gpurun_out/r4_configs.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); [print(k, v) for k, v in d.items()]"
timeout -k 10 200 python scripts/hand_profile_layers.py > gpurun_out/r4_hand_layers.log 2>&1 && head -1 gpurun_out/r4_hand_layers.log
