# All GPU tests, smoke, then the secondary-config measurements (C2/C3/C5/fast mode).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
bash scripts/r2_full.sh || exit 1
timeout -k 10 600 python scripts/bench_configs.py > gpurun_out/configs.log 2>&1 || { tail -5 gpurun_out/configs.log; exit 1; }
grep '^{' gpurun_out/configs.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); [print(k, v) for k, v in d.items()]"
