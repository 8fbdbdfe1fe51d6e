cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 200 python scripts/hand_profile_layers.py > gpurun_out/r4_hand_layers.log 2>&1 && head -1 gpurun_out/r4_hand_layers.log &&
OPOSE_BIG_TBL=1 timeout -k 10 200 python scripts/hand_profile_layers.py > gpurun_out/r4_hand_layers_big.log 2>&1 && head -1 gpurun_out/r4_hand_layers_big.log &&
timeout -k 10 600 python scripts/bench_configs.py > gpurun_out/r4_configs.log 2>&1 && grep '^{' gpurun_out/r4_configs.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); [print(k, v) for k, v in d.items()]"
