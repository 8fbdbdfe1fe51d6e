cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u scripts/bench_configs.py > gpurun_out/configs.json 2> gpurun_out/configs.err; rc=$?; tail -c 2000 gpurun_out/configs.json; tail -3 gpurun_out/configs.err; exit $rc
