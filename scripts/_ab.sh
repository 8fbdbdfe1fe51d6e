cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1; tail -c 1500 gpurun_out/bench_full.log
