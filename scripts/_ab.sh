cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
AB_LAYERS=tiny3,tiny7_236,k7_c32 timeout -k 10 120 python scripts/x6_ab.py > gpurun_out/ab.log 2>&1; cat gpurun_out/ab.log
AB_TILE=128x256 AB_LAYERS=tiny3 timeout -k 10 120 python scripts/x6_ab.py > gpurun_out/ab.log 2>&1; cat gpurun_out/ab.log
