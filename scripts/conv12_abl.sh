# conv12_pool_x6 phase ablations (timing only): 0 full, 1 no conv1_1 math, 2 no conv1_2 loop, 3 neither
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for a in ${ABLS:-0 1 2 3}; do
  OPOSE_CONV12_ABL=$a timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --latency-iters 0 --detail > gpurun_out/ba_$a.log 2>gpurun_out/bda_$a.log || exit 1
  echo "abl $a: $(grep 'conv1_1+conv1_2' gpurun_out/bda_$a.log)"
done
