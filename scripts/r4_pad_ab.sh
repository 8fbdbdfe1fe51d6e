# Same-box A/B of the X6P row pad, measured while the tree had kX6PPad = 16: alt_lib/pad3.so was
# that tree built with 3 (scripts/build_alt.sh on a worktree edited to 3).  The tree now has 3.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for r in 1 2; do for v in pad3 pad16; do
  if [ $v = pad3 ]; then export OPOSE_LIB=alt_lib/pad3.so; else unset OPOSE_LIB; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/ab_$v_$r.log 2>&1 || { echo fail; tail -3 gpurun_out/ab_$v_$r.log; exit 1; }
  echo "$v: $(grep '^{' gpurun_out/ab_$v_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), d['roofline']['mean_launch_ms'], d['roofline']['frac'])")"
done; done
