# C2 planner A/B (temporary env switches): device batch-1 latency + top layers per variant
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for v in "OPOSE_BIG_TBL=1" "X=0" "OPOSE_SMALL_WIN=1" "OPOSE_SMALL_WIN=1 OPOSE_BIG_TBL=1"; do
  env $v timeout -k 10 120 python scripts/c2_profile.py > "gpurun_out/c2ab_$v.log" 2>&1 || { echo "fail $v"; tail -3 "gpurun_out/c2ab_$v.log"; exit 1; }
  echo "== $v"; grep -v amdgpu "gpurun_out/c2ab_$v.log" | sed -n '1,2p;4,9p' | cut -c1-150
done
