# Hand() slab-table sweep (OPOSE_HAND_SLABS, temporary): one crop latency per table
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for t in "16,12,8,7,4,2,1" "24,16,12,8,4,2,1" "28,21,12,7,4,2,1" "24,20,12,6,4,2,1" "12,8,6,5,4,2,1"; do
  OPOSE_HAND_SLABS=$t timeout -k 10 120 python scripts/hand_profile_layers.py > gpurun_out/hs_$t.log 2>&1 || { echo "fail $t"; tail -5 gpurun_out/hs_$t.log; exit 1; }
  echo "$t: $(head -1 gpurun_out/hs_$t.log)"
done
