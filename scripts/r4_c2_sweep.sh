# TEMP: C2 7x7 (tile, slabs) sweep via OPOSE_FORCE7
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
for v in "128,64,16" "128,64,20" "128,64,24" "128,64,32" "64,64,16" "64,64,24" "64,128,24" "64,128,32"; do
  OPOSE_FORCE7=$v timeout -k 10 120 python scripts/c2_profile.py > "gpurun_out/c2s_$v.log" 2>&1 || { echo "fail $v"; tail -3 "gpurun_out/c2s_$v.log"; exit 1; }
  echo "[$v] $(grep -v amdgpu "gpurun_out/c2s_$v.log" | head -1) | $(grep -v amdgpu "gpurun_out/c2s_$v.log" | sed -n 2p | cut -c1-40) | $(grep -m1 'Mconv2_stage3' "gpurun_out/c2s_$v.log" | cut -c1-100)"
done
