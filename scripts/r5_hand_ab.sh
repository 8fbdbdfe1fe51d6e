#!/bin/bash
# same-box A/B of Hand(): the build in pytorch-openpose_amd/lib/ab_base.so against the tree's
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for L in pytorch-openpose_amd/lib/ab_base.so "" pytorch-openpose_amd/lib/ab_base.so ""; do
  if [ -n "$L" ]; then OPOSE_LIB=$L timeout -k 10 120 python scripts/hand_ab.py || exit 1
  else timeout -k 10 120 python scripts/hand_ab.py || exit 1; fi
done 2>&1 | grep -v amdgpu.ids
