#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for L in pytorch-openpose_amd/lib/ab_base.so "" pytorch-openpose_amd/lib/ab_base.so ""; do
  if [ -n "$L" ]; then OPOSE_LIB=$L timeout -k 10 200 python scripts/c5_ab.py || exit 1
  else timeout -k 10 200 python scripts/c5_ab.py || exit 1; fi
done 2>&1 | grep "^lib"
