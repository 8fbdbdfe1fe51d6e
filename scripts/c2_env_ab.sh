#!/bin/bash
# C2 (one 368x656 frame, graph replay) under several environment settings, alternated twice:
# arguments are "NAME=VALUE" strings ("-" for none); scripts/c2_profile.py per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2; do
for E in "$@"; do
  echo "== $E"
  if [ "$E" = "-" ]; then timeout -k 10 200 python scripts/c2_profile.py 2>&1 | grep -v amdgpu.ids | head -${LINES_OUT:-4} || exit 1
  else env "$E" timeout -k 10 200 python scripts/c2_profile.py 2>&1 | grep -v amdgpu.ids | head -${LINES_OUT:-4} || exit 1; fi
done
done
