#!/bin/bash
# Build libopose.so of a given commit (default HEAD) into alt_lib/<name>.so for same-box A/B runs
# (OPOSE_LIB=alt_lib/<name>.so python scripts/x6_ab.py).
set -e
REV=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/opose_alt && git -C "$ROOT" worktree add -f --detach /tmp/opose_alt "$REV" > /dev/null
make -C /tmp/opose_alt/pytorch-openpose_amd -j8 > /tmp/opose_alt_build.log 2>&1
mkdir -p "$ROOT/alt_lib" && cp /tmp/opose_alt/pytorch-openpose_amd/lib/libopose.so "$ROOT/alt_lib/$NAME.so"
git -C "$ROOT" worktree remove --force /tmp/opose_alt
echo "alt_lib/$NAME.so"
