#!/bin/bash
# Timing-ablation builds of libopose (conv_x6.hip compiled with -DOPOSE_X6_ABL=<mask>) into
# alt_lib/abl<mask>.so; compare with OPOSE_LIB=alt_lib/abl<mask>.so python scripts/x6_ab.py.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/pytorch-openpose_amd
mkdir -p "$ROOT/alt_lib" /tmp/opose_abl
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -DOPOSE_X6_ABL=$m \
    -c "$PKG/csrc/conv_x6.hip" -o /tmp/opose_abl/conv_x6_$m.o
  objs=$(ls $PKG/build/*.o | grep -v conv_x6.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/alt_lib/abl$m.so" $objs /tmp/opose_abl/conv_x6_$m.o
  echo "alt_lib/abl$m.so"
done
