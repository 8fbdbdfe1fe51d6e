"""Times the split-bf16 conv kernel on the bench's layer shapes (32 frames of 184x328 input),
default tile/stream-K choice; one JSON line per shape.  A/B: OPOSE_LIB=<other build> (build_alt.sh),
AB_TILE=MTxPT, AB_SPLITS=<stream-K grids>."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src import _native  # noqa: E402

h = _native.Handle(0)
tag = os.environ.get("AB_TAG", "")
ms = C.c_float()
layers = os.environ.get("AB_LAYERS")
for name, N, Cin, H, W, Cout, ks, ng in [("Mconv2-5", 32, 128, 23, 41, 128, 7, 2), ("Mconv1", 32, 185, 23, 41, 256, 7, 1),
                                          ("conv1_2", 32, 64, 184, 328, 64, 3, 1),
                                          ("conv2_2", 32, 128, 92, 164, 128, 3, 1),
                                          ("conv3_x", 32, 256, 46, 82, 256, 3, 1),
                                          ("conv4_2", 32, 512, 23, 41, 512, 3, 1),
                                          ("stage1_3x3", 32, 128, 23, 41, 128, 3, 2),
                                          # K scan of the Mconv shape (intercept = per-launch fixed cost)
                                          ("k7_c32", 32, 32, 23, 41, 128, 7, 2), ("k7_c64", 32, 64, 23, 41, 128, 7, 2),
                                          ("k7_c256", 32, 256, 23, 41, 128, 7, 2),
                                          # tiny launches: per-launch overhead floor
                                          ("tiny3", 1, 32, 8, 8, 128, 3, 1), ("tiny7_236", 32, 32, 23, 41, 128, 7, 2)]:
    if layers and name not in layers.split(","):
        continue
    flops = 2.0 * N * H * W * Cout * Cin * ks * ks * ng
    for sp in [int(v) for v in os.environ.get("AB_SPLITS", "0").split(",")]:
        mt, pt = (128, 256) if sp else (0, 0)
        if os.environ.get("AB_TILE"):  # e.g. AB_TILE=256x128
            mt, pt = (int(v) for v in os.environ["AB_TILE"].split("x"))
        h.check(_native.lib.opose_debug_conv_x6_time(h.h, N, Cin, H, W, Cout, ks, ng, mt, pt, sp, 20, C.byref(ms)))
        print(json.dumps(dict(tag=tag + (f"sk{sp}" if sp else ""), layer=name, ms=round(ms.value, 4),
                              tf=round(flops / ms.value / 1e9, 1))), flush=True)
