"""Conv kernel timing sweep on the GPU (tile configs, split-K, ablations)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src import _native  # noqa: E402

h = _native.Handle(0)
cases = [  # name, N, Cin, H, W, Cout, ks, ngroups
    ("Mconv2-5 (grouped)", 32, 128, 23, 41, 128, 7, 2),
    ("Mconv1 (M=256)", 32, 185, 23, 41, 256, 7, 1),
    ("conv3_x", 32, 256, 46, 82, 256, 3, 1),
    ("conv1_2", 32, 64, 184, 328, 64, 3, 1),
    ("Mconv2 1 frame", 1, 128, 23, 41, 128, 7, 2),
]
variants = [(0, 0, 0, 0), (128, 128, 0, 0), (128, 128, 512, 0), (128, 256, 0, 0), (128, 256, 256, 0),
            (256, 128, 0, 0), (256, 128, 256, 0),
            (128, 128, 0, 3), (128, 128, 512, 3),
            (64, 128, 0, 0), (128, 64, 0, 0), (64, 64, 0, 0)]
only = sys.argv[1:] or None
for name, N, Cin, H, W, Cout, ks, ng in cases:
    flops = 2.0 * N * H * W * Cout * Cin * ks * ks * ng
    for mt, pt, sp, ab in variants:
        if mt and Cout % mt and not (Cout < 64):
            continue
        ms = C.c_float()
        rc = _native.lib.opose_debug_conv_time(h.h, N, Cin, H, W, Cout, ks, ng, mt, pt, sp, ab, 10, C.byref(ms))
        if rc:
            print(name, mt, pt, sp, ab, "rc", rc, _native.lib.opose_last_error(h.h))
            continue
        print(f"{name:22s} tile {mt:3d}x{pt:3d} s{sp} ablate {ab}: {ms.value:8.3f} ms  {flops / ms.value / 1e9:7.1f} TF/s",
              flush=True)
