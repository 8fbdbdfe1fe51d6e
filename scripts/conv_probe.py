"""Run one conv configuration repeatedly (for rocprofv3 counter passes).
usage: python scripts/conv_probe.py ABLATE [N Cin H W Cout ks ngroups]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src import _native  # noqa: E402

ab = int(sys.argv[1])
N, Cin, H, W, Cout, ks, ng = (int(v) for v in (sys.argv[2:9] if len(sys.argv) > 2 else (32, 128, 23, 41, 128, 7, 2)))
h = _native.Handle(0)
ms = C.c_float()
rc = _native.lib.opose_debug_conv_time(h.h, N, Cin, H, W, Cout, ks, ng, 128, 128, 512, ab, 5, C.byref(ms))
flops = 2.0 * N * H * W * Cout * Cin * ks * ks * ng
print(f"ablate {ab}: {ms.value:.3f} ms {flops / ms.value / 1e9:.1f} TF/s rc={rc}")
