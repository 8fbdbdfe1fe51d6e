import ctypes as C, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src import _native
h = _native.Handle(0)
for name, N, Cin, H, W, Cout, ks, ng in [("Mconv2-5", 32, 128, 23, 41, 128, 7, 2), ("Mconv big", 64, 128, 32, 64, 128, 7, 2)]:
    flops = 2.0 * N * H * W * Cout * Cin * ks * ks * ng
    for ab in (0, 128, 8, 1, 2, 3, 7):
        ms = C.c_float()
        rc = _native.lib.opose_debug_conv_time(h.h, N, Cin, H, W, Cout, ks, ng, 128, 128, 512, ab, 10, C.byref(ms))
        print(f"{name:10s} ablate {ab:2d}: {ms.value:7.3f} ms {flops / ms.value / 1e9:7.1f} TF/s rc={rc}", flush=True)
