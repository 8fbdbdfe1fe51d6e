"""A/B of the 7x7 / 3x3 conv kernels (im2col vs window) on the bench shapes."""
import ctypes as C, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src import _native
h = _native.Handle(0)
for name, N, Cin, H, W, Cout, ks, ng in [("Mconv2-5", 32, 128, 23, 41, 128, 7, 2), ("Mconv1", 32, 185, 23, 41, 256, 7, 1),
                                          ("conv4_2", 32, 512, 23, 41, 512, 3, 1), ("conv3_x", 32, 256, 46, 82, 256, 3, 1)]:
    flops = 2.0 * N * H * W * Cout * Cin * ks * ks * ng
    for sp in (0, 256):
        ms = C.c_float()
        rc = _native.lib.opose_debug_conv_time(h.h, N, Cin, H, W, Cout, ks, ng, 128, 256, sp, 0, 10, C.byref(ms))
        print(f"{os.environ.get('OPOSE_CONV_WINDOW', '1')} {name:9s} s{sp:<4d} {ms.value:7.3f} ms {flops / ms.value / 1e9:7.1f} TF/s rc={rc}", flush=True)
