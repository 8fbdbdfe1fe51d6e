import ctypes as C, os, sys
sys.path.insert(0, "/root/repo/pytorch-openpose_amd")
from src import _native
h = _native.Handle(0)
N, Cin, H, W, Cout, ks, ng = 32, 128, 23, 41, 128, 7, 2
flops = 2.0 * N * H * W * Cout * Cin * ks * ks * ng
for mt, pt, sp in ((128, 128, 512), (128, 128, 256), (128, 256, 256), (128, 256, 128)):
    ms = C.c_float()
    rc = _native.lib.opose_debug_conv_time(h.h, N, Cin, H, W, Cout, ks, ng, mt, pt, sp, 0, 10, C.byref(ms))
    print(f"{mt}x{pt} grid {sp}: {ms.value:.3f} ms {flops / ms.value / 1e9:.1f} TF/s", flush=True)
