"""One conv configuration (Mconv2-5 shape, 128x256, stream-K 256) for counter passes;
window vs im2col via OPOSE_CONV_WINDOW, ablation via argv[1]."""
import ctypes as C, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src import _native
ab = int(sys.argv[1]) if len(sys.argv) > 1 else 0
mt, pt = (128, 128) if ab else (128, 256)
h = _native.Handle(0)
ms = C.c_float()
rc = _native.lib.opose_debug_conv_time(h.h, 32, 128, 23, 41, 128, 7, 2, mt, pt, 256 if pt == 256 else 512, ab, 5, C.byref(ms))
print(f"win={os.environ.get('OPOSE_CONV_WINDOW', '1')} ab={ab}: {ms.value:.3f} ms rc={rc}")
