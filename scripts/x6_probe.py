"""Split-bf16 (x6) conv kernel: accuracy vs float64 and the fp32 MFMA kernel, and timing.

python scripts/x6_probe.py  -> one JSON line per case."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src import _native  # noqa: E402

lib = _native.lib
h = _native.Handle(0)


def ref64(x, w, b, pad, relu):
    y = torch.nn.functional.conv2d(torch.from_numpy(x).double(), torch.from_numpy(w).double(),
                                   torch.from_numpy(b).double(), padding=pad)
    return (y.clamp_min(0) if relu else y).numpy()


def run(fn, x, w, b, N, Cin, H, W, Cout, ks, relu, mt, pt, splits, *extra):
    out = np.empty((N, Cout, H, W), np.float32)
    rc = fn(h.h, x.ctypes.data, w.ctypes.data, b.ctypes.data, N, Cin, H, W, Cout, ks, ks // 2, relu, mt, pt, splits,
            *extra, out.ctypes.data)
    h.check(rc)
    return out


rng = np.random.default_rng(0)
cases = [(2, 64, 20, 24, 96, 3, 0, 0, 0), (2, 128, 23, 41, 128, 7, 0, 0, 0), (1, 3, 37, 45, 64, 3, 0, 0, 0),
         (2, 185, 17, 19, 128, 7, 128, 256, 0), (2, 128, 17, 19, 38, 1, 64, 64, 0), (3, 64, 30, 33, 128, 3, 128, 128, 37),
         (2, 128, 23, 41, 256, 7, 256, 128, 0), (2, 96, 23, 41, 128, 3, 128, 64, 0), (2, 96, 23, 41, 128, 3, 64, 128, 300)]
for (N, Cin, H, W, Cout, ks, mt, pt, splits) in cases:
    x = np.maximum(rng.standard_normal((N, Cin, H, W)).astype(np.float32), 0)
    w = (rng.standard_normal((Cout, Cin, ks, ks)) * np.sqrt(2.0 / (Cin * ks * ks))).astype(np.float32)
    b = rng.standard_normal(Cout).astype(np.float32) * 0.1
    r = ref64(x, w, b, ks // 2, 1)
    scale = np.abs(r).max()
    y32 = run(lib.opose_debug_conv, x, w, b, N, Cin, H, W, Cout, ks, 1, mt, pt, splits)
    y6 = run(lib.opose_debug_conv_x6, x, w, b, N, Cin, H, W, Cout, ks, 1, mt, pt, splits, 0)
    y6x = run(lib.opose_debug_conv_x6, x, w, b, N, Cin, H, W, Cout, ks, 1, mt, pt, splits, 1)
    absw = ref64(np.abs(x), np.abs(w), np.abs(b), ks // 2, 0)  # sum |a b|: the fp32 error scale
    e32 = np.abs(y32 - r) / np.maximum(absw, 1e-30)
    e6 = np.abs(y6 - r) / np.maximum(absw, 1e-30)
    print(json.dumps(dict(case=[N, Cin, H, W, Cout, ks, mt, pt, splits], f32_err_max=float(e32.max()),
                          f32_err_mean=float(e32.mean()), x6_err_max=float(e6.max()), x6_err_mean=float(e6.mean()),
                          x6_out_x6_equal=bool(np.array_equal(y6, y6x)), scale=float(scale))), flush=True)

ms = C.c_float()
for (N, Cin, H, W, Cout, ks, ng) in [(32, 128, 46, 82, 128, 7, 2), (32, 185, 46, 82, 256, 7, 1),
                                     (32, 256, 92, 164, 256, 3, 1), (32, 64, 368 // 2, 656 // 2, 64, 3, 1),
                                     (32, 128, 46, 82, 128, 3, 2), (1, 128, 46, 82, 128, 7, 2)]:
    flops = 2.0 * Cout * Cin * ks * ks * N * H * W * ng
    h.check(lib.opose_debug_conv_time(h.h, N, Cin, H, W, Cout, ks, ng, 0, 0, 0, 0, 10, C.byref(ms)))
    t32 = ms.value
    h.check(lib.opose_debug_conv_x6_time(h.h, N, Cin, H, W, Cout, ks, ng, 0, 0, 0, 10, C.byref(ms)))
    t6 = ms.value
    res = dict(shape=[N, Cin, H, W, Cout, ks, ng], f32_ms=t32, f32_tf=flops / t32 / 1e9, x6_ms=t6,
               x6_tf=flops / t6 / 1e9)
    for mt, pt in ((128, 256), (256, 128), (128, 128), (64, 128), (128, 64)):
        if (Cout if ng == 1 else Cout) % mt and Cout > 64:
            continue
        try:
            h.check(lib.opose_debug_conv_x6_time(h.h, N, Cin, H, W, Cout, ks, ng, mt, pt, 0, 10, C.byref(ms)))
            res["x6_%dx%d_dp_tf" % (mt, pt)] = flops / ms.value / 1e9
        except Exception as e:  # noqa: BLE001
            res["x6_%dx%d" % (mt, pt)] = str(e)[:60]
    print(json.dumps(res), flush=True)
