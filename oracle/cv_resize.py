"""ORACLE (test infrastructure only): OpenCV ``cv2.resize(..., INTER_CUBIC)`` restated in NumPy.

The reference calls cv2.resize at `src/body.py:38,55,57,61,63` and
`src/hand.py:38,53,55`.  opencv-python is unpinned (`requirements.txt:3`) and
absent from this image, so this module restates the *generic scalar* path of
OpenCV's `resizeGeneric_` (imgproc/resize.cpp) as published:

* dsize = (cvRound(w*fx), cvRound(h*fy)) when dsize is empty, and the inverse
  scale used for the source mapping is 1/fx; otherwise scale = 1/(dw/sw).
* src coordinate  f = (float)((d + 0.5) * scale - 0.5);  s = floor(f);  f -= s
* coefficients    interpolateCubic(f) with A = -0.75, float32, no FMA.
* border          replicate (tap index clamped to [0, n-1]).
* uint8 images    coefficients saturate_cast<short>(c*2048); horizontal int sum,
                  vertical int sum, (v + 2^21) >> 22, saturate to [0,255].
* float32 images  horizontal ((p0+p1)+p2)+p3 then vertical ((q0+q1)+q2)+q3 in
                  float32.
* dsize == ssize  plain copy.

Parity status: UNPINNED against real OpenCV (no cv2 build or golden resize
output exists in the reference); OpenCV's SIMD uint8 vertical pass (float
muladd) can differ by 1 LSB from the generic path restated here.  The golden
fixtures produced by `oracle/gen_golden.py` route the reference's cv2.resize
calls through this module, so they pin everything *around* the resize.
"""
from __future__ import annotations

import numpy as np

_A = np.float32(-0.75)
_F32 = np.float32


def cubic_coeffs(fx: np.ndarray) -> np.ndarray:
    """OpenCV `interpolateCubic` in float32 arithmetic; returns [n, 4] float32."""
    x = np.asarray(fx, dtype=np.float32)
    one = _F32(1.0)
    a5, a8, a4 = _F32(5.0) * _A, _F32(8.0) * _A, _F32(4.0) * _A
    ap2, ap3 = _A + _F32(2.0), _A + _F32(3.0)
    x1 = x + one
    c0 = ((_A * x1 - a5) * x1 + a8) * x1 - a4
    c1 = ((ap2 * x - ap3) * x) * x + one
    omx = one - x
    c2 = ((ap2 * omx - ap3) * omx) * omx + one
    c3 = ((one - c0) - c1) - c2
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.float32)


def axis_table(dsize: int, ssize: int, scale: float):
    """Per destination index: 4 clamped source taps and float32 cubic coefficients."""
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    taps = np.clip(s[:, None] - 1 + np.arange(4)[None, :], 0, ssize - 1)
    return taps, cubic_coeffs(f)


def _round_half_even(v: float) -> int:
    return int(round(v))


def output_size(src_hw, dsize=None, fx=None, fy=None):
    """Return (dh, dw, scale_y, scale_x) exactly as cv::resize computes them."""
    sh, sw = src_hw
    if dsize is None or tuple(dsize) == (0, 0):
        dw, dh = _round_half_even(sw * fx), _round_half_even(sh * fy)
        inv_x, inv_y = float(fx), float(fy)
    else:
        dw, dh = int(dsize[0]), int(dsize[1])
        inv_x, inv_y = dw / sw, dh / sh
    if dw <= 0 or dh <= 0:
        raise ValueError("resize: empty destination")
    return dh, dw, 1.0 / inv_y, 1.0 / inv_x


def resize_cubic(src: np.ndarray, dsize=None, fx=None, fy=None) -> np.ndarray:
    """cv2.resize(src, dsize, fx=fx, fy=fy, interpolation=cv2.INTER_CUBIC)."""
    squeeze = src.ndim == 2
    img = src[:, :, None] if squeeze else src
    sh, sw = img.shape[:2]
    dh, dw, scale_y, scale_x = output_size((sh, sw), dsize, fx, fy)
    if (dh, dw) == (sh, sw):
        out = img.copy()
        return out[:, :, 0] if squeeze else out
    xt, xc = axis_table(dw, sw, scale_x)
    yt, yc = axis_table(dh, sh, scale_y)
    if img.dtype == np.uint8:
        ia = np.rint(xc * _F32(2048.0)).astype(np.int64)
        ib = np.rint(yc * _F32(2048.0)).astype(np.int64)
        ia = np.clip(ia, -32768, 32767)
        ib = np.clip(ib, -32768, 32767)
        S = img.astype(np.int64)
        h = np.zeros((sh, dw, img.shape[2]), np.int64)
        for j in range(4):
            h += S[:, xt[:, j], :] * ia[None, :, j, None]
        v = np.zeros((dh, dw, img.shape[2]), np.int64)
        for j in range(4):
            v += h[yt[:, j], :, :] * ib[:, j, None, None]
        out = np.clip((v + (1 << 21)) >> 22, 0, 255).astype(np.uint8)
    elif img.dtype == np.float32:
        S = img
        h = S[:, xt[:, 0], :] * xc[None, :, 0, None]
        for j in range(1, 4):
            h = h + S[:, xt[:, j], :] * xc[None, :, j, None]
        v = h[yt[:, 0], :, :] * yc[:, 0, None, None]
        for j in range(1, 4):
            v = v + h[yt[:, j], :, :] * yc[:, j, None, None]
        out = v.astype(np.float32)
    else:
        raise TypeError("oracle resize supports uint8 and float32 only")
    return out[:, :, 0] if squeeze else out


class Cv2Shim:
    """Minimal stand-in exposing the two cv2 names the reference hot path uses."""

    INTER_CUBIC = 2

    @staticmethod
    def resize(src, dsize, dst=None, fx=None, fy=None, interpolation=None):
        if interpolation not in (None, 2):
            raise NotImplementedError("only INTER_CUBIC is restated")
        return resize_cubic(np.asarray(src), dsize, fx, fy)

    @staticmethod
    def flip(src, code):
        if code == 1:
            return np.ascontiguousarray(src[:, ::-1])
        if code == 0:
            return np.ascontiguousarray(src[::-1])
        return np.ascontiguousarray(src[::-1, ::-1])
