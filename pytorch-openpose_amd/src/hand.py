"""Hand keypoints with the reference's call surface (hitmaxiang/pytorch-openpose src/hand.py).

    hand = Hand('hand_pose_model.pth')
    peaks = hand(crop)            # crop: uint8 h x w x 3 (BGR), normally from util.handDetect

Returns what `Hand.__call__` (src/hand.py:25-75) returns: a [21, 3] array of (x, y, score)
per hand part, float64 — or int64 when no part was found (np.array of [0, 0, 0] rows).

On the GPU (libopose): uint8 cubic resize/pad/normalise for the 4 scales, the 6-stage hand
CPM network (implicit-GEMM fp32 MFMA), x8 cubic upsample + resize + scale average, Gaussian
smoothing, threshold, 8-connected component labelling (union-find), component selection by
raw-heat sum and the first row-major maximum (util.npmax).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native, util
from .model import handpose_model


def _load_state(model_path):
    if isinstance(model_path, dict):
        return model_path
    import torch
    return torch.load(model_path, map_location="cpu", weights_only=True)


def _as_reference_array(peaks: np.ndarray, found: np.ndarray) -> np.ndarray:
    """np.array(all_peaks) semantics: int64 when every row is the [0, 0, 0] placeholder."""
    if not found.any():
        return np.zeros((21, 3), dtype=np.int64)
    out = peaks.copy()
    out[~found.astype(bool)] = 0.0
    return out


class Hand(object):
    def __init__(self, model_path, device: int = 0, scale_search=(0.5, 1.0, 1.5, 2.0), boxsize=368, stride=8,
                 padValue=128, thre=0.03):
        self.model = handpose_model(device)
        self.model.load_state_dict(util.transfer(self.model, _load_state(model_path)))
        self.model.eval()
        self.handle = self.model.handle
        self.params = _native.default_params(_native.NET_HAND, scale_search=scale_search, boxsize=float(boxsize),
                                             stride=int(stride), pad_value=int(padValue), thre_hand=float(thre))

    def __call__(self, oriImg):
        return self.batch(np.asarray(oriImg)[None])[0]

    def batch(self, crops):
        """crops: uint8 [N, h, w, 3] of equal size -> list of [21, 3] arrays."""
        crops = np.asarray(crops)
        if crops.dtype != np.uint8 or crops.ndim != 4 or crops.shape[3] != 3:
            raise ValueError("expected uint8 crops [N, h, w, 3]")
        if not (crops.strides[3] == 1 and crops.strides[2] == 3 and crops.strides[1] >= 3 * crops.shape[2]
                and (crops.shape[0] == 1 or crops.strides[0] >= crops.strides[1] * crops.shape[1])):
            crops = np.ascontiguousarray(crops)
        N, H, W, _ = crops.shape
        fs = crops.strides[0] if N > 1 else crops.strides[1] * H
        peaks = np.empty((N, 21, 3), np.float64)
        found = np.empty((N, 21), np.int32)
        self.handle.check(_native.lib.opose_hand_infer(self.handle.h, crops.ctypes.data, N, H, W, crops.strides[1], fs,
                                                       self.params, peaks.ctypes.data, found.ctypes.data, 0))
        return [_as_reference_array(peaks[i], found[i]) for i in range(N)]

    def batch_crops(self, crops):
        """Square crops of different sizes (e.g. all hands util.handDetect found in a batch of
        frames) -> list of [21, 3] arrays; the network runs once per scale for all of them."""
        crops = [np.asarray(c) for c in crops]
        if not crops:
            return []
        arrs = []
        for c in crops:
            if c.dtype != np.uint8 or c.ndim != 3 or c.shape[2] != 3 or c.shape[0] != c.shape[1]:
                raise ValueError("expected square uint8 crops [w, w, 3]")
            if not (c.strides[2] == 1 and c.strides[1] == 3):
                c = np.ascontiguousarray(c)
            arrs.append(c)
        n = len(arrs)
        ptrs = (C.c_void_p * n)(*[a.ctypes.data for a in arrs])
        sizes = np.array([a.shape[0] for a in arrs], np.int32)
        strides = np.array([a.strides[0] for a in arrs], np.int64)
        peaks = np.empty((n, 21, 3), np.float64)
        found = np.empty((n, 21), np.int32)
        self.handle.check(_native.lib.opose_hand_infer_crops(self.handle.h, ptrs, sizes.ctypes.data, strides.ctypes.data,
                                                             n, self.params, peaks.ctypes.data, found.ctypes.data, 0))
        return [_as_reference_array(peaks[i], found[i]) for i in range(n)]

    def post(self, maps, pads, H, W):
        """Post-network path only (src/hand.py:51-75).

        maps: list (one per scale) of float32 [N, 22, h, w] network outputs; pads: per-scale
        util.padRightDownCorner pads; H, W: crop size."""
        arrs = [np.ascontiguousarray(m, dtype=np.float32) for m in maps]
        ns = len(arrs)
        N = arrs[0].shape[0]
        ptrs = (C.c_void_p * ns)(*[a.ctypes.data for a in arrs])
        hl = np.array([a.shape[2] for a in arrs], np.int32)
        wl = np.array([a.shape[3] for a in arrs], np.int32)
        pd = np.array([p[2] for p in pads], np.int32)
        pr = np.array([p[3] for p in pads], np.int32)
        peaks = np.empty((N, 21, 3), np.float64)
        found = np.empty((N, 21), np.int32)
        self.handle.check(_native.lib.opose_hand_post(self.handle.h, ptrs, hl.ctypes.data, wl.ctypes.data,
                                                      pd.ctypes.data, pr.ctypes.data, ns, N, int(H), int(W),
                                                      self.params, peaks.ctypes.data, found.ctypes.data, 0))
        return [_as_reference_array(peaks[i], found[i]) for i in range(N)]
