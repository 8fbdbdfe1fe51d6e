"""The reference's batched "fast mode" (hitmaxiang/pytorch-openpose srcmx/Batch_model.py),
on the GPU.

    bb = Batch_body('body_pose_model.pth')
    results = bb(batch_images)       # [(candidate, subset), ...], one per frame

`Batch_body.__call__` (srcmx/Batch_model.py:137-204) differs from `Body` in numerics, not in
its person model: torch bicubic resizing of ToTensor'd frames (uint8 / 255), floor instead of
round image sizes, a single scale (0.5), a 5x5 Gaussian (srcmx/utilmx.py:246-263) instead of
scipy's sigma-3 filter, and peak scores read from the blurred map; limb scoring, greedy
matching and assembly are Body's (`FindBody_frame`, :206-300).  Here the whole call is one
libopose launch sequence (`opose_batch_body_infer`): torch-convention bicubic kernels,
the same conv network, a blur+NMS kernel, then the shared PAF / matching / assembly kernels.

Inputs: what the reference's DataLoader yields -- a float tensor [B, 3, h, w] in [0, 1]
(transforms.ToTensor of uint8 BGR frames; converted back to the exact uint8 values) -- or
uint8 frames [B, h, w, 3] directly.
"""
from __future__ import annotations

import numpy as np

from . import _native
from .body import Body


def size_pad(g_scale, height, width, boxsize=368, stride=8):
    """Batch_body.calculate_size_pad (srcmx/Batch_model.py:302-307)."""
    scale = boxsize * g_scale / height
    h, w = int(height * scale), int(width * scale)
    return scale, h, w, (stride - (h % stride)) % stride, (stride - (w % stride)) % stride


def _as_uint8_frames(batch_images) -> np.ndarray:
    if hasattr(batch_images, "detach"):  # torch tensor [B, 3, h, w] float in [0, 1]
        t = batch_images.detach()
        if t.dtype.is_floating_point:
            t = (t * 255).round().clamp(0, 255).to(dtype=__import__("torch").uint8)
        return np.ascontiguousarray(t.permute(0, 2, 3, 1).cpu().numpy())
    a = np.asarray(batch_images)
    if a.dtype == np.uint8 and a.ndim == 4 and a.shape[3] == 3:
        return a
    if a.ndim == 4 and a.shape[1] == 3:
        return np.ascontiguousarray(np.clip(np.rint(a * 255), 0, 255).astype(np.uint8).transpose(0, 2, 3, 1))
    raise ValueError("expected a [B,3,h,w] float batch in [0,1] or uint8 frames [B,h,w,3]")


class Batch_body(Body):
    def __init__(self, model_path, device: int = 0, scale_search=0.5, boxsize=368, stride=8, thre1=0.1, thre2=0.05,
                 peaks_per_part=128, max_people=96):
        super().__init__(model_path, device, scale_search=(float(scale_search),), boxsize=boxsize, stride=stride,
                         padValue=128, thre1=thre1, thre2=thre2, peaks_per_part=peaks_per_part,
                         max_people=max_people)
        self.scale_search, self.boxsize, self.stride = float(scale_search), boxsize, stride

    def __call__(self, batch_images):
        return self.batch(_as_uint8_frames(batch_images))

    def batch(self, frames):
        frames = np.ascontiguousarray(frames)
        N, H, W, _ = frames.shape
        while True:
            rec = np.empty((N, self.handle.record_bytes()), np.uint8)
            rc = _native.lib.opose_batch_body_infer(self.handle.h, frames.ctypes.data, N, H, W, frames.strides[1],
                                                    frames.strides[1] * H, self.params, rec.ctypes.data, 0)
            if rc == _native.OPOSE_E_CAPACITY and self._grow():
                continue
            if rc not in (_native.OPOSE_OK, _native.OPOSE_E_CAPACITY, _native.OPOSE_E_ASSEMBLY):
                self.handle.check(rc)
            return [self._decode(r) for r in rec]

    def post(self, maps, H, W):
        """Post-network part only (srcmx/Batch_model.py:159-204): maps float32 [N, 57, hl, wl]
        (PAF 0..37, heat 38..56) for frames of H x W."""
        maps = np.ascontiguousarray(maps, dtype=np.float32)
        N, c, hl, wl = maps.shape
        assert c == 57
        _, nh, nw, _, _ = size_pad(self.scale_search, H, W, self.boxsize, self.stride)
        while True:
            rec = np.empty((N, self.handle.record_bytes()), np.uint8)
            rc = _native.lib.opose_batch_body_post(self.handle.h, maps.ctypes.data, N, hl, wl, nh, nw, int(H), int(W),
                                                   self.params, rec.ctypes.data, 0)
            if rc == _native.OPOSE_E_CAPACITY and self._grow():
                continue
            if rc not in (_native.OPOSE_OK, _native.OPOSE_E_CAPACITY, _native.OPOSE_E_ASSEMBLY):
                self.handle.check(rc)
            return [self._decode(r) for r in rec]

    def infer_records(self, frames_dev, records_dev=None):
        """Device-resident uint8 frames [N, H, W, 3] -> device records (asynchronous)."""
        import torch
        N, H, W, _ = frames_dev.shape
        if frames_dev.stride(3) != 1 or frames_dev.stride(2) != 3:
            frames_dev = frames_dev.contiguous()
        row_stride = frames_dev.stride(1) if H > 1 else 3 * W  # size-1 axes: any stride (numpy newaxis: 0)
        frame_stride = frames_dev.stride(0) if N > 1 else row_stride * H
        if records_dev is None:
            records_dev = torch.empty((N, self.handle.record_bytes()), dtype=torch.uint8, device=frames_dev.device)
        self.handle.wait_torch()
        self.handle.check(_native.lib.opose_batch_body_infer(
            self.handle.h, frames_dev.data_ptr(), N, H, W, row_stride, frame_stride, self.params,
            records_dev.data_ptr(), _native.IN_DEVICE | _native.OUT_DEVICE))
        self.handle.signal_torch()
        return records_dev


class Batch_hand(object):
    """srcmx/Batch_model.py:310-354: crops already resized to boxsize (the data loader's
    HandImageDataset does that with cv2) -> np.array [B, 21, 3] of (x, y, score) in crop
    pixels, float64 (int64 when nothing is found anywhere, as np.array of [0, 0, 0] rows)."""

    def __init__(self, model_path, device: int = 0, thre=0.035):
        from .hand import _load_state
        from .model import handpose_model
        from . import util
        self.model = handpose_model(device)
        self.model.load_state_dict(util.transfer(self.model, _load_state(model_path)))
        self.model.eval()
        self.handle = self.model.handle
        self.params = _native.default_params(_native.NET_HAND, scale_search=(1.0,), thre_hand=float(thre))

    def __call__(self, batch_imgs):
        crops = np.ascontiguousarray(_as_uint8_frames(batch_imgs))
        N, H, W, _ = crops.shape
        peaks = np.empty((N, 21, 3), np.float64)
        found = np.empty((N, 21), np.int32)
        self.handle.check(_native.lib.opose_batch_hand_infer(self.handle.h, crops.ctypes.data, N, H, W,
                                                             crops.strides[1], crops.strides[1] * H, self.params,
                                                             peaks.ctypes.data, found.ctypes.data, 0))
        return self._as_reference(peaks, found)

    def post(self, heat):
        """Post-network part only (srcmx/Batch_model.py:334-354): heat float32 [B, 22, hl, wl]."""
        heat = np.ascontiguousarray(heat, dtype=np.float32)
        N, c, hl, wl = heat.shape
        assert c == 22
        peaks = np.empty((N, 21, 3), np.float64)
        found = np.empty((N, 21), np.int32)
        self.handle.check(_native.lib.opose_batch_hand_post(self.handle.h, heat.ctypes.data, N, hl, wl, self.params,
                                                            peaks.ctypes.data, found.ctypes.data, 0))
        return self._as_reference(peaks, found)

    @staticmethod
    def _as_reference(peaks, found):
        if not found.any():
            return np.zeros(peaks.shape, dtype=np.int64)
        peaks[~found.astype(bool)] = 0.0
        return peaks
