"""Body pose estimation with the reference's call surface (hitmaxiang/pytorch-openpose src/body.py).

    body = Body('body_pose_model.pth')
    candidate, subset = body(oriImg)          # oriImg: uint8 H x W x 3, BGR

Returns exactly what `Body.__call__` (src/body.py:24-212) returns:
* candidate: float64 [N, 4] rows (x, y, score, id), or shape (0,) when no peak exists;
* subset:    float64 [P, 20]: candidate ids per part (-1 = missing), total score, part count.

Everything after weight loading runs on the GPU in libopose: uint8 cubic resize + pad +
normalise, the VGG-19/CPM network (implicit-GEMM fp32 MFMA), x8 cubic upsample, resize
and scale averaging, Gaussian(sigma=3) peak NMS, PAF line integrals, greedy matching and
person assembly.  Only the fixed-size per-frame record crosses PCIe.

Extras beyond the reference (defaults = reference values, src/body.py:25-31):
scale_search, boxsize, stride, padValue, thre1, thre2, device; `Body.batch(frames)` runs
a video batch through one launch sequence; `Body.infer_records` keeps inputs/outputs on
the device (multi-GPU gather, benchmark).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native, util
from .model import bodypose_model


def _load_state(model_path):
    if isinstance(model_path, dict):
        return model_path
    import torch
    return torch.load(model_path, map_location="cpu", weights_only=True)


ctypes_int4 = ctypes.c_int * 4


class Body(object):
    def __init__(self, model_path, device: int = 0, scale_search=(0.5,), boxsize=368, stride=8, padValue=128,
                 thre1=0.1, thre2=0.05, peaks_per_part=128, max_people=96):
        self.model = bodypose_model(device)
        model_dict = util.transfer(self.model, _load_state(model_path))
        self.model.load_state_dict(model_dict)
        self.model.eval()
        self.handle = self.model.handle
        self.params = _native.default_params(_native.NET_BODY, scale_search=scale_search, boxsize=float(boxsize),
                                             stride=int(stride), pad_value=int(padValue), thre1=float(thre1),
                                             thre2=float(thre2))
        self.peaks_per_part, self.max_people = peaks_per_part, max_people
        self.handle.set_capacity(peaks_per_part, max_people)

    # ------------------------------------------------------------------ host API
    def __call__(self, oriImg):
        return self.batch(oriImg[None])[0]

    def batch(self, frames):
        """frames: uint8 [N, H, W, 3] (or a list of equally sized frames) -> list of (candidate, subset)."""
        if isinstance(frames, (list, tuple)):
            frames = np.stack(frames)
        frames = np.asarray(frames)
        if frames.dtype != np.uint8 or frames.ndim != 4 or frames.shape[3] != 3:
            raise ValueError("expected uint8 frames [N, H, W, 3]")
        if not (frames.strides[3] == 1 and frames.strides[2] == 3 and frames.strides[1] >= 3 * frames.shape[2]
                and (frames.shape[0] == 1 or frames.strides[0] >= frames.strides[1] * frames.shape[1])):
            frames = np.ascontiguousarray(frames)
        N, H, W, _ = frames.shape
        frame_stride = frames.strides[0] if N > 1 else frames.strides[1] * H
        while True:
            rb = self.handle.record_bytes()
            rec = np.empty((N, rb), np.uint8)
            rc = _native.lib.opose_body_infer(self.handle.h, frames.ctypes.data, N, H, W, frames.strides[1],
                                              frame_stride, self.params, rec.ctypes.data, 0)
            if rc == _native.OPOSE_E_CAPACITY and self._grow():
                continue
            if rc not in (_native.OPOSE_OK, _native.OPOSE_E_CAPACITY, _native.OPOSE_E_ASSEMBLY):
                self.handle.check(rc)
            return [self._decode(r) for r in rec]

    def post(self, maps, pad, H, W):
        """Post-network path only (src/body.py:52-212) on one scale.

        maps: float32 [N, 57, h, w] (PAF channels 0..37, heat 38..56); pad: util.padRightDownCorner pad."""
        maps = np.ascontiguousarray(maps, dtype=np.float32)
        N, c, hl, wl = maps.shape
        assert c == 57
        while True:
            rec = np.empty((N, self.handle.record_bytes()), np.uint8)
            rc = _native.lib.opose_body_post(self.handle.h, maps.ctypes.data, N, hl, wl, int(pad[2]), int(pad[3]),
                                             int(H), int(W), self.params, rec.ctypes.data, 0)
            if rc == _native.OPOSE_E_CAPACITY and self._grow():
                continue
            if rc not in (_native.OPOSE_OK, _native.OPOSE_E_CAPACITY, _native.OPOSE_E_ASSEMBLY):
                self.handle.check(rc)
            return [self._decode(r) for r in rec]

    # ------------------------------------------------------------------ per-scale split
    def scale_geom(self, H, W):
        """[(hl, wl, pad_down, pad_right)] per scale of scale_search for an H x W frame."""
        out = []
        for s in range(self.params.n_scales):
            g = (ctypes_int4)()
            self.handle.check(_native.lib.opose_body_scale_geom(int(H), int(W), self.params, s, g))
            out.append(tuple(int(v) for v in g))
        return out

    def scale_maps(self, frames, s, out=None):
        """Network maps of scale index `s` only: [N, 57, hl, wl] float32 (PAF 38 | heat 19).

        frames: uint8 [N,H,W,3] numpy (-> numpy) or a torch cuda tensor (-> torch cuda tensor,
        written into `out` when given, complete in torch's current-stream order)."""
        if hasattr(frames, "data_ptr"):
            import torch
            if frames.dim() == 3:
                frames = frames[None]
            N, H, W, _ = frames.shape
            if frames.stride(2) != 3 or frames.stride(3) != 1 or (N > 1 and frames.stride(0) < frames.stride(1) * H):
                raise ValueError("expected uint8 frames [N, H, W, 3] with packed pixels")
            hl, wl, _, _ = self.scale_geom(H, W)[s]
            if out is None:
                out = torch.empty((N, 57, hl, wl), dtype=torch.float32, device=frames.device)
            assert out.is_contiguous() and tuple(out.shape) == (N, 57, hl, wl)
            self.handle.wait_torch()
            self.handle.check(_native.lib.opose_body_scale_maps(
                self.handle.h, frames.data_ptr(), N, H, W, frames.stride(1), max(frames.stride(0), frames.stride(1) * H),
                self.params, s, out.data_ptr(), _native.IN_DEVICE | _native.OUT_DEVICE))
            self.handle.signal_torch()  # `out` complete in torch's stream order (e.g. an isend)
            return out
        frames = np.ascontiguousarray(frames if np.ndim(frames) == 4 else np.asarray(frames)[None])
        N, H, W, _ = frames.shape
        hl, wl, _, _ = self.scale_geom(H, W)[s]
        maps = np.empty((N, 57, hl, wl), np.float32)
        self.handle.check(_native.lib.opose_body_scale_maps(
            self.handle.h, frames.ctypes.data, N, H, W, frames.strides[1], frames.strides[1] * H, self.params, s,
            maps.ctypes.data, 0))
        return maps

    def band_maps(self, frame, s, r0, r1, exchange=None):
        """Rows [r0, r1) of scale `s`'s network maps for one frame: [1, 57, r1-r0, wl] float32
        (opose_body_band_maps; src/body.py:36-50 for one m, cut into output rows).

        frame: uint8 [H,W,3] numpy (-> numpy) or torch cuda tensor (-> torch cuda tensor in
        torch's current-stream order).  exchange(xbuf, cap, nbytes, stream) moves the halo rows
        between neighbouring bands (src.dist.band_exchange): xbuf is the uint8 device tensor
        [send_up | send_dn | recv_up | recv_dn] of `cap` bytes each, `stream` the library's
        hipStream_t, on which the send halves are being packed.  Not needed when one band covers
        every row.  exchange="rccl": the library's own RCCL send/recv on its stream, with the
        communicator and neighbours of src.dist.init_band_comm / Handle.set_band_peers (no Python
        between the layers).  The bands of a frame put together are scale_maps(frame, s) bit for
        bit: every conv sums a pixel in the whole frame's order."""
        import torch
        dev = hasattr(frame, "data_ptr")
        if dev:
            frame = frame[0] if frame.dim() == 4 else frame
            if frame.stride(1) != 3 or frame.stride(2) != 1:
                raise ValueError("expected a uint8 frame [H, W, 3] with packed pixels")
            H, W, _ = frame.shape
            ptr, rs = frame.data_ptr(), frame.stride(0)
        else:
            frame = np.ascontiguousarray(np.asarray(frame)[0] if np.ndim(frame) == 4 else frame)
            H, W, _ = frame.shape
            ptr, rs = frame.ctypes.data, frame.strides[0]
        hl, wl, _, _ = self.scale_geom(H, W)[s]
        cap = int(_native.lib.opose_body_band_halo_bytes(wl))
        xbuf = getattr(self, "_band_xbuf", None)  # kept across calls (27 exchanges per call)
        if xbuf is None or xbuf.numel() < 4 * cap:
            xbuf = self._band_xbuf = torch.empty(4 * cap, dtype=torch.uint8,
                                                 device=torch.device("cuda", self.handle.device))
        err = []

        def _cb(user, nbytes, stream):
            try:
                if exchange is None:
                    raise RuntimeError("row band with neighbours but no exchange")
                exchange(xbuf[:4 * cap], cap, int(nbytes), stream)
                return 0
            except BaseException as e:  # reported after the call returns
                err.append(e)
                return 1

        cb = _native.HALO_FN() if exchange == "rccl" else _native.HALO_FN(_cb)  # NULL: the library's RCCL
        flags = 0
        if dev:
            out = torch.empty((1, 57, r1 - r0, wl), dtype=torch.float32, device=frame.device)
            self.handle.wait_torch()
            rc = _native.lib.opose_body_band_maps(self.handle.h, ptr, H, W, rs, self.params, s, r0, r1,
                                                  out.data_ptr(), cb, None, xbuf.data_ptr(), 4 * cap,
                                                  flags | _native.IN_DEVICE | _native.OUT_DEVICE)
            if err:
                raise err[0]
            self.handle.check(rc)
            self.handle.signal_torch()
            return out
        self.handle.wait_torch()  # xbuf was allocated on torch's stream
        out = np.empty((1, 57, r1 - r0, wl), np.float32)
        rc = _native.lib.opose_body_band_maps(self.handle.h, ptr, H, W, rs, self.params, s, r0, r1, out.ctypes.data,
                                              cb, None, xbuf.data_ptr(), 4 * cap, flags)
        if err:
            raise err[0]
        self.handle.check(rc)
        return out

    def post_scales(self, maps, H, W):
        """Multi-scale post-network path (src/body.py:51-212): maps[s] = [N,57,hl,wl] for every
        scale of scale_search (numpy, or torch cuda tensors) -> list of (candidate, subset)."""
        geoms = self.scale_geom(H, W)
        if len(maps) != len(geoms):
            raise ValueError("expected %d scale maps, got %d" % (len(geoms), len(maps)))
        dev = hasattr(maps[0], "data_ptr")
        if not dev:
            maps = [np.ascontiguousarray(m, dtype=np.float32) for m in maps]
        for m, (hl, wl, _, _) in zip(maps, geoms):
            if tuple(m.shape[1:]) != (57, hl, wl):
                raise ValueError("scale maps of shape %s, expected (N, 57, %d, %d)" % (tuple(m.shape), hl, wl))
        N = maps[0].shape[0]
        ns = len(maps)
        ptrs = (ctypes.c_void_p * ns)(*[m.data_ptr() if dev else m.ctypes.data for m in maps])
        if dev:
            self.handle.wait_torch()  # e.g. maps received by an irecv on torch's stream
        arr = [(ctypes.c_int * ns)(*[g[i] for g in geoms]) for i in range(4)]
        while True:
            rec = np.empty((N, self.handle.record_bytes()), np.uint8)
            rc = _native.lib.opose_body_post_scales(self.handle.h, ptrs, arr[0], arr[1], arr[2], arr[3], ns, N,
                                                    int(H), int(W), self.params, rec.ctypes.data,
                                                    _native.IN_DEVICE if dev else 0)
            if rc == _native.OPOSE_E_CAPACITY and self._grow():
                continue
            if rc not in (_native.OPOSE_OK, _native.OPOSE_E_CAPACITY, _native.OPOSE_E_ASSEMBLY):
                self.handle.check(rc)
            return [self._decode(r) for r in rec]

    # ------------------------------------------------------------------ device API
    def infer_records(self, frames_dev, records_dev=None, pipeline=False, wait=True):
        """frames_dev: torch.uint8 cuda [N,H,W,3]; returns a torch.uint8 cuda [N, record_bytes] tensor.

        Asynchronous (no host synchronisation): ordered after torch's current stream, and the
        records are complete in that stream's order on return (opose_wait_stream /
        opose_signal_stream).  pipeline=True
        (OPOSE_PIPELINE, include/opose.h): the frames are complete now and are not modified until
        the handle's stream passes this call; the call's network then overlaps the previous
        call's post-processing (video-batch throughput).  pipeline="defer"
        (OPOSE_PIPELINE_DEFER): this call's post-processing is enqueued by the next pipelined
        call once that call's network reaches conv3_1, or by handle.flush() / synchronize() /
        decode_records(); keep frames and records alive until then.
        wait=False (pipelined calls only): do not order the call after torch's current stream.
        The caller guarantees that the frames are complete and that the records buffer is free
        (e.g. it synchronized the host on the upload's event): opose_wait_stream would put a
        marker on the caller's stream, and a stream that shares a hardware queue with the
        handle's post-processing stream then holds the next network back behind that work."""
        import torch
        N, H, W, _ = frames_dev.shape
        if frames_dev.stride(3) != 1 or frames_dev.stride(2) != 3:
            frames_dev = frames_dev.contiguous()  # pixels must be packed BGR; rows / frames may be strided
        # a size-1 axis may carry any stride (0 for a numpy newaxis): give it the dense one
        row_stride = frames_dev.stride(1) if H > 1 else 3 * W
        frame_stride = frames_dev.stride(0) if N > 1 else row_stride * H
        rb = self.handle.record_bytes()
        if records_dev is None:
            records_dev = torch.empty((N, rb), dtype=torch.uint8, device=frames_dev.device)
        if wait or not pipeline:
            self.handle.wait_torch()  # frames / records produced or last used on torch's stream
        rc = _native.lib.opose_body_infer(self.handle.h, frames_dev.data_ptr(), N, H, W, row_stride,
                                          frame_stride, self.params, records_dev.data_ptr(),
                                          _native.IN_DEVICE | _native.OUT_DEVICE
                                          | (_native.PIPELINE if pipeline else 0)
                                          | (_native.PIPELINE_DEFER if pipeline == "defer" else 0))
        self.handle.check(rc)
        if pipeline:
            # outputs stay in the handle's stream order (torch's stream must not wait for them, or
            # the next call's network could not overlap this call's post-processing): consumers
            # order themselves on handle.stream() (bench.py, src/dist.py) or call decode_records
            self.handle.hold(records_dev, frames_dev)
        else:
            self.handle.signal_torch()
        return records_dev

    def decode_records(self, records):
        """uint8 [N, record_bytes] (numpy or torch) -> list of (candidate, subset)."""
        if hasattr(records, "cpu"):
            if records.is_cuda:
                self.handle.signal_torch()  # pipelined records complete on the handle's stream
            records = records.cpu().numpy()
        return [self._decode(r) for r in np.asarray(records)]

    # ------------------------------------------------------------------ helpers
    def _grow(self) -> bool:
        if self.peaks_per_part >= 1024 and self.max_people >= 256:
            return False
        self.peaks_per_part = min(1024, self.peaks_per_part * 2)
        self.max_people = min(256, self.max_people * 2)
        self.handle.set_capacity(self.peaks_per_part, self.max_people)
        return True

    def _decode(self, rec):
        status, cand, subset = _native.decode_record(rec, self.peaks_per_part, self.max_people)
        if status == _native.OPOSE_E_ASSEMBLY:
            # the reference raises here when a third subset row matches (src/body.py:170-173)
            raise IndexError("list assignment index out of range")
        if status == _native.OPOSE_E_CAPACITY:
            raise RuntimeError("libopose: per-frame capacity exceeded (peaks_per_part=%d, max_people=%d)"
                               % (self.peaks_per_part, self.max_people))
        if status != 0:
            raise _native.OposeError(status, "frame failed")
        return cand, subset
