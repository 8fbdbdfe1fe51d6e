"""Video motion-matrix extraction (SURVEY §8 f rank 2) on the GPU Body/Hand.

Restates `Extract_MotionData_from_Video` (hitmaxiang/pytorch-openpose
srcmx/MotionEstimation.py:25-76) and the frame source `VideoDataset`
(srcmx/Batch_model.py:36-52): frames are read in order, cropped to the region of interest
`recpoint = [(x0, y0), (x1, y1)]` (frame[y0:y1, x0:x1]), run through the Body (+Hand)
pipeline, and stacked into MotionMat [frames, 18 or 60, 3] (x, y, score per joint: 18 body
joints, then 21 left-hand and 21 right-hand joints in "bodyhand" mode), saved with
joblib.dump like the reference.

Frames are processed in batches (one Body launch sequence per batch, all hands of a batch in
one crop-batched Hand pass) instead of one frame at a time; per-frame results are those of
`src.pipeline.motion_data_every_frame`.  Any iterable of uint8 BGR frames works as a source;
`VideoFrames` reads a video file through OpenCV when it is installed (it is not part of this
image: decode elsewhere and pass the frames, or pass any cv2.VideoCapture-like `capture`).

Like the reference, the matrix has one row per frame the container *reports*
(CAP_PROP_FRAME_COUNT, srcmx/MotionEstimation.py:45-50): rows of frames that never decode stay
zero, a video that decodes more frames than it reports raises IndexError, and a video that does
not open is reported and yields None (`Extract_MotionData_from_Video`, the reference's entry
point, :25-76).

Ingest (the reference's DataLoader over decoded frames, srcmx/Batch_model.py:36-52, 409-412, into
the per-video loop of srcmx/MotionEstimation.py:61-76): with a GPU, `extract_motion_data` streams
the batches through two pinned host buffers and two device frame buffers.  While batch k runs
Body on the GPU (Body.infer_records, pipelined with batch k-1's post-processing), batch k+1 is
cropped into the other pinned buffer and uploaded on its own copy stream, and batch k-1's
records (downloaded asynchronously to pinned memory) are decoded into poses on the host, its
hands running through Hand on the Hand handle's stream.  The poses are those of the host path
(`device=False`: Body.batch per batch), bit for bit.
"""
from __future__ import annotations

import numpy as np



CAP_PROP_FRAME_COUNT = 7  # cv2.CAP_PROP_FRAME_COUNT


class VideoFrames(object):
    """Sequential BGR frames of a video file, optionally cropped (VideoDataset semantics).

    capture: a cv2.VideoCapture-like factory (isOpened / get(CAP_PROP_FRAME_COUNT) / read);
    default cv2.VideoCapture.  len() is the count the container reports; `opened` is False for a
    file that does not open (then it has no frames)."""

    def __init__(self, videopath, crop=None, capture=None):
        if capture is None:
            try:
                import cv2
            except ImportError as e:  # pragma: no cover - cv2 is absent in this image
                raise ImportError("VideoFrames needs OpenCV (cv2) to decode video; pass decoded frames "
                                  "to extract_motion_data instead, or a capture factory") from e
            capture = cv2.VideoCapture
        self.video = capture(videopath)
        self.opened = bool(self.video.isOpened())
        self.crop = crop

    def __len__(self):
        return int(self.video.get(CAP_PROP_FRAME_COUNT)) if self.opened else 0

    def __iter__(self):
        while self.opened:
            ok, image = self.video.read()
            if not ok:
                return
            if self.crop is not None:
                image = image[self.crop[0][1]:self.crop[1][1], self.crop[0][0]:self.crop[1][0], :]
            yield image


def crop_roi(frame, recpoint):
    """frame[y0:y1, x0:x1] for recpoint [(x0, y0), (x1, y1)] (MotionEstimation.py:66)."""
    if recpoint is None:
        return frame
    return frame[recpoint[0][1]:recpoint[1][1], recpoint[0][0]:recpoint[1][0], :]


def _batches(frames, recpoint, batch):
    buf = []
    for frame in frames:
        buf.append(crop_roi(np.asarray(frame), recpoint))
        if len(buf) == batch:
            yield buf
            buf = []
    if buf:
        yield buf


def _host_poses(frames, body, hand, recpoint, mode, batch):
    from .pipeline import poses_from_results
    out = []
    for b in _batches(frames, recpoint, batch):
        arr = np.stack([np.ascontiguousarray(f) for f in b])
        out.append(poses_from_results(body.batch(arr), arr, hand, mode))
    return out


class _DeviceIngest(object):
    """Two pinned host frame buffers -> two device frame buffers (one copy stream each) ->
    Body.infer_records(pipeline=True) -> records downloaded to pinned host memory on the
    handle's stream; at most two batches in flight.

    A frame whose peaks or people overflow the record capacity (the reference has no limit) is
    run again through Body.batch, which grows the capacity and retries like Body(); later
    batches then get records of the grown size (a batch decodes with the layout it was
    submitted with)."""

    def __init__(self, body, batch, H, W):
        import torch
        self.torch = torch
        self.body = body
        self.batch = batch
        self.devc = torch.device("cuda", body.handle.device)
        self.host = [torch.empty((batch, H, W, 3), dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.dev = [torch.empty((batch, H, W, 3), dtype=torch.uint8, device=self.devc) for _ in range(2)]
        self.rdev, self.rhost, self.layout = [None, None], [None, None], [None, None]
        self.cps = [torch.cuda.Stream(device=self.devc) for _ in range(2)]
        self.up_done = [None, None]    # upload of buffer i finished with host[i]
        self.rec_done = [None, None]   # records of buffer i on the host
        self.lib = body.handle.torch_stream()

    def submit(self, i, frames):
        torch = self.torch
        n = len(frames)
        if self.up_done[i] is not None:
            self.up_done[i].synchronize()  # host[i] free: its previous upload completed
        rb = self.body.handle.record_bytes()
        if self.rdev[i] is None or self.rdev[i].shape[1] != rb:  # (first use, or the capacity grew)
            self.rdev[i] = torch.empty((self.batch, rb), dtype=torch.uint8, device=self.devc)
            self.rhost[i] = torch.empty((self.batch, rb), dtype=torch.uint8).pin_memory()
        self.layout[i] = (self.body.peaks_per_part, self.body.max_people)
        np.stack(frames, out=self.host[i][:n].numpy())
        cp = self.cps[i]
        cp.wait_stream(self.lib)  # the call that last read dev[i] / wrote rdev[i] is done with them
        with torch.cuda.stream(cp):
            self.dev[i][:n].copy_(self.host[i][:n], non_blocking=True)
            self.up_done[i] = torch.cuda.Event()
            self.up_done[i].record(cp)
            # the library orders itself after this stream (opose_wait_stream): the upload above
            self.body.infer_records(self.dev[i][:n], self.rdev[i][:n], pipeline=True)
        with torch.cuda.stream(self.lib):
            self.rhost[i][:n].copy_(self.rdev[i][:n], non_blocking=True)
            self.rec_done[i] = torch.cuda.Event()
            self.rec_done[i].record(self.lib)

    def results(self, i, frames):
        from . import _native
        self.rec_done[i].synchronize()
        out = []
        for r, f in zip(self.rhost[i][:len(frames)].numpy(), frames):
            status, cand, subset = _native.decode_record(r, *self.layout[i])
            if status == _native.OPOSE_E_CAPACITY:
                out.extend(self.body.batch(np.ascontiguousarray(f)[None]))
            elif status == _native.OPOSE_E_ASSEMBLY:
                raise IndexError("list assignment index out of range")  # src/body.py:170-173
            elif status != 0:
                raise _native.OposeError(status, "frame failed")
            else:
                out.append((cand, subset))
        return out


def _device_poses(frames, body, hand, recpoint, mode, batch):
    from .pipeline import poses_from_results
    out, ing, pending, k = [], None, None, 0
    for b in _batches(frames, recpoint, batch):
        if ing is None:
            H, W = b[0].shape[:2]
            ing = _DeviceIngest(body, batch, H, W)
        if any(f.shape != b[0].shape for f in b) or b[0].shape[:2] != tuple(ing.host[0].shape[1:3]):
            raise ValueError("frames must have equal sizes after cropping")
        i = k % 2
        ing.submit(i, b)
        if pending is not None:  # the previous batch's poses while this one runs on the GPU
            pi, pframes = pending
            out.append(poses_from_results(ing.results(pi, pframes), pframes, hand, mode))
        pending = (i, b)
        k += 1
    if pending is not None:
        pi, pframes = pending
        out.append(poses_from_results(ing.results(pi, pframes), pframes, hand, mode))
    return out


def extract_motion_data(frames, body, hand=None, outpath=None, recpoint=None, mode="body", batch=32, device=None,
                        count=None):
    """MotionMat [count, 18 | 60, 3] float64 for an iterable of uint8 BGR frames (equal sizes
    after cropping).  mode "body" (18 joints) or "bodyhand" (needs `hand`); saved with
    joblib.dump when `outpath` is given, like Extract_MotionData_from_Video.  device=None: the
    pinned, double-buffered GPU ingest when torch sees a GPU, else host batches (Body.batch).

    count: rows of the matrix, the frame count the source reports (default len(frames) when it
    has one -- a VideoFrames' CAP_PROP_FRAME_COUNT -- else the frames decoded).  Frames past the
    decoded ones stay zero rows; more decoded frames than `count` raise IndexError, as the
    reference's preallocated MotionMat does (srcmx/MotionEstimation.py:45-50, 72-73)."""
    if mode not in ("body", "bodyhand"):
        raise ValueError("mode must be 'body' or 'bodyhand'")
    if mode == "bodyhand" and hand is None:
        raise ValueError("'bodyhand' mode needs a Hand")
    if device is None:
        try:
            import torch
            device = torch.cuda.is_available()
        except ImportError:
            device = False
    if count is None and hasattr(frames, "__len__"):
        count = len(frames)
    out = (_device_poses if device else _host_poses)(frames, body, hand, recpoint, mode, batch)
    joints = 60 if mode == "bodyhand" else 18
    poses = np.concatenate(out) if out else np.zeros((0, joints, 3))
    if count is None:
        count = len(poses)
    if len(poses) > count:
        raise IndexError("index %d is out of bounds for axis 0 with size %d" % (count, count))
    motion = np.zeros((count, joints, 3))
    motion[:len(poses)] = poses
    if outpath is not None:
        import joblib
        joblib.dump(motion, outpath)
    return motion


def Extract_MotionData_from_Video(videopath, outpath, Recpoint, mode="body", overwrite=False, *, body, hand=None,
                                  batch=32, device=None, capture=None):
    """The reference's entry point (srcmx/MotionEstimation.py:25-76) on the GPU Body / Hand:
    the video's frames cropped to Recpoint [(x0, y0), (x1, y1)], MotionMat [count, 18 | 60, 3]
    (count = CAP_PROP_FRAME_COUNT; frames that do not decode leave zero rows) written to
    `outpath` with joblib.dump.  Returns None, like the reference (the matrix is the file); a
    video that does not open is reported on stdout and nothing is written.  `overwrite` is
    unused, as in the reference.  body / hand: the estimators (the reference's module-level
    body_estimation / hand_estimation); capture: see VideoFrames."""
    import os
    del overwrite
    video = VideoFrames(videopath, crop=Recpoint, capture=capture)
    if not video.opened:
        print('the file %s is not exist' % videopath)
        return None
    count = len(video)
    outname = os.path.split(outpath)[1]

    def progress():
        for index, frame in enumerate(video):
            if index % 100 == 0:
                print('%s-%d/%d' % (outname, index, count))
            yield frame

    extract_motion_data(progress(), body, hand, outpath=outpath, mode=mode, batch=batch, device=device, count=count)
    print('%s is saved!' % outpath)
    return None
