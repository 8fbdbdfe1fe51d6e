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
image: decode elsewhere and pass the frames).
"""
from __future__ import annotations

import numpy as np

from .pipeline import motion_data_frames


class VideoFrames(object):
    """Sequential BGR frames of a video file, optionally cropped (VideoDataset semantics)."""

    def __init__(self, videopath, crop=None):
        try:
            import cv2
        except ImportError as e:  # pragma: no cover - cv2 is absent in this image
            raise ImportError("VideoFrames needs OpenCV (cv2) to decode video; pass decoded frames "
                              "to extract_motion_data instead") from e
        self._cv2 = cv2
        self.video = cv2.VideoCapture(videopath)
        if not self.video.isOpened():
            raise FileNotFoundError(videopath)
        self.crop = crop

    def __len__(self):
        return int(self.video.get(self._cv2.CAP_PROP_FRAME_COUNT))

    def __iter__(self):
        while True:
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


def extract_motion_data(frames, body, hand=None, outpath=None, recpoint=None, mode="body", batch=32):
    """MotionMat [n_frames, 18 | 60, 3] for an iterable of uint8 BGR frames (equal sizes after
    cropping).  mode "body" (18 joints) or "bodyhand" (needs `hand`); saved with joblib.dump
    when `outpath` is given, like Extract_MotionData_from_Video."""
    if mode not in ("body", "bodyhand"):
        raise ValueError("mode must be 'body' or 'bodyhand'")
    if mode == "bodyhand" and hand is None:
        raise ValueError("'bodyhand' mode needs a Hand")
    out, buf = [], []

    def flush():
        if buf:
            out.append(motion_data_frames(body, hand, np.stack(buf), mode))
            buf.clear()

    for frame in frames:
        buf.append(np.ascontiguousarray(crop_roi(np.asarray(frame), recpoint)))
        if len(buf) == batch:
            flush()
    flush()
    joints = 60 if mode == "bodyhand" else 18
    motion = np.concatenate(out) if out else np.zeros((0, joints, 3))
    if outpath is not None:
        import joblib
        joblib.dump(motion, outpath)
    return motion
