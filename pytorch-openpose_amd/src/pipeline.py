"""Per-frame Body + Hand pipeline (SURVEY §8 f, rank 1).

Restates `MotionData_every_frame` (hitmaxiang/pytorch-openpose srcmx/MotionEstimation.py:126-216)
on top of the GPU `Body` / `Hand`:
  body -> the person with the largest left-shoulder x (subset column 5; an absent shoulder
  reads candidate[-1] as the reference does) -> the other subset rows blanked ->
  util.handDetect -> Hand on the right-hand crop and on the horizontally flipped left-hand
  crop, x mapped back as w - x - 1 + x0 -> PoseMat (18 body rows, then left 21, right 21).
"""
from __future__ import annotations

import numpy as np

from . import util


def motion_data_every_frame(body, hand, oriImg, mode: str = "body") -> np.ndarray:
    candidate, subset = body(oriImg)
    pose = np.zeros((60, 3))
    best = None
    if len(subset) >= 1:
        shoulder_x = np.zeros((len(subset),))
        for person in range(len(subset)):
            shoulder_x[person] = candidate[int(subset[person][5])][0]
        best = np.argmax(shoulder_x)
    if best is not None:
        for part in range(18):
            idx = int(subset[best][part])
            if idx != -1:
                pose[part, :] = candidate[idx][:3]
    for i in range(len(subset)):
        if i != best:
            subset[i, :] = -1
    if mode == "bodyhand":
        for x, y, w, is_left in util.handDetect(candidate, subset, oriImg):
            crop = oriImg[y:y + w, x:x + w, :]
            if not is_left:
                peaks = hand(crop)
                peaks[:, 0] = np.where(peaks[:, 0] == 0, peaks[:, 0], peaks[:, 0] + x)
                peaks[:, 1] = np.where(peaks[:, 1] == 0, peaks[:, 1], peaks[:, 1] + y)
                pose[39:60, :] = peaks
            else:
                peaks = hand(np.ascontiguousarray(crop[:, ::-1]))  # cv2.flip(crop, 1)
                peaks[:, 0] = np.where(peaks[:, 0] == 0, peaks[:, 0], w - peaks[:, 0] - 1 + x)
                peaks[:, 1] = np.where(peaks[:, 1] == 0, peaks[:, 1], peaks[:, 1] + y)
                pose[18:39, :] = peaks
    if mode != "bodyhand":
        pose = pose[:18, :]
    return pose


def motion_data_frames(body, hand, frames, mode: str = "bodyhand") -> np.ndarray:
    """Batched `motion_data_every_frame` over equal-size frames [T, H, W, 3]: one Body launch
    sequence for all frames, then every selected hand of every frame in one crop-batched Hand
    launch per scale (SURVEY §8 f rank 1).  Returns [T, 60, 3] ("bodyhand") or [T, 18, 3]."""
    frames = np.asarray(frames)
    return poses_from_results(body.batch(frames), frames, hand, mode)


def poses_from_results(results, frames, hand, mode: str = "bodyhand") -> np.ndarray:
    """The glue of `MotionData_every_frame` (srcmx/MotionEstimation.py:139-216) after Body:
    results[t] = (candidate, subset) of frames[t] -> [T, 60, 3] ("bodyhand") or [T, 18, 3]; the
    hands of all frames go through one crop-batched Hand call."""
    T = len(results)
    poses = np.zeros((T, 60, 3))
    jobs = []  # (frame, crop, x0, y0, w, is_left)
    for t, (candidate, subset) in enumerate(results):
        subset = subset.copy()
        best = None
        if len(subset) >= 1:
            shoulder_x = np.array([candidate[int(subset[q][5])][0] for q in range(len(subset))])
            best = np.argmax(shoulder_x)
        if best is not None:
            for part in range(18):
                idx = int(subset[best][part])
                if idx != -1:
                    poses[t, part, :] = candidate[idx][:3]
        for i in range(len(subset)):
            if i != best:
                subset[i, :] = -1
        if mode == "bodyhand":
            for x, y, w, is_left in util.handDetect(candidate, subset, frames[t]):
                crop = frames[t][y:y + w, x:x + w, :]
                jobs.append((t, np.ascontiguousarray(crop[:, ::-1]) if is_left else crop, x, y, w, is_left))
    if jobs:
        peaks_all = hand.batch_crops([j[1] for j in jobs])
        for (t, _, x, y, w, is_left), peaks in zip(jobs, peaks_all):
            if is_left:
                peaks[:, 0] = np.where(peaks[:, 0] == 0, peaks[:, 0], w - peaks[:, 0] - 1 + x)
                peaks[:, 1] = np.where(peaks[:, 1] == 0, peaks[:, 1], peaks[:, 1] + y)
                poses[t, 18:39, :] = peaks
            else:
                peaks[:, 0] = np.where(peaks[:, 0] == 0, peaks[:, 0], peaks[:, 0] + x)
                peaks[:, 1] = np.where(peaks[:, 1] == 0, peaks[:, 1], peaks[:, 1] + y)
                poses[t, 39:60, :] = peaks
    return poses if mode == "bodyhand" else poses[:, :18, :]
