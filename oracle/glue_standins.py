"""ORACLE (test infrastructure only): planted stand-ins for Body / Hand that pin the host glue
of the reference's per-frame Body+Hand pipeline, `MotionData_every_frame`
(srcmx/MotionEstimation.py:126-216), independently of the networks.

The reference function is run (oracle/gen_golden.py glue) with these stand-ins in place of its
module-level `body_estimation` / `hand_estimation`, and `src/pipeline.py` is run with the same
stand-ins in tests/test_pipeline_glue.py.  The scenes exercise the glue's quirks:
* a person whose left shoulder (subset column 5) is missing: the reference reads
  candidate[-1][0] for it (src index -1), and that value decides the chosen person;
* hand boxes clamped at the bottom / right image edges (crops cut from the frame's corner);
* the left-hand crop flipped before Hand and x mapped back as w - x - 1 + x0;
* zero-preserving back-mapping (np.where(peaks == 0, ...)): a peak at x == 0 stays 0, and an
  all-missing hand comes back as the reference's int64 [[0, 0, 0]] * 21;
* no person at all (candidate shape (0,), subset (0, 20)).
"""
from __future__ import annotations

import zlib

import numpy as np

SCENES = (  # (seed, H, W)
    (900, 240, 320), (901, 240, 320), (902, 240, 320), (903, 240, 320), (904, 240, 320))

# arm template in units of person height: shoulder, elbow, wrist (right then left), neck-relative
_ARM = {2: (-0.14, 0.0), 3: (-0.20, 0.22), 4: (-0.24, 0.44), 5: (0.14, 0.0), 6: (0.20, 0.22), 7: (0.24, 0.44)}


def frame(seed, H, W):
    return np.random.default_rng(seed).integers(0, 256, (H, W, 3), dtype=np.uint8)


def scene(seed, H, W):
    """(candidate [n,4] float64 (x, y, score, id) or shape (0,), subset [p,20] float64)."""
    rng = np.random.default_rng(seed + 1)
    n_people = {902: 0, 903: 1}.get(seed, 3)
    people = []
    for p in range(n_people):
        ph = rng.uniform(0.35, 0.6) * H
        cx = rng.uniform(0.2, 0.8) * W
        cy = rng.uniform(0.15, 0.35) * H
        if seed == 901 and p == 0:  # hands clamped at the bottom-right corner
            cx, cy, ph = W - 0.16 * H, H - 0.45 * H, 0.9 * H
        pts = {}
        for part in range(18):
            if part in _ARM:
                ox, oy = _ARM[part]
            else:
                ox, oy = rng.uniform(-0.15, 0.15), rng.uniform(-0.2, 0.9)
            pts[part] = (float(np.clip(round(cx + ox * ph + rng.normal(0, 2)), 0, W - 1)),
                         float(np.clip(round(cy + oy * ph + rng.normal(0, 2)), 0, H - 1)))
        vis = {part: True for part in range(18)}
        for part in range(18):
            if part not in _ARM and rng.random() < 0.2:
                vis[part] = False
        if seed == 900 and p == 1:
            vis[5] = False  # left shoulder missing: the reference reads candidate[-1][0]
        if seed == 904 and p == 2:
            vis[5] = vis[4] = False
        people.append((pts, vis))
    cand, subset = [], []
    for p in range(n_people):
        subset.append([-1.0] * 20)
    for part in range(18):  # candidate ids run part by part, as src/body.py:89-92 assigns them
        for p, (pts, vis) in enumerate(people):
            if vis[part]:
                x, y = pts[part]
                score = float(rng.uniform(0.2, 1.0))
                cand.append([x, y, score, float(len(cand))])
                subset[p][part] = float(len(cand) - 1)
    for p in range(n_people):
        ids = [int(i) for i in subset[p][:18] if i >= 0]
        subset[p][18] = float(sum(cand[i][2] for i in ids) + rng.uniform(0, 2))
        subset[p][19] = float(len(ids))
    if seed == 900:  # make the last candidate's x the largest: the shoulder-less person wins
        cand[-1][0] = float(W - 1)
    c = np.array(cand, dtype=np.float64) if cand else np.array([])
    s = np.array(subset, dtype=np.float64).reshape(-1, 20) if subset else -1 * np.ones((0, 20))
    return c, s


class StandInBody:
    """Body(...)(img) -> the planted scene of the frame (looked up by content)."""
    scenes: dict = {}

    def __init__(self, *args, **kwargs):
        pass

    @classmethod
    def register(cls, img, cand, subset):
        cls.scenes[zlib.crc32(np.ascontiguousarray(img).tobytes())] = (cand, subset)

    def __call__(self, img):
        cand, subset = self.scenes[zlib.crc32(np.ascontiguousarray(img).tobytes())]
        return cand.copy(), subset.copy()

    def batch(self, frames):
        return [self(f) for f in frames]


class StandInHand:
    """Hand(...)(crop) -> 21 peaks derived from the crop's bytes (deterministic)."""

    def __init__(self, *args, **kwargs):
        pass

    def __call__(self, crop):
        crop = np.ascontiguousarray(crop)
        key = zlib.crc32(crop.tobytes()) ^ (crop.shape[0] << 16) ^ crop.shape[1]
        rng = np.random.default_rng(key)
        if key % 7 == 0:  # nothing found: the reference returns int64 zeros (src/hand.py:66-67)
            return np.array([[0, 0, 0]] * 21)
        w = crop.shape[1]
        rows = []
        for _ in range(21):
            u = rng.random()
            if u < 0.15:
                rows.append([0, 0, 0])
            elif u < 0.25:
                rows.append([0, int(rng.integers(1, max(2, w))), float(rng.random())])
            else:
                rows.append([int(rng.integers(1, max(2, w))), int(rng.integers(1, max(2, w))), float(rng.random())])
        return np.array(rows)

    def batch_crops(self, crops):
        return [self(c) for c in crops]


# ---------------------------------------------------------------- video front end
# Extract_MotionData_from_Video (srcmx/MotionEstimation.py:25-76) reads cv2.VideoCapture: the
# frame count the container reports sizes MotionMat, the frames that decode fill it.
CAP_PROP_FRAME_COUNT = 7  # cv2.CAP_PROP_FRAME_COUNT
ROI = [(40, 30), (360, 270)]  # Recpoint [(x0, y0), (x1, y1)]: a 240 x 320 crop of 300 x 400 frames


def video_frame(seed):
    """A 300 x 400 frame whose ROI crop is frame(seed, 240, 320) (a registered scene)."""
    full = np.random.default_rng(seed + 7).integers(0, 256, (300, 400, 3), dtype=np.uint8)
    full[ROI[0][1]:ROI[1][1], ROI[0][0]:ROI[1][0]] = frame(seed, 240, 320)
    return full


# path -> (seeds of the frames that decode, the count the container reports)
VIDEOS = {
    "clip_short.avi": ((900, 901, 902, 903, 904), 7),     # two frames fewer than reported: zero rows
    "clip_exact.avi": ((903, 900, 904), 3),
    "clip_overflow.avi": ((900, 901, 902, 903, 904), 3),  # more than reported: IndexError
}


class FakeCapture:
    """cv2.VideoCapture stand-in over VIDEOS (a path not in it does not open)."""

    def __init__(self, path):
        import os
        self.v = VIDEOS.get(os.path.basename(path))
        self.i = 0

    def isOpened(self):
        return self.v is not None

    def get(self, prop):
        assert prop == CAP_PROP_FRAME_COUNT
        return float(self.v[1])

    def read(self):
        if self.v is None or self.i >= len(self.v[0]):
            return False, None
        self.i += 1
        return True, video_frame(self.v[0][self.i - 1])
