"""CPU: host-side helpers against the reference's own outputs (util.handDetect golden) and
the record/pipeline glue (no GPU)."""
import glob
import json
import os

import numpy as np

from conftest import GOLDEN


def test_hand_detect_matches_reference():
    from src.util import handDetect
    cases = json.load(open(os.path.join(GOLDEN, "hand_detect.json")))
    assert len(cases) >= 10 and any(c["boxes"] for c in cases)
    for c in cases:
        d = np.load(os.path.join(GOLDEN, c["fixture"]))
        H, W = (int(v) for v in d["img_hw"])
        boxes = handDetect(d["candidate"], d["subset"], np.zeros((H, W, 3), np.uint8))
        assert [[int(x), int(y), int(w), bool(l)] for x, y, w, l in boxes] == c["boxes"], c["fixture"]


def test_pad_right_down_corner():
    from oracle.body_post import pad_right_down
    from src.util import padRightDownCorner
    img = np.arange(5 * 7 * 3, dtype=np.uint8).reshape(5, 7, 3)
    a, pa = padRightDownCorner(img, 8, 128)
    b, pb = pad_right_down(img, 8, 128)
    assert pa == pb == [0, 0, 3, 1] and np.array_equal(a, b)


def test_npmax_first_occurrence():
    from src.util import npmax
    a = np.array([[0, 3, 3], [3, 1, 0]], float)
    assert npmax(a) == (0, 1)


class _FakeBody:
    def __init__(self, cand, subset):
        self.c, self.s = cand, subset

    def __call__(self, img):
        return self.c.copy(), self.s.copy()


def test_pipeline_body_mode_picks_rightmost_left_shoulder():
    from src.pipeline import motion_data_every_frame
    p = sorted(glob.glob(os.path.join(GOLDEN, "body_planted_112_*.npz")))[0]
    d = np.load(p)
    pose = motion_data_every_frame(_FakeBody(d["candidate"], d["subset"]), None, np.zeros((368, 656, 3), np.uint8))
    sub, cand = d["subset"], d["candidate"]
    best = int(np.argmax([cand[int(r[5])][0] for r in sub]))
    assert pose.shape == (18, 3)
    for k in range(18):
        idx = int(sub[best][k])
        assert np.array_equal(pose[k], cand[idx][:3] if idx != -1 else np.zeros(3))


def test_draw_bodypose_marks_keypoints_and_limbs():
    """src/util.py:44-77 (OpenCV pixel parity unpinned: cv2 is absent): discs of the part colours
    at every keypoint, blended limb ellipses between connected parts, nothing elsewhere."""
    from src import util
    canvas = np.zeros((120, 160, 3), np.uint8)
    # one person: neck (1) at (80, 40), right shoulder (2) at (60, 40), right elbow (3) at (55, 70)
    candidate = np.array([[80.0, 40.0, 0.9, 0], [60.0, 40.0, 0.8, 1], [55.0, 70.0, 0.7, 2]])
    subset = -1 * np.ones((1, 20))
    subset[0, 1], subset[0, 2], subset[0, 3] = 0, 1, 2
    out = util.draw_bodypose(canvas, candidate, subset)
    assert out.shape == canvas.shape and out.dtype == np.uint8
    assert tuple(canvas[40, 80]) == (255, 85, 0)  # the neck disc (part 1 colour), drawn in place (as cv2.circle)
    assert out[40, 70].any()  # the neck-shoulder limb between them
    assert not out[110, 150].any() and not out[5, 5].any()


def test_draw_handpose_renders_rgb():
    from src import util
    canvas = np.zeros((60, 80, 3), np.uint8)
    peaks = np.zeros((21, 2))
    peaks[0], peaks[1], peaks[2] = (10, 10), (20, 15), (30, 25)
    img = util.draw_handpose(canvas, [peaks])
    assert img.ndim == 3 and img.shape[2] == 3 and img.dtype == np.uint8 and img.any()
