"""CPU: the video front end (src/motion.py) against the reference's own
`Extract_MotionData_from_Video` (srcmx/MotionEstimation.py:25-76), both reading the same fake
videos through a cv2.VideoCapture stand-in and driven by the same planted Body / Hand
stand-ins (oracle/glue_standins.py; golden from oracle/gen_golden.py motion).

Pins the reference's file semantics bit for bit: MotionMat has CAP_PROP_FRAME_COUNT rows and
frames that never decode leave zero rows (a container reporting 7 frames with 5 decodable), a
video that decodes more frames than it reports raises IndexError (and writes nothing), a file
that does not open is reported on stdout and returns None, the ROI crop, body and bodyhand
modes, and the joblib file itself (read back).  The GPU ingest into the seeded-network golden
is tests/test_gpu_pipeline.py::test_extract_motion_video_device_ingest_matches_reference."""
import contextlib
import io
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import glue_standins as gs
from src import motion


@pytest.fixture(scope="module")
def golden():
    for seed, H, W in gs.SCENES:
        gs.StandInBody.register(gs.frame(seed, H, W), *gs.scene(seed, H, W))
    return np.load(os.path.join(GOLDEN, "motion_extract.npz"))


def _run(tmp_path, clip, mode):
    import joblib
    dst = os.path.join(str(tmp_path), "%s-%s.pkl" % (clip, mode))
    log = io.StringIO()
    with contextlib.redirect_stdout(log):
        ret = motion.Extract_MotionData_from_Video(os.path.join(str(tmp_path), clip), dst, gs.ROI, mode=mode,
                                                   body=gs.StandInBody(), hand=gs.StandInHand(),
                                                   capture=gs.FakeCapture, device=False, batch=2)
    out = joblib.load(dst) if os.path.exists(dst) else None
    text = log.getvalue().replace(str(tmp_path) + os.sep, "")
    return ret, out, text


def _progress_lines(text):
    # the reference's per-frame timing prints (MotionData_every_frame) are not part of the contract
    return [ln for ln in text.splitlines() if ln and not ln.startswith("each const time")]


@pytest.mark.parametrize("clip", ["clip_short", "clip_exact"])
@pytest.mark.parametrize("mode", ["body", "bodyhand"])
def test_motion_file_matches_reference(golden, tmp_path, clip, mode):
    ret, out, text = _run(tmp_path, clip + ".avi", mode)
    key = "%s_%s" % (clip, mode)
    assert ret is None and bool(golden[key + "_ret_none"])
    exp = golden[key]
    assert out.shape == exp.shape and out.dtype == exp.dtype
    assert np.array_equal(out, exp)
    assert _progress_lines(text) == _progress_lines(str(golden[key + "_stdout"]))


def test_short_container_leaves_zero_rows(golden):
    exp = golden["clip_short_bodyhand"]
    assert exp.shape[0] == 7 and not exp[5:].any() and exp[:5].any()


@pytest.mark.parametrize("mode", ["body", "bodyhand"])
def test_more_frames_than_reported_raises_index_error(golden, tmp_path, mode):
    assert str(golden["clip_overflow_%s_error" % mode]) == "IndexError"
    with pytest.raises(IndexError):
        _run(tmp_path, "clip_overflow.avi", mode)
    assert not os.listdir(str(tmp_path))  # nothing written, as the reference


@pytest.mark.parametrize("mode", ["body", "bodyhand"])
def test_missing_video_returns_none(golden, tmp_path, mode):
    ret, out, text = _run(tmp_path, "clip_missing.avi", mode)
    assert ret is None and out is None
    assert bool(golden["clip_missing_%s_ret_none" % mode]) and not bool(golden["clip_missing_%s_written" % mode])
    assert text.strip() == str(golden["clip_missing_%s_stdout" % mode]).strip()


def test_frame_list_keeps_decoded_count():
    """Without a container count (a plain list of frames), the matrix has one row per frame."""
    frames = [gs.frame(seed, 240, 320) for seed, _, _ in gs.SCENES[:3]]
    for seed, H, W in gs.SCENES:
        gs.StandInBody.register(gs.frame(seed, H, W), *gs.scene(seed, H, W))
    m = motion.extract_motion_data(frames, gs.StandInBody(), mode="body", device=False, batch=2)
    assert m.shape == (3, 18, 3)
    with pytest.raises(IndexError):
        motion.extract_motion_data(frames, gs.StandInBody(), mode="body", device=False, count=2)
