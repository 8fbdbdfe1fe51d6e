"""CPU: the host glue of the Body+Hand frame pipeline (src/pipeline.py) against the reference's
own `MotionData_every_frame` (srcmx/MotionEstimation.py:126-216), both driven by the same planted
Body / Hand stand-ins (oracle/glue_standins.py; golden from oracle/gen_golden.py glue).

Pins the glue's quirks bit for bit: the left-shoulder pick through candidate[-1] when a
person's shoulder is missing, hand boxes clamped at the frame edges, the flipped left-hand crop
and its w - x - 1 + x0 back-mapping, zero-preserving offsets (x == 0 stays 0; an all-missing hand
is int64 zeros), and the empty frame.  The GPU Body / Hand are pinned separately."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import glue_standins as gs
from src import pipeline


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "glue_motion_every_frame.npz"))


@pytest.fixture(scope="module")
def frames():
    out = []
    for seed, H, W in gs.SCENES:
        img = gs.frame(seed, H, W)
        gs.StandInBody.register(img, *gs.scene(seed, H, W))
        out.append((seed, img))
    return out


@pytest.mark.parametrize("mode", ["body", "bodyhand"])
def test_motion_data_every_frame_matches_reference(golden, frames, mode):
    body, hand = gs.StandInBody(), gs.StandInHand()
    for seed, img in frames:
        got = pipeline.motion_data_every_frame(body, hand, img, mode=mode)
        exp = golden[f"pose_{seed}_{mode}"]
        assert got.shape == exp.shape and got.dtype == exp.dtype
        assert np.array_equal(got, exp), seed


@pytest.mark.parametrize("mode", ["body", "bodyhand"])
def test_motion_data_frames_matches_reference(golden, frames, mode):
    """The batched variant (one Body launch sequence, one crop-batched Hand pass)."""
    got = pipeline.motion_data_frames(gs.StandInBody(), gs.StandInHand(), np.stack([f for _, f in frames]), mode=mode)
    exp = np.stack([golden[f"pose_{seed}_{mode}"] for seed, _ in frames])
    assert np.array_equal(got, exp)


def test_scenes_exercise_the_quirks(golden, frames):
    c, s = gs.scene(900, 240, 320)
    assert s[1][5] == -1 and c[-1][0] == 319  # shoulder-less person, largest candidate[-1] x
    assert np.array_equal(golden["pose_900_body"][:18], golden["pose_900_body"])
    assert not golden["pose_902_bodyhand"].any()  # empty frame
    assert (golden["pose_903_bodyhand"][18:] != 0).any()  # hands were found and mapped back
