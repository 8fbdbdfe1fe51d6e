"""GPU: the north-star bar at the configurations' full sizes (verdict r3 item 2).

* C5: Body() on one 1080x1920 frame with scale_search [0.5, 1.0, 1.5, 2.0] (the C5 calibration:
  ~200 keypoints, 10 people), four networks of 184x328 .. 736x1312;
* C3: Hand() on one 368x368 crop, the four pyramid networks 184^2 .. 736^2;
against the oracle (oracle/network.py + body_post / hand_post, pinned to the reference's own
goldens by tests/test_oracle_golden.py) run on the CPU in this container
(tests/golden/fullsize_c3_c5.npz, oracle/gen_golden.py fullsize; the inputs are regenerated from
their seeds).  The oracle's float32 and float64 networks place every keypoint identically on
these inputs (no plateau ties), so the bar is the exact one: every keypoint's pixel and id, every
person's parts and part count identical; scores within fp32 network noise (rtol 1e-3)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "fullsize_c3_c5.npz"))


def test_fixture_has_no_plateau_ties(golden):
    assert np.array_equal(golden["c5_cand_f32"][:, [0, 1, 3]], golden["c5_cand_f64"][:, [0, 1, 3]])
    assert np.array_equal(golden["c5_subset_f32"][:, :18], golden["c5_subset_f64"][:, :18])
    assert np.array_equal(golden["c3_peaks_f32"][:, :2], golden["c3_peaks_f64"][:, :2])


def test_body_1080p_four_scales_vs_oracle(golden):
    from src.body import Body
    from src.weights import c5_out_scale, seeded_state_dict
    body = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=(0.5, 1.0, 1.5, 2.0))
    img = np.random.default_rng(int(golden["c5_seed"])).integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
    cand, subset = body(img)
    rc, rs = golden["c5_cand_f32"], golden["c5_subset_f32"]
    assert len(rc) > 150 and len(rs) >= 8
    assert cand.shape == rc.shape and subset.shape == rs.shape
    assert np.array_equal(cand[:, [0, 1, 3]], rc[:, [0, 1, 3]])
    np.testing.assert_allclose(cand[:, 2], rc[:, 2], rtol=1e-3, atol=1e-4)
    assert np.array_equal(subset[:, :18], rs[:, :18]) and np.array_equal(subset[:, 19], rs[:, 19])
    np.testing.assert_allclose(subset[:, 18], rs[:, 18], rtol=1e-3)


def test_hand_368_crop_vs_oracle(golden):
    from src.hand import Hand
    from src.weights import seeded_state_dict
    hand = Hand(seeded_state_dict("hand", 0))
    crop = np.random.default_rng(int(golden["c3_seed"])).integers(0, 256, (368, 368, 3), dtype=np.uint8)
    peaks = hand(crop)
    ref = golden["c3_peaks_f32"]
    assert (ref[:, 2] > 0).sum() >= 10
    assert peaks.shape == ref.shape and peaks.dtype == ref.dtype
    assert np.array_equal(peaks[:, :2], ref[:, :2])
    np.testing.assert_allclose(peaks[:, 2], ref[:, 2], rtol=1e-3, atol=1e-4)
