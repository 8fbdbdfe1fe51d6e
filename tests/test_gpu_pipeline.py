"""GPU: multi-scale Body (the 1080p pyramid path of config C5, on a small frame) and the
per-frame Body+Hand pipeline (srcmx/MotionEstimation.py:126-216, config C3) against the oracle
with the same seeded networks (bar: identical keypoint pixels / assignment, scores within
fp32 network noise)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nets():
    from src.body import Body
    from src.hand import Hand
    from src.weights import seeded_state_dict
    return seeded_state_dict("body", 0), seeded_state_dict("hand", 0), Body, Hand


def _oracle_body(scales):
    from oracle import body_post, network
    sd = network.seeded_state_dict("body", 0)

    def run(img):
        def net_fn(x):
            p, h = network.body_forward(torch.from_numpy(x), sd)
            return p.numpy(), h.numpy()
        return body_post.body_infer(img, net_fn, scale_search=scales)
    return run


def _oracle_hand():
    from oracle import hand_post, network
    sd = network.seeded_state_dict("hand", 0)
    return lambda img: hand_post.hand_infer(img, lambda x: network.hand_forward(torch.from_numpy(x), sd).numpy())


def _same(a, b):
    ca, sa = a
    cb, sb = b
    assert ca.shape == cb.shape and sa.shape == sb.shape
    if ca.size:
        assert np.array_equal(ca[:, [0, 1, 3]], cb[:, [0, 1, 3]])
        np.testing.assert_allclose(ca[:, 2], cb[:, 2], rtol=1e-3, atol=1e-4)
    assert np.array_equal(sa[:, :18], sb[:, :18]) and np.array_equal(sa[:, 19], sb[:, 19])
    np.testing.assert_allclose(sa[:, 18], sb[:, 18], rtol=1e-3)


@pytest.mark.parametrize("scales", [(0.5, 1.0), (0.5, 1.0, 1.5, 2.0)])
def test_multiscale_body_vs_oracle(nets, scales):
    bsd, _, Body, _ = nets
    body = Body(bsd, scale_search=scales)
    img = np.random.default_rng(31).integers(0, 256, (72, 96, 3), dtype=np.uint8)
    _same(body(img), _oracle_body(scales)(img))


def test_body_hand_pipeline_vs_oracle(nets):
    from src.pipeline import motion_data_every_frame
    bsd, hsd, Body, Hand = nets
    body, hand = Body(bsd), Hand(hsd)
    img = np.random.default_rng(21).integers(0, 256, (96, 128, 3), dtype=np.uint8)
    got = motion_data_every_frame(body, hand, img, mode="bodyhand")
    ref = motion_data_every_frame(_oracle_body((0.5,)), _oracle_hand(), img, mode="bodyhand")
    assert got.shape == ref.shape == (60, 3)
    assert np.array_equal(got[:, :2], ref[:, :2])
    np.testing.assert_allclose(got[:, 2], ref[:, 2], rtol=1e-3, atol=1e-4)


def test_hand_batch_crops_matches_single(nets):
    _, hsd, _, Hand = nets
    hand = Hand(hsd)
    rng = np.random.default_rng(41)
    crops = [rng.integers(0, 256, (w, w, 3), dtype=np.uint8) for w in (40, 57, 96, 128)]
    crops.append(np.ascontiguousarray(crops[2][:, ::-1]))  # flipped left hand
    crops.append(rng.integers(0, 256, (80, 80, 3), dtype=np.uint8)[10:60, 5:55])  # strided view
    batch = hand.batch_crops(crops)
    for c, b in zip(crops, batch):
        single = hand(np.ascontiguousarray(c))
        assert b.dtype == single.dtype and b.shape == (21, 3)
        np.testing.assert_allclose(b, single, rtol=1e-4, atol=1e-5)


def test_pipeline_frames_matches_per_frame(nets):
    from src.pipeline import motion_data_every_frame, motion_data_frames
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    _, hsd, Body, Hand = nets
    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
    hand = Hand(hsd)
    frames = np.random.default_rng(51).integers(0, 256, (3, 184, 240, 3), dtype=np.uint8)
    got = motion_data_frames(body, hand, frames)
    ref = np.stack([motion_data_every_frame(body, hand, f, mode="bodyhand") for f in frames])
    assert got.shape == ref.shape == (3, 60, 3)
    assert (ref[:, 18:, 2] > 0).any(), "no hand found: the test would not exercise the crop batch"
    assert np.array_equal(got[:, :, :2], ref[:, :, :2])
    np.testing.assert_allclose(got[:, :, 2], ref[:, :, 2], rtol=1e-3, atol=1e-4)


def test_extract_motion_data_matches_per_frame(nets, tmp_path):
    import joblib
    from src.motion import extract_motion_data
    from src.pipeline import motion_data_every_frame
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    _, hsd, Body, Hand = nets
    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
    hand = Hand(hsd)
    video = np.random.default_rng(61).integers(0, 256, (5, 200, 260, 3), dtype=np.uint8)
    rec = [(10, 8), (250, 192)]  # [(x0, y0), (x1, y1)]
    out = tmp_path / "motion.pkl"
    got = extract_motion_data(iter(video), body, hand, outpath=str(out), recpoint=rec, mode="bodyhand", batch=2)
    ref = np.stack([motion_data_every_frame(body, hand, f[8:192, 10:250], mode="bodyhand") for f in video])
    assert got.shape == (5, 60, 3)
    assert np.array_equal(got[:, :, :2], ref[:, :, :2])
    np.testing.assert_allclose(got[:, :, 2], ref[:, :, 2], rtol=1e-3, atol=1e-4)
    assert np.array_equal(joblib.load(out), got)
    body_only = extract_motion_data(video, body, recpoint=rec, mode="body", batch=4)
    assert body_only.shape == (5, 18, 3) and np.array_equal(body_only[:, :, :2], got[:, :18, :2])


def test_extract_motion_data_device_ingest_equals_host(nets):
    """The pinned, double-buffered GPU ingest (device=True: uploads on copy streams, pipelined
    Body.infer_records, records downloaded asynchronously, poses of batch k-1 decoded while batch
    k runs) against host batches (device=False: Body.batch): identical poses, both modes, a
    ragged last batch, and more batches than buffers."""
    from src.motion import extract_motion_data
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    _, hsd, Body, Hand = nets
    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
    hand = Hand(hsd)
    video = np.random.default_rng(62).integers(0, 256, (11, 200, 260, 3), dtype=np.uint8)
    rec = [(4, 6), (248, 190)]
    for mode in ("body", "bodyhand"):
        dev = extract_motion_data(iter(video), body, hand, recpoint=rec, mode=mode, batch=3, device=True)
        host = extract_motion_data(iter(video), body, hand, recpoint=rec, mode=mode, batch=3, device=False)
        assert dev.shape == host.shape == (11, 60 if mode == "bodyhand" else 18, 3)
        assert np.array_equal(dev, host), mode


def test_hand_batch_crops_beyond_one_launch(nets):
    """More crops than one network launch holds (at the 736-pixel scale ten crops fill the 2 GiB
    the conv kernels address): the batch is cut into launches of at most ten, every crop's
    result equals its single-crop Hand()."""
    _, hsd, _, Hand = nets
    hand = Hand(hsd)
    rng = np.random.default_rng(43)
    crops = [rng.integers(0, 256, (64, 64, 3), dtype=np.uint8) for _ in range(12)]
    batch = hand.batch_crops(crops)
    assert len(batch) == 12
    for c, b in zip(crops, batch):
        np.testing.assert_allclose(b, hand(c), rtol=1e-4, atol=1e-5)


def test_extract_motion_video_device_ingest_matches_reference(nets, tmp_path):
    """f2 end to end against the reference's own Extract_MotionData_from_Video
    (srcmx/MotionEstimation.py:25-76) run with its Body / Hand on the seeded networks
    (tests/golden/motion_extract_seeded.npz, oracle/gen_golden.py motion): a fake container that
    reports 4 frames and decodes 3 (the last row stays zero), the ROI crop, bodyhand mode (a
    flipped left hand on frame 2), read through src.motion's pinned double-buffered device ingest
    in batches of 2 and written with joblib.  Bar: the north-star one -- every joint's pixel
    identical, scores within fp32 network noise (rtol 1e-3)."""
    import contextlib
    import io
    import os

    import joblib

    from conftest import GOLDEN
    from oracle import glue_standins as gs
    from src.motion import Extract_MotionData_from_Video
    bsd, hsd, Body, Hand = nets
    g = np.load(os.path.join(GOLDEN, "motion_extract_seeded.npz"))
    gs.VIDEOS["clip_seeded.avi"] = (tuple(int(s) for s in g["seeds"]), int(g["count"]))
    dst = os.path.join(str(tmp_path), "seeded.pkl")
    with contextlib.redirect_stdout(io.StringIO()):
        assert Extract_MotionData_from_Video(os.path.join(str(tmp_path), "clip_seeded.avi"), dst, gs.ROI,
                                             mode="bodyhand", body=Body(bsd), hand=Hand(hsd), batch=2,
                                             device=True, capture=gs.FakeCapture) is None
    got, exp = joblib.load(dst), g["motion"]
    assert got.shape == exp.shape == (4, 60, 3) and got.dtype == exp.dtype
    assert (exp[2, 18:39] != 0).any() and not exp[3].any()
    assert np.array_equal(got[..., :2], exp[..., :2])
    np.testing.assert_allclose(got[..., 2], exp[..., 2], rtol=1e-3, atol=1e-6)
