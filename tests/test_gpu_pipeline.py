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
