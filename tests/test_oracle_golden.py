"""CPU: pin the oracle (CPU restatement) against fixtures recorded from the imported reference."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from oracle import body_post, hand_post, network
from oracle.cv_resize import cubic_coeffs, resize_cubic

from conftest import GOLDEN, golden_image


def _files(pat):
    fs = sorted(glob.glob(os.path.join(GOLDEN, pat)))
    assert fs, pat
    return fs


@pytest.mark.parametrize("path", _files("net_*.npz"), ids=os.path.basename)
def test_network_matches_reference_model(path):
    d = np.load(path)
    net = "body" if "body" in os.path.basename(path) else "hand"
    sd = network.seeded_state_dict(net, 0)
    x = torch.from_numpy(d["x"])
    if net == "body":
        paf, heat = network.body_forward(x, sd)
        np.testing.assert_allclose(paf.numpy(), d["paf"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(heat.numpy(), d["heat"], rtol=1e-5, atol=1e-6)
        assert (heat.numpy() >= 0).all()   # ReLU after Mconv7_stage6_L2 (src/model.py:30-33)
    else:
        np.testing.assert_allclose(network.hand_forward(x, sd).numpy(), d["heat"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("path", _files("body_planted_*.npz"), ids=os.path.basename)
def test_body_post_matches_reference(path):
    d = np.load(path)
    lowres = [(d["paf"], d["heat"], list(d["pad"]), tuple(d["padded_hw"]))]
    if str(d["error"]):
        with pytest.raises(IndexError):
            body_post.post_from_lowres(tuple(d["img_hw"]), lowres)
        return
    cand, subset = body_post.post_from_lowres(tuple(d["img_hw"]), lowres)
    assert cand.shape == d["candidate"].shape and cand.dtype == d["candidate"].dtype
    assert np.array_equal(cand, d["candidate"])
    assert np.array_equal(subset, d["subset"])


def _c5_lowres(d):
    n = len(d["scales"])
    return [(d[f"paf{i}"], d[f"heat{i}"], list(d[f"pad{i}"]), tuple(d[f"padded{i}"])) for i in range(n)]


def test_body_post_c5_matches_reference():
    """C5 (BASELINE.json): 1080x1920, scale_search [0.5, 1, 1.5, 2], the reference's multi-scale
    Body on planted per-scale maps (oracle/gen_golden.py c5).  The 3-person case only here (the
    float64 full-resolution NumPy path takes ~20 s); the GPU test covers both."""
    d = np.load(os.path.join(GOLDEN, "body_c5_701_1080x1920_p3.npz"))
    cand, subset = body_post.post_from_lowres(tuple(d["img_hw"]), _c5_lowres(d))
    assert np.array_equal(cand, d["candidate"]) and np.array_equal(subset, d["subset"])


@pytest.mark.slow
@pytest.mark.parametrize("path", _files("body_e2e_*.npz"), ids=os.path.basename)
def test_body_end_to_end_matches_reference(path):
    d = np.load(path)
    sd = network.seeded_state_dict("body", 0)

    def net_fn(x):
        p, h = network.body_forward(torch.from_numpy(x), sd)
        return p.numpy(), h.numpy()

    nt = torch.get_num_threads()
    torch.set_num_threads(8)  # the goldens' thread count (the reference's order depends on it)
    try:
        cand, subset = body_post.body_infer(golden_image(d), net_fn)
    finally:
        torch.set_num_threads(nt)
    assert np.array_equal(cand, d["candidate"])
    assert np.array_equal(subset, d["subset"])


@pytest.mark.parametrize("path", _files("hand_planted_*.npz"), ids=os.path.basename)
def test_hand_post_matches_reference(path):
    d = np.load(path)
    size = int(d["size"])
    calls = iter([d[f"heat{i}"] for i in range(4)])
    peaks = hand_post.hand_infer(np.zeros((size, size, 3), np.uint8), lambda x: next(calls)[None])
    assert peaks.dtype == d["peaks"].dtype
    assert np.array_equal(peaks, d["peaks"])


def test_hand_output_size_table():
    """Known-answer artefact shipped by the reference (src/hand_model_output_size.json)."""
    with open(os.path.join(GOLDEN, "hand_model_output_size.json")) as f:
        table = {int(k): v for k, v in json.load(f).items()}
    assert len(table) == 990
    for i, v in table.items():
        assert v == i // 2 // 2 // 2   # three floor-mode 2x2 pools (src/model.py:147,150,155)


def test_cubic_coeffs_partition_of_unity():
    f = np.linspace(0, 1, 257, dtype=np.float32)[:-1]
    c = cubic_coeffs(f)
    assert np.allclose(c.sum(1), 1, atol=1e-6)
    assert np.array_equal(cubic_coeffs(np.float32([0]))[0], np.float32([0, 1, 0, 0]))


def test_resize_identity_and_sizes():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    assert np.array_equal(resize_cubic(img, (53, 37)), img)
    out = resize_cubic(img, (0, 0), fx=0.5, fy=0.5)
    assert out.shape == (round(37 * 0.5), round(53 * 0.5), 3)
    f = rng.random((5, 7, 19), dtype=np.float32)
    up = resize_cubic(f, (0, 0), fx=8, fy=8)
    assert up.shape == (40, 56, 19) and up.dtype == np.float32
    # a constant map stays constant through the cubic kernel (coefficients sum to ~1)
    c = np.full((5, 7, 2), 0.25, np.float32)
    assert np.allclose(resize_cubic(c, (0, 0), fx=8, fy=8), 0.25, atol=1e-6)


def test_flops_match_survey():
    assert network.body_flops(184, 328) == 121158571264
    assert network.body_flops(184, 184) == 67967003392
    assert network.hand_flops(368, 368) == 206375342080


# ---- Batch_body fast mode (srcmx/Batch_model.py:137-204) ---------------------------------
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "batch_body_planted_*.npz"))),
                         ids=os.path.basename)
def test_batch_oracle_planted_matches_reference(path):
    import torch
    from oracle import batch_post
    d = np.load(path)
    H, W = (int(v) for v in d["img_hw"])
    _, nh, nw, _, _ = batch_post.size_pad(0.5, H, W)
    res = batch_post.post(torch.from_numpy(d["paf"]), torch.from_numpy(d["heat"]), (H, W, nh, nw))
    for i, (c, s) in enumerate(res):
        assert np.array_equal(np.asarray(c, np.float64).reshape(-1, 4) if len(c) else c, d[f"candidate{i}"])
        assert np.array_equal(s, d[f"subset{i}"])


def test_batch_oracle_e2e_matches_reference():
    import torch
    from oracle import batch_post, network
    d = np.load(os.path.join(GOLDEN, "batch_body_e2e_23_96x128_b2.npz"))
    sd = network.seeded_state_dict("body", 0)

    def net_fn(x):
        p, h = network.body_forward(torch.from_numpy(x), sd)
        return p.numpy(), h.numpy()
    res = batch_post.batch_body_infer(d["frames"], net_fn)
    for i, (c, s) in enumerate(res):
        ref_c, ref_s = d[f"candidate{i}"], d[f"subset{i}"]
        # the torch-CPU network here vs the reference's nn.Module: same ops, fp32 noise only
        assert c.shape == ref_c.shape and s.shape == ref_s.shape
        assert np.array_equal(c[:, [0, 1, 3]], ref_c[:, [0, 1, 3]])
        np.testing.assert_allclose(c[:, 2], ref_c[:, 2], rtol=1e-5, atol=1e-6)
        assert np.array_equal(s[:, :18], ref_s[:, :18])


def test_batch_hand_oracle_matches_reference():
    import torch
    from oracle import batch_post
    d = np.load(os.path.join(GOLDEN, "batch_hand_planted_b4.npz"))
    got = batch_post.hand_post(torch.from_numpy(d["heat"]))
    assert got.dtype == d["peaks"].dtype and np.array_equal(got, d["peaks"])
    d = np.load(os.path.join(GOLDEN, "batch_hand_e2e_b2_64.npz"))
    sd = network.seeded_state_dict("hand", 0)
    got = batch_post.batch_hand_infer(d["crops"], lambda x: network.hand_forward(torch.from_numpy(x), sd).numpy())
    assert np.array_equal(got[:, :, :2], d["peaks"][:, :, :2])
    np.testing.assert_allclose(got[:, :, 2], d["peaks"][:, :, 2], rtol=1e-5)
