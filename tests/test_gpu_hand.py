"""GPU parity for Hand(): planted 4-scale heat maps (reference fixtures, bit-exact) and an
end-to-end seeded-network run against the oracle (keypoints equal, scores within fp32 noise)."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

SCALES = (0.5, 1.0, 1.5, 2.0)


@pytest.fixture(scope="module")
def hand():
    from src.hand import Hand
    from src.weights import seeded_state_dict
    return Hand(seeded_state_dict("hand", 0))


def _pads(S):
    out = []
    for s in SCALES:
        m = s * 368 / S
        hs = round(S * m)
        out.append([0, 0, (8 - hs % 8) % 8, (8 - hs % 8) % 8])
    return out


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "hand_planted_*.npz"))), ids=os.path.basename)
def test_hand_post_matches_reference_exactly(hand, path):
    d = np.load(path)
    S = int(d["size"])
    maps = [d[f"heat{i}"][None] for i in range(4)]
    peaks = hand.post(maps, _pads(S), S, S)[0]
    assert peaks.dtype == d["peaks"].dtype
    assert np.array_equal(peaks, d["peaks"])


def test_hand_end_to_end_vs_oracle(hand):
    from oracle import hand_post, network
    sd = network.seeded_state_dict("hand", 0)
    img = np.random.default_rng(3).integers(0, 256, (64, 64, 3), dtype=np.uint8)
    ref = hand_post.hand_infer(img, lambda x: network.hand_forward(torch.from_numpy(x), sd).numpy())
    out = hand(img)
    assert out.shape == (21, 3) and out.dtype == ref.dtype
    assert np.array_equal(out[:, :2], ref[:, :2])
    np.testing.assert_allclose(out[:, 2], ref[:, 2], rtol=1e-3, atol=1e-4)


def test_hand_batch_and_all_missing(hand):
    # a flat grey crop: whatever the seeded network says, batch == single
    crops = np.random.default_rng(4).integers(0, 256, (3, 48, 48, 3), dtype=np.uint8)
    batch = hand.batch(crops)
    for c, b in zip(crops, batch):
        np.testing.assert_allclose(hand(c), b, rtol=1e-4, atol=1e-5)
    # all-missing -> int64 zeros like np.array([[0, 0, 0]] * 21)
    from src.hand import _as_reference_array
    z = _as_reference_array(np.zeros((21, 3)), np.zeros(21, np.int32))
    assert z.dtype == np.int64 and not z.any()


@pytest.mark.parametrize("seed,S", [(0, 120), (1, 120), (2, 120), (3, 120), (4, 368), (5, 368)])
def test_hand_post_intricate_components(hand, seed, S):
    """Heat maps hovering around the threshold: many components with holes, diagonal-only
    contacts and long snakes after the x8 upsample + Gaussian -- the labelling (per 64 x 32
    tile in LDS, then joined across tile edges: 2 x 4 tiles at S = 120, 6 x 12 at 368), the
    sums and the selection must match the oracle (scipy.ndimage.label) exactly."""
    from scipy.ndimage import gaussian_filter
    from oracle import hand_post
    from oracle.body_post import preprocess
    rng = np.random.default_rng(100 + seed)
    maps, lowres, pads = [], [], []
    for s in SCALES:
        _, pad, padded_hw = preprocess(np.zeros((S, S, 3), np.uint8), s * 368 / S)
        h, w = padded_hw[0] // 8, padded_hw[1] // 8
        noise = gaussian_filter(rng.standard_normal((22, h, w)), (0, 0.7, 0.7))
        heat = (0.03 + 0.08 * noise / noise.std()).astype(np.float32)
        maps.append(heat[None])
        lowres.append((heat, pad, padded_hw))
        pads.append(pad)
    ref = hand_post.post_from_lowres((S, S), lowres)
    out = hand.post(maps, pads, S, S)[0]
    assert out.dtype == ref.dtype
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("shape", [(368, 368), (100, 70), (33, 200)])
def test_hand_labels_match_scipy(hand, shape):
    """The labelling itself (gauss_threshold's per-tile components in LDS + cc_border across tile
    edges + cc_compress_sum), label for label: binary = gaussian_filter(map, 3) > thre and
    scipy.ndimage.label(binary, 8-connectivity) (src/hand.py:62-64), each component named by its
    first pixel in raster order (scipy's numbering order).  Maps hover around the threshold so
    the components are many, holed, snaking and diagonal-only-connected; the shapes leave ragged
    64 x 32 tiles at the right and bottom edges.  Component sums against numpy at 1e-12."""
    from scipy.ndimage import gaussian_filter, label
    from src import _native
    H, W = shape
    rng = np.random.default_rng(H * 7 + W)
    NP = 3
    noise = gaussian_filter(rng.standard_normal((NP, H, W)), (0, 2.5, 2.5))
    maps = np.ascontiguousarray(0.05 + 0.1 * noise / noise.std())
    thre = 0.05
    labels = np.empty((NP, H, W), np.int32)
    sums = np.empty((NP, H, W), np.float64)
    hand.handle.check(_native.lib.opose_debug_hand_label(hand.handle.h, maps.ctypes.data, NP, H, W, thre,
                                                         labels.ctypes.data, sums.ctypes.data))
    ncomp = 0
    for k in range(NP):
        binary = gaussian_filter(maps[k], sigma=3) > thre
        lab, n = label(binary, structure=np.ones((3, 3), int))
        ncomp += n
        flat = lab.ravel()
        first = np.zeros(n + 1, np.int64)  # first (raster-order) pixel of each scipy label
        idx = np.flatnonzero(flat)
        first[1:] = np.full(n, flat.size)
        np.minimum.at(first, flat[idx], idx)
        expect = np.where(flat > 0, first[flat], -1).reshape(H, W)
        assert np.array_equal(labels[k], expect.astype(np.int32)), k
        ref_sums = np.bincount(flat, weights=maps[k].ravel(), minlength=n + 1)[1:]
        np.testing.assert_allclose(sums[k].ravel()[first[1:]], ref_sums, rtol=1e-12, atol=1e-12)
    assert ncomp > 10
