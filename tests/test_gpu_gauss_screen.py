"""GPU: the Gaussian NMS stage (csrc/post.hip gauss_nms_wide) against the oracle's scipy
gaussian_filter + 4-neighbour NMS (src/body.py:70-94) on maps built to stress float64
near-ties: flat plateaus (neighbours within float32 noise of each other), dense noise (many
local maxima), values hugging the threshold, a single-pixel spike, and the two-scale float64
average.  Bar: the candidate and subset arrays are identical (bit-exact), as for every
post-network test."""
import numpy as np
import pytest

from oracle import body_post

pytestmark = pytest.mark.gpu

HL, WL = 12, 16  # low-res maps -> 96 x 128 frames (pad 0)


@pytest.fixture(scope="module")
def body():
    from src.body import Body
    from src.weights import seeded_state_dict
    return Body(seeded_state_dict("body", 0))


def _maps(kind, rng):
    heat = np.zeros((19, HL, WL), np.float32)
    paf = (rng.standard_normal((38, HL, WL)) * 0.3).astype(np.float32)
    if kind == "plateau":  # near-flat tops: neighbours within float32 noise of each other
        heat[:18] = np.float32(0.5) + rng.random((18, HL, WL), dtype=np.float32) * np.float32(1e-6)
        heat[:18, 4:8, 4:10] = np.float32(0.8) + rng.random((18, 4, 6), dtype=np.float32) * np.float32(1e-6)
    elif kind == "noise":
        heat[:18] = rng.random((18, HL, WL), dtype=np.float32)
    elif kind == "threshold":
        heat[:18] = np.float32(0.1) + (rng.random((18, HL, WL), dtype=np.float32) - 0.5) * np.float32(2e-6)
    elif kind == "spike":
        heat[:18, 6, 8] = 3.0
        heat[:18, 2, 3] = 0.11
    return paf, heat


@pytest.mark.parametrize("kind", ["plateau", "noise", "threshold", "spike"])
def test_screened_nms_single_scale(body, kind):
    rng = np.random.default_rng({"plateau": 1, "noise": 2, "threshold": 3, "spike": 4}[kind])
    paf, heat = _maps(kind, rng)
    H, W = HL * 8, WL * 8
    pad = [0, 0, 0, 0]
    maps = np.concatenate([paf, heat], 0)[None]
    cand, subset = body.post(maps, pad, H, W)[0]
    ref_c, ref_s = body_post.post_from_lowres((H, W), [(paf, heat, pad, (H, W))])
    assert np.array_equal(cand, ref_c) and np.array_equal(subset, ref_s)


def test_screened_nms_two_scales_float64_average():
    from src.body import Body
    from src.weights import seeded_state_dict
    rng = np.random.default_rng(7)
    H, W = 120, 168
    body2 = Body(seeded_state_dict("body", 0), scale_search=(0.5, 1.0))
    geoms = body2.scale_geom(H, W)
    lowres, maps = [], []
    for (hl, wl, pd, pr) in geoms:
        heat = np.zeros((19, hl, wl), np.float32)  # ~12 blobs per part, heights 0.05-0.9
        for part in range(18):
            ys, xs = rng.integers(0, hl, 12), rng.integers(0, wl, 12)
            heat[part, ys, xs] = rng.random(12, dtype=np.float32) * np.float32(0.85) + np.float32(0.05)
        paf = (rng.standard_normal((38, hl, wl)) * 0.3).astype(np.float32)
        lowres.append((paf, heat, [0, 0, pd, pr], (8 * hl, 8 * wl)))
        maps.append(np.concatenate([paf, heat], 0)[None])
    cand, subset = body2.post_scales(maps, H, W)[0]
    ref_c, ref_s = body_post.post_from_lowres((H, W), lowres)
    assert np.array_equal(cand, ref_c) and np.array_equal(subset, ref_s)


@pytest.mark.parametrize("hw", [(2, 5), (3, 14), (16, 2)], ids=lambda v: f"{v[0]}x{v[1]}")
def test_nms_maps_smaller_than_one_reflection(body, hw):
    """Maps so small that the 13-pixel filter footprint wraps more than once (scipy's periodic
    reflect; the kernel's division-based index path)."""
    hl, wl = hw
    rng = np.random.default_rng(11 + hl)
    heat = (rng.random((19, hl, wl), dtype=np.float32) * np.float32(0.9)).astype(np.float32)
    paf = (rng.standard_normal((38, hl, wl)) * 0.3).astype(np.float32)
    H, W = hl * 8, wl * 8
    pad = [0, 0, 0, 0]
    cand, subset = body.post(np.concatenate([paf, heat], 0)[None], pad, H, W)[0]
    ref_c, ref_s = body_post.post_from_lowres((H, W), [(paf, heat, pad, (H, W))])
    assert np.array_equal(cand, ref_c) and np.array_equal(subset, ref_s)
