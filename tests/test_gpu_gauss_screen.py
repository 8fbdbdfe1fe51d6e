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


def _blob_maps(rng, hl, wl, per_part=12):
    heat = np.zeros((19, hl, wl), np.float32)  # sparse blobs, heights 0.05-0.9
    for part in range(18):
        ys, xs = rng.integers(0, hl, per_part), rng.integers(0, wl, per_part)
        heat[part, ys, xs] = rng.random(per_part, dtype=np.float32) * np.float32(0.85) + np.float32(0.05)
    paf = (rng.standard_normal((38, hl, wl)) * 0.3).astype(np.float32)
    return paf, heat


# (hl, wl, pad_down, pad_right, H, W): the x8 map (8hl - pad_down) x (8wl - pad_right) resized to
# H x W.  A true upsampling resize (source step <= 0.618) runs gauss_nms_resize (the heat-map
# resize fused into the NMS tiles, cold tiles dropped on a bound of their sources); the last two
# cases run the separate heat_full_f32 + gauss_nms_wide (a source step too large for the fused
# kernel's staged rows, and the identity size); (2, 3, ...) wraps the filter footprint (H < 56).
RESIZE_CASES = [(12, 16, 0, 0, 200, 260), (46, 82, 0, 0, 368, 656), (23, 41, 3, 5, 331, 587),
                (46, 82, 2, 0, 1080, 1920), (2, 3, 0, 0, 40, 50), (23, 41, 0, 0, 200, 300),
                (12, 16, 0, 0, 96, 128)]


@pytest.mark.parametrize("case", RESIZE_CASES, ids=lambda c: "%dx%d_from_%dx%d" % (c[4], c[5], c[0], c[1]))
def test_resize_nms_matches_oracle(body, case):
    hl, wl, pd, pr, H, W = case
    rng = np.random.default_rng(hl * 1000 + W)
    paf, heat = _blob_maps(rng, hl, wl, per_part=12 if H < 1000 else 30)
    pad = [0, 0, pd, pr]
    cand, subset = body.post(np.concatenate([paf, heat], 0)[None], pad, H, W)[0]
    ref_c, ref_s = body_post.post_from_lowres((H, W), [(paf, heat, pad, (8 * hl, 8 * wl))])
    assert len(ref_c) > 0
    assert np.array_equal(cand, ref_c) and np.array_equal(subset, ref_s)


@pytest.mark.parametrize("level", [0.0526, 0.0527, 0.1, 0.3])
def test_cold_tile_bound_at_the_threshold(body, level):
    """Sources just below / above the skip bound (1.9 * max|source| vs thre1 = 0.1): a flat
    patch of height `level` whose resized values overshoot around its edges, so peaks may sit
    anywhere in the tile; records equal the oracle's either way (skipping is exact)."""
    hl, wl, H, W = 23, 41, 368, 656
    rng = np.random.default_rng(int(level * 1e4))
    heat = np.zeros((19, hl, wl), np.float32)
    for part in range(18):
        y, x = rng.integers(2, hl - 4), rng.integers(2, wl - 4)
        heat[part, y:y + 2, x:x + 3] = np.float32(level)
        heat[part, rng.integers(0, hl), rng.integers(0, wl)] = -np.float32(level)
    paf = (rng.standard_normal((38, hl, wl)) * 0.3).astype(np.float32)
    pad = [0, 0, 0, 0]
    cand, subset = body.post(np.concatenate([paf, heat], 0)[None], pad, H, W)[0]
    ref_c, ref_s = body_post.post_from_lowres((H, W), [(paf, heat, pad, (8 * hl, 8 * wl))])
    assert np.array_equal(cand, ref_c) and np.array_equal(subset, ref_s)
