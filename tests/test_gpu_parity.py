"""GPU parity: libopose (HIP on cuda:0) against the oracle and the reference's golden fixtures.

Tolerances:
* integer / index / float64 post-processing and the OpenCV-cubic resize chain: bit-exact.
* network (fp32 MFMA vs the reference's torch-CPU conv, different summation order):
  |gpu - ref| <= 2e-4 * max|ref| + 2e-4 * |ref| over the stacked 92-conv graph; single convs
  against a float64 reference within 4e-6 * conv(|x|, |w|) (fp32 rounding of K-term sums).
"""
import ctypes as C
import glob
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN, golden_image, report

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from src import _native
    return _native


@pytest.fixture(scope="module")
def handle(native):
    return native.Handle(0)


@pytest.fixture(scope="module")
def body():
    from src.body import Body
    from src.weights import seeded_state_dict
    return Body(seeded_state_dict("body", 0))


def _conv_case(native, handle, N, Cin, H, W, Cout, ks, relu, mt=0, pt=0, splits=0, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((N, Cin, H, W), dtype=np.float32)
    w = (rng.standard_normal((Cout, Cin, ks, ks), dtype=np.float32) * np.float32(1 / np.sqrt(Cin * ks * ks)))
    b = rng.standard_normal(Cout, dtype=np.float32)
    out = np.empty((N, Cout, H, W), np.float32)
    pad = ks // 2
    handle.check(native.lib.opose_debug_conv(handle.h, x.ctypes.data, w.ctypes.data, b.ctypes.data, N, Cin, H, W,
                                             Cout, ks, pad, int(relu), mt, pt, splits, out.ctypes.data))
    xd, wd, bd = (torch.from_numpy(a).double() for a in (x, w, b))
    ref = F.conv2d(xd, wd, bd, padding=pad)
    if relu:
        ref = ref.clamp_min(0)
    bound = F.conv2d(xd.abs(), wd.abs(), bd.abs(), padding=pad) * 4e-6 + 1e-6
    err = (torch.from_numpy(out).double() - ref).abs()
    assert (err <= bound).all(), float((err / bound).max())


@pytest.mark.parametrize("N,Cin,H,W,Cout,ks", [
    (1, 3, 40, 72, 64, 3),      # conv1_1 (K = 27 -> padded 32)
    (2, 64, 23, 41, 128, 3),
    (1, 185, 23, 41, 128, 7),   # Mconv1 (K = 9065, ragged)
    (3, 128, 11, 13, 38, 1),    # Mconv7 (Cout < 64)
    (1, 512, 9, 9, 19, 1),
    (2, 128, 23, 41, 256, 7),
])
def test_conv_heuristic_tiles(native, handle, N, Cin, H, W, Cout, ks):
    _conv_case(native, handle, N, Cin, H, W, Cout, ks, relu=True)


@pytest.mark.parametrize("mt,pt,splits", [(128, 128, 1), (128, 64, 1), (64, 128, 1), (64, 64, 1), (128, 256, 1),
                                          (128, 128, 4), (64, 64, 7), (128, 64, 3), (128, 256, 5), (128, 256, 0)])
def test_conv_every_tile_and_split(native, handle, mt, pt, splits):
    _conv_case(native, handle, 2, 96, 17, 29, 128, 3, relu=False, mt=mt, pt=pt, splits=splits, seed=3)


@pytest.mark.parametrize("cout,mt,pt,splits", [(128, 128, 256, 0), (128, 128, 256, 7), (128, 128, 128, 9),
                                               (256, 256, 128, 0), (256, 256, 128, 5), (192, 256, 128, 3)])
def test_conv_7x7_tiles(native, handle, cout, mt, pt, splits):
    # Mconv shapes (128 -> 128 / 256, 7x7) on a ragged pixel count
    _conv_case(native, handle, 3, 128, 23, 41, cout, 7, relu=True, mt=mt, pt=pt, splits=splits, seed=4)


@pytest.mark.parametrize("splits", [0, 1, 6])
def test_conv_256_rows(native, handle, splits):
    _conv_case(native, handle, 2, 96, 17, 29, 256, 3, relu=False, mt=256, pt=128, splits=splits, seed=5)


def test_preprocess_bit_exact(native, handle):
    from oracle.body_post import preprocess
    rng = np.random.default_rng(5)
    # (H, W, scale_search entry); multiplier = s * 368 / H as src/body.py:32
    for (H, W, s) in [(368, 656, 0.5), (240, 320, 0.5), (97, 131, 1.0), (1080, 1920, 1.5),
                      (368, 368, 1.0), (100, 180, 2.0), (53, 97, 0.5),
                      # C5's smallest scale (a 5.9x source step) and a 41x source step
                      (1080, 1920, 0.5), (1500, 2999, 0.1),
                      # frames whose byte size is a whole number of pages (no slack after the
                      # buffer's last byte)
                      (128, 128, 1.0), (256, 256, 0.5)]:
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        hw = np.zeros(2, np.int32)
        handle.check(native.lib.opose_debug_preprocess(handle.h, img.ctypes.data, H, W, s, 128, None,
                                                       hw.ctypes.data))
        out = np.empty((3, hw[0], hw[1]), np.float32)
        handle.check(native.lib.opose_debug_preprocess(handle.h, img.ctypes.data, H, W, s, 128, out.ctypes.data,
                                                       hw.ctypes.data))
        ref, _, _ = preprocess(img, s * 368 / H)
        assert ref.shape == (1,) + out.shape, (ref.shape, out.shape)
        assert np.array_equal(out, ref[0]), (H, W, s)


def test_heat_chain_bit_exact(native, handle):
    from oracle.body_post import upsample_map
    from oracle.cv_resize import resize_cubic
    for path in sorted(glob.glob(os.path.join(GOLDEN, "body_planted_*.npz")))[:6]:
        d = np.load(path)
        H, W = (int(v) for v in d["img_hw"])
        pad, padded = list(d["pad"]), tuple(d["padded_hw"])
        maps = np.ascontiguousarray(np.concatenate([d["paf"], d["heat"]], 0))
        hl, wl = maps.shape[1:]
        heat = np.empty((18, H, W), np.float64)
        Hs, Ws = padded[0] - pad[2], padded[1] - pad[3]
        paf_mid = np.empty((38, Hs, Ws), np.float32)
        handle.check(native.lib.opose_debug_heat(handle.h, maps.ctypes.data, hl, wl, pad[2], pad[3], H, W,
                                                 heat.ctypes.data, paf_mid.ctypes.data))
        ref = np.zeros((H, W, 19)) + upsample_map(d["heat"], pad, padded, (H, W)) / 1
        assert np.array_equal(heat, np.transpose(ref[:, :, :18], (2, 0, 1))), path
        mid = resize_cubic(np.ascontiguousarray(np.transpose(d["paf"], (1, 2, 0))), (0, 0), fx=8, fy=8)[:Hs, :Ws]
        assert np.array_equal(paf_mid, np.transpose(mid, (2, 0, 1))), path


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "body_planted_*.npz"))),
                         ids=os.path.basename)
def test_body_post_matches_reference_exactly(body, path):
    d = np.load(path)
    H, W = (int(v) for v in d["img_hw"])
    maps = np.concatenate([d["paf"], d["heat"]], 0)[None]
    if str(d["error"]):
        with pytest.raises(IndexError):
            body.post(maps, list(d["pad"]), H, W)
        return
    cand, subset = body.post(maps, list(d["pad"]), H, W)[0]
    assert cand.shape == d["candidate"].shape
    assert np.array_equal(cand, d["candidate"])
    assert np.array_equal(subset, d["subset"])


def test_body_post_batch_equals_single(body):
    paths = sorted(glob.glob(os.path.join(GOLDEN, "body_planted_*_368x656_*.npz")))[:8]
    ds = [np.load(p) for p in paths]
    maps = np.stack([np.concatenate([d["paf"], d["heat"]], 0) for d in ds])
    outs = body.post(maps, list(ds[0]["pad"]), 368, 656)
    for d, (cand, subset) in zip(ds, outs):
        assert np.array_equal(cand, d["candidate"]) and np.array_equal(subset, d["subset"])


def _net_tol(gpu, ref):
    ref = np.asarray(ref)
    np.testing.assert_allclose(gpu, ref, rtol=2e-4, atol=2e-4 * float(np.abs(ref).max()))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "net_*.npz"))), ids=os.path.basename)
def test_network_matches_reference_model(path):
    from src.model import bodypose_model, handpose_model
    from src.util import transfer
    from src.weights import seeded_state_dict
    d = np.load(path)
    if "body" in os.path.basename(path):
        m = bodypose_model()
        m.load_state_dict(transfer(m, seeded_state_dict("body", 0)))
        paf, heat = m(d["x"])
        _net_tol(paf, d["paf"])
        _net_tol(heat, d["heat"])
        assert (heat >= 0).all()
    else:
        m = handpose_model()
        m.load_state_dict(transfer(m, seeded_state_dict("hand", 0)))
        _net_tol(m(d["x"]), d["heat"])


def test_network_full_size_and_batch_vs_oracle():
    from oracle import network as onet
    from src.model import bodypose_model
    from src.util import transfer
    from src.weights import seeded_state_dict
    x = np.random.default_rng(7).random((3, 3, 184, 328), dtype=np.float32) - np.float32(0.5)
    m = bodypose_model()
    m.load_state_dict(transfer(m, seeded_state_dict("body", 0)))
    paf, heat = m(x)
    rp, rh = onet.body_forward(torch.from_numpy(x[:1]), onet.seeded_state_dict("body", 0))
    _net_tol(paf[:1], rp.numpy())
    _net_tol(heat[:1], rh.numpy())
    # batching: frame 0 alone vs inside a batch of 3 (tile / split-K choices depend on the batch,
    # so the fp32 summation order may differ; the network tolerance applies)
    p1, h1 = m(x[:1])
    _net_tol(p1, paf[:1])
    _net_tol(h1, heat[:1])
    p2, _ = m(x[2:3])
    _net_tol(p2, paf[2:3])


# Keypoints the GPU may place on the other pixel of a float64 plateau (oracle/ties.py: smoothed
# values within 1e-6 of the part map's max), per fixture -- the count observed on hardware (rounds
# 5 and 6: 3 of 1,350), within what the reference moves against itself at that size
# (profiles/r5_ref_thread_noise.json: body_e2e_31 at 1 / 16 torch threads moves 4 / 2 of its own
# keypoints, all onto such plateaus).  Every other fixture, body_e2e_21 / 22 included (the
# reference never tips them, and the library's summation order is fixed per layer): exact pixels.
_TIE_ALLOWANCE = {"body_e2e_31_368x656.npz": 3}


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "body_e2e_*.npz"))), ids=os.path.basename)
def test_body_end_to_end_vs_reference(body, path):
    """Full Body() on a random image with seeded weights against the reference's own run (its
    src/body.py Body.__call__ on src/model.py's network, 8 torch threads): the north-star bar,
    identical keypoint pixels and identical person/subset assignment -- except on fixtures listed in
    _TIE_ALLOWANCE, where at most that many keypoints may sit one pixel from the reference's on a
    float64 plateau of the smoothed heat map (body_e2e_31: three of 1,350; the fp32 summation order
    decides them, as the reference's own thread count does at C2's size).  Such keypoints' ids
    are mapped; the people and their assignment must still be identical, and only the scores of
    the people holding a moved keypoint may change beyond rtol 1e-3 (to 3e-2: the keypoint's heat
    value and its limbs' PAF integrals move with it)."""
    from oracle import ties
    from oracle.network import seeded_state_dict as oracle_sd
    d = np.load(path)
    img = golden_image(d)
    cand, subset = body(img)
    ref_c, ref_s = d["candidate"], d["subset"]
    assert cand.shape == ref_c.shape
    ids = np.arange(len(cand), dtype=np.float64)
    moved = []  # reference ids of keypoints on another (tied) pixel
    allowance = _TIE_ALLOWANCE.get(os.path.basename(path), 0)
    same = np.array_equal(cand[:, :2], ref_c[:, :2])
    if same:  # the driver's log shows the count for every fixture, zero included
        report(f"{os.path.basename(path)}: 0 of {len(ref_c)} keypoints across float64 plateaus (allowed {allowance})")
    if not same:
        assert allowance, "keypoint pixels differ on a fixture with no tie allowance"
        up, blur = ties.f64_smoothed(img, oracle_sd("body", 0))
        pairs = ties.tie_pairs(up, blur, cand, ref_c)
        assert pairs is not None, "keypoints moved away from float64 ties"
        for i, j in pairs.items():
            ids[i] = j
            if not np.array_equal(cand[i, :2], ref_c[j, :2]):
                moved.append(j)
        report(f"{os.path.basename(path)}: {len(moved)} of {len(ref_c)} keypoints across float64 plateaus "
               f"(allowed {allowance})")
        assert len(moved) <= allowance, (len(moved), allowance)
        keep = np.setdiff1d(np.arange(len(cand)), list(pairs))
        assert np.array_equal(cand[keep, :2], ref_c[keep, :2])
        np.testing.assert_allclose(cand[keep, 2], ref_c[keep, 2], rtol=1e-3, atol=1e-4)
    else:
        np.testing.assert_allclose(cand[:, 2], ref_c[:, 2], rtol=1e-3, atol=1e-4)
    assert np.array_equal(cand[:, 3], np.arange(len(cand)))
    assert subset.shape == ref_s.shape
    mapped = np.where(subset[:, :18] >= 0, ids[np.maximum(subset[:, :18], 0).astype(int)], -1)
    assert np.array_equal(mapped, ref_s[:, :18]) and np.array_equal(subset[:, 19], ref_s[:, 19])
    touched = np.isin(ref_s[:, :18], moved).any(1)
    np.testing.assert_allclose(subset[~touched, 18], ref_s[~touched, 18], rtol=1e-3)
    np.testing.assert_allclose(subset[touched, 18], ref_s[touched, 18], rtol=3e-2)


def test_body_call_surface_and_empty_frame(body):
    img = np.zeros((368, 656, 3), np.uint8)
    cand, subset = body(img)
    assert cand.dtype == np.float64 and subset.dtype == np.float64 and subset.shape[1] == 20
    # non-contiguous input is accepted like cv2 arrays
    big = np.random.default_rng(1).integers(0, 256, (200, 300, 3), dtype=np.uint8)
    a = body(big[::1, 10:250])
    b = body(np.ascontiguousarray(big[:, 10:250]))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_capacity_overflow_grows_and_matches(native):
    """Records too small for the frame: the library flags OPOSE_E_CAPACITY, the facade grows
    the capacity and re-runs; the result still equals the reference fixture."""
    from src.body import Body
    from src.weights import seeded_state_dict
    small = Body(seeded_state_dict("body", 0), peaks_per_part=2, max_people=2)
    for path in sorted(glob.glob(os.path.join(GOLDEN, "body_planted_5*_368x656_p14.npz")))[:2]:
        d = np.load(path)
        maps = np.concatenate([d["paf"], d["heat"]], 0)[None]
        cand, subset = small.post(maps, list(d["pad"]), 368, 656)[0]
        assert np.array_equal(cand, d["candidate"]) and np.array_equal(subset, d["subset"])
    assert small.peaks_per_part > 2 and small.max_people > 2


@pytest.mark.parametrize("hw", [(10, 12), (9, 40), (200, 11)])
def test_tiny_frames_vs_oracle(body, hw):
    """Frames smaller than the 25-tap Gaussian (scipy 'reflect' wraps more than once)."""
    from oracle import body_post, network
    sd = network.seeded_state_dict("body", 0)
    img = np.random.default_rng(hw[0] * 7 + hw[1]).integers(0, 256, hw + (3,), dtype=np.uint8)

    def net_fn(x):
        p, h = network.body_forward(torch.from_numpy(x), sd)
        return p.numpy(), h.numpy()

    ref_c, ref_s = body_post.body_infer(img, net_fn)
    cand, subset = body(img)
    assert cand.shape == ref_c.shape and subset.shape == ref_s.shape
    if cand.size:
        assert np.array_equal(cand[:, [0, 1, 3]], ref_c[:, [0, 1, 3]])
    assert np.array_equal(subset[:, :18], ref_s[:, :18])


def test_graph_replay_matches_eager(native):
    """The launch-sequence cache: call 1 eager, call 2 captured, calls 3+ replayed -- all equal,
    also when two shapes alternate and when a larger shape reallocates the workspace."""
    from src.body import Body
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
    rng = np.random.default_rng(9)
    a = rng.integers(0, 256, (184, 328, 3), dtype=np.uint8)
    b = rng.integers(0, 256, (120, 200, 3), dtype=np.uint8)
    big = rng.integers(0, 256, (368, 656, 3), dtype=np.uint8)
    ra, rb = body(a), body(b)
    for img, ref in ((a, ra), (b, rb), (a, ra), (b, rb), (big, None), (a, ra), (a, ra), (b, rb)):
        out = body(img)
        if ref is not None:
            assert np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1])
