"""GPU: the split-bf16 ("x6") convolution that runs the network by default (csrc/conv_x6.hip).

Every fp32 operand is carried as three bf16 pieces (exact) and each product is rebuilt from
six bf16 MFMA piece products; the claim is fp32 accuracy.  Tolerances:
* single convs against a float64 reference: |err| <= 4e-6 * conv(|x|, |w|) + 1e-6 — the bound
  the fp32 MFMA kernel is held to (tests/test_gpu_parity.py) — and the mean relative error
  within 3x the fp32 kernel's on the same inputs;
* the X6 epilogue (split store) + rebuild is lossless: identical to the fp32-output epilogue;
* the whole network on the x6 path vs the fp32 MFMA path (OPOSE_CONV=f32): within the
  network tolerance of test_gpu_parity (2e-4 * max|ref| + 2e-4 * |ref|); the e2e golden
  fixtures of the reference (test_gpu_parity / test_gpu_pipeline) run on the x6 path too.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from src import _native
    return _native


@pytest.fixture(scope="module")
def handle(native):
    return native.Handle(0)


def _run(native, handle, fn, x, w, b, relu, mt, pt, splits, *extra):
    N, Cin, H, W = x.shape
    Cout, _, ks, _ = w.shape
    out = np.empty((N, Cout, H, W), np.float32)
    handle.check(fn(handle.h, x.ctypes.data, w.ctypes.data, b.ctypes.data, N, Cin, H, W, Cout, ks, ks // 2,
                    int(relu), mt, pt, splits, *extra, out.ctypes.data))
    return out


CASES = [
    (1, 3, 40, 72, 64, 3, 0, 0, 0),          # conv1_1: one channel group, chunks of 4 taps
    (2, 64, 20, 24, 96, 3, 0, 0, 0),         # Mpad 128 > Cout
    (2, 128, 23, 41, 128, 7, 128, 256, 0),   # 8-wave tile, data parallel
    (2, 128, 23, 41, 256, 7, 256, 128, 0),
    (2, 185, 17, 19, 128, 7, 128, 128, 0),   # ragged channel groups (185 -> 24 groups, clamped reads)
    (3, 64, 30, 33, 128, 3, 128, 64, 37),    # stream-K: partial slabs + fixup
    (2, 96, 23, 41, 128, 3, 64, 128, 300),   # stream-K, more workgroups than tiles
    (2, 128, 17, 19, 38, 1, 64, 64, 0),      # 1x1, Cout 38 (PAF head)
    (1, 150, 9, 13, 128, 7, 64, 64, 5),      # hand Mconv1-like, tiny frame, 5 workgroups
    (2, 64, 23, 41, 64, 3, 64, 128, 0),      # conv1_2-like M = 64
    (3, 64, 30, 33, 64, 3, 64, 128, 40),     # the same tile stream-K
]


@pytest.mark.parametrize("N,Cin,H,W,Cout,ks,mt,pt,splits", CASES)
def test_x6_conv_fp32_accuracy(native, handle, N, Cin, H, W, Cout, ks, mt, pt, splits):
    rng = np.random.default_rng(Cin * 7 + ks)
    x = np.maximum(rng.standard_normal((N, Cin, H, W), dtype=np.float32), 0)  # post-ReLU activations
    w = (rng.standard_normal((Cout, Cin, ks, ks), dtype=np.float32) * np.float32(np.sqrt(2 / (Cin * ks * ks))))
    b = rng.standard_normal(Cout, dtype=np.float32) * np.float32(0.1)
    y6 = _run(native, handle, native.lib.opose_debug_conv_x6, x, w, b, True, mt, pt, splits, 0)
    y6x = _run(native, handle, native.lib.opose_debug_conv_x6, x, w, b, True, mt, pt, splits, 1)
    y32 = _run(native, handle, native.lib.opose_debug_conv, x, w, b, True, mt, pt, splits)
    xd, wd, bd = (torch.from_numpy(a).double() for a in (x, w, b))
    ref = F.conv2d(xd, wd, bd, padding=ks // 2).clamp_min(0).numpy()
    mag = F.conv2d(xd.abs(), wd.abs(), bd.abs(), padding=ks // 2).numpy()
    e6 = np.abs(y6 - ref)
    e32 = np.abs(y32 - ref)
    assert (e6 <= 4e-6 * mag + 1e-6).all(), float((e6 / (4e-6 * mag + 1e-6)).max())
    assert (e6 / np.maximum(mag, 1e-30)).mean() <= 3 * (e32 / np.maximum(mag, 1e-30)).mean() + 1e-9
    assert np.array_equal(y6, y6x)  # split epilogue + rebuild is lossless


WINO_CASES = [
    (2, 128, 23, 41, 256),   # H/8 of the bench: odd W, tile blocks across frames
    (2, 256, 46, 82, 128),   # H/4: windows across frames too long -> frame-aligned tile blocks
    (1, 64, 17, 30, 128),    # one frame, even W, 6 chunks (two four-group periods)
    (3, 40, 11, 13, 128),    # 5 channel groups: 15 pairs, the last chunk padded
    (1, 512, 23, 41, 512),   # conv4_2 on one frame
    (2, 128, 9, 7, 96),      # Cout < 128 (Mpad 128), W = 7
]


@pytest.mark.parametrize("N,Cin,H,W,Cout", WINO_CASES)
def test_wino_conv_fp32_accuracy(native, handle, N, Cin, H, W, Cout):
    """conv_wino_x6 (Winograd F(2,3) along x, csrc/conv_wino.hip) on padded X6P inputs through the
    engine's launch path (opose_debug_conv_x6 with mt = -3 forces the family) against a float64
    reference: the same bar as the direct kernels -- |err| <= 4e-6 * conv(|x|, |w|) + 1e-6 and
    the mean relative error within 3x the fp32 MFMA kernel's.  The window kernel on the same
    padded inputs (mt = -2) is checked to the same bar beside it."""
    rng = np.random.default_rng(Cin * 3 + W)
    x = np.maximum(rng.standard_normal((N, Cin, H, W), dtype=np.float32), 0)
    w = rng.standard_normal((Cout, Cin, 3, 3), dtype=np.float32) * np.float32(np.sqrt(2 / (Cin * 9)))
    b = rng.standard_normal(Cout, dtype=np.float32) * np.float32(0.1)
    yw = _run(native, handle, native.lib.opose_debug_conv_x6, x, w, b, True, -3, 0, 0, 1)
    yd = _run(native, handle, native.lib.opose_debug_conv_x6, x, w, b, True, -2, 0, 0, 1)
    y32 = _run(native, handle, native.lib.opose_debug_conv, x, w, b, True, 0, 0, 0)
    xd, wd, bd = (torch.from_numpy(a).double() for a in (x, w, b))
    ref = F.conv2d(xd, wd, bd, padding=1).clamp_min(0).numpy()
    mag = F.conv2d(xd.abs(), wd.abs(), bd.abs(), padding=1).numpy()
    e32 = (np.abs(y32 - ref) / np.maximum(mag, 1e-30)).mean()
    for y in (yw, yd):
        e = np.abs(y - ref)
        assert (e <= 4e-6 * mag + 1e-6).all(), float((e / (4e-6 * mag + 1e-6)).max())
        assert (e / np.maximum(mag, 1e-30)).mean() <= 3 * e32 + 1e-9
    print(f"wino mean rel err {(np.abs(yw - ref) / np.maximum(mag, 1e-30)).mean():.3e}, "
          f"window {(np.abs(yd - ref) / np.maximum(mag, 1e-30)).mean():.3e}, fp32 {e32:.3e}")


@pytest.mark.parametrize("kind,shape", [("body", (4, 3, 184, 328)), ("body", (1, 3, 368, 656)),
                                        ("hand", (1, 3, 368, 368))], ids=["body4x184x328", "body368x656", "hand368"])
def test_network_wino_vs_window(native, kind, shape):
    """The network with its 3x3 layers on conv_wino_x6 (OPOSE_WINO=1, opt-in) against the default
    window kernel: a different summation order, so the bar is the network tolerance and a maximum
    deviation below 1e-5 of the map's range."""
    from src.model import bodypose_model, handpose_model
    cls = bodypose_model if kind == "body" else handpose_model
    x = np.random.default_rng(12).random(shape, dtype=np.float32) - np.float32(0.5)
    on = _model_outputs(cls, kind, x, {"OPOSE_WINO": "1"})
    off = _model_outputs(cls, kind, x, {"OPOSE_WINO": "0"})
    for a, r in zip(on, off):
        tol = 2e-4 * np.abs(r).max() + 2e-4 * np.abs(r)
        assert (np.abs(a - r) <= tol).all(), kind
        assert np.abs(a - r).max() <= 1e-5 * np.abs(r).max(), kind


def test_x6_split_roundtrip_exact(native, handle):
    """A 1x1 identity conv through the X6 epilogue reproduces every fp32 input bit-exactly
    (subnormal-free, both signs, magnitudes over 2^-60 .. 2^60)."""
    rng = np.random.default_rng(3)
    C, H, W = 16, 8, 8
    mant = rng.uniform(1, 2, (1, C, H, W))
    expo = rng.integers(-60, 60, (1, C, H, W))
    sign = rng.choice([-1.0, 1.0], (1, C, H, W))
    x = (sign * mant * np.exp2(expo)).astype(np.float32)
    w = np.eye(C, dtype=np.float32).reshape(C, C, 1, 1)
    b = np.zeros(C, np.float32)
    y = _run(native, handle, native.lib.opose_debug_conv_x6, x, w, b, False, 64, 64, 0, 1)
    assert np.array_equal(y, x)


def test_network_x6_vs_f32_path(native):
    """The default x6 network against the fp32 MFMA network (OPOSE_CONV=f32, read at handle
    creation) on the same input: same maps within the network tolerance."""
    from src import util
    from src.model import bodypose_model
    from src.weights import seeded_state_dict
    sd = seeded_state_dict("body", 0)
    x = np.random.default_rng(11).random((2, 3, 64, 96), dtype=np.float32) - np.float32(0.5)
    m6 = bodypose_model(0)
    m6.load_state_dict(util.transfer(m6, sd))
    p6, h6 = m6(x)
    old = os.environ.get("OPOSE_CONV")
    os.environ["OPOSE_CONV"] = "f32"
    try:
        m32 = bodypose_model(0)
    finally:
        if old is None:
            del os.environ["OPOSE_CONV"]
        else:
            os.environ["OPOSE_CONV"] = old
    m32.load_state_dict(util.transfer(m32, sd))
    p32, h32 = m32(x)
    for a, r in ((p6, p32), (h6, h32)):
        tol = 2e-4 * np.abs(r).max() + 2e-4 * np.abs(r)
        assert (np.abs(a - r) <= tol).all()


@pytest.mark.parametrize("env", ["OPOSE_FUSED_POOL", "OPOSE_FIRST_DIRECT"])
def test_network_variants(native, env):
    """Default network against the variant with one optimisation switched off (read at handle
    creation): OPOSE_FUSED_POOL=0 runs MaxPool2d as separate launches instead of in the conv
    epilogue (max then bias + ReLU is the same value as bias + ReLU then max: equal whenever the
    conv sums in the same order; the fused launch always runs whole tiles while the separate conv
    may be split over k at these small sizes); OPOSE_FIRST_DIRECT=0 runs conv1_1 as an implicit
    GEMM instead of the direct fp32-FMA kernel.  Bar: fp32 summation-order noise -- the network
    tolerance, and a maximum deviation below 1e-5 of the map's range."""
    from src import util
    from src.model import bodypose_model, handpose_model
    from src.weights import seeded_state_dict
    for kind, cls, shape in (("body", bodypose_model, (2, 3, 72, 104)), ("hand", handpose_model, (1, 3, 88, 88))):
        sd = seeded_state_dict(kind, 0)
        x = np.random.default_rng(5).random(shape, dtype=np.float32) - np.float32(0.5)
        outs = []
        for on in ("1", "0"):
            old = os.environ.get(env)
            os.environ[env] = on
            try:
                m = cls(0)
            finally:
                if old is None:
                    del os.environ[env]
                else:
                    os.environ[env] = old
            m.load_state_dict(util.transfer(m, sd))
            y = m(x)
            outs.append(y if isinstance(y, tuple) else (y,))
        for a, r in zip(*outs):
            tol = 2e-4 * np.abs(r).max() + 2e-4 * np.abs(r)
            assert (np.abs(a - r) <= tol).all(), kind
            assert np.abs(a - r).max() <= 1e-5 * np.abs(r).max(), kind


def _model_outputs(cls, kind, x, env):
    from src import util
    from src.weights import seeded_state_dict
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = cls(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    m.load_state_dict(util.transfer(m, seeded_state_dict(kind, 0)))
    y = m(x)
    return y if isinstance(y, tuple) else (y,)


@pytest.mark.parametrize("kind,shape", [("body", (2, 3, 72, 104)), ("body", (1, 3, 80, 88)),
                                        ("body", (1, 3, 184, 328)), ("hand", (1, 3, 88, 88)),
                                        ("body", (3, 3, 8, 8)), ("body", (1, 3, 16, 120)),
                                        ("hand", (2, 3, 40, 24)), ("hand", (1, 3, 56, 200))],
                         ids=["body72x104", "body80x88", "body184x328", "hand88", "body3x8x8", "body16x120",
                              "hand2x40x24", "hand56x200"])
def test_conv12_window_bit_identical(native, kind, shape):
    """conv1_2 + pool with the input window in LDS (conv3_pool_win_x6, default) against conv_x6's
    pooled launch over the im2col stream (OPOSE_CONV12_WIN=0): the same weight chunks and MFMA
    sequence per output, so the network outputs are bit-identical.  Partial tiles in the column
    direction (88 / 104 columns) and the bench's 184 x 328 network input."""
    from src.model import bodypose_model, handpose_model
    cls = bodypose_model if kind == "body" else handpose_model
    x = np.random.default_rng(10).random(shape, dtype=np.float32) - np.float32(0.5)
    on = _model_outputs(cls, kind, x, {"OPOSE_CONV12_WIN": "1"})
    off = _model_outputs(cls, kind, x, {"OPOSE_CONV12_WIN": "0"})
    for a, r in zip(on, off):
        assert np.array_equal(a, r), kind


@pytest.mark.parametrize("kind,shape", [("body", (2, 3, 72, 104)), ("body", (32, 3, 184, 328)),
                                        ("hand", (1, 3, 88, 88))], ids=["body72x104", "bench32", "hand88"])
def test_conv11_fp32_handoff_bit_identical(native, kind, shape):
    """conv1_1 -> conv1_2 hand-off as fp32 units split inside conv3_pool_win_x6 (default) against
    the X6 tensor split in conv1_1's epilogue (OPOSE_C11_F32=0): split3 of the same fp32 values
    either way, so the network outputs are bit-identical (ragged 8 x 16 tiles at 72 x 104 / 88 x 88;
    the bench's batch)."""
    from src.model import bodypose_model, handpose_model
    cls = bodypose_model if kind == "body" else handpose_model
    x = np.random.default_rng(12).random(shape, dtype=np.float32) - np.float32(0.5)
    on = _model_outputs(cls, kind, x, {"OPOSE_C11_F32": "1"})
    off = _model_outputs(cls, kind, x, {"OPOSE_C11_F32": "0"})
    for a, r in zip(on, off):
        assert np.array_equal(a, r), kind


@pytest.mark.parametrize("kind,shape", [("body", (32, 3, 184, 328)), ("body", (30, 3, 184, 328)),
                                        ("body", (88, 3, 136, 152)), ("hand", (120, 3, 184, 184))],
                         ids=["bench32", "partial_tile30", "frame_crossing88", "hand120"])
def test_conv7_window_vs_im2col(native, kind, shape):
    """The batched 7x7 CPM convs and the padded-input 3x3 convs (trunk conv3_x / conv4_x, stage-1
    CPM) on the LDS-window kernel (conv_win_x6, default when a layer has >= 192 whole 128 x 256
    tiles filling >= 85 % of their rounds) against conv_x6 over the im2col stream (OPOSE_CONV7_WIN=0):
    the same split-bf16 products in another k order (pair order), so fp32 summation-order noise
    only -- the network tolerance, and a maximum deviation below 5e-5 of the map's range (every
    one of the 25 7x7 layers sums in another order; measured ~1.1e-5).  Shapes:
    the bench's batch, a partial last tile, 17 x 19 maps whose tiles span two frames, and 120 hand
    crops (hand Mconv1: 19 input groups, the last chunk padded)."""
    from src.model import bodypose_model, handpose_model
    cls = bodypose_model if kind == "body" else handpose_model
    x = np.random.default_rng(12).random(shape, dtype=np.float32) - np.float32(0.5)
    win = _model_outputs(cls, kind, x, {"OPOSE_CONV7_WIN": "1"})
    ref = _model_outputs(cls, kind, x, {"OPOSE_CONV7_WIN": "0"})
    for a, r in zip(win, ref):
        tol = 2e-4 * np.abs(r).max() + 2e-4 * np.abs(r)
        assert (np.abs(a - r) <= tol).all()
        assert np.abs(a - r).max() <= 5e-5 * np.abs(r).max()


def _hand_model(env):
    from src import util
    from src.model import handpose_model
    from src.weights import seeded_state_dict
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = handpose_model(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    m.load_state_dict(util.transfer(m, seeded_state_dict("hand", 0)))
    return m


@pytest.mark.parametrize("crops,sizes", [(1, (184, 368, 552, 736)), (2, (184, 368, 552, 736)), (3, (48, 96, 144))],
                         ids=["one_crop_368", "two_crops_368", "three_crops_96"])
@pytest.mark.parametrize("env", [{}, {"OPOSE_CONV7_WIN": "0"}], ids=["default", "no_window"])
def test_hand_pyramid_lockstep_vs_per_scale(native, crops, sizes, env):
    """Hand()'s scale pyramid in lockstep (opose_hand_forward_pyramid: one conv launch per layer
    for every scale, X6 groups of different geometry in one grid, the work units of all scales
    scheduled together) against each scale's network on its own (opose_hand_forward): bit for
    bit -- a pixel's k slabs and kernel family are fixed by its layer and its scale's geometry,
    not by the launch.  The 368-crop pyramid is C3's; three 96-crops the
    crop-batched Hand of a frame with hands."""
    rng = np.random.default_rng(17)
    xs = [rng.random((crops, 3, s, s), dtype=np.float32) - np.float32(0.5) for s in sizes]
    m = _hand_model(env)
    pyr = m.forward_pyramid(xs)
    for x, a in zip(xs, pyr):
        assert np.array_equal(a, m(x))


@pytest.mark.parametrize("crops", [2, 3])
def test_hand_crop_batch_per_frame_windows(native, crops):
    """A crop batch's largest scale (N x 92 x 92 at the 7x7 layers): 256-pixel tiles that
    straddle two crops need a window larger than the LDS, so the planner runs that segment as
    one segment per crop (frame views of the same X6P buffers) on the window kernel (default) --
    against the whole launch on conv_x6 (OPOSE_SPLIT_FRAMES=0): summation-order noise only
    (3 smaller scales + one group per crop: up to 5 crops split)."""
    rng = np.random.default_rng(19)
    xs = [rng.random((crops, 3, s, s), dtype=np.float32) - np.float32(0.5) for s in (184, 368, 552, 736)]
    a = _hand_model({}).forward_pyramid(xs)
    r = _hand_model({"OPOSE_SPLIT_FRAMES": "0"}).forward_pyramid(xs)
    for x, y in zip(a, r):
        tol = 2e-4 * np.abs(y).max() + 2e-4 * np.abs(y)
        assert (np.abs(x - y) <= tol).all()
        assert np.abs(x - y).max() <= 5e-5 * np.abs(y).max()


def test_hand_pyramid_vs_oracle(native):
    """The lockstep pyramid against the oracle network (oracle/network.py hand_forward, the
    reference's handpose_model restated) at small sizes: the network tolerance."""
    from oracle import network
    sd = network.seeded_state_dict("hand", 0)
    rng = np.random.default_rng(18)
    xs = [rng.random((2, 3, s, s), dtype=np.float32) - np.float32(0.5) for s in (40, 80, 120, 160)]
    pyr = _hand_model({}).forward_pyramid(xs)
    for x, a in zip(xs, pyr):
        r = network.hand_forward(torch.from_numpy(x), sd).numpy()
        np.testing.assert_allclose(a, r, rtol=2e-4, atol=2e-4 * float(np.abs(r).max()))


@pytest.mark.parametrize("kind,shape,exact", [("body", (32, 3, 184, 328), True), ("body", (2, 3, 72, 104), False),
                                              ("hand", (1, 3, 88, 88), False), ("hand", (120, 3, 184, 184), False)],
                         ids=["bench32", "body72x104", "hand88", "hand120"])
def test_fused_1x1_chain(native, kind, shape, exact):
    """The closing 1x1 pair of every CPM stage in one launch (conv1x1_chain_x6, default) against
    two conv_x6 launches through an HBM intermediate (OPOSE_FUSE_1X1=0): the same piece products
    in the same order, so on the bench's batch -- where conv_x6 runs both convs on whole tiles --
    the network outputs are bit-identical; at small sizes conv_x6 splits k (stream-K) and the bar
    is fp32 summation-order noise."""
    from src.model import bodypose_model, handpose_model
    cls = bodypose_model if kind == "body" else handpose_model
    x = np.random.default_rng(14).random(shape, dtype=np.float32) - np.float32(0.5)
    fused = _model_outputs(cls, kind, x, {"OPOSE_FUSE_1X1": "1"})
    split = _model_outputs(cls, kind, x, {"OPOSE_FUSE_1X1": "0"})
    for a, r in zip(fused, split):
        if exact:
            assert np.array_equal(a, r), kind
        else:
            tol = 2e-4 * np.abs(r).max() + 2e-4 * np.abs(r)
            assert (np.abs(a - r) <= tol).all()
            assert np.abs(a - r).max() <= 5e-5 * np.abs(r).max()


@pytest.mark.parametrize("crops", [1, 2])
def test_hand_pyramid_window_vs_im2col(native, crops):
    """A 368 crop's pyramid in lockstep on the window kernel (stream-K 128 x 256 window tiles over
    the four scales' groups) against conv_x6 over the im2col stream (OPOSE_CONV7_WIN=0):
    pair-order vs group-tap-order summation, the network tolerance and a maximum deviation below
    5e-5 of the map's range."""
    rng = np.random.default_rng(19)
    xs = [rng.random((crops, 3, s, s), dtype=np.float32) - np.float32(0.5) for s in (184, 368, 552, 736)]
    win = _hand_model({"OPOSE_CONV7_WIN": "1"}).forward_pyramid(xs)
    ref = _hand_model({"OPOSE_CONV7_WIN": "0"}).forward_pyramid(xs)
    for a, r in zip(win, ref):
        tol = 2e-4 * np.abs(r).max() + 2e-4 * np.abs(r)
        assert (np.abs(a - r) <= tol).all()
        assert np.abs(a - r).max() <= 5e-5 * np.abs(r).max()
