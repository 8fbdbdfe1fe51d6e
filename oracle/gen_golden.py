"""ORACLE harness (test infrastructure only; runs in the build container only).

Imports the reference's own `src/model.py`, `src/body.py` and `src/hand.py` from
/root/reference (read-only, never copied) and records their outputs as small
golden fixtures under tests/golden/.  The reference never travels to the GPU box:
only the .npz / .json data written here does.

Shims (the reference's third-party imports that are absent from this image):
* cv2          -> oracle.cv_resize.Cv2Shim (resize INTER_CUBIC, flip).  Resize parity
                  is therefore self-consistent only ("unpinned").
* torchvision  -> empty module (imported but unused at src/body.py:9).
* skimage.measure.label -> scipy.ndimage.label with a 3x3 structure (connectivity=2).

Usage:  PYTHONDONTWRITEBYTECODE=1 python -m oracle.gen_golden
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, REPO)
from oracle import network as onet  # noqa: E402
from oracle import planted  # noqa: E402
from oracle.cv_resize import Cv2Shim  # noqa: E402
from oracle.hand_post import label8  # noqa: E402


def install_shims():
    cv2 = types.ModuleType("cv2")
    cv2.INTER_CUBIC = Cv2Shim.INTER_CUBIC
    cv2.resize = Cv2Shim.resize
    cv2.flip = Cv2Shim.flip
    sys.modules["cv2"] = cv2
    tv = types.ModuleType("torchvision")
    tv.transforms = types.ModuleType("torchvision.transforms")
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tv.transforms
    sk = types.ModuleType("skimage")
    skm = types.ModuleType("skimage.measure")

    def label(binary, return_num=False, connectivity=None):
        assert connectivity == binary.ndim == 2
        lab, n = label8(binary)
        return (lab, n) if return_num else lab

    skm.label = label
    sk.measure = skm
    sys.modules["skimage"] = sk
    sys.modules["skimage.measure"] = skm


class PlantedBody:
    """Stand-in for bodypose_model returning fixed low-res maps (ignores the input)."""

    def __init__(self, paf, heat):
        self.paf, self.heat = torch.from_numpy(paf[None]), torch.from_numpy(heat[None])

    def __call__(self, data):
        h, w = data.shape[2] // 8, data.shape[3] // 8
        assert self.paf.shape[2:] == (h, w), (self.paf.shape, data.shape)
        return self.paf, self.heat


class PlantedHand:
    """Stand-in for handpose_model: renders the same normalised hand at every scale."""

    def __init__(self, pts, vis, seed, extra):
        self.pts, self.vis, self.seed, self.extra = pts, vis, seed, extra
        self.calls = []

    def __call__(self, data):
        h, w = data.shape[2] // 8, data.shape[3] // 8
        rng = np.random.default_rng(self.seed + len(self.calls))
        heat = planted.render_hand(h, w, self.pts, self.vis, rng, extra_blobs=self.extra)
        self.calls.append(heat)
        return torch.from_numpy(heat[None])


def ref_body(model):
    from src.body import Body
    b = Body.__new__(Body)
    b.model = model
    return b


def ref_hand(model):
    from src.hand import Hand
    h = Hand.__new__(Hand)
    h.model = model
    return h


def gen_network():
    from src.model import bodypose_model, handpose_model
    for net, cls, shape in (("body", bodypose_model, (1, 3, 64, 96)), ("hand", handpose_model, (1, 3, 64, 64)),
                            ("body", bodypose_model, (2, 3, 48, 40))):
        m = cls().eval()
        sd = onet.seeded_state_dict(net, 0)
        m.load_state_dict({k: sd[".".join(k.split(".")[1:])] for k in m.state_dict().keys()})
        x = np.random.default_rng(11).random(shape, dtype=np.float32) - np.float32(0.5)
        with torch.no_grad():
            out = m(torch.from_numpy(x))
        name = f"net_{net}_{shape[0]}x{shape[2]}x{shape[3]}.npz"
        if net == "body":
            np.savez_compressed(os.path.join(OUT, name), x=x, paf=out[0].numpy(), heat=out[1].numpy())
        else:
            np.savez_compressed(os.path.join(OUT, name), x=x, heat=out.numpy())
        print("wrote", name)


def body_case(seed, img_hw, n_people, **kw):
    from oracle.body_post import preprocess
    rng = np.random.default_rng(seed)
    H, W = img_hw
    scale = 0.5 * 368 / H
    _, pad, padded = preprocess(np.zeros((H, W, 3), np.uint8), scale)
    h, w = padded[0] // 8, padded[1] // 8
    people, vis = planted.random_people(rng, n_people, h, w)
    paf, heat = planted.render_body(h, w, people, vis, rng, **kw)
    body = ref_body(PlantedBody(paf, heat))
    err = ""
    try:
        cand, subset = body(np.zeros((H, W, 3), np.uint8))
    except IndexError as e:  # the reference's latent 3-row-match failure (src/body.py:173)
        cand, subset, err = np.zeros((0,)), np.zeros((0, 20)), "IndexError: " + str(e)
    return dict(img_hw=np.array(img_hw), paf=paf, heat=heat, pad=np.array(pad), padded_hw=np.array(padded),
                candidate=cand, subset=subset, error=np.array(err))


def gen_body_planted():
    cases = []
    # (seed, image, people, render kwargs)
    cases += [(100 + p, (368, 656), p, {}) for p in (0, 1, 3, 6, 12)]
    cases += [(200, (368, 368), 2, {}), (201, (368, 368), 5, {"drop_limb_p": 0.3})]
    cases += [(300 + i, (368, 656), 8, {"drop_limb_p": 0.35, "band": 1.3}) for i in range(6)]
    cases += [(400, (240, 320), 4, {"amp": (0.1, 0.2)})]           # near-threshold scores
    cases += [(401, (368, 656), 4, {"sigma": 1.6, "noise": 0.0})]  # broad blobs / plateaus
    cases += [(402, (100, 180), 3, {}), (403, (53, 97), 2, {})]    # ragged sizes, padding
    cases += [(500 + i, (368, 656), 14, {"drop_limb_p": 0.5, "band": 1.6}) for i in range(6)]
    for seed, hw, n, kw in cases:
        d = body_case(seed, hw, n, **kw)
        name = f"body_planted_{seed}_{hw[0]}x{hw[1]}_p{n}.npz"
        np.savez_compressed(os.path.join(OUT, name), **d)
        print("wrote", name, "cand", d["candidate"].shape, "subset", d["subset"].shape, d["error"])


def gen_body_e2e():
    """Full Body() on a small random uint8 image with the seeded reference network."""
    from src.model import bodypose_model
    m = bodypose_model().eval()
    sd = onet.seeded_state_dict("body", 0)
    m.load_state_dict({k: sd[".".join(k.split(".")[1:])] for k in m.state_dict().keys()})
    for seed, hw in ((21, (96, 128)), (22, (120, 90))):
        img = np.random.default_rng(seed).integers(0, 256, size=hw + (3,), dtype=np.uint8)
        body = ref_body(m)
        cand, subset = body(img)
        name = f"body_e2e_{seed}_{hw[0]}x{hw[1]}.npz"
        np.savez_compressed(os.path.join(OUT, name), img=img, candidate=cand, subset=subset)
        print("wrote", name, cand.shape, subset.shape)


def gen_hand_planted(cases=((600, 96, 0.9, 0), (601, 150, 0.7, 2), (602, 64, 0.0, 0), (603, 200, 1.0, 3))):
    rng0 = np.random.default_rng(77)
    for seed, size, vis_p, extra in cases:
        rng = np.random.default_rng(seed)
        pts = rng0.uniform(0.15, 0.85, size=(21, 2))
        vis = rng.random(21) < vis_p
        hand = ref_hand(PlantedHand(pts, vis, seed, extra))
        img = np.zeros((size, size, 3), np.uint8)
        peaks = hand(img)
        calls = hand.model.calls
        name = f"hand_planted_{seed}_{size}.npz"
        np.savez_compressed(os.path.join(OUT, name), size=np.array(size), peaks=peaks,
                            **{f"heat{i}": c for i, c in enumerate(calls)})
        print("wrote", name, peaks.dtype, peaks.shape)


def main():
    os.makedirs(OUT, exist_ok=True)
    install_shims()
    sys.path.insert(0, REF)
    torch.set_num_threads(8)
    gen_network()
    gen_body_planted()
    gen_body_e2e()
    gen_hand_planted()
    shutil.copyfile(os.path.join(REF, "src", "hand_model_output_size.json"),
                    os.path.join(OUT, "hand_model_output_size.json"))
    with open(os.path.join(OUT, "README.json"), "w") as f:
        json.dump({"generator": "oracle/gen_golden.py", "reference": "hitmaxiang/pytorch-openpose src/ (imported read-only)",
                   "weights": "oracle.network.seeded_state_dict(seed=0)",
                   "resize": "cv2.resize routed through oracle.cv_resize (OpenCV parity unpinned)"}, f, indent=1)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def gen_hand_detect():
    """util.handDetect (src/util.py:133-201) on the planted Body fixtures' outputs."""
    from src import util as ref_util
    cases = []
    for p in sorted(glob.glob(os.path.join(OUT, "body_planted_*.npz"))):
        d = np.load(p)
        if d["subset"].shape[0] == 0:
            continue
        H, W = (int(v) for v in d["img_hw"])
        boxes = ref_util.handDetect(d["candidate"], d["subset"], np.zeros((H, W, 3), np.uint8))
        cases.append({"fixture": os.path.basename(p), "boxes": [[int(x), int(y), int(w), bool(l)] for x, y, w, l in boxes]})
    with open(os.path.join(OUT, "hand_detect.json"), "w") as f:
        json.dump(cases, f, indent=0)
    print("wrote hand_detect.json", len(cases))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "hand_detect":
    install_shims()
    sys.path.insert(0, REF)
    gen_hand_detect()


def install_batch_shims():
    """Extra stand-ins for srcmx/Batch_model.py + srcmx/utilmx.py imports absent here (none of
    them is used by Batch_body.__call__): numba.jit, h5py, tslearn.metrics,
    torchvision.transforms(.functional)."""
    install_shims()
    nb = types.ModuleType("numba")
    nb.jit = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
    sys.modules["numba"] = nb
    sys.modules["h5py"] = types.ModuleType("h5py")
    tsl = types.ModuleType("tslearn")
    tsl.metrics = types.ModuleType("tslearn.metrics")
    sys.modules["tslearn"] = tsl
    sys.modules["tslearn.metrics"] = tsl.metrics
    tv = sys.modules["torchvision"]
    tv.transforms.functional = types.ModuleType("torchvision.transforms.functional")
    sys.modules["torchvision.transforms.functional"] = tv.transforms.functional
    sys.path.insert(0, os.path.join(REF, "srcmx"))


class PlantedBatch:
    """Stand-in bodypose_model for Batch_body: fixed low-res maps per frame."""

    def __init__(self, paf, heat):
        self.paf, self.heat = torch.from_numpy(paf), torch.from_numpy(heat)

    def __call__(self, x):
        assert tuple(self.paf.shape[2:]) == (x.shape[2] // 8, x.shape[3] // 8), (self.paf.shape, x.shape)
        return self.paf, self.heat


def ref_batch_body(model):
    import Batch_model as BM
    import utilmx
    b = BM.Batch_body.__new__(BM.Batch_body)
    b.model = model
    # Batch_body.__init__ (srcmx/Batch_model.py:116-135) without torch.load of the .pth
    b.scale_search, b.boxsize, b.stride, b.padvalue, b.thre1, b.thre2 = 0.5, 368, 8, 128, 0.1, 0.05
    b.limbSeq = [[2, 3], [2, 6], [3, 4], [4, 5], [6, 7], [7, 8], [2, 9], [9, 10], [10, 11], [2, 12], [12, 13],
                 [13, 14], [2, 1], [1, 15], [15, 17], [1, 16], [16, 18], [3, 17], [6, 18]]
    b.mapIdx = [[31, 32], [39, 40], [33, 34], [35, 36], [41, 42], [43, 44], [19, 20], [21, 22], [23, 24], [25, 26],
                [27, 28], [29, 30], [47, 48], [49, 50], [53, 54], [51, 52], [55, 56], [37, 38], [45, 46]]
    b.guassian_filter_conv = utilmx.GaussianBlurConv(19)
    return b


def gen_batch_body():
    """Batch_body (srcmx/Batch_model.py:137-204) on planted maps and with the seeded network."""
    from oracle.batch_post import size_pad, to_tensor
    from src.model import bodypose_model
    for seed, hw, B, n_people in ((700, (368, 656), 3, 6), (701, (240, 320), 2, 3), (702, (100, 180), 2, 2)):
        rng = np.random.default_rng(seed)
        H, W = hw
        _, nh, nw, ph, pw = size_pad(0.5, H, W)
        h, w = (nh + ph) // 8, (nw + pw) // 8
        pafs, heats = [], []
        for _ in range(B):
            people, vis = planted.random_people(rng, n_people, h, w)
            paf, heat = planted.render_body(h, w, people, vis, rng)
            pafs.append(paf)
            heats.append(heat)
        paf, heat = np.stack(pafs), np.stack(heats)
        frames = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
        res = ref_batch_body(PlantedBatch(paf, heat))(to_tensor(frames))
        d = dict(img_hw=np.array(hw), paf=paf, heat=heat)
        for i, (c, sset) in enumerate(res):
            d[f"candidate{i}"], d[f"subset{i}"] = np.asarray(c, np.float64), np.asarray(sset, np.float64)
        name = f"batch_body_planted_{seed}_{H}x{W}_b{B}.npz"
        np.savez_compressed(os.path.join(OUT, name), **d)
        print("wrote", name, [r[0].shape for r in res], [r[1].shape for r in res])
    m = bodypose_model().eval()
    sd = onet.seeded_state_dict("body", 0)
    m.load_state_dict({k: sd[".".join(k.split(".")[1:])] for k in m.state_dict().keys()})
    frames = np.random.default_rng(23).integers(0, 256, (2, 96, 128, 3), dtype=np.uint8)
    res = ref_batch_body(m)(to_tensor(frames))
    d = dict(frames=frames)
    for i, (c, sset) in enumerate(res):
        d[f"candidate{i}"], d[f"subset{i}"] = np.asarray(c, np.float64), np.asarray(sset, np.float64)
    np.savez_compressed(os.path.join(OUT, "batch_body_e2e_23_96x128_b2.npz"), **d)
    print("wrote batch_body_e2e", [r[0].shape for r in res], [r[1].shape for r in res])


class PlantedHandBatch:
    """Stand-in handpose_model for Batch_hand: fixed [B, 22, 46, 46] maps."""

    def __init__(self, heat):
        self.heat = torch.from_numpy(heat)

    def __call__(self, x):
        assert tuple(self.heat.shape[2:]) == (x.shape[2] // 8, x.shape[3] // 8)
        return self.heat


def ref_batch_hand(model):
    import Batch_model as BM
    import utilmx
    b = BM.Batch_hand.__new__(BM.Batch_hand)
    b.model = model
    # Batch_hand.__init__ (srcmx/Batch_model.py:311-324) without torch.load of the .pth
    b.scale_search, b.boxsize, b.stride, b.padValue, b.thre = [1.0], 368, 8, 128, 0.035
    b.guassian_filter_conv = utilmx.GaussianBlurConv(22)
    return b


def gen_batch_hand():
    """Batch_hand (srcmx/Batch_model.py:326-354) on planted hand maps and the seeded network."""
    from oracle.batch_post import to_tensor
    from src.model import handpose_model
    rng0 = np.random.default_rng(88)
    heats = []
    for seed, vis_p, extra in ((800, 0.9, 0), (801, 0.7, 2), (802, 0.0, 0), (803, 1.0, 3)):
        rng = np.random.default_rng(seed)
        pts = rng0.uniform(0.15, 0.85, size=(21, 2))
        vis = rng.random(21) < vis_p
        heats.append(planted.render_hand(46, 46, pts, vis, rng, extra_blobs=extra))
    heat = np.stack(heats)
    crops = np.random.default_rng(9).integers(0, 256, (len(heats), 368, 368, 3), dtype=np.uint8)
    peaks = ref_batch_hand(PlantedHandBatch(heat))(to_tensor(crops))
    np.savez_compressed(os.path.join(OUT, "batch_hand_planted_b4.npz"), heat=heat, peaks=peaks)
    print("wrote batch_hand_planted", peaks.dtype, peaks.shape)
    m = handpose_model().eval()
    sd = onet.seeded_state_dict("hand", 0)
    m.load_state_dict({k: sd[".".join(k.split(".")[1:])] for k in m.state_dict().keys()})
    crops = np.random.default_rng(10).integers(0, 256, (2, 64, 64, 3), dtype=np.uint8)
    peaks = ref_batch_hand(m)(to_tensor(crops))
    np.savez_compressed(os.path.join(OUT, "batch_hand_e2e_b2_64.npz"), crops=crops, peaks=peaks)
    print("wrote batch_hand_e2e", peaks.dtype, peaks.shape)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "batch":
    install_batch_shims()
    sys.path.insert(0, REF)
    torch.set_num_threads(8)
    gen_batch_body()
    gen_batch_hand()


# ---------------------------------------------------------------- C5: 1080p four-scale pyramid
C5_SCALES = [0.5, 1.0, 1.5, 2.0]


def ref_body_scales(model, scales):
    """The reference's Body.__call__ with its commented-out multi-scale line active
    (src/body.py:25-26): the method's own source, one assignment changed, compiled in the
    reference module's namespace (nothing is written anywhere)."""
    import inspect
    import textwrap
    import src.body as rb
    code = textwrap.dedent(inspect.getsource(rb.Body.__call__))
    old = "    scale_search = [0.5]\n"
    assert code.count(old) == 1
    code = code.replace(old, f"    scale_search = {list(scales)!r}\n")
    ns = dict(vars(rb))
    exec(compile(code, rb.__file__, "exec"), ns)
    b = ref_body(model)
    b.__class__ = type("BodyScales", (rb.Body,), {"__call__": ns["__call__"]})
    return b


class PlantedBodyScales:
    """Stand-in network returning each scale's planted low-res maps, selected by input size."""

    def __init__(self, by_shape):
        self.by_shape = by_shape

    def __call__(self, data):
        paf, heat = self.by_shape[(data.shape[2] // 8, data.shape[3] // 8)]
        return torch.from_numpy(paf[None]), torch.from_numpy(heat[None])


def gen_body_c5():
    """Planted 1080x1920 frame at scale_search = [0.5, 1, 1.5, 2] (BASELINE.json C5): the same
    people rendered at every scale's low-res grid, the reference's multi-scale Body on them."""
    from oracle.body_post import preprocess
    H, W = 1080, 1920
    for seed, n_people in ((700, 8), (701, 3)):
        rng = np.random.default_rng(seed)
        geo = []
        for s in C5_SCALES:
            _, pad, padded = preprocess(np.zeros((H, W, 3), np.uint8), s * 368 / H)
            geo.append((padded[0] // 8, padded[1] // 8, pad, padded))
        hl, wl = geo[-1][0], geo[-1][1]
        people, vis = planted.random_people(rng, n_people, hl, wl, min_h=0.3, max_h=0.7)
        maps, by_shape = {}, {}
        for i, (h, w, pad, padded) in enumerate(geo):
            # the 2.0-scale people mapped onto this scale's grid (pixel centres)
            sy, sx = h / hl, w / wl
            pts = (people + 0.5) * np.array([sx, sy]) - 0.5
            paf, heat = planted.render_body(h, w, pts, vis, np.random.default_rng(seed * 10 + i),
                                            sigma=0.9 * max(sy, 0.5), band=0.9 * max(sy, 0.6), noise=0.0)
            by_shape[(h, w)] = (paf, heat)
            maps[f"paf{i}"], maps[f"heat{i}"] = paf, heat
            maps[f"pad{i}"], maps[f"padded{i}"] = np.array(pad), np.array(padded)
        body = ref_body_scales(PlantedBodyScales(by_shape), C5_SCALES)
        cand, subset = body(np.zeros((H, W, 3), np.uint8))
        name = f"body_c5_{seed}_{H}x{W}_p{n_people}.npz"
        np.savez_compressed(os.path.join(OUT, name), img_hw=np.array([H, W]), scales=np.array(C5_SCALES),
                            candidate=cand, subset=subset, **maps)
        print("wrote", name, "cand", cand.shape, "subset", subset.shape)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "c5":
    install_shims()
    sys.path.insert(0, REF)
    torch.set_num_threads(8)
    gen_body_c5()


# ---------------------------------------------------------------- Body+Hand frame-pipeline glue
def gen_glue():
    """The reference's MotionData_every_frame (srcmx/MotionEstimation.py:126-216) with planted
    Body / Hand stand-ins (oracle/glue_standins.py) in place of its module-level estimators."""
    install_batch_shims()
    from oracle import glue_standins as gs
    import src.body
    import src.hand
    src.body.Body, src.hand.Hand = gs.StandInBody, gs.StandInHand
    import MotionEstimation as me
    assert isinstance(me.body_estimation, gs.StandInBody) and isinstance(me.hand_estimation, gs.StandInHand)
    out = {}
    for seed, H, W in gs.SCENES:
        img = gs.frame(seed, H, W)
        cand, subset = gs.scene(seed, H, W)
        gs.StandInBody.register(img, cand, subset)
        for mode in ("body", "bodyhand"):
            out[f"pose_{seed}_{mode}"] = me.MotionData_every_frame(img, mode=mode)
    np.savez_compressed(os.path.join(OUT, "glue_motion_every_frame.npz"),
                        scenes=np.array(gs.SCENES), **out)
    print("wrote glue_motion_every_frame.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "glue":
    sys.path.insert(0, REF)
    gen_glue()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "hand368":
    # C3's crop size (BASELINE.json: per-detected-hand 368x368 crops)
    install_shims()
    sys.path.insert(0, REF)
    gen_hand_planted(((604, 368, 0.85, 2),))


# ---------------------------------------------------------------- video front end (f2)
def gen_motion():
    """The reference's Extract_MotionData_from_Video (srcmx/MotionEstimation.py:25-76) on fake
    videos (oracle/glue_standins.py FakeCapture as cv2.VideoCapture): frame counts above and at
    the decoded count, one above it (IndexError), a file that does not open; ROI crop; body and
    bodyhand modes; the joblib file it writes, read back.  Planted Body / Hand stand-ins."""
    import contextlib
    import io
    import tempfile
    import joblib
    install_batch_shims()
    from oracle import glue_standins as gs
    import cv2
    cv2.VideoCapture = gs.FakeCapture
    cv2.CAP_PROP_FRAME_COUNT = gs.CAP_PROP_FRAME_COUNT
    import src.body
    import src.hand
    src.body.Body, src.hand.Hand = gs.StandInBody, gs.StandInHand
    import MotionEstimation as me
    me.body_estimation, me.hand_estimation = gs.StandInBody(), gs.StandInHand()
    me.cv2.VideoCapture, me.cv2.CAP_PROP_FRAME_COUNT = gs.FakeCapture, gs.CAP_PROP_FRAME_COUNT
    for seed, H, W in gs.SCENES:
        gs.StandInBody.register(gs.frame(seed, H, W), *gs.scene(seed, H, W))
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for clip in ("clip_short.avi", "clip_exact.avi", "clip_overflow.avi", "clip_missing.avi"):
            for mode in ("body", "bodyhand"):
                dst = os.path.join(td, "%s-%s.pkl" % (clip, mode))
                key = "%s_%s" % (clip.split(".")[0], mode)
                log = io.StringIO()
                try:
                    with contextlib.redirect_stdout(log):
                        ret = me.Extract_MotionData_from_Video(os.path.join(td, clip), dst, gs.ROI, mode=mode)
                    out[key + "_ret_none"] = np.array(ret is None)
                    out[key + "_written"] = np.array(os.path.exists(dst))
                    if os.path.exists(dst):
                        out[key] = joblib.load(dst)  # (written by the reference just now)
                except IndexError:
                    out[key + "_error"] = np.array("IndexError")
                out[key + "_stdout"] = np.array(log.getvalue().replace(td + os.sep, ""))
    np.savez_compressed(os.path.join(OUT, "motion_extract.npz"), **out)
    print("wrote motion_extract.npz", {k: v.shape for k, v in out.items()})


def gen_motion_seeded():
    """Extract_MotionData_from_Video with the reference's own Body / Hand on the seeded networks
    (bodyhand mode, 3 decoded frames of a 4-frame container, ROI crop): the golden the GPU
    device ingest is held to (tests/test_gpu_pipeline.py)."""
    import contextlib
    import io
    import tempfile
    import joblib
    install_batch_shims()
    from oracle import glue_standins as gs
    import cv2
    from src.model import bodypose_model, handpose_model
    bm = bodypose_model().eval()
    sd = onet.seeded_state_dict("body", 0)
    bm.load_state_dict({k: sd[".".join(k.split(".")[1:])] for k in bm.state_dict().keys()})
    hm = handpose_model().eval()
    sd = onet.seeded_state_dict("hand", 0)
    hm.load_state_dict({k: sd[".".join(k.split(".")[1:])] for k in hm.state_dict().keys()})
    body, hand = ref_body(bm), ref_hand(hm)
    import src.body
    import src.hand
    src.body.Body = lambda *a, **k: body
    src.hand.Hand = lambda *a, **k: hand
    seeds = (910, 911, 912)
    gs.VIDEOS["clip_seeded.avi"] = (seeds, 4)
    cv2.VideoCapture = gs.FakeCapture
    cv2.CAP_PROP_FRAME_COUNT = gs.CAP_PROP_FRAME_COUNT
    import MotionEstimation as me
    # (the module may already be imported by gen_motion with the stand-ins)
    me.body_estimation, me.hand_estimation = body, hand
    me.cv2.VideoCapture, me.cv2.CAP_PROP_FRAME_COUNT = gs.FakeCapture, gs.CAP_PROP_FRAME_COUNT
    with tempfile.TemporaryDirectory() as td:
        dst = os.path.join(td, "seeded.pkl")
        with contextlib.redirect_stdout(io.StringIO()):
            me.Extract_MotionData_from_Video(os.path.join(td, "clip_seeded.avi"), dst, gs.ROI, mode="bodyhand")
        motion = joblib.load(dst)
    np.savez_compressed(os.path.join(OUT, "motion_extract_seeded.npz"), seeds=np.array(seeds), count=np.array(4),
                        motion=motion)
    print("wrote motion_extract_seeded.npz", motion.shape, (motion != 0).any(2).sum(1))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "motion":
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "srcmx"))
    torch.set_num_threads(8)
    gen_motion_seeded()  # (first: gen_motion replaces src.body.Body / src.hand.Hand by stand-ins)
    gen_motion()


# ---------------------------------------------------------------- full-size C3 / C5 (verdict r3 item 2)
def gen_fullsize():
    """Body() on one 1080x1920 frame with scale_search [0.5, 1, 1.5, 2] (C5, the C5 calibration)
    and Hand() on one 368x368 crop (C3's four pyramid networks 184^2 .. 736^2), through the oracle
    (oracle/network.py + oracle/body_post.py / hand_post.py, pinned to the reference's goldens by
    tests/test_oracle_golden.py) in float32 -- the reference's arithmetic -- and in float64 (the
    exact answer near ties).  The GPU tests regenerate the inputs from the seeds; only the outputs
    are stored (tests/golden/fullsize_c3_c5.npz)."""
    sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
    from oracle import body_post, hand_post
    from src.weights import c5_out_scale
    torch.set_num_threads(8)
    out = {}
    img = np.random.default_rng(53).integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
    sd = onet.seeded_state_dict("body", 0, out_scale=c5_out_scale())
    for tag, d, dbl in (("f32", sd, False), ("f64", {k: v.double() for k, v in sd.items()}, True)):
        def fn(x, d=d, dbl=dbl):
            xx = torch.from_numpy(x)
            p, h = onet.body_forward(xx.double() if dbl else xx, d)
            return p.float().numpy(), h.float().numpy()
        c, s = body_post.body_infer(img, fn, scale_search=(0.5, 1.0, 1.5, 2.0))
        out["c5_cand_" + tag], out["c5_subset_" + tag] = np.asarray(c, np.float64), s
        print("C5", tag, np.shape(c), s.shape)
    crop = np.random.default_rng(54).integers(0, 256, (368, 368, 3), dtype=np.uint8)
    hsd = onet.seeded_state_dict("hand", 0)
    for tag, d, dbl in (("f32", hsd, False), ("f64", {k: v.double() for k, v in hsd.items()}, True)):
        def hfn(x, d=d, dbl=dbl):
            xx = torch.from_numpy(x)
            return onet.hand_forward(xx.double() if dbl else xx, d).float().numpy()
        out["c3_peaks_" + tag] = hand_post.hand_infer(crop, hfn)
        print("C3", tag, out["c3_peaks_" + tag][:3])
    np.savez_compressed(os.path.join(OUT, "fullsize_c3_c5.npz"), c5_seed=np.array(53), c3_seed=np.array(54), **out)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "fullsize":
    gen_fullsize()


# ---------------------------------------------------------------- C2-size end to end + the reference's own tie noise
def gen_e2e_c2():
    """Verdict r4 item 6.  (a) C2's frame size, 368x656, through the reference's own Body() with
    the seeded network at 8 torch threads (as every golden here): tests/golden/body_e2e_31_368x656.npz
    (the image is regenerated from its seed).  (b) The reference against itself: every body_e2e
    golden's image through the reference's Body() at 1, 2, 4, 8 and 16 threads, each run's keypoints
    against the 8-thread golden, and whether every keypoint it moves sits on a float64 plateau
    (oracle/ties.py) -> profiles/r5_ref_thread_noise.json."""
    from src.model import bodypose_model
    from oracle import ties
    assert "reference" in sys.modules["src.model"].__file__
    m = bodypose_model().eval()
    sd = onet.seeded_state_dict("body", 0)
    m.load_state_dict({k: sd[".".join(k.split(".")[1:])] for k in m.state_dict().keys()})
    seed, hw = 31, (368, 656)
    img31 = np.random.default_rng(seed).integers(0, 256, size=hw + (3,), dtype=np.uint8)
    torch.set_num_threads(8)
    cand, subset = ref_body(m)(img31)
    name = f"body_e2e_{seed}_{hw[0]}x{hw[1]}.npz"
    np.savez_compressed(os.path.join(OUT, name), img_seed=np.array(seed), img_hw=np.array(hw),
                        img_sum=np.array(int(img31.astype(np.int64).sum())), candidate=cand, subset=subset)
    print("wrote", name, cand.shape, subset.shape)
    rows = []
    for path in sorted(glob.glob(os.path.join(OUT, "body_e2e_*.npz"))):
        d = np.load(path)
        img = d["img"] if "img" in d else img31
        up, blur = ties.f64_smoothed(img, sd)
        for th in (1, 2, 4, 8, 16):
            torch.set_num_threads(th)
            c, s = ref_body(m)(img)
            r = {"golden": os.path.basename(path), "threads": th, "keypoints": len(c),
                 "people": len(s), "golden_people": len(d["subset"])}
            if len(c) == len(d["candidate"]):
                moved = int((c[:, :2] != d["candidate"][:, :2]).any(1).sum())
                pairs = ties.tie_pairs(up, blur, c, d["candidate"])
                r.update(moved_vs_8_threads=moved, moves_on_f64_ties=pairs is not None and len(pairs) == moved,
                         identical_to_golden=bool(np.array_equal(c, d["candidate"]) and np.array_equal(s, d["subset"])))
            rows.append(r)
            print(json.dumps(r), flush=True)
    torch.set_num_threads(8)
    with open(os.path.join(REPO, "profiles", "r5_ref_thread_noise.json"), "w") as fh:
        json.dump({"generator": "oracle/gen_golden.py e2e_c2", "reference": "src/body.py Body.__call__ with src/model.py "
                   "bodypose_model (imported read-only), seeded weights", "torch": torch.__version__,
                   "tie_rule": "oracle/ties.py: float64 smoothed values within 1e-6 of the part map's max", "rows": rows},
                  fh, indent=1)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "e2e_c2":
    install_shims()
    sys.path.insert(0, REF)
    gen_e2e_c2()
