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


def gen_hand_planted():
    rng0 = np.random.default_rng(77)
    for seed, size, vis_p, extra in ((600, 96, 0.9, 0), (601, 150, 0.7, 2), (602, 64, 0.0, 0), (603, 200, 1.0, 3)):
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
