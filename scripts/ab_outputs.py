"""Raw network outputs of the engine on seeded inputs, for bit-exact A/B between two builds
(OPOSE_LIB=<other .so> picks the library): a Hand() scale pyramid (stream-K 7x7 layers and their
fixup), one 368x656 body frame (stream-K everywhere) and a 4-frame body batch.

  python scripts/ab_outputs.py save out.npz
  python scripts/ab_outputs.py compare a.npz b.npz     # exit 1 unless every array is bit-identical
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))


def save(path):
    from src import util
    from src.model import bodypose_model, handpose_model
    from src.weights import seeded_state_dict

    rng = np.random.default_rng(11)
    out = {}
    hand = handpose_model()
    hand.load_state_dict(util.transfer(hand, seeded_state_dict("hand", 0)))
    xs = [rng.standard_normal((1, 3, s, s)).astype(np.float32) * 0.5 for s in (184, 368, 552, 736)]
    for i, h in enumerate(hand.forward_pyramid(xs)):
        out["hand_pyr%d" % i] = h
    body = bodypose_model(handle=hand.handle)
    body.load_state_dict(util.transfer(body, seeded_state_dict("body", 0)))
    for n in (1, 4):
        x = rng.standard_normal((n, 3, 368, 656)).astype(np.float32) * 0.5
        paf, heat = body(x)
        out["body%d_paf" % n] = paf
        out["body%d_heat" % n] = heat
    # the bench's layer shapes: 8 frames at the network input of a 368x656 frame at scale 0.5
    x = rng.standard_normal((8, 3, 184, 328)).astype(np.float32) * 0.5
    paf, heat = body(x)
    out["body8s_paf"] = paf
    out["body8s_heat"] = heat
    np.savez(path, **out)
    print("saved", path, {k: v.shape for k, v in out.items()})


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        same = np.array_equal(A[k].view(np.uint32), B[k].view(np.uint32))
        diff = float(np.max(np.abs(A[k] - B[k])))
        print("%-12s %s max|diff| %.3g" % (k, "bit-identical" if same else "DIFFERS", diff))
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
