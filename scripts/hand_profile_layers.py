"""Per-layer kernel times of one Hand() call on a 368x368 crop (scales one after another)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
os.environ.setdefault("OPOSE_SCALE_STREAMS", "0")
from src.hand import Hand
from src.weights import seeded_state_dict
hand = Hand(seeded_state_dict("hand", 0))
crop = np.random.default_rng(5).integers(0, 256, (368, 368, 3), dtype=np.uint8)
for _ in range(3):
    hand(crop)
hand.handle.check(__import__("src._native", fromlist=["lib"]).lib.opose_profile_enable(hand.handle.h, 2))
hand.handle.profile_reset()
for _ in range(3):
    hand(crop)
prof = hand.handle.profile_read()
rows = sorted(((k, v) for k, v in prof.items() if k.startswith("layer/")), key=lambda kv: -kv[1]["ms"])
tot = sum(v["ms"] for k, v in rows) / 3
print("total layer ms per call %.3f" % tot)
for k, v in rows[:45]:
    tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
    print("%-72s %7.3f ms %6.1f TF/s" % (k, v["ms"] / 3, tf))
