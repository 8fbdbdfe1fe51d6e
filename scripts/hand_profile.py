"""Per-layer kernel times of one Hand() call (4 scales, one 368x368 crop)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.hand import Hand
from src.weights import seeded_state_dict
hand = Hand(seeded_state_dict("hand", 0))
crop = np.random.default_rng(3).integers(0, 256, (368, 368, 3), dtype=np.uint8)
for _ in range(3):
    hand(crop)
hand.handle.profile(2); hand.handle.profile_reset()
R = 5
for _ in range(R):
    hand(crop)
prof = hand.handle.profile_read(); hand.handle.profile(False)
tot = 0
for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"]):
    if not k.startswith("layer/"):
        tot += v["ms"] / R
        print(f"{k:20s} {v['ms'] / R:8.3f} ms x{v['count'] // R}  {v['flops'] / max(v['ms'], 1e-9) / 1e9:7.1f} TF/s")
print("sum", tot)
for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"])[:40]:
    if k.startswith("layer/"):
        print(f"{k:70s} {v['ms'] / R:8.3f} ms {v['flops'] / max(v['ms'], 1e-9) / 1e9:7.1f} TF/s")
