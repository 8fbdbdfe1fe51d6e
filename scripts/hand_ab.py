"""Hand() one crop: host-to-host latency and the per-stage GPU times of a profiled pass, for a
same-box A/B between two builds (OPOSE_LIB=<other .so>).  python scripts/hand_ab.py"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.hand import Hand  # noqa: E402
from src.weights import seeded_state_dict  # noqa: E402

hand = Hand(seeded_state_dict("hand", 0))
crop = np.random.default_rng(5).integers(0, 256, (368, 368, 3), dtype=np.uint8)
for _ in range(5):
    hand(crop)
t = []
for _ in range(20):
    t0 = time.perf_counter()
    hand(crop)
    t.append(time.perf_counter() - t0)
hand.handle.profile(1)
hand.handle.profile_reset()
for _ in range(3):
    hand(crop)
prof = hand.handle.profile_read()
hand.handle.profile(False)
stages = {k: round(v["ms"] / 3, 4) for k, v in sorted(prof.items())}
print("lib %s: one crop %.3f ms; stages %s" % (os.environ.get("OPOSE_LIB", "default"), float(np.median(t)) * 1e3, stages))
