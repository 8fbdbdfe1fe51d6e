"""Graph-launch crash repro: Hand handle A runs (graph captured, with per-scale stream branches),
is destroyed (or kept), then Hand handle B runs 4 calls (eager, capture, replays)."""
import faulthandler
import gc
import os
import sys

import numpy as np

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.hand import Hand  # noqa: E402
from src.weights import seeded_state_dict  # noqa: E402

mode = sys.argv[1]
sd = seeded_state_dict("hand", 0)
crop = np.random.default_rng(1).integers(0, 256, (128, 128, 3), dtype=np.uint8)
a = Hand(sd)
for _ in range(4):
    ra = a(crop)
if mode != "keep":
    del a
    gc.collect()
print("A done", file=sys.stderr, flush=True)
b = Hand(sd)
for i in range(4):
    rb = b(crop)
    print("B call", i, file=sys.stderr, flush=True)
assert np.array_equal(ra, rb)
print("ok", mode, file=sys.stderr, flush=True)
