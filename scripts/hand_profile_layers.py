"""Hand() on a 368x368 crop (4 scales): host-to-host latency of one crop and of two crops
batched (Hand.batch_crops), then per-layer kernel times of profiled passes (events around every
launch, graphs off) of one crop and of the two-crop batch.  The engine configuration comes from
the environment (OPOSE_LOCKSTEP, OPOSE_SPLIT_FRAMES, ...), so an A/B is two runs
of this script."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.hand import Hand  # noqa: E402
from src.weights import seeded_state_dict  # noqa: E402


def median_ms(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    t = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return float(np.median(t)) * 1e3


hand = Hand(seeded_state_dict("hand", 0))
rng = np.random.default_rng(5)
crop = rng.integers(0, 256, (368, 368, 3), dtype=np.uint8)
crop2 = rng.integers(0, 256, (256, 256, 3), dtype=np.uint8)
env = {k: v for k, v in os.environ.items() if k.startswith("OPOSE_")}
one = median_ms(lambda: hand(crop))
two = median_ms(lambda: hand.batch_crops([crop, crop2]), iters=6)
print("env %s: one crop %.3f ms, two crops batched %.3f ms (%.2fx)" % (env, one, two, two / one))
hand.handle.check(__import__("src._native", fromlist=["lib"]).lib.opose_profile_enable(hand.handle.h, 2))


def layers(title, fn, nrows):
    hand.handle.profile_reset()
    for _ in range(3):
        fn()
    prof = hand.handle.profile_read()
    conv = [v for k, v in prof.items() if k.startswith("conv")]
    print("%s: conv class ms per call %.3f, %.3f TFLOP" % (title, sum(v["ms"] for v in conv) / 3,
                                                           sum(v["flops"] for v in conv) / 3e12))
    rows = sorted(((k, v) for k, v in prof.items() if k.startswith("layer/")), key=lambda kv: -kv[1]["ms"])
    print("total layer ms per call %.3f" % (sum(v["ms"] for k, v in rows) / 3))
    for k, v in rows[:nrows]:
        tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
        print("%-84s %7.3f ms %6.1f TF/s" % (k, v["ms"] / 3, tf))


layers("one crop", lambda: hand(crop), 60)
layers("two crops batched", lambda: hand.batch_crops([crop, crop2]), 16)
