"""Per-layer GPU times of one C5 scale network (opose_body_scale_maps on one 1080x1920 frame,
events around every launch, graphs off).  argv[1]: scale index (default 3 = the 2.0 scale).
OPOSE_LIB selects the library, so a same-box A/B is two runs."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body  # noqa: E402
from src.weights import c5_out_scale, seeded_state_dict  # noqa: E402
import src._native as nat  # noqa: E402

s = int(sys.argv[1]) if len(sys.argv) > 1 else 3
b = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=(0.5, 1.0, 1.5, 2.0))
img = np.random.default_rng(53).integers(0, 256, (1, 1080, 1920, 3), dtype=np.uint8)
for _ in range(3):
    b.scale_maps(img, s)
t = []
for _ in range(5):
    t0 = time.perf_counter()
    b.scale_maps(img, s)
    t.append(time.perf_counter() - t0)
print("scale %d: %.3f ms host to host (median of 5)" % (s, np.median(t) * 1e3))
b.handle.check(nat.lib.opose_profile_enable(b.handle.h, 2))
b.handle.profile_reset()
R = 3
for _ in range(R):
    b.scale_maps(img, s)
prof = b.handle.profile_read()
rows = sorted(((k, v) for k, v in prof.items() if k.startswith("layer/")), key=lambda kv: -kv[1]["ms"])
print("sum of layer ms %.3f" % (sum(v["ms"] for k, v in rows) / R))
for k, v in rows[:25]:
    tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
    print("%-76s %7.3f ms %6.1f TF/s" % (k, v["ms"] / R, tf))
