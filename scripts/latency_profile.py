"""Single-frame Body() latency breakdown (GPU kernel time per class vs wall)."""
import os, sys, time, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body
from src.weights import BENCH_OUT_SCALE, seeded_state_dict
body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
img = np.random.default_rng(1).integers(0, 256, (368, 656, 3), dtype=np.uint8)
for _ in range(5):
    body(img)
t = []
for _ in range(20):
    t0 = time.perf_counter(); body(img); t.append(time.perf_counter() - t0)
print("wall ms median", np.median(t) * 1e3, "min", np.min(t) * 1e3)
body.handle.profile(2); body.handle.profile_reset()
for _ in range(10):
    body(img)
prof = body.handle.profile_read(); body.handle.profile(False)
tot = 0
for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"]):
    if not k.startswith("layer/"):
        tot += v["ms"] / 10
        print(f"{k:20s} {v['ms'] / 10:8.3f} ms  x{v['count'] // 10}")
print("sum of kernel classes", tot)
for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"])[:12]:
    if k.startswith("layer/"):
        print(f"{k:70s} {v['ms'] / 10:8.3f} ms")
