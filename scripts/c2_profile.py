"""C2 (one 368x656 frame through Body()) per-stage / per-layer GPU times, device-resident
batch 1, seeded weights with the bench calibration."""
import os, sys, time
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body
from src.weights import BENCH_OUT_SCALE, seeded_state_dict
import src._native as nat

body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
img = np.random.default_rng(3).integers(0, 256, (368, 656, 3), dtype=np.uint8)
dev = torch.device("cuda", 0)
f1 = torch.from_numpy(img[None].copy()).to(dev)
rec = torch.empty((1, body.handle.record_bytes()), dtype=torch.uint8, device=dev)
for _ in range(5):
    body.infer_records(f1, rec)
body.handle.synchronize()
t = []
for _ in range(30):
    t0 = time.perf_counter(); body.infer_records(f1, rec); body.handle.synchronize(); t.append(time.perf_counter() - t0)
print("device batch-1 wall ms %.3f (graph replay)" % (np.median(t) * 1e3))
body.handle.check(nat.lib.opose_profile_enable(body.handle.h, 2))
body.handle.profile_reset()
R = 10
for _ in range(R):
    body.infer_records(f1, rec)
body.handle.synchronize()
prof = body.handle.profile_read()
body.handle.check(nat.lib.opose_profile_enable(body.handle.h, 0))
stages = {k: v["ms"] / R for k, v in prof.items() if not k.startswith("layer/")}
print("stages ms:", {k: round(v, 4) for k, v in sorted(stages.items(), key=lambda kv: -kv[1])})
print("sum of stage ms %.3f" % sum(stages.values()))
rows = sorted(((k, v) for k, v in prof.items() if k.startswith("layer/")), key=lambda kv: -kv[1]["ms"])
for k, v in rows[:30]:
    tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
    print("%-66s %7.4f ms %6.1f TF/s" % (k, v["ms"] / R, tf))
