"""C2 (one 368x656 frame through Body(), device-resident batch 1) as graph replays only, for a
rocprofv3 kernel trace: 5 warm-up calls (eager, capture, replays), then REPS timed replays."""
import os, sys, time
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body
from src.weights import BENCH_OUT_SCALE, seeded_state_dict

REPS = int(os.environ.get("REPS", "20"))
body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
img = np.random.default_rng(3).integers(0, 256, (368, 656, 3), dtype=np.uint8)
dev = torch.device("cuda", 0)
f1 = torch.from_numpy(img[None].copy()).to(dev)
rec = torch.empty((1, body.handle.record_bytes()), dtype=torch.uint8, device=dev)
for _ in range(5):
    body.infer_records(f1, rec)
body.handle.synchronize()
t = []
for _ in range(REPS):
    t0 = time.perf_counter(); body.infer_records(f1, rec); body.handle.synchronize(); t.append(time.perf_counter() - t0)
print("replays %d, median wall ms %.3f" % (REPS, np.median(t) * 1e3))
