"""C5 (1920x1080, scale_search [0.5, 1, 1.5, 2]) batch of 4 device-resident frames: ms per batch
and the post-network stage times, for a same-box A/B between builds (OPOSE_LIB=<other .so>)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body  # noqa: E402
from src.weights import c5_out_scale, seeded_state_dict  # noqa: E402

b = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=(0.5, 1.0, 1.5, 2.0))
f = torch.from_numpy(np.random.default_rng(53).integers(0, 256, (4, 1080, 1920, 3), dtype=np.uint8)).cuda()
rec = torch.empty((4, b.handle.record_bytes()), dtype=torch.uint8, device="cuda")
for _ in range(3):
    b.infer_records(f, rec)
b.handle.synchronize()
t = []
for _ in range(8):
    t0 = time.perf_counter()
    b.infer_records(f, rec)
    b.handle.synchronize()
    t.append(time.perf_counter() - t0)
b.handle.profile(1)
b.handle.profile_reset()
for _ in range(2):
    b.infer_records(f, rec)
b.handle.synchronize()
prof = b.handle.profile_read()
b.handle.profile(False)
st = {k: round(v["ms"] / 2, 3) for k, v in sorted(prof.items()) if not k.startswith("conv")}
print("lib %s: %.2f ms per batch of 4; post stages %s" % (os.environ.get("OPOSE_LIB", "default"), float(np.median(t)) * 1e3, st))
