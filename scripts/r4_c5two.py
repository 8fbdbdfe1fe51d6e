"""Repro of the bench_configs C5 sequence: a 4-frame lockstep handle, a per-scale handle created,
used and destroyed, then single frames on the first handle."""
import faulthandler
import os
import sys

import numpy as np
import torch

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body  # noqa: E402
from src.weights import c5_out_scale, seeded_state_dict  # noqa: E402

step = sys.argv[1] if len(sys.argv) > 1 else "all"
sd = seeded_state_dict("body", 0, out_scale=c5_out_scale())
b = Body(sd, scale_search=(0.5, 1.0, 1.5, 2.0))
f = torch.from_numpy(np.random.default_rng(3).integers(0, 256, (4, 1080, 1920, 3), dtype=np.uint8)).cuda()
rb = b.handle.record_bytes()
recs = [torch.empty((4, rb), dtype=torch.uint8, device="cuda") for _ in range(2)]
for i in range(3):
    b.infer_records(f, recs[i % 2]); b.handle.synchronize()
print("batch ok", flush=True)
for i in range(3):
    b.infer_records(f, recs[i % 2], pipeline=True)
b.handle.synchronize()
print("pipelined ok", flush=True)
if step in ("all", "second"):
    os.environ["OPOSE_LOCKSTEP"] = "0"
    b2 = Body(sd, scale_search=(0.5, 1.0, 1.5, 2.0))
    del os.environ["OPOSE_LOCKSTEP"]
    for i in range(3):
        b2.infer_records(f, recs[0]); b2.handle.synchronize()
    for i in range(3):
        b2.infer_records(f[:1].contiguous(), recs[0][:1]); b2.handle.synchronize()
    del b2
    print("second handle ok", flush=True)
f1 = f[:1].contiguous()
for i in range(4):
    print("single", i, flush=True)
    b.infer_records(f1, recs[0][:1]); b.handle.synchronize()
print("ok", flush=True)
