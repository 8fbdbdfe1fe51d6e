"""Repro: single-frame multi-scale Body (C5, 1080p, 4 scales) through infer_records, a few calls."""
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

b = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=(0.5, 1.0, 1.5, 2.0))
f = torch.from_numpy(np.random.default_rng(3).integers(0, 256, (1, 1080, 1920, 3), dtype=np.uint8)).cuda()
rec = torch.empty((1, b.handle.record_bytes()), dtype=torch.uint8, device="cuda")
for i in range(4):
    print("call", i, flush=True)
    b.infer_records(f, rec)
    b.handle.synchronize()
print("ok", flush=True)
