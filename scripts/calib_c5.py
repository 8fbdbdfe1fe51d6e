"""Pick the heat-bias offset for the C5 (1080p, 4-scale) synthetic workload: peaks/people per frame."""
import os, sys, copy
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body
from src.weights import BENCH_OUT_SCALE, seeded_state_dict
img = np.random.default_rng(3).integers(0, 256, (1, 1080, 1920, 3), dtype=np.uint8)
dev = torch.device("cuda", 0)
f = torch.from_numpy(img).to(dev)
for off in (-2.5, -3.0, -3.5):
    for paf in (0.8,):
        cal = copy.deepcopy(BENCH_OUT_SCALE)
        w, b = cal["Mconv7_stage6_L2"]
        cal["Mconv7_stage6_L2"] = (w, [v + off for v in b])
        cal["Mconv7_stage6_L1"] = (1.0, paf)
        body = Body(seeded_state_dict("body", 0, out_scale=cal), scale_search=(0.5, 1.0, 1.5, 2.0), peaks_per_part=1024, max_people=256)
        rec = torch.empty((1, body.handle.record_bytes()), dtype=torch.uint8, device=dev)
        body.infer_records(f, rec)
        body.handle.synchronize()
        print(off, paf, "status/peaks/people", rec.view(torch.int32)[0, :3].tolist(), flush=True)
