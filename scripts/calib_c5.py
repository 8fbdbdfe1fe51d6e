"""Pick the heat-bias shift / PAF offset for the C5 (1080p, 4-scale) synthetic workload:
status, peaks and people per frame on two random frames (src/weights.py:c5_out_scale)."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body
from src.weights import c5_out_scale, seeded_state_dict
img = np.random.default_rng(3).integers(0, 256, (2, 1080, 1920, 3), dtype=np.uint8)
dev = torch.device("cuda", 0)
f = torch.from_numpy(img).to(dev)
# heat = gain * z + shift with z the 368x656-calibrated pre-activation: the threshold 0.1 is
# crossed at z* = (0.1 - shift) / gain; the gain sets how far peaks rise above it
zs = [float(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2.9,2.75").split(",")]
gains = [float(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,3,6").split(",")]
pafs = [float(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0.8").split(",")]
for z in zs:
    for gain in gains:
      for paf in pafs:
        off = 0.1 - gain * z
        body = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale(off, paf, gain)), scale_search=(0.5, 1.0, 1.5, 2.0),
                    peaks_per_part=1024, max_people=256)
        rec = body.infer_records(f)
        hdr = rec.view(torch.int32)[:, :3].cpu().tolist()
        print(f"z*={z} gain={gain} shift={off:.3f} paf={paf}", "status/peaks/people", hdr, flush=True)
