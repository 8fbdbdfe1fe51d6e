"""Per-channel heat pre-activation statistics of the seeded body network on 1080p frames at
scale_search [0.5, 1, 1.5, 2] (C5): the 95th percentile and the max of each heat channel over the
four scales' maps.  An affine map per channel (p95 -> 0, max -> 1) then gives the C5 synthetic
workload ~a dozen peaks per part, as BENCH_OUT_SCALE does at 368x656 (src/weights.py)."""
import os, sys, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body
from src.weights import seeded_state_dict
SCALES = (0.5, 1.0, 1.5, 2.0)
q = float(sys.argv[1]) if len(sys.argv) > 1 else 99.0
# +100 on the heat biases keeps every pre-activation above the final ReLU: z = out - 100
body = Body(seeded_state_dict("body", 0, out_scale={"Mconv7_stage6_L2": (1.0, 100.0)}), scale_search=SCALES)
zs = [[] for _ in range(19)]
for seed in (3, 4):
    img = np.random.default_rng(seed).integers(0, 256, (1, 1080, 1920, 3), dtype=np.uint8)
    for s in range(len(SCALES)):
        m = body.scale_maps(img, s)[0, 38:] - 100.0
        for c in range(19):
            zs[c].append(m[c].ravel())
lo = [float(np.percentile(np.concatenate(z), q)) for z in zs]
hi = [float(np.concatenate(z).max()) for z in zs]
gain = [round(1.0 / max(h - l, 1e-3), 3) for l, h in zip(lo, hi)]
shift = [round(-l * g, 3) for l, g in zip(lo, gain)]
print(json.dumps({"q": q, "p": lo, "max": hi, "gain": gain, "shift": shift}))
