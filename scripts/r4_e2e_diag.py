"""Body() on the e2e golden images; saves candidates/subsets and the scale-0 maps."""
import glob, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body
from src.weights import seeded_state_dict
body = Body(seeded_state_dict("body", 0))
out = {}
for p in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "body_e2e_*.npz"))):
    d = np.load(p)
    c, s = body(d["img"])
    k = os.path.basename(p)[:-4]
    out[k + "_cand"] = c
    out[k + "_subset"] = s
    out[k + "_maps"] = body.scale_maps(d["img"][None], 0)
    print(k, c.shape, d["candidate"].shape, "equal xy" if c.shape == d["candidate"].shape and np.array_equal(c[:, :2], d["candidate"][:, :2]) else "DIFF")
np.savez(os.path.join(REPO, "gpurun_out", "e2e_gpu.npz"), **out)
