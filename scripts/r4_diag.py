"""Diagnose Body.batch (concurrent multi-scale infer) against post_scales(scale_maps)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "pytorch-openpose_amd"), REPO]
from src.body import Body  # noqa: E402
from src.weights import c5_out_scale, seeded_state_dict  # noqa: E402

SCALES = (0.5, 1.0, 1.5, 2.0)
img = np.random.default_rng(43).integers(0, 256, (368, 656, 3), dtype=np.uint8)
sd = seeded_state_dict("body", 0, out_scale=c5_out_scale())
b = Body(sd, scale_search=SCALES)
(ca, sa), = b.batch(img[None])
(cb, sb), = b.batch(img[None])
maps = [b.scale_maps(img, s) for s in range(4)]
cc, sc = b.post_scales(maps, 368, 656)[0]
print("batch twice equal", np.array_equal(ca, cb), len(ca), len(cb))
print("batch vs post(scale_maps)", np.array_equal(ca, cc), len(ca), len(cc))
(cd, sd_), = b.batch(img[None])
print("batch after scale_maps", np.array_equal(cd, cc), len(cd))
for s in range(4):
    m2 = b.scale_maps(img, s)
    print("scale_maps repeat", s, np.array_equal(m2, maps[s]))
os.environ["OPOSE_SCALE_STREAMS"] = "0"
b2 = Body(sd, scale_search=SCALES)
(ce, se), = b2.batch(img[None])
print("serial-scales batch vs post(scale_maps)", np.array_equal(ce, cc), len(ce))
maps2 = [b2.scale_maps(img, s) for s in range(4)]
print("serial handle scale_maps equal", [np.array_equal(x, y) for x, y in zip(maps, maps2)])
