"""Diagnostic: the balanced 4-rank plan's banded maps (threads on one GPU) against scale_maps,
per scale, and the records of post_scales on them against Body.batch."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "pytorch-openpose_amd")
import test_gpu_band as T
from src.body import Body
from src.dist import band_rows, split_plan
from src.weights import c5_out_scale, seeded_state_dict

sd = seeded_state_dict("body", 0, out_scale=c5_out_scale())
bodies = [Body(sd, scale_search=T.SCALES) for _ in range(5)]
img = np.random.default_rng(43).integers(0, 256, T.HW + (3,), dtype=np.uint8)
geo = bodies[0].scale_geom(*T.HW)
_, owners, _ = split_plan([g[0] * g[1] for g in geo], 4, [g[0] for g in geo])
print("owners", owners)
maps = []
for s, rs in enumerate(owners):
    ref = bodies[0].scale_maps(img, s)
    if len(rs) == 1:
        maps.append(ref)
        continue
    got = T._run_bands(bodies, img, s, band_rows(geo[s][0], len(rs)), exact=False)
    d = np.abs(got - ref)
    print("scale", s, "max abs", d.max(), "max rel", (d / (np.abs(ref) + 1e-6)).max(), "ref max", np.abs(ref).max())
    maps.append(got)
np.savez("gpurun_out/thread_maps.npz", *maps)
(c, su), = bodies[0].post_scales(maps, *T.HW)
(rc, rsu), = bodies[0].batch(img[None])
print("cand equal", np.array_equal(c, rc), c.shape, rc.shape)
if c.shape == rc.shape:
    dd = np.where((c != rc).any(1))[0]
    print("cand rows differing", dd[:10], c[dd[:5]], rc[dd[:5]])
if c.shape == rc.shape:
    mv = np.where((c[:, :2] != rc[:, :2]).any(1))[0]
    print("moved peaks", len(mv), c[mv][:5], rc[mv][:5])
print("subset equal", np.array_equal(su, rsu))
if su.shape == rsu.shape:
    dd = np.where((su != rsu).any(1))[0]
    print("subset rows differing", dd[:10], su[dd[:3]], rsu[dd[:3]])
