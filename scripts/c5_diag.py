import os, sys, numpy as np, torch
sys.path.insert(0, "pytorch-openpose_amd"); sys.path.insert(0, ".")
from src.body import Body
from src.weights import c5_out_scale, seeded_state_dict
from oracle import body_post as bp
img = np.random.default_rng(3).integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
body = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale(-2.8, 2.0, 1.0)), scale_search=(0.5, 1.0, 1.5, 2.0), peaks_per_part=1024, max_people=256)
geo = body.scale_geom(1080, 1920)
lowres = []
for s in range(4):
    m = body.scale_maps(img[None], s)[0]
    hl, wl, pd, pr = geo[s]
    lowres.append((m[:38], m[38:], [0, 0, pd, pr], (hl * 8, wl * 8)))
    print("scale", s, "paf mean/std", m[:38].mean(), m[:38].std(), "heat max", m[38:56].max(), flush=True)
h, w = 1080, 1920
heat_avg = np.zeros((h, w, 19)); paf_avg = np.zeros((h, w, 38))
for paf, heat, pad, phw in lowres:
    heat_avg += bp.upsample_map(heat, pad, phw, (h, w)) / 4
    paf_avg += bp.upsample_map(paf, pad, phw, (h, w)) / 4
print("paf_avg mean", paf_avg.mean(), "std", paf_avg.std(), flush=True)
peaks = bp.find_peaks(heat_avg, 0.1)
print("peaks per part", [len(p) for p in peaks], flush=True)
for p in peaks[:3]:
    print("sample peaks", p[:5], flush=True)
conns, special = bp.connect_limbs(peaks, paf_avg, h, 0.05)
print("connections per limb", [len(c) for c in conns], "special", special, flush=True)
cand, subset = bp.assemble(peaks, conns, special)
print("cand", np.shape(cand), "subset", np.shape(subset), flush=True)
