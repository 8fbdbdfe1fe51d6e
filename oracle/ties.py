"""ORACLE (test infrastructure only): float64 plateau ties of the smoothed heat maps.

The reference finds peaks on `gaussian_filter(heatmap_avg[:, :, part], sigma=3)` of its float32
network's maps (src/body.py:76-94).  Where two neighbouring pixels of that smoothed map differ by
less than the network's float32 summation noise, the order of the conv sums decides which one is
the peak: the reference itself moves such keypoints between torch thread counts
(profiles/r5_ref_thread_noise.json).  These helpers evaluate the network in float64 (the exact
answer up to 1e-16), smooth its x8 maps like the reference, and pair up keypoints that two runs
put on different pixels of such a plateau.  Used by tests/ (GPU vs reference goldens) and
oracle/gen_golden.py (the reference against itself); never by the product path.
"""
from __future__ import annotations

import numpy as np
import torch
from scipy.ndimage import gaussian_filter

from oracle import body_post, network


def f64_smoothed(img: np.ndarray, sd: dict, scale: float | None = None):
    """(x8 heat maps [H, W, 19] of the float64 network, the 18 smoothed part maps) for one
    single-scale Body() call (scale 0.5*368/H as src/body.py:25-31)."""
    H, W = img.shape[:2]
    x, pad, phw = body_post.preprocess(img, 0.5 * 368 / H if scale is None else scale)
    sd64 = {k: v.double() for k, v in sd.items()}
    _, heat = network.body_forward(torch.from_numpy(x).double(), sd64)
    up = body_post.upsample_map(heat.float().numpy()[0], pad, phw, (H, W))
    blur = [gaussian_filter(up[:, :, p].astype(np.float64), sigma=3) for p in range(18)]
    return up, blur


def tie_pairs(up, blur, cand, ref_c, tol: float = 1e-6):
    """Rows where `cand` and `ref_c` (same length, same order) put a keypoint on different
    pixels, paired up: each ref_c row with a cand row one pixel away whose float64 smoothed values
    differ by at most tol of that part map's maximum.  Returns {cand row: ref_c row}, or None if a
    differing row is not such a move."""
    H, W = up.shape[:2]
    gi = [i for i in range(len(cand)) if not np.array_equal(cand[i, :2], ref_c[i, :2])]
    pairs = {}
    for j in gi:
        xr, yr = (int(v) for v in ref_c[j, :2])
        hit = None
        for i in gi:
            xg, yg = (int(v) for v in cand[i, :2])
            if i in pairs or abs(xg - xr) > 1 or abs(yg - yr) > 1 or not (0 <= xg < W and 0 <= yg < H):
                continue
            # the keypoint's part: the one whose map holds its score (the raw heat value) there
            p = int(np.argmin(np.abs(up[yg, xg, :18] - cand[i, 2])))
            if abs(up[yg, xg, p] - cand[i, 2]) > 1e-4 or abs(up[yr, xr, p] - ref_c[j, 2]) > 1e-4:
                continue
            if abs(blur[p][yg, xg] - blur[p][yr, xr]) <= tol * blur[p].max():
                hit = i
                break
        if hit is None:
            return None
        pairs[hit] = j
    return pairs
