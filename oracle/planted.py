"""ORACLE (test infrastructure only): synthetic 'planted' network outputs.

Real OpenPose weights and test images are unavailable offline, so
post-network parity is pinned on low-resolution PAF/heat maps with planted
people: Gaussian part blobs in the heat channels and unit-vector bands along the
19 limbs in the PAF channels (channel pairs from src/body.py:101-103).
"""
from __future__ import annotations

import numpy as np

from .body_post import LIMB_SEQ, MAP_IDX

# rough COCO-18 skeleton (x, y) in units of person height, origin at the neck
_TEMPLATE = np.array([
    [0.00, -0.18],  # 0 nose
    [0.00, 0.00],   # 1 neck
    [-0.14, 0.00],  # 2 r shoulder
    [-0.18, 0.22],  # 3 r elbow
    [-0.20, 0.42],  # 4 r wrist
    [0.14, 0.00],   # 5 l shoulder
    [0.18, 0.22],   # 6 l elbow
    [0.20, 0.42],   # 7 l wrist
    [-0.09, 0.45],  # 8 r hip
    [-0.10, 0.68],  # 9 r knee
    [-0.10, 0.92],  # 10 r ankle
    [0.09, 0.45],   # 11 l hip
    [0.10, 0.68],   # 12 l knee
    [0.10, 0.92],   # 13 l ankle
    [-0.03, -0.21],  # 14 r eye
    [0.03, -0.21],  # 15 l eye
    [-0.07, -0.19],  # 16 r ear
    [0.07, -0.19],  # 17 l ear
])


def random_people(rng, n, h, w, min_h=0.45, max_h=0.9):
    """n people as [n, 18, 2] low-res coordinates plus a visibility mask."""
    people, vis = [], []
    for _ in range(n):
        ph = rng.uniform(min_h, max_h) * h
        cx = rng.uniform(0.1, 0.9) * w
        cy = rng.uniform(0.2 * ph, max(0.2 * ph + 1.0, h - 0.6 * ph))
        jitter = rng.normal(0, 0.03, size=_TEMPLATE.shape)
        pts = (_TEMPLATE + jitter) * ph + np.array([cx, cy])
        people.append(pts)
        vis.append(rng.random(18) > 0.1)
    return np.array(people).reshape(n, 18, 2), np.array(vis).reshape(n, 18)


def render_body(h, w, people, vis, rng, sigma=0.9, band=0.9, drop_limb_p=0.05,
                noise=0.01, amp=(0.6, 1.0)):
    """Low-res (paf[38,h,w], heat[19,h,w]) float32 for the given people."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    heat = np.zeros((19, h, w))
    paf = np.zeros((38, h, w))
    cnt = np.zeros((38, h, w))
    for p in range(len(people)):
        for part in range(18):
            if not vis[p, part]:
                continue
            x, y = people[p, part]
            a = rng.uniform(*amp)
            heat[part] = np.maximum(heat[part], a * np.exp(-((xx - x) ** 2 + (yy - y) ** 2) / (2 * sigma ** 2)))
        for k, (pa, pb) in enumerate(LIMB_SEQ):
            if not (vis[p, pa - 1] and vis[p, pb - 1]) or rng.random() < drop_limb_p:
                continue
            a, b = people[p, pa - 1], people[p, pb - 1]
            d = b - a
            ln = np.hypot(*d)
            if ln < 1e-6:
                continue
            u = d / ln
            t = ((xx - a[0]) * u[0] + (yy - a[1]) * u[1]) / ln
            px = a[0] + np.clip(t, 0, 1) * d[0]
            py = a[1] + np.clip(t, 0, 1) * d[1]
            m = (np.hypot(xx - px, yy - py) <= band) & (t >= -0.1) & (t <= 1.1)
            cx, cy = MAP_IDX[k][0] - 19, MAP_IDX[k][1] - 19
            paf[cx][m] += u[0]
            paf[cy][m] += u[1]
            cnt[cx][m] += 1
            cnt[cy][m] += 1
    paf = np.where(cnt > 0, paf / np.maximum(cnt, 1), 0.0)
    heat[18] = np.clip(1 - heat[:18].max(0), 0, 1)
    heat[:18] += rng.normal(0, noise, size=heat[:18].shape)
    paf += rng.normal(0, noise, size=paf.shape)
    # the reference's final heat conv is followed by ReLU (src/model.py:30-33)
    heat = np.maximum(heat, 0)
    return paf.astype(np.float32), heat.astype(np.float32)


def render_hand(h, w, pts, vis, rng, sigma=0.8, noise=0.004, extra_blobs=0):
    """Low-res hand heat [22, h, w] float32; pts in normalised [0,1] crop coordinates."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    heat = np.zeros((22, h, w))
    for part in range(21):
        if not vis[part]:
            continue
        x, y = pts[part][0] * w, pts[part][1] * h
        heat[part] += rng.uniform(0.3, 0.9) * np.exp(-((xx - x) ** 2 + (yy - y) ** 2) / (2 * sigma ** 2))
        for _ in range(extra_blobs):
            ex, ey = rng.uniform(0, w), rng.uniform(0, h)
            heat[part] += rng.uniform(0.1, 0.5) * np.exp(-((xx - ex) ** 2 + (yy - ey) ** 2) / (2 * sigma ** 2))
    heat[21] = np.clip(1 - heat[:21].max(0), 0, 1)
    heat += rng.normal(0, noise, size=heat.shape)
    return heat.astype(np.float32)
