"""ORACLE (test infrastructure only): NumPy/SciPy restatement of `Body.__call__`.

Follows `src/body.py` of hitmaxiang/pytorch-openpose step by step:

* constants                         src/body.py:25-32
* resize / pad / normalise          src/body.py:36-41, src/util.py:12-32
* network call boundary             src/body.py:43-50
* x8 upsample, crop, resize, avg    src/body.py:52-68   (float32 maps, float64 sums)
* Gaussian(sigma=3) + 4-nbr NMS     src/body.py:70-94   (scipy.ndimage.gaussian_filter)
* PAF line integral, 19 limbs       src/body.py:96-141
* stable sort + greedy matching     src/body.py:143-155
* person assembly                   src/body.py:157-202 (incl. merge '+1' quirk :186 and
                                                        the IndexError when a 3rd row matches)
* prune + return                    src/body.py:203-212

The PAF scoring is vectorised over (i, j) pairs but performs the very same
float64 operations in the same order as the reference's Python loop (checked
bit-exactly against the imported reference by tests/test_oracle_golden.py).
"""
from __future__ import annotations


import numpy as np
from scipy.ndimage import gaussian_filter

from .cv_resize import resize_cubic

# src/body.py:97-103 (1-based part pairs; PAF channel pairs offset by 19)
LIMB_SEQ = [[2, 3], [2, 6], [3, 4], [4, 5], [6, 7], [7, 8], [2, 9], [9, 10],
            [10, 11], [2, 12], [12, 13], [13, 14], [2, 1], [1, 15], [15, 17],
            [1, 16], [16, 18], [3, 17], [6, 18]]
MAP_IDX = [[31, 32], [39, 40], [33, 34], [35, 36], [41, 42], [43, 44], [19, 20], [21, 22],
           [23, 24], [25, 26], [27, 28], [29, 30], [47, 48], [49, 50], [53, 54], [51, 52],
           [55, 56], [37, 38], [45, 46]]
MID_NUM = 10


def pad_right_down(img: np.ndarray, stride: int, pad_value: int):
    """util.padRightDownCorner (src/util.py:12-32): pad bottom/right to a stride multiple."""
    h, w = img.shape[:2]
    pd = 0 if h % stride == 0 else stride - h % stride
    pr = 0 if w % stride == 0 else stride - w % stride
    out = np.full((h + pd, w + pr) + img.shape[2:], pad_value, dtype=img.dtype)
    out[:h, :w] = img
    return out, [0, 0, pd, pr]


def preprocess(ori: np.ndarray, scale: float, stride=8, pad_value=128):
    """src/body.py:38-41 -> (NCHW float32 input, pad, padded (h, w))."""
    img = resize_cubic(ori, (0, 0), fx=scale, fy=scale)
    padded, pad = pad_right_down(img, stride, pad_value)
    x = np.transpose(np.float32(padded[:, :, :, None]), (3, 2, 0, 1)) / 256 - 0.5
    return np.ascontiguousarray(x), pad, padded.shape[:2]


def upsample_map(lowres_chw: np.ndarray, pad, padded_hw, out_hw, stride=8):
    """src/body.py:54-57: x8 cubic, crop the padding, cubic resize to (H, W); float32."""
    m = np.transpose(lowres_chw, (1, 2, 0))
    m = resize_cubic(np.ascontiguousarray(m), (0, 0), fx=stride, fy=stride)
    m = m[:padded_hw[0] - pad[2], :padded_hw[1] - pad[3], :]
    return resize_cubic(np.ascontiguousarray(m), (out_hw[1], out_hw[0]))


def find_peaks(heat_avg: np.ndarray, thre1: float):
    """src/body.py:70-94 -> list (per part) of (x, y, score, id) tuples."""
    all_peaks, counter = [], 0
    for part in range(18):
        ori = heat_avg[:, :, part]
        g = gaussian_filter(ori, sigma=3)
        nb = np.zeros((4,) + g.shape)
        nb[0, 1:, :] = g[:-1, :]
        nb[1, :-1, :] = g[1:, :]
        nb[2, :, 1:] = g[:, :-1]
        nb[3, :, :-1] = g[:, 1:]
        mask = (g >= nb[0]) & (g >= nb[1]) & (g >= nb[2]) & (g >= nb[3]) & (g > thre1)
        ys, xs = np.nonzero(mask)
        peaks = [(xs[i], ys[i], ori[ys[i], xs[i]], counter + i) for i in range(len(ys))]
        all_peaks.append(peaks)
        counter += len(ys)
    return all_peaks


def limb_scores(cand_a, cand_b, paf_x: np.ndarray, paf_y: np.ndarray, img_h: int, thre2: float):
    """PAF line integral for every (i, j) pair (src/body.py:118-141).

    Returns (score[nA, nB] float64, accept[nA, nB] bool)."""
    xa = np.array([c[0] for c in cand_a], np.int64)[:, None]
    ya = np.array([c[1] for c in cand_a], np.int64)[:, None]
    xb = np.array([c[0] for c in cand_b], np.int64)[None, :]
    yb = np.array([c[1] for c in cand_b], np.int64)[None, :]
    vx, vy = xb - xa, yb - ya
    norm = np.sqrt((vx * vx + vy * vy).astype(np.float64)) + 1e-10
    ux, uy = vx / norm, vy / norm
    t = np.arange(MID_NUM, dtype=np.float64)

    def lin(a, b):
        a = np.broadcast_to(a, vx.shape).astype(np.float64)
        b = np.broadcast_to(b, vx.shape).astype(np.float64)
        step = (b - a) / (MID_NUM - 1)
        pts = t[None, None, :] * step[..., None] + a[..., None]
        pts[..., -1] = b
        return np.rint(pts).astype(np.int64)

    sx, sy = lin(xa, xb), lin(ya, yb)
    s = paf_x[sy, sx] * ux[..., None] + paf_y[sy, sx] * uy[..., None]
    acc = 0.0 + s[..., 0]
    for k in range(1, MID_NUM):
        acc = acc + s[..., k]
    prior = 0.5 * img_h / norm - 1
    score = acc / MID_NUM + np.where(prior > 0, 0.0, prior)
    accept = ((s > thre2).sum(-1) > 0.8 * MID_NUM) & (score > 0)
    return score, accept


def connect_limbs(all_peaks, paf_avg: np.ndarray, img_h: int, thre2: float):
    """src/body.py:105-155 -> (connection_all, special_k)."""
    connection_all, special_k = [], []
    for k, (pa, pb) in enumerate(LIMB_SEQ):
        cand_a, cand_b = all_peaks[pa - 1], all_peaks[pb - 1]
        n_a, n_b = len(cand_a), len(cand_b)
        if n_a == 0 or n_b == 0:
            special_k.append(k)
            connection_all.append([])
            continue
        ch = [c - 19 for c in MAP_IDX[k]]
        score, accept = limb_scores(cand_a, cand_b, paf_avg[:, :, ch[0]], paf_avg[:, :, ch[1]], img_h, thre2)
        ii, jj = np.nonzero(accept)              # row-major == the reference's i-then-j order
        sc = score[ii, jj]
        order = np.argsort(-sc, kind="stable")   # sorted(..., reverse=True) is stable
        used_a, used_b, rows = set(), set(), []
        for o in order:
            i, j = int(ii[o]), int(jj[o])
            if i in used_a or j in used_b:
                continue
            rows.append([cand_a[i][3], cand_b[j][3], sc[o], i, j])
            used_a.add(i)
            used_b.add(j)
            if len(rows) >= min(n_a, n_b):
                break
        connection_all.append(np.array(rows, dtype=np.float64).reshape(-1, 5))
    return connection_all, special_k


def assemble(all_peaks, connection_all, special_k):
    """Person assembly + pruning (src/body.py:157-212) -> (candidate, subset)."""
    candidate = np.array([p for part in all_peaks for p in part])
    people = []                                   # list of float64[20] rows
    for k, (pa, pb) in enumerate(LIMB_SEQ):
        if k in special_k:
            continue
        conn = connection_all[k]
        ia, ib = pa - 1, pb - 1
        for c in range(len(conn)):
            id_a, id_b, s = conn[c, 0], conn[c, 1], conn[c, 2]
            hits = [r for r in range(len(people)) if people[r][ia] == id_a or people[r][ib] == id_b]
            if len(hits) > 2:
                # the reference writes subset_idx[2] and raises (src/body.py:170-173)
                raise IndexError("list assignment index out of range")
            if len(hits) == 1:
                row = people[hits[0]]
                if row[ib] != id_b:
                    row[ib] = id_b
                    row[19] += 1
                    row[18] += candidate[int(id_b), 2] + s
            elif len(hits) == 2:
                r1, r2 = people[hits[0]], people[hits[1]]
                both = ((r1[:18] >= 0).astype(int) + (r2[:18] >= 0).astype(int)) == 2
                if not both.any():
                    r1[:18] += r2[:18] + 1
                    r1[18:] += r2[18:]
                    r1[18] += s
                    del people[hits[1]]
                else:
                    r1[ib] = id_b
                    r1[19] += 1
                    r1[18] += candidate[int(id_b), 2] + s
            elif k < 17:
                row = -1 * np.ones(20)
                row[ia], row[ib] = id_a, id_b
                row[19] = 2
                row[18] = sum(candidate[conn[c, :2].astype(int), 2]) + s
                people.append(row)
    keep = [r for r in people if not (r[19] < 4 or r[18] / r[19] < 0.4)]
    subset = np.array(keep, dtype=np.float64).reshape(-1, 20) if keep else -1 * np.ones((0, 20))
    return candidate, subset


def post_from_lowres(img_hw, lowres, thre1=0.1, thre2=0.05, stride=8):
    """Everything after the network (src/body.py:52-212).

    lowres: list (one per scale) of (paf[38,h,w] f32, heat[19,h,w] f32, pad, padded_hw)."""
    h, w = img_hw
    heat_avg = np.zeros((h, w, 19))
    paf_avg = np.zeros((h, w, 38))
    n = len(lowres)
    for paf, heat, pad, padded_hw in lowres:
        heat_avg += upsample_map(heat, pad, padded_hw, (h, w), stride) / n
        paf_avg += upsample_map(paf, pad, padded_hw, (h, w), stride) / n
    peaks = find_peaks(heat_avg, thre1)
    conns, special = connect_limbs(peaks, paf_avg, h, thre2)
    return assemble(peaks, conns, special)


def body_infer(ori: np.ndarray, net_fn, scale_search=(0.5,), boxsize=368, stride=8,
               pad_value=128, thre1=0.1, thre2=0.05):
    """Body.__call__ (src/body.py:24-212); net_fn(x NCHW f32) -> (paf, heat) numpy [1,C,h,w]."""
    lowres = []
    for s in scale_search:
        scale = s * boxsize / ori.shape[0]
        x, pad, padded_hw = preprocess(ori, scale, stride, pad_value)
        paf, heat = net_fn(x)
        lowres.append((np.asarray(paf)[0], np.asarray(heat)[0], pad, padded_hw))
    return post_from_lowres(ori.shape[:2], lowres, thre1, thre2, stride)
