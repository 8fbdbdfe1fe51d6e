"""ORACLE (test infrastructure only): NumPy/SciPy restatement of `Hand.__call__`.

Follows `src/hand.py:25-75` of hitmaxiang/pytorch-openpose:
* 4 scales, multiplier = s*368/h                 src/hand.py:26-32
* resize / pad / normalise (as Body)             src/hand.py:38-41
* x8 upsample, crop, resize, average (22 ch)     src/hand.py:51-57
* per part: Gaussian sigma=3, > thre,            src/hand.py:60-67
  8-connected labelling (skimage.measure.label,  src/hand.py:68
  connectivity=2 -> scipy.ndimage.label with a 3x3 structure: same labels and
  numbering), keep the component with the largest raw-heat sum, zero the rest,
  first row-major argmax (util.npmax)            src/hand.py:69-74, src/util.py:205-210
* return np.array(all_peaks): float64, or int64 when every part is missing.
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import gaussian_filter, label as nd_label

from .body_post import preprocess, upsample_map

EIGHT = np.ones((3, 3), dtype=int)


def label8(binary: np.ndarray):
    """skimage.measure.label(binary, return_num=True, connectivity=2) equivalent."""
    lab, n = nd_label(binary, structure=EIGHT)
    return lab, n


def npmax(a: np.ndarray):
    """util.npmax (src/util.py:205-210): first max in row-major order -> (row, col)."""
    cols = a.argmax(1)
    vals = a.max(1)
    i = vals.argmax()
    return i, cols[i]


def peaks_from_avg(heat_avg: np.ndarray, thre=0.03):
    """src/hand.py:59-75 on the averaged [h, w, 22] float64 map."""
    out = []
    for part in range(21):
        ori = heat_avg[:, :, part]
        g = gaussian_filter(ori, sigma=3)
        binary = np.ascontiguousarray(g > thre, dtype=np.uint8)
        if np.sum(binary) == 0:
            out.append([0, 0, 0])
            continue
        lab, n = label8(binary)
        sums = [np.sum(ori[lab == i]) for i in range(1, n + 1)]
        best = int(np.argmax(sums)) + 1
        lab[lab != best] = 0
        ori[lab == 0] = 0
        y, x = npmax(ori)
        out.append([x, y, np.max(ori)])
    return np.array(out)


def post_from_lowres(img_hw, lowres, thre=0.03, stride=8):
    """lowres: list of (heat[22,h,w] f32, pad, padded_hw) per scale."""
    h, w = img_hw
    avg = np.zeros((h, w, 22))
    n = len(lowres)
    for heat, pad, padded_hw in lowres:
        avg += upsample_map(heat, pad, padded_hw, (h, w), stride) / n
    return peaks_from_avg(avg, thre)


def hand_infer(ori: np.ndarray, net_fn, scale_search=(0.5, 1.0, 1.5, 2.0), boxsize=368,
               stride=8, pad_value=128, thre=0.03):
    """Hand.__call__ (src/hand.py:25-75); net_fn(x NCHW f32) -> heat numpy [1,22,h,w]."""
    lowres = []
    for s in scale_search:
        scale = s * boxsize / ori.shape[0]
        x, pad, padded_hw = preprocess(ori, scale, stride, pad_value)
        lowres.append((np.asarray(net_fn(x))[0], pad, padded_hw))
    return post_from_lowres(ori.shape[:2], lowres, thre, stride)
