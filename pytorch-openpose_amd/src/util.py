"""Helpers with the reference's names and behaviour (hitmaxiang/pytorch-openpose src/util.py).

* padRightDownCorner  src/util.py:12-32   (host reference of what the preprocess kernel does)
* transfer            src/util.py:36-40   (Caffe key names -> module key names)
* handDetect          src/util.py:133-201 (hand boxes from body keypoints)
* npmax               src/util.py:205-210 (first row-major argmax)
Drawing helpers (draw_bodypose / draw_handpose) are rendering only and out of scope.
"""
from __future__ import annotations

import math

import numpy as np


def padRightDownCorner(img, stride, padValue):
    """Pad bottom/right to a multiple of `stride` with `padValue`; returns (img, pad[4])."""
    h, w = img.shape[0], img.shape[1]
    pad = [0, 0, 0 if h % stride == 0 else stride - h % stride, 0 if w % stride == 0 else stride - w % stride]
    out = np.empty((h + pad[2], w + pad[3]) + img.shape[2:], dtype=img.dtype)
    out[...] = padValue
    out[:h, :w] = img
    return out, pad


def transfer(model, model_weights):
    """Map the .pth file's keys ('conv1_1.weight') onto the model's ('model0.conv1_1.weight')."""
    return {k: model_weights[".".join(k.split(".")[1:])] for k in model.state_dict().keys()}


def handDetect(candidate, subset, oriImg):
    """Hand boxes [x, y, w, is_left] (ints) from shoulder/elbow/wrist (src/util.py:133-201)."""
    ratio = 0.33
    out = []
    img_h, img_w = oriImg.shape[0:2]
    for person in subset.astype(int):
        arms = []
        if np.sum(person[[5, 6, 7]] == -1) == 0:
            arms.append(([int(i) for i in person[[5, 6, 7]]], True))
        if np.sum(person[[2, 3, 4]] == -1) == 0:
            arms.append(([int(i) for i in person[[2, 3, 4]]], False))
        for (sh, el, wr), is_left in arms:
            x1, y1 = candidate[sh][:2]
            x2, y2 = candidate[el][:2]
            x3, y3 = candidate[wr][:2]
            x = x3 + ratio * (x3 - x2)
            y = y3 + ratio * (y3 - y2)
            d_we = math.sqrt((x3 - x2) ** 2 + (y3 - y2) ** 2)
            d_es = math.sqrt((x2 - x1) ** 2 + (y2 - y1) ** 2)
            width = 1.5 * max(d_we, 0.9 * d_es)
            x -= width / 2
            y -= width / 2
            x = 0 if x < 0 else x
            y = 0 if y < 0 else y
            w1 = img_w - x if x + width > img_w else width
            w2 = img_h - y if y + width > img_h else width
            out.append([int(x), int(y), int(min(w1, w2)), is_left])
    return out


def npmax(array):
    """(row, col) of the first maximum in row-major order."""
    cols = array.argmax(1)
    vals = array.max(1)
    i = vals.argmax()
    return i, cols[i]
