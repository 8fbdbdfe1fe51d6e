"""Helpers with the reference's names and behaviour (hitmaxiang/pytorch-openpose src/util.py).

* padRightDownCorner  src/util.py:12-32   (host reference of what the preprocess kernel does)
* transfer            src/util.py:36-40   (Caffe key names -> module key names)
* handDetect          src/util.py:133-201 (hand boxes from body keypoints)
* npmax               src/util.py:205-210 (first row-major argmax)
* draw_bodypose       src/util.py:44-77   (keypoint discs + translucent limb ellipses)
* draw_handpose       src/util.py:80-113  (matplotlib hand skeleton)
The drawing helpers are host-side rendering of the results, not part of the GPU
path.  OpenCV is absent here, so draw_bodypose rasterises the reference's cv2.circle /
cv2.ellipse2Poly / cv2.fillConvexPoly / cv2.addWeighted calls itself (pixel parity with OpenCV
unpinned); draw_handpose uses matplotlib as the reference does (its FigureCanvas.tostring_rgb
is gone from this image's matplotlib 3.10, so the RGB buffer is read through buffer_rgba).
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


# ---------------------------------------------------------------- drawing (src/util.py:44-128)
_LIMBS = [[2, 3], [2, 6], [3, 4], [4, 5], [6, 7], [7, 8], [2, 9], [9, 10], [10, 11], [2, 12], [12, 13], [13, 14],
          [2, 1], [1, 15], [15, 17], [1, 16], [16, 18], [3, 17], [6, 18]]
_COLORS = [[255, 0, 0], [255, 85, 0], [255, 170, 0], [255, 255, 0], [170, 255, 0], [85, 255, 0], [0, 255, 0],
           [0, 255, 85], [0, 255, 170], [0, 255, 255], [0, 170, 255], [0, 85, 255], [0, 0, 255], [85, 0, 255],
           [170, 0, 255], [255, 0, 255], [255, 0, 170], [255, 0, 85]]
_HAND_EDGES = [[0, 1], [1, 2], [2, 3], [3, 4], [0, 5], [5, 6], [6, 7], [7, 8], [0, 9], [9, 10], [10, 11], [11, 12],
               [0, 13], [13, 14], [14, 15], [15, 16], [0, 17], [17, 18], [18, 19], [19, 20]]


def _fill_disc(canvas, cx, cy, r, color):
    h, w = canvas.shape[:2]
    y0, y1, x0, x1 = max(cy - r, 0), min(cy + r + 1, h), max(cx - r, 0), min(cx + r + 1, w)
    if y0 >= y1 or x0 >= x1:
        return
    yy, xx = np.mgrid[y0:y1, x0:x1]
    m = (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
    canvas[y0:y1, x0:x1][m] = color


def _ellipse_poly(center, axes, angle_deg):
    """cv2.ellipse2Poly(center, axes, angle, 0, 360, delta=1): one vertex per degree, rounded."""
    t = np.deg2rad(np.arange(0, 361))
    a = np.deg2rad(angle_deg)
    x = center[0] + axes[0] * np.cos(t) * np.cos(a) - axes[1] * np.sin(t) * np.sin(a)
    y = center[1] + axes[0] * np.cos(t) * np.sin(a) + axes[1] * np.sin(t) * np.cos(a)
    return np.stack([np.round(x), np.round(y)], 1)


def _fill_convex(canvas, poly, color):
    from matplotlib.path import Path
    h, w = canvas.shape[:2]
    x0, y0 = np.floor(poly.min(0)).astype(int)
    x1, y1 = np.ceil(poly.max(0)).astype(int)
    x0, y0, x1, y1 = max(x0, 0), max(y0, 0), min(x1 + 1, w), min(y1 + 1, h)
    if x0 >= x1 or y0 >= y1:
        return
    yy, xx = np.mgrid[y0:y1, x0:x1]
    pts = np.stack([xx.ravel(), yy.ravel()], 1)
    m = Path(poly).contains_points(pts, radius=0.5).reshape(yy.shape)  # boundary pixels included
    canvas[y0:y1, x0:x1][m] = color


def draw_bodypose(canvas, candidate, subset):
    """Keypoint discs (radius 4) drawn into `canvas` in place, then each of the first 17 limbs as
    a filled ellipse (stick width 4) blended 0.4 canvas / 0.6 limb; returns the final canvas."""
    stickwidth = 4
    for i in range(18):
        for n in range(len(subset)):
            index = int(subset[n][i])
            if index == -1:
                continue
            x, y = candidate[index][0:2]
            _fill_disc(canvas, int(x), int(y), 4, _COLORS[i])
    for i in range(17):
        for n in range(len(subset)):
            index = subset[n][np.array(_LIMBS[i]) - 1]
            if -1 in index:
                continue
            cur = canvas.copy()
            Y = candidate[index.astype(int), 0]
            X = candidate[index.astype(int), 1]
            mX, mY = np.mean(X), np.mean(Y)
            length = ((X[0] - X[1]) ** 2 + (Y[0] - Y[1]) ** 2) ** 0.5
            angle = math.degrees(math.atan2(X[0] - X[1], Y[0] - Y[1]))
            poly = _ellipse_poly((int(mY), int(mX)), (int(length / 2), stickwidth), int(angle))
            _fill_convex(cur, poly, _COLORS[i])
            canvas = np.clip(np.rint(canvas.astype(np.float64) * 0.4 + cur.astype(np.float64) * 0.6), 0,
                             255).astype(np.uint8)
    return canvas


def draw_handpose(canvas, all_hand_peaks, show_number=False):
    """The hand skeletons (20 edges in HSV colours, red keypoints) drawn over `canvas` with
    matplotlib, as the reference does; returns the rendered RGB image."""
    import matplotlib
    import matplotlib.pyplot as plt
    from matplotlib.backends.backend_agg import FigureCanvasAgg
    from matplotlib.figure import Figure
    fig = Figure(figsize=plt.figaspect(canvas))
    fig.subplots_adjust(0, 0, 1, 1)
    fig.subplots_adjust(bottom=0, top=1, left=0, right=1)
    bg = FigureCanvasAgg(fig)
    ax = fig.subplots()
    ax.axis("off")
    ax.imshow(canvas)
    width, height = ax.figure.get_size_inches() * ax.figure.get_dpi()
    for peaks in all_hand_peaks:
        for ie, e in enumerate(_HAND_EDGES):
            if np.sum(np.all(peaks[e], axis=1) == 0) == 0:
                x1, y1 = peaks[e[0]]
                x2, y2 = peaks[e[1]]
                ax.plot([x1, x2], [y1, y2], color=matplotlib.colors.hsv_to_rgb([ie / float(len(_HAND_EDGES)), 1.0, 1.0]))
        for i, keypoint in enumerate(peaks):
            x, y = keypoint
            ax.plot(x, y, "r.")
            if show_number:
                ax.text(x, y, str(i))
    bg.draw()
    rgba = np.asarray(bg.buffer_rgba())
    return np.ascontiguousarray(rgba[..., :3]).reshape(int(height), int(width), 3)
