"""Deterministic synthetic weights.

The real `body_pose_model.pth` / `hand_pose_model.pth` are not available offline
(SURVEY.md §0), so tests and the benchmark use seeded He-normal weights generated from
numpy's default_rng(seed) in reference state_dict order (keys as in the .pth files, i.e.
before util.transfer).  Bit-identical to oracle/network.py:seeded_state_dict.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .model import conv_specs

# Bench calibration of the two output convs (timing of the convolutions is value independent):
# * heat (Mconv7_stage6_L2): per-channel affine map sending each channel's 95th percentile of
#   pre-activations on a uniform-noise 368x656 frame to 0 and its max to 1, so the seeded
#   network yields ~17 peaks per part instead of a dense carpet of ~75;
# * PAF (Mconv7_stage6_L1): +0.8 on every channel so that PAF vectors are coherent enough for
#   limbs to connect (~20 assembled people per frame: a crowded-scene workload).
BENCH_OUT_SCALE = {
    "Mconv7_stage6_L2": (
        [4.278, 4.923, 3.501, 1.921, 3.771, 5.688, 3.714, 3.656, 2.007, 3.603, 2.861, 4.452, 3.519, 4.595,
         6.164, 3.614, 3.665, 2.856, 2.23],
        [-3.625, -2.142, 0.815, -1.009, -0.328, -4.451, -2.318, -0.451, -1.747, -2.233, 0.418, -1.766, 0.657,
         -6.417, -5.763, -0.264, -0.099, -1.635, 1.118]),
    "Mconv7_stage6_L1": (1.0, 0.8),
}


# C5 (1080p, scale_search [0.5, 1, 1.5, 2]): the 368x656 calibration leaves most heat channels of
# the averaged 1080p maps empty, so the heat conv gets its own per-channel affine, measured on
# 1080p frames over the four scales' maps (scripts/calib_c5_stats.py: the 99.7th percentile of
# each channel's pre-activations -> 0, its max -> 1; a one-off round-4 check: ~190 peaks and
# ~10 assembled people per frame).  PAF as BENCH_OUT_SCALE.
C5_OUT_SCALE = {
    "Mconv7_stage6_L2": (
        [6.799, 6.869, 4.388, 1.824, 4.797, 6.222, 4.417, 3.631, 5.173, 2.862, 2.307, 3.628, 5.313, 3.598, 3.523, 6.004, 4.872, 3.888, 2.677],
        [-8.361, -6.269, 0.551, -2.099, -1.307, -7.711, -4.217, -1.382, -7.498, -2.706, 0.151, -2.059, 0.503, -7.834, -4.97, -1.486, -0.688, -4.525, 1.209]),
    "Mconv7_stage6_L1": (1.0, 0.8),
}


def c5_out_scale() -> dict:
    return C5_OUT_SCALE


def seeded_state_dict(net: str = "body", seed: int = 0, out_scale: dict | None = None, as_torch: bool = False):
    rng = np.random.default_rng(seed)
    sd = OrderedDict()
    for name, cin, cout, k, _ in conv_specs(net):
        fan_in = cin * k * k
        w = rng.standard_normal((cout, cin, k, k), dtype=np.float32) * np.float32(np.sqrt(2.0 / fan_in))
        b = rng.standard_normal((cout,), dtype=np.float32) * np.float32(0.01)
        if out_scale and name in out_scale:  # per-output-channel (or scalar) w*wm, b*wm + ba
            wm, ba = (np.asarray(v, np.float32) for v in out_scale[name])
            w = (w * (wm.reshape(-1, 1, 1, 1) if wm.ndim else wm)).astype(np.float32)
            b = (b * wm + ba).astype(np.float32)
        sd[name + ".weight"] = np.ascontiguousarray(w)
        sd[name + ".bias"] = np.ascontiguousarray(b)
    if as_torch:
        import torch
        sd = OrderedDict((k, torch.from_numpy(v)) for k, v in sd.items())
    return sd
