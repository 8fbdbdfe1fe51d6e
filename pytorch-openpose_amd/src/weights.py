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

# Bench calibration: a negative bias on the final heat-map conv so that the random-weight
# network yields a sparse, person-like number of peaks (tens per part) instead of a dense
# carpet.  Timing of the convolutions is value independent.
BENCH_OUT_SCALE = {"Mconv7_stage6_L2": (1.0, 0.0)}


def seeded_state_dict(net: str = "body", seed: int = 0, out_scale: dict | None = None, as_torch: bool = False):
    rng = np.random.default_rng(seed)
    sd = OrderedDict()
    for name, cin, cout, k, _ in conv_specs(net):
        fan_in = cin * k * k
        w = rng.standard_normal((cout, cin, k, k), dtype=np.float32) * np.float32(np.sqrt(2.0 / fan_in))
        b = rng.standard_normal((cout,), dtype=np.float32) * np.float32(0.01)
        if out_scale and name in out_scale:
            wm, ba = out_scale[name]
            w = w * np.float32(wm)
            b = b + np.float32(ba)
        sd[name + ".weight"] = np.ascontiguousarray(w)
        sd[name + ".bias"] = np.ascontiguousarray(b)
    if as_torch:
        import torch
        sd = OrderedDict((k, torch.from_numpy(v)) for k, v in sd.items())
    return sd
