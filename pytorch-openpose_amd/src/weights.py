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


def c5_out_scale(heat_shift: float = -3.5, paf_offset: float = 0.8, heat_gain: float = 1.0) -> dict:
    """BENCH_OUT_SCALE re-aimed at C5 (1080p, scale_search [0.5, 1, 1.5, 2]): the 368x656 heat
    calibration carpets some channels of the averaged 1080p maps with plateau peaks, so the heat
    pre-activations z become heat_gain * z + heat_shift (scripts/calib_c5.py picks them on the
    GPU)."""
    w, b = BENCH_OUT_SCALE["Mconv7_stage6_L2"]
    return {"Mconv7_stage6_L2": ([v * heat_gain for v in w], [v * heat_gain + heat_shift for v in b]),
            "Mconv7_stage6_L1": (1.0, paf_offset)}


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
