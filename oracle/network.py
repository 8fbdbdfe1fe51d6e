"""ORACLE (test infrastructure only): torch-CPU restatement of `src/model.py`.

Topology restated from the reference:
* `make_layers`            src/model.py:7-22   (conv stride 1, ReLU unless listed)
* `bodypose_model`         src/model.py:25-104 (VGG-19 trunk, stage 1, stages 2-6)
  - no-ReLU list quirk     src/model.py:30-33  ('Mconv7_stage6_L1' listed twice,
                                               'Mconv7_stage6_L2' missing => the final
                                               heatmap conv IS followed by ReLU)
* `bodypose_model.forward` src/model.py:106-133
* `handpose_model`         src/model.py:136-214

State-dict keys follow the reference's *file* naming (`conv1_1.weight`, ...), i.e.
the keys of `body_pose_model.pth` before `util.transfer` (src/util.py:36-40).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

# (name, cin, cout, ksize, pad) ; a ('pool', ...) entry is MaxPool2d(2, 2)
_VGG_BODY = [
    ("conv1_1", 3, 64, 3, 1), ("conv1_2", 64, 64, 3, 1), ("pool1_stage1",),
    ("conv2_1", 64, 128, 3, 1), ("conv2_2", 128, 128, 3, 1), ("pool2_stage1",),
    ("conv3_1", 128, 256, 3, 1), ("conv3_2", 256, 256, 3, 1), ("conv3_3", 256, 256, 3, 1),
    ("conv3_4", 256, 256, 3, 1), ("pool3_stage1",),
    ("conv4_1", 256, 512, 3, 1), ("conv4_2", 512, 512, 3, 1),
    ("conv4_3_CPM", 512, 256, 3, 1), ("conv4_4_CPM", 256, 128, 3, 1),
]

_VGG_HAND = [
    ("conv1_1", 3, 64, 3, 1), ("conv1_2", 64, 64, 3, 1), ("pool1_stage1",),
    ("conv2_1", 64, 128, 3, 1), ("conv2_2", 128, 128, 3, 1), ("pool2_stage1",),
    ("conv3_1", 128, 256, 3, 1), ("conv3_2", 256, 256, 3, 1), ("conv3_3", 256, 256, 3, 1),
    ("conv3_4", 256, 256, 3, 1), ("pool3_stage1",),
    ("conv4_1", 256, 512, 3, 1), ("conv4_2", 512, 512, 3, 1), ("conv4_3", 512, 512, 3, 1),
    ("conv4_4", 512, 512, 3, 1), ("conv5_1", 512, 512, 3, 1), ("conv5_2", 512, 512, 3, 1),
    ("conv5_3_CPM", 512, 128, 3, 1),
]

BODY_NO_RELU = {"conv5_5_CPM_L1", "conv5_5_CPM_L2"} | {
    f"Mconv7_stage{s}_L{b}" for s in range(2, 6) for b in (1, 2)} | {"Mconv7_stage6_L1"}
HAND_NO_RELU = {"conv6_2_CPM"} | {f"Mconv7_stage{s}" for s in range(2, 7)}


def body_branch(stage: int, branch: int):
    out = 38 if branch == 1 else 19
    if stage == 1:
        return [(f"conv5_1_CPM_L{branch}", 128, 128, 3, 1), (f"conv5_2_CPM_L{branch}", 128, 128, 3, 1),
                (f"conv5_3_CPM_L{branch}", 128, 128, 3, 1), (f"conv5_4_CPM_L{branch}", 128, 512, 1, 0),
                (f"conv5_5_CPM_L{branch}", 512, out, 1, 0)]
    sfx = f"stage{stage}_L{branch}"
    return ([(f"Mconv1_{sfx}", 185, 128, 7, 3)] +
            [(f"Mconv{i}_{sfx}", 128, 128, 7, 3) for i in range(2, 6)] +
            [(f"Mconv6_{sfx}", 128, 128, 1, 0), (f"Mconv7_{sfx}", 128, out, 1, 0)])


def hand_stage(stage: int):
    if stage == 1:
        return [("conv6_1_CPM", 128, 512, 1, 0), ("conv6_2_CPM", 512, 22, 1, 0)]
    sfx = f"stage{stage}"
    return ([(f"Mconv1_{sfx}", 150, 128, 7, 3)] +
            [(f"Mconv{i}_{sfx}", 128, 128, 7, 3) for i in range(2, 6)] +
            [(f"Mconv6_{sfx}", 128, 128, 1, 0), (f"Mconv7_{sfx}", 128, 22, 1, 0)])


def conv_specs(net: str):
    """All conv layers of `net` ('body'|'hand') in reference state_dict order."""
    if net == "body":
        seq = list(_VGG_BODY)
        for s in range(1, 7):
            seq += body_branch(s, 1)
        for s in range(1, 7):
            seq += body_branch(s, 2)
        # reference module order: model0, model1_1, model2_1..model6_1, model1_2, ...
        # (src/model.py:92-104 assigns _1 blocks first) -> matches the loop above.
    elif net == "hand":
        seq = list(_VGG_HAND)
        for s in range(1, 7):
            seq += hand_stage(s)
    else:
        raise ValueError(net)
    return [e for e in seq if len(e) == 5]


def seeded_state_dict(net: str, seed: int = 0, out_scale: dict | None = None):
    """Deterministic synthetic weights (real .pth files are not available offline).

    Weight ~ N(0, 2/fan_in) via numpy default_rng(seed); bias = 0.01*N(0,1).
    `out_scale` optionally overrides {layer_name: (weight_mul, bias_add)}.
    Identical to `src/weights.py` in the product package (checked by a test).
    """
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
        sd[name + ".weight"] = torch.from_numpy(np.ascontiguousarray(w))
        sd[name + ".bias"] = torch.from_numpy(np.ascontiguousarray(b))
    return sd


def _run(seq, x, sd, no_relu):
    for e in seq:
        if len(e) == 1:
            x = F.max_pool2d(x, 2, 2)
            continue
        name, _, _, _, pad = e
        x = F.conv2d(x, sd[name + ".weight"], sd[name + ".bias"], stride=1, padding=pad)
        if name not in no_relu:
            x = F.relu(x)
    return x


@torch.no_grad()
def body_forward(x: torch.Tensor, sd) -> tuple:
    """bodypose_model.forward (src/model.py:106-133): returns (paf[N,38], heat[N,19])."""
    trunk = _run(_VGG_BODY, x, sd, BODY_NO_RELU)
    l1 = _run(body_branch(1, 1), trunk, sd, BODY_NO_RELU)
    l2 = _run(body_branch(1, 2), trunk, sd, BODY_NO_RELU)
    for s in range(2, 7):
        cat = torch.cat([l1, l2, trunk], 1)
        l1 = _run(body_branch(s, 1), cat, sd, BODY_NO_RELU)
        l2 = _run(body_branch(s, 2), cat, sd, BODY_NO_RELU)
    return l1, l2


@torch.no_grad()
def hand_forward(x: torch.Tensor, sd) -> torch.Tensor:
    """handpose_model.forward (src/model.py:197-214): returns heat[N,22]."""
    trunk = _run(_VGG_HAND, x, sd, HAND_NO_RELU)
    out = _run(hand_stage(1), trunk, sd, HAND_NO_RELU)
    for s in range(2, 7):
        out = _run(hand_stage(s), torch.cat([out, trunk], 1), sd, HAND_NO_RELU)
    return out


def body_flops(h: int, w: int) -> int:
    """Algorithmic FLOPs (2*MAC) of one body forward at input h x w."""
    return _flops(conv_specs("body"), _VGG_BODY, h, w)


def hand_flops(h: int, w: int) -> int:
    return _flops(conv_specs("hand"), _VGG_HAND, h, w)


def _flops(specs, vgg, h, w):
    total = 0
    hh, ww = h, w
    trunk_names = {e[0] for e in vgg if len(e) == 5}
    for e in vgg:
        if len(e) == 1:
            hh, ww = hh // 2, ww // 2
        else:
            total += 2 * e[1] * e[2] * e[3] * e[3] * hh * ww
    for name, cin, cout, k, _ in specs:
        if name not in trunk_names:
            total += 2 * cin * cout * k * k * hh * ww
    return total
