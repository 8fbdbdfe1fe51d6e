"""Network modules with the reference's interface (hitmaxiang/pytorch-openpose src/model.py).

`bodypose_model` / `handpose_model` keep the reference's module names (so `state_dict()`
keys such as 'model0.conv1_1.weight' and `util.transfer` work unchanged), but hold their
weights on the GPU inside libopose and run `forward` as hand-written HIP kernels
(implicit-GEMM convolutions on the gfx950 fp32 matrix cores; see csrc/conv.hip).

Topology (restated from src/model.py:25-104 and :136-195):
* body: VGG-19 conv1_1..conv4_2 + conv4_3_CPM + conv4_4_CPM, stage 1 (two branches:
  3x conv3x3 128, conv1x1 512, conv1x1 38|19), stages 2-6 (two branches: 5x conv7x7 128,
  conv1x1 128, conv1x1 38|19).  ReLU after every conv except the branch outputs - but the
  reference's no-ReLU list names 'Mconv7_stage6_L1' twice and omits 'Mconv7_stage6_L2'
  (src/model.py:30-33), so the final heat-map conv IS followed by a ReLU.  Reproduced.
* hand: VGG-19 conv1_1..conv5_2 + conv5_3_CPM, stage 1 (conv1x1 512, conv1x1 22), stages
  2-6 (5x conv7x7 128, conv1x1 128, conv1x1 22); no ReLU on stage outputs.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from . import _native

_VGG_BODY = [("conv1_1", 3, 64, 3, 1), ("conv1_2", 64, 64, 3, 1), ("conv2_1", 64, 128, 3, 1),
             ("conv2_2", 128, 128, 3, 1), ("conv3_1", 128, 256, 3, 1), ("conv3_2", 256, 256, 3, 1),
             ("conv3_3", 256, 256, 3, 1), ("conv3_4", 256, 256, 3, 1), ("conv4_1", 256, 512, 3, 1),
             ("conv4_2", 512, 512, 3, 1), ("conv4_3_CPM", 512, 256, 3, 1), ("conv4_4_CPM", 256, 128, 3, 1)]
_VGG_HAND = _VGG_BODY[:10] + [("conv4_3", 512, 512, 3, 1), ("conv4_4", 512, 512, 3, 1),
                              ("conv5_1", 512, 512, 3, 1), ("conv5_2", 512, 512, 3, 1),
                              ("conv5_3_CPM", 512, 128, 3, 1)]


def _body_block(stage, branch):
    out = 38 if branch == 1 else 19
    if stage == 1:
        return [(f"conv5_{i}_CPM_L{branch}", 128, 128, 3, 1) for i in (1, 2, 3)] + [
            (f"conv5_4_CPM_L{branch}", 128, 512, 1, 0), (f"conv5_5_CPM_L{branch}", 512, out, 1, 0)]
    sfx = f"stage{stage}_L{branch}"
    return ([(f"Mconv1_{sfx}", 185, 128, 7, 3)] + [(f"Mconv{i}_{sfx}", 128, 128, 7, 3) for i in range(2, 6)]
            + [(f"Mconv6_{sfx}", 128, 128, 1, 0), (f"Mconv7_{sfx}", 128, out, 1, 0)])


def _hand_block(stage):
    if stage == 1:
        return [("conv6_1_CPM", 128, 512, 1, 0), ("conv6_2_CPM", 512, 22, 1, 0)]
    sfx = f"stage{stage}"
    return ([(f"Mconv1_{sfx}", 150, 128, 7, 3)] + [(f"Mconv{i}_{sfx}", 128, 128, 7, 3) for i in range(2, 6)]
            + [(f"Mconv6_{sfx}", 128, 128, 1, 0), (f"Mconv7_{sfx}", 128, 22, 1, 0)])


def module_layout(net: str):
    """[(module_name, [conv specs])] in the reference's registration (= state_dict) order."""
    if net == "body":
        return ([("model0", _VGG_BODY)] + [(f"model{s}_1", _body_block(s, 1)) for s in range(1, 7)]
                + [(f"model{s}_2", _body_block(s, 2)) for s in range(1, 7)])
    if net == "hand":
        return ([("model1_0", _VGG_HAND), ("model1_1", _hand_block(1))]
                + [(f"model{s}", _hand_block(s)) for s in range(2, 7)])
    raise ValueError(net)


def conv_specs(net: str):
    return [spec for _, specs in module_layout(net) for spec in specs]


class _DeviceNet:
    """Weights resident in libopose; forward runs the HIP network."""

    NET = "body"

    def __init__(self, device: int = 0, handle: "_native.Handle | None" = None):
        self.handle = handle or _native.Handle(device)
        self._state = OrderedDict()
        for mod, specs in module_layout(self.NET):
            for name, cin, cout, k, _ in specs:
                self._state[f"{mod}.{name}.weight"] = np.zeros((cout, cin, k, k), np.float32)
                self._state[f"{mod}.{name}.bias"] = np.zeros((cout,), np.float32)
        self._loaded = False

    # --- nn.Module-like surface used by the reference's callers (src/body.py:17-22)
    def state_dict(self):
        return self._state

    def load_state_dict(self, sd, strict: bool = True):
        missing = [k for k in self._state if k not in sd]
        if strict and (missing or len(sd) != len(self._state)):
            raise KeyError(f"state_dict mismatch: missing {missing[:4]}...")
        tensors = []
        for k, ref in self._state.items():
            v = sd[k]
            v = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
            if tuple(v.shape) != ref.shape:
                raise ValueError(f"{k}: expected {ref.shape}, got {tuple(v.shape)}")
            tensors.append(np.ascontiguousarray(v, dtype=np.float32))
        self.handle.load_weights(_native.NET_BODY if self.NET == "body" else _native.NET_HAND, tensors)
        self._loaded = True
        return self

    def eval(self):
        return self

    def cuda(self, device=None):
        return self

    def __call__(self, x):
        return self.forward(x)


class bodypose_model(_DeviceNet):
    """forward(x[N,3,H,W] fp32) -> (paf[N,38,H/8,W/8], heat[N,19,H/8,W/8]) (src/model.py:106-133)."""

    NET = "body"

    def forward(self, x):
        N, c, H, W = x.shape
        if c != 3 or H % 8 or W % 8:
            raise ValueError("input must be [N,3,H,W] with H, W multiples of 8")
        if hasattr(x, "is_cuda") and x.is_cuda:
            import torch
            xt = x.contiguous().float()
            paf = torch.empty((N, 38, H // 8, W // 8), device=x.device)
            heat = torch.empty((N, 19, H // 8, W // 8), device=x.device)
            self.handle.wait_torch()  # xt may still be in flight on torch's stream
            self.handle.check(_native.lib.opose_body_forward(self.handle.h, xt.data_ptr(), N, H, W, paf.data_ptr(),
                                                             heat.data_ptr(), _native.IN_DEVICE | _native.OUT_DEVICE))
            self.handle.signal_torch()  # outputs ready (and xt free to reuse) in torch's stream order
            return paf, heat
        xn = np.ascontiguousarray(x.numpy() if hasattr(x, "numpy") else x, dtype=np.float32)
        paf = np.empty((N, 38, H // 8, W // 8), np.float32)
        heat = np.empty((N, 19, H // 8, W // 8), np.float32)
        self.handle.check(_native.lib.opose_body_forward(self.handle.h, xn.ctypes.data, N, H, W, paf.ctypes.data,
                                                         heat.ctypes.data, 0))
        return paf, heat


class handpose_model(_DeviceNet):
    """forward(x[N,3,H,W] fp32) -> heat[N,22,H/8,W/8] (src/model.py:197-214)."""

    NET = "hand"

    def forward(self, x):
        N, c, H, W = x.shape
        if c != 3 or H % 8 or W % 8:
            raise ValueError("input must be [N,3,H,W] with H, W multiples of 8")
        if hasattr(x, "is_cuda") and x.is_cuda:
            import torch
            xt = x.contiguous().float()
            heat = torch.empty((N, 22, H // 8, W // 8), device=x.device)
            self.handle.wait_torch()
            self.handle.check(_native.lib.opose_hand_forward(self.handle.h, xt.data_ptr(), N, H, W, heat.data_ptr(),
                                                             _native.IN_DEVICE | _native.OUT_DEVICE))
            self.handle.signal_torch()
            return heat
        xn = np.ascontiguousarray(x.numpy() if hasattr(x, "numpy") else x, dtype=np.float32)
        heat = np.empty((N, 22, H // 8, W // 8), np.float32)
        self.handle.check(_native.lib.opose_hand_forward(self.handle.h, xn.ctypes.data, N, H, W, heat.ctypes.data, 0))
        return heat

    def forward_pyramid(self, xs):
        """The networks of a scale pyramid in one lockstep pass (what Hand() runs for its
        scale_search): xs = list of [N,3,H,W] fp32 host arrays -> list of heat [N,22,H/8,W/8]
        (opose_hand_forward_pyramid; one conv launch per layer covers every scale)."""
        import ctypes as C
        xn = [np.ascontiguousarray(x, dtype=np.float32) for x in xs]
        for x in xn:
            if x.ndim != 4 or x.shape[1] != 3 or x.shape[2] % 8 or x.shape[3] % 8:
                raise ValueError("inputs must be [N,3,H,W] with H, W multiples of 8")
        heats = [np.empty((x.shape[0], 22, x.shape[2] // 8, x.shape[3] // 8), np.float32) for x in xn]
        n = len(xn)
        P = C.c_void_p * n
        Iv = C.c_int * n
        self.handle.check(_native.lib.opose_hand_forward_pyramid(
            self.handle.h, n, P(*[x.ctypes.data for x in xn]), Iv(*[x.shape[0] for x in xn]),
            Iv(*[x.shape[2] for x in xn]), Iv(*[x.shape[3] for x in xn]), P(*[o.ctypes.data for o in heats]), 0))
        return heats
