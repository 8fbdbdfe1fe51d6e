"""ORACLE (test infrastructure only; never imported by the product path).

Restatement of the reference's batched "fast mode" `Batch_body.__call__`
(hitmaxiang/pytorch-openpose srcmx/Batch_model.py:137-204) with the same torch CPU image ops
it calls:
* frames -> `transforms.ToTensor()` (uint8 BGR / 255, CHW; :242-245 GetVideoDataLoader)
* `F.interpolate(bicubic, scale_factor = 0.5·368/h)` - 0.5, zero pad right/bottom to /8 (:147-150)
* network; heat and PAF: bicubic x8, crop to (int(h·s), int(w·s)), bicubic to (h, w) (:159-168)
* heat: 5x5 Gaussian `GaussianBlurConv` with reflect padding (srcmx/utilmx.py:246-263)
* peaks: `findpeaks_torch` (srcmx/utilmx.py:230-243): > thre1 and >= the 4 neighbours (zero
  outside), torch.nonzero order (frame, part, y, x); score = the BLURRED value (:182-191)
* `FindBody_frame` (:206-300) = src/body.py's limb scoring / greedy matching / assembly,
  reused from oracle.body_post (identical code in the reference).
Pinned by tests/golden/batch_body_*.npz (oracle/gen_golden.py `batch` imports the reference's
Batch_model with shims for its absent imports and runs it on planted maps).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .body_post import assemble, connect_limbs

# srcmx/utilmx.py:251-255
GAUSS5 = [[0.00078633, 0.00655965, 0.01330373, 0.00655965, 0.00078633],
          [0.00655965, 0.05472157, 0.11098164, 0.05472157, 0.00655965],
          [0.01330373, 0.11098164, 0.22508352, 0.11098164, 0.01330373],
          [0.00655965, 0.05472157, 0.11098164, 0.05472157, 0.00655965],
          [0.00078633, 0.00655965, 0.01330373, 0.00655965, 0.00078633]]


def size_pad(g_scale, h, w, boxsize=368, stride=8):
    """Batch_body.calculate_size_pad (srcmx/Batch_model.py:302-307)."""
    scale = boxsize * g_scale / h
    nh, nw = int(h * scale), int(w * scale)
    return scale, nh, nw, (stride - nh % stride) % stride, (stride - nw % stride) % stride


def to_tensor(frames_u8: np.ndarray) -> torch.Tensor:
    """transforms.ToTensor() on each uint8 BGR HWC frame, stacked: [B, 3, h, w] float32."""
    return torch.from_numpy(np.ascontiguousarray(frames_u8.transpose(0, 3, 1, 2))).float().div(255)


def net_input(frames_u8: np.ndarray, g_scale=0.5, boxsize=368, stride=8):
    x = to_tensor(frames_u8)
    _, _, h, w = x.shape
    scale, nh, nw, ph, pw = size_pad(g_scale, h, w, boxsize, stride)
    x = F.interpolate(x, scale_factor=scale, mode="bicubic") - 0.5
    return F.pad(x, [0, pw, 0, ph], mode="constant", value=0), (h, w, nh, nw)


def blur5(heat: torch.Tensor) -> torch.Tensor:
    c = heat.shape[1]
    k = torch.tensor(GAUSS5, dtype=torch.float32)[None, None].expand(c, 1, 5, 5)
    return F.conv2d(F.pad(heat, (2, 2, 2, 2), mode="reflect"), k, groups=c)


def find_peaks(data: torch.Tensor, thre: float) -> torch.Tensor:
    b = data > thre
    b &= data >= F.pad(data, (1, 0))[:, :, :, :-1]
    b &= data >= F.pad(data, (0, 1))[:, :, :, 1:]
    b &= data >= F.pad(data, (0, 0, 1, 0))[:, :, :-1, :]
    b &= data >= F.pad(data, (0, 0, 0, 1))[:, :, 1:, :]
    return torch.nonzero(b, as_tuple=False)


def post(paf_low: torch.Tensor, heat_low: torch.Tensor, geo, thre1=0.1, thre2=0.05, stride=8):
    """Everything after the network for a batch: list of (candidate, subset)."""
    h, w, nh, nw = geo
    heat = F.interpolate(heat_low, scale_factor=stride, mode="bicubic")[:, :, :nh, :nw]
    heat = F.interpolate(heat, size=(h, w), mode="bicubic")
    paf = F.interpolate(paf_low, scale_factor=stride, mode="bicubic")[:, :, :nh, :nw]
    paf = F.interpolate(paf, size=(h, w), mode="bicubic").numpy().transpose(0, 2, 3, 1)
    heat = blur5(heat)
    peaks = find_peaks(heat[:, :-1], thre1).numpy()
    heat = heat.numpy().transpose(0, 2, 3, 1)
    B = heat.shape[0]
    all_peaks = [[[] for _ in range(18)] for _ in range(B)]
    counter, b_num = 0, None
    for b, c, y, x in peaks:
        counter = 0 if b != b_num else counter + 1
        b_num = b
        all_peaks[b][c].append((x, y, heat[b, y, x, c], counter))
    out = []
    for b in range(B):
        conns, special = connect_limbs(all_peaks[b], paf[b], h, thre2)
        out.append(assemble(all_peaks[b], conns, special))
    return out


def batch_body_infer(frames_u8: np.ndarray, net_fn, g_scale=0.5, thre1=0.1, thre2=0.05):
    """net_fn(x [B,3,Hp,Wp] float32 numpy) -> (paf, heat) numpy."""
    x, geo = net_input(frames_u8, g_scale)
    paf, heat = net_fn(x.numpy())
    return post(torch.from_numpy(np.asarray(paf)), torch.from_numpy(np.asarray(heat)), geo, thre1, thre2)


def hand_post(heat_low: torch.Tensor, thre=0.035, stride=8):
    """Batch_hand.__call__ after the network (srcmx/Batch_model.py:334-354) -> np.array [B, 21, 3]."""
    from .hand_post import label8, npmax
    heat = F.interpolate(heat_low, scale_factor=stride, mode="bicubic")
    heat = blur5(heat).numpy().transpose(0, 2, 3, 1)
    out = []
    for i in range(heat.shape[0]):
        peaks = []
        for part in range(21):
            m = heat[i, :, :, part]
            binary = m > thre
            if np.sum(binary) == 0:
                peaks.append([0, 0, 0])
                continue
            lab, n = label8(binary)
            best = np.argmax([np.sum(m[lab == k]) for k in range(1, n + 1)]) + 1
            m[lab != best] = 0
            y, x = npmax(m)
            peaks.append([x, y, np.max(m)])
        out.append(peaks)
    return np.array(out)


def batch_hand_infer(crops_u8: np.ndarray, net_fn, thre=0.035):
    """crops already at the data loader's size; net_fn(x [B,3,h,w] numpy) -> heat numpy."""
    x = to_tensor(crops_u8) - 0.5
    return hand_post(torch.from_numpy(np.asarray(net_fn(x.numpy()))), thre)
