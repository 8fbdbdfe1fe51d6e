"""Repro of the bench_configs crash: C2 body + Hand handles used first, then the C5 handle."""
import faulthandler
import os
import sys

import numpy as np
import torch

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body  # noqa: E402
from src.hand import Hand  # noqa: E402
from src.weights import BENCH_OUT_SCALE, c5_out_scale, seeded_state_dict  # noqa: E402

stages = sys.argv[1].split(",") if len(sys.argv) > 1 else ["c2", "hand", "c5"]
rng = np.random.default_rng(3)
dev = torch.device("cuda", 0)
if "c2" in stages:
    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
    img = rng.integers(0, 256, (368, 656, 3), dtype=np.uint8)
    for _ in range(5):
        body(img)
    f1 = torch.from_numpy(img[None].copy()).to(dev)
    rec = torch.empty((1, body.handle.record_bytes()), dtype=torch.uint8, device=dev)
    for _ in range(5):
        body.infer_records(f1, rec); body.handle.synchronize()
    print("c2 ok", file=sys.stderr, flush=True)
if "hand" in stages:
    hand = Hand(seeded_state_dict("hand", 0))
    crop = rng.integers(0, 256, (368, 368, 3), dtype=np.uint8)
    for _ in range(5):
        hand(crop)
    print("hand ok", file=sys.stderr, flush=True)
b = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=(0.5, 1.0, 1.5, 2.0))
f = torch.from_numpy(rng.integers(0, 256, (4, 1080, 1920, 3), dtype=np.uint8)).to(dev)
rec5 = torch.empty((4, b.handle.record_bytes()), dtype=torch.uint8, device=dev)
for i in range(4):
    b.infer_records(f, rec5); b.handle.synchronize()
print("c5 batch ok", file=sys.stderr, flush=True)
if "l0" in stages:
    os.environ["OPOSE_LOCKSTEP"] = "0"
    b2 = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=(0.5, 1.0, 1.5, 2.0))
    del os.environ["OPOSE_LOCKSTEP"]
    if "unused" not in stages:
        for i in range(4):
            b2.infer_records(f, rec5); b2.handle.synchronize()
        for i in range(4):
            b2.infer_records(f[:1].contiguous(), rec5[:1]); b2.handle.synchronize()
    else:
        b2.handle.wait_torch()
    print("streams", b.handle.stream(), b2.handle.stream(), file=sys.stderr, flush=True)
    if "keep" not in stages:
        del b2
    print("l0 ok", file=sys.stderr, flush=True)
f1 = f[:1].contiguous()
for i in range(6):
    print("c5 single", i, file=sys.stderr, flush=True)
    b.infer_records(f1, rec5[:1]); b.handle.synchronize()
print("ok", file=sys.stderr, flush=True)
