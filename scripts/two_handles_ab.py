"""Throughput A/B: one Body handle (the bench's pipelined step) against two handles on the same
GPU taking alternate 32-frame batches, so one handle's network can fill the CUs the other's
launches leave idle (236-tile 7x7 grids on 256 CUs, partial last rounds of the 3x3 grids).

    python scripts/two_handles_ab.py [--steps 20] [--rounds 3]   (one JSON line per leg)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "pytorch-openpose_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--handles", type=int, default=2)
    a = ap.parse_args()
    from src.body import Body
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    sd = seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE)
    bodies = [Body(sd, device=0) for _ in range(a.handles)]
    dev = torch.device("cuda", 0)
    frames = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (32, 368, 656, 3), dtype=np.uint8)).to(dev)
    rb = bodies[0].handle.record_bytes()
    recs = [torch.empty((32, rb), dtype=torch.uint8, device=dev) for _ in bodies]
    torch.cuda.synchronize()

    def run(nh, n):
        for k in range(n):
            i = k % nh
            bodies[i].infer_records(frames, recs[i], pipeline=True, wait=False)
        for b in bodies[:nh]:
            b.handle.synchronize()

    for nh in (1, a.handles):
        run(nh, 4)
    for r in range(a.rounds):
        for nh in (1, a.handles):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(nh, a.steps)
            dt = time.perf_counter() - t0
            print(json.dumps({"handles": nh, "round": r, "frames_per_s": 32 * a.steps / dt,
                              "ms_per_step": dt / a.steps * 1e3}), flush=True)
    # the records of the two-handle run equal the one-handle run's (same frames)
    run(1, 1)
    ref = recs[0].clone()
    run(a.handles, a.handles)
    print(json.dumps({"records_equal": all(bool(torch.equal(ref, r)) for r in recs[:a.handles])}))


if __name__ == "__main__":
    main()
