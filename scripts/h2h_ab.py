"""Host-to-host pass A/B (round-6 verdict item 1): device-resident rate, bench.host_to_host (round 6:
uploads ordered on the network's input read, downloads on their own stream) and round 5's pass
(uploads wait for the handle's whole stream, downloads queued on it), alternated on one box.

    python scripts/h2h_ab.py [--steps 10] [--rounds 2] [--only sync|stream|old]   (one JSON line per leg)
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
import bench  # noqa: E402


def old_host_to_host(body, frames_np, steps, dev):
    B = len(frames_np)
    host = torch.from_numpy(frames_np).pin_memory()
    rb = body.handle.record_bytes()
    dbuf = [torch.empty_like(host, device=dev) for _ in range(2)]
    rdev = [torch.empty((B, rb), dtype=torch.uint8, device=dev) for _ in range(2)]
    rhost = [torch.empty((B, rb), dtype=torch.uint8).pin_memory() for _ in range(2)]
    cps = [torch.cuda.Stream(device=dev) for _ in range(2)]
    lib_stream = body.handle.torch_stream()

    def upload(i):
        cps[i].wait_stream(lib_stream)
        with torch.cuda.stream(cps[i]):
            dbuf[i].copy_(host, non_blocking=True)

    def run(n):
        for i in range(2):
            upload(i)
        for k in range(n):
            i = k % 2
            with torch.cuda.stream(cps[i]):
                body.infer_records(dbuf[i], rdev[i], pipeline=True)
            with torch.cuda.stream(lib_stream):
                rhost[i].copy_(rdev[i], non_blocking=True)
            if k + 2 < n:
                upload(i)
        body.handle.synchronize()
        torch.cuda.synchronize()

    run(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    dt = time.perf_counter() - t0
    return B * steps / dt, dt / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    from src.body import Body
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    dev = torch.device("cuda", 0)
    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE), device=0)
    frames_np = np.random.default_rng(1).integers(0, 256, (32, bench.H, bench.W, 3), dtype=np.uint8)
    frames = torch.from_numpy(frames_np).to(dev)
    rec = torch.empty((32, body.handle.record_bytes()), dtype=torch.uint8, device=dev)

    def resident(n):
        for _ in range(3):
            body.infer_records(frames, rec, pipeline=True)
        body.handle.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            body.infer_records(frames, rec, pipeline=True)
        body.handle.synchronize()
        dt = time.perf_counter() - t0
        return 32 * n / dt, dt / n * 1e3

    for r in range(a.rounds):
        v, ms = resident(a.steps)
        print(json.dumps({"leg": "resident", "round": r, "value": v, "ms": ms}), flush=True)
        for mode in ("sync", "stream"):
            if a.only in (None, mode):
                v, ms, info = bench.host_to_host(body, frames_np, a.steps, dev, 0, 1, mode=mode)
                print(json.dumps({"leg": "h2h_" + mode, "round": r, "value": v, "ms": ms, "info": info}), flush=True)
        if a.only in (None, "old"):
            v, ms = old_host_to_host(body, frames_np, a.steps, dev)
            print(json.dumps({"leg": "h2h_old", "round": r, "value": v, "ms": ms}), flush=True)


if __name__ == "__main__":
    main()
