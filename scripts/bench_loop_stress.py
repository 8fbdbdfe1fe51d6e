"""Race stress of bench.py's timed loop: N pipelined steps on one resident 32-frame batch and
one records buffer, calls without torch-stream markers (wait=False), each step's records copied
out on the handle's stream; every copy must equal the serial records.

    python scripts/bench_loop_stress.py [--steps 200]
"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    from src.body import Body
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
    d = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (32, 368, 656, 3), dtype=np.uint8)).cuda()
    ref = body.infer_records(d).clone()
    body.handle.synchronize()
    rec = torch.empty_like(ref)
    lib = body.handle.torch_stream()
    bad, chunk = 0, 20
    for s0 in range(0, a.steps, chunk):
        outs = [torch.empty_like(rec) for _ in range(chunk)]
        torch.cuda.synchronize()
        for k in range(chunk):
            body.infer_records(d, rec, pipeline=True, wait=False)
            with torch.cuda.stream(lib):
                outs[k].copy_(rec)
        body.handle.synchronize()
        torch.cuda.synchronize()
        bad += sum(not torch.equal(o, ref) for o in outs)
        print(f"steps {s0 + chunk}: mismatching steps so far {bad}", flush=True)
    print("records equal in every step" if bad == 0 else f"MISMATCH in {bad} steps")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
