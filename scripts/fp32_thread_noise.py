"""Evidence for DESIGN §2's near-tie statement: on the bench's crowded calibrated frames the
reference's own fp32 network (torch CPU, the oracle restatement of src/model.py) run on 8 threads
and on 1 thread puts keypoints at different pixels -- its summation order changes with the thread
count, and the smoothed heat maps have 1-2 px plateaus.  Prints, per frame, how many keypoints the
two fp32 runs place identically, one pixel apart, or not at all, and each run against the float64
network; writes the table to profiles/r4_fp32_thread_noise.json.  CPU only.

    python scripts/fp32_thread_noise.py [n_frames]
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "pytorch-openpose_amd"), REPO]
from oracle import body_post, network  # noqa: E402
from src.weights import BENCH_OUT_SCALE  # noqa: E402


def agreement(c1, c2):
    """Keypoints of c1 matched in c2 at the same pixel (score within 1e-3), within one pixel, or
    not at all (+ c2's leftovers): (exact, within_1px, unmatched) -- tests/test_gpu_c4_shard.py."""
    free = [tuple(r[:3]) for r in c2]
    exact = near = 0
    rest = []

    def close(p, q, tol):
        return abs(q[0] - p[0]) <= tol and abs(q[1] - p[1]) <= tol and abs(q[2] - p[2]) <= 1e-3 * abs(q[2]) + 1e-6

    for r in c1:
        p = tuple(r[:3])
        hit = next((q for q in free if close(p, q, 0)), None)
        if hit is None:
            rest.append(p)
        else:
            free.remove(hit)
            exact += 1
    unmatched = 0
    for p in rest:
        hit = next((q for q in free if close(p, q, 1)), None)
        if hit is None:
            unmatched += 1
        else:
            free.remove(hit)
            near += 1
    return exact, near, unmatched + len(free)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    frames = np.random.default_rng(1).integers(0, 256, (32, 368, 656, 3), dtype=np.uint8)[:n]  # bench.py rank 0
    sd = network.seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE)
    sd64 = {k: v.double() for k, v in sd.items()}

    def run(img, d, threads, dbl=False):
        torch.set_num_threads(threads)

        def fn(x):
            xx = torch.from_numpy(x)
            p, h = network.body_forward(xx.double() if dbl else xx, d)
            return p.float().numpy(), h.float().numpy()
        return body_post.body_infer(img, fn)[0]

    rows = []
    for f, img in enumerate(frames):
        c8, c1 = run(img, sd, 8), run(img, sd, 1)
        c64 = run(img, sd64, 8, True)
        r = {"frame": f, "keypoints_8threads": len(c8), "keypoints_1thread": len(c1), "keypoints_f64": len(c64),
             "8t_vs_1t": agreement(c8, c1), "8t_vs_f64": agreement(c8, c64), "1t_vs_f64": agreement(c1, c64)}
        e, nb, u = r["8t_vs_1t"]
        r["8t_vs_1t_moved_frac"] = (nb + u) / max(1, len(c8))
        rows.append(r)
        print(json.dumps(r), flush=True)
    out = {"script": "scripts/fp32_thread_noise.py", "frames": "bench.py rank-0 frames (rng seed 1), 368x656",
           "weights": "seeded body net, BENCH_OUT_SCALE", "torch": torch.__version__,
           "mean_moved_frac_8t_vs_1t": float(np.mean([r["8t_vs_1t_moved_frac"] for r in rows])), "rows": rows}
    with open(os.path.join(REPO, "profiles", "r4_fp32_thread_noise.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("mean fraction of keypoints that move between 8 and 1 threads: %.3f" % out["mean_moved_frac_8t_vs_1t"])


if __name__ == "__main__":
    main()
