"""Pipelined vs host-path records on the same batches, many trials: counts frames whose candidates
or subsets differ (OPOSE_LIB selects the library, for A/B against an older build)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, "pytorch-openpose_amd")
from src.body import Body
from src.weights import BENCH_OUT_SCALE, seeded_state_dict
# MULTI=1: a two-scale pyramid (scale_search 0.5, 1.0: the scales' networks run concurrently)
scales = (0.5, 1.0) if os.environ.get("MULTI") == "1" else (0.5,)
body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE), scale_search=scales)
rng = np.random.default_rng(21)
# BENCH=1: the bench's shape (32 frames of 368x656 per call) instead of 3 frames of 184x328
NB, HB, WB = (32, 368, 656) if os.environ.get("BENCH") == "1" else (3, 184, 328)
batches = [rng.integers(0, 256, (NB, HB, WB, 3), dtype=np.uint8) for _ in range(3)]
exp = [body.batch(f) for f in batches]
dev = [torch.from_numpy(f).cuda() for f in batches]
torch.cuda.synchronize()
T = int(os.environ.get("TRIALS", "20"))
bad_c = bad_s = frames = 0
for trial in range(T):
    order = [0, 1, 2, 0, 1, 2, 1]
    recs = [body.infer_records(dev[i], pipeline=True) for i in order]
    body.handle.synchronize()
    for call, (i, rec) in enumerate(zip(order, recs)):
        for f, ((c, s), (ec, es)) in enumerate(zip(body.decode_records(rec), exp[i])):
            frames += 1
            if not np.array_equal(c, ec):
                bad_c += 1
            elif not np.array_equal(s, es):
                bad_s += 1
                if bad_s <= 3:
                    rows = min(len(s), len(es))
                    d = [r for r in range(rows) if not np.array_equal(s[r], es[r])]
                    print(f"  trial {trial} call {call} b{i} f{f}: subset {s.shape} vs {es.shape}, first diff row "
                          f"{d[:1]}: {s[d[0]] if d else None} vs {es[d[0]] if d else None}", flush=True)
print(f"lib={os.environ.get('OPOSE_LIB', 'head')} "
      f"shape={NB}x{HB}x{WB} scales={len(scales)}: "
      f"{frames} frames, candidate mismatches {bad_c}, subset-only mismatches {bad_s}", flush=True)
