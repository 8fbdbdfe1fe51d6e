# Pipelined vs serial records on the same batches (OPOSE_PIPELINE): prints every frame whose
# candidates differ from the host batch path.  Run on the GPU box (scripts/gauss_screen_ab.sh).
import sys, os, numpy as np, torch
sys.path.insert(0, "pytorch-openpose_amd"); sys.path.insert(0, ".")
from src.body import Body
from src.weights import BENCH_OUT_SCALE, seeded_state_dict
body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
rng = np.random.default_rng(21)
batches = [rng.integers(0, 256, (3, 184, 328, 3), dtype=np.uint8) for _ in range(3)]
exp = [body.batch(f) for f in batches]
def cmp(tag, got, e):
    bad = 0
    for f, ((c, s), (ec, es)) in enumerate(zip(got, e)):
        if not (np.array_equal(c, ec) and np.array_equal(s, es)):
            bad += 1
            print(f"{tag} frame {f}: cand {c.shape} vs {ec.shape}", flush=True)
            A = {tuple(r[:3]) for r in c}; B = {tuple(r[:3]) for r in ec}
            print("   missing:", sorted(B - A)[:4], " extra:", sorted(A - B)[:4], flush=True)
    return bad
for t in range(4):
    for i in range(3):
        cmp(f"serial-host t{t} b{i}", body.batch(batches[i]), exp[i])
dev = [torch.from_numpy(f).cuda() for f in batches]
torch.cuda.synchronize()
for t in range(4):
    for i in range(3):
        r = body.infer_records(dev[i]); body.handle.synchronize()
        cmp(f"serial-dev t{t} b{i}", body.decode_records(r), exp[i])
for trial in range(6):
    order = [0, 1, 2, 0, 1, 2, 1]
    recs = [body.infer_records(dev[i], pipeline=True) for i in order]
    body.handle.synchronize()
    for call, (i, rec) in enumerate(zip(order, recs)):
        cmp(f"pipe trial {trial} call {call} b{i}", body.decode_records(rec), exp[i])
    # interleave a host call
    body.batch(batches[1])
print("done")
