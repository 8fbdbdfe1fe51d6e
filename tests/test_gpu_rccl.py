"""GPU: the RCCL ('nccl') branches of src/dist.py, executed for real on the one MI355X of a test
box: a one-rank nccl process group (RCCL refuses two ranks on one device, and the 8-GPU runs are
the driver's).  World size 1 still runs the library's collective path end to end -- RCCL
communicator setup, all_gather_into_tensor on device records enqueued behind the library's
stream -- and the device-tensor branch of body_scale_sharded (maps kept on the GPU)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "pytorch-openpose_amd")


def _worker(port, q):
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from src.body import Body
    from src.dist import all_gather_padded, body_scale_sharded, gather_records, shard_bounds
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        res = {"backend": dist.get_backend()}
        body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
        frames = np.random.default_rng(7).integers(0, 256, (5, 184, 240, 3), dtype=np.uint8)
        dev = torch.from_numpy(frames).cuda()
        lo, hi = shard_bounds(5, 0, 1)
        rec = body.infer_records(dev[lo:hi])  # async, in the handle's stream order
        body.handle.synchronize()
        parts = all_gather_padded(rec, 1)  # the RCCL collective itself
        torch.cuda.synchronize()
        res["gather_equal"] = bool(torch.equal(parts[0], rec))
        res["records_equal_host_path"] = all(
            np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
            for a, b in zip(body.decode_records(gather_records(rec, 5, 1)), body.batch(frames)))
        # device-tensor scale sharding on RCCL (maps stay on the GPU)
        b2 = Body(seeded_state_dict("body", 0), scale_search=(0.5, 1.0))
        img = np.random.default_rng(31).integers(0, 256, (90, 160, 3), dtype=np.uint8)
        out = body_scale_sharded(b2, torch.from_numpy(img).cuda(), 0, 1)
        ref = b2.batch(img[None])
        res["scale_shard_equal"] = all(np.array_equal(ca, cb) and np.array_equal(sa, sb)
                                       for (ca, sa), (cb, sb) in zip(out, ref))
        q.put(res)
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_gather_and_scale_shard():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(29900 + os.getpid() % 90, q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res == {"backend": "nccl", "gather_equal": True, "records_equal_host_path": True,
                   "scale_shard_equal": True}, res
