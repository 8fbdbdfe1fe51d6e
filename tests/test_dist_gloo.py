"""CPU, world_size 2 (gloo): frame sharding + record gather of the multi-GPU Body path.

Each rank 'processes' its contiguous shard of a synthetic video (oracle results encoded as
libopose records, since the build container has no GPU), gathers with src.dist.gather_records
and checks that every rank ends up with every frame, in frame order, bit-identical."""
import glob
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG, REPO

PPP, MAXP = 16, 24


def _frames():
    """Per-frame (candidate, subset) from the golden planted fixtures (reference outputs)."""
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "body_planted_*.npz")))[:7]:
        d = np.load(p)
        out.append((d["candidate"], d["subset"]))
    return out


def _worker(rank, world, port, n_frames, q):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    from src import _native
    from src.dist import gather_records, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = _frames()
        frames = [frames[i % len(frames)] for i in range(n_frames)]
        lo, hi = shard_bounds(n_frames, rank, world)
        local = np.stack([_native.encode_record(c, s, PPP, MAXP) for c, s in frames[lo:hi]]) if hi > lo else \
            np.zeros((0, _native.record_bytes(PPP, MAXP)), np.uint8)
        allrec = gather_records(torch.from_numpy(local), n_frames, world).numpy()
        ok = allrec.shape[0] == n_frames
        for i, (c, s) in enumerate(frames):
            st, c2, s2 = _native.decode_record(allrec[i], PPP, MAXP)
            ok &= st == 0 and np.array_equal(np.asarray(c, np.float64).reshape(c2.shape), c2) and np.array_equal(s, s2)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [8, 7, 1])
def test_gather_records_two_ranks(n_frames):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + n_frames * 7 + os.getpid() % 200
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_frames, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_shard_bounds_cover_exactly():
    import sys
    sys.path.insert(0, PKG)
    from src.dist import shard_bounds
    for n in range(0, 40):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


# ------------------------------------------------------------- single-frame scale sharding
GEOMS = [(12, 20, 4, 0), (23, 40, 0, 0), (35, 60, 4, 4), (46, 80, 0, 0)]   # C5-like pyramid, scaled down


class _FakeBody:
    """Stands in for Body: per-scale maps are a function of the scale only, post returns them."""

    def __init__(self):
        self.computed = []

    def scale_geom(self, H, W):
        return GEOMS

    def scale_maps(self, frame, s):
        self.computed.append(s)
        hl, wl = GEOMS[s][:2]
        rng = np.random.default_rng(100 + s)
        return rng.standard_normal((frame.shape[0], 57, hl, wl)).astype(np.float32)

    def post_scales(self, maps, H, W):
        return [np.asarray(m) for m in maps]


def _scale_worker(rank, world, port, q):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    from src.dist import body_scale_sharded, scale_plan
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        body = _FakeBody()
        frame = np.zeros((90, 160, 3), np.uint8)
        out = body_scale_sharded(body, frame, rank, world, dst=0)
        owner = scale_plan([g[0] * g[1] for g in GEOMS], world)
        ok = sorted(body.computed) == [s for s, r in enumerate(owner) if r == rank]
        if rank == 0:
            ok &= len(out) == len(GEOMS)
            for s, m in enumerate(out):
                ok &= np.array_equal(m, _FakeBody().scale_maps(frame[None], s))
        else:
            ok &= out is None
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scale_sharded_gathers_lowres_maps(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29900 + world * 13 + os.getpid() % 200
    procs = [ctx.Process(target=_scale_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def test_scale_plan_balances_largest_first():
    import sys
    sys.path.insert(0, PKG)
    from src.dist import scale_plan
    costs = [0.25, 1.0, 2.25, 4.0]          # scale_search = [0.5, 1, 1.5, 2]: cost ~ scale^2
    assert scale_plan(costs, 1) == [0, 0, 0, 0]
    assert scale_plan(costs, 2) == [1, 1, 1, 0]           # 4.0 | 3.5
    assert scale_plan(costs, 4) == [3, 2, 1, 0]
    assert scale_plan(costs, 8) == [3, 2, 1, 0]
    for w in (2, 3, 5):
        own = scale_plan(costs, w)
        load = [sum(c for c, r in zip(costs, own) if r == k) for k in range(w)]
        assert max(load) == 4.0
