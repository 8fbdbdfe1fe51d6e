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
        self.bands = []

    def scale_geom(self, H, W):
        return GEOMS

    def scale_maps(self, frame, s):
        self.computed.append(s)
        hl, wl = GEOMS[s][:2]
        rng = np.random.default_rng(100 + s)
        return rng.standard_normal((frame.shape[0], 57, hl, wl)).astype(np.float32)

    def band_maps(self, frame, s, r0, r1, exchange=None):
        """Rows [r0, r1) of scale_maps(s); drives the real halo exchange with a host xbuf whose
        send halves carry (scale, first row / last row) tags, and checks what comes back."""
        self.bands.append((s, r0, r1))  # (scale_maps below records s in computed)
        hl = GEOMS[s][0]
        cap, n = 64, 40
        xbuf = torch.zeros(4 * cap, dtype=torch.uint8)
        xbuf[0:n] = s * 16 + r0 % 16             # my top rows, for the band above
        xbuf[cap:cap + n] = s * 16 + (r1 - 1) % 16  # my bottom rows, for the band below
        for _ in range(3):
            exchange(xbuf, cap, n, None)
        if r0 > 0:   # the band above sent its last row's tag
            assert (xbuf[2 * cap:2 * cap + n] == s * 16 + (r0 - 1) % 16).all()
        if r1 < hl:  # the band below sent its first row's tag
            assert (xbuf[3 * cap:3 * cap + n] == s * 16 + r1 % 16).all()
        return self.scale_maps(frame[None], s)[:, :, r0:r1].copy()

    def post_scales(self, maps, H, W):
        return [np.asarray(m) for m in maps]


def _scale_worker(rank, world, port, q, split="scales"):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    from src.dist import band_rows, body_scale_sharded, scale_plan, split_plan
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        body = _FakeBody()
        frame = np.zeros((90, 160, 3), np.uint8)
        out = body_scale_sharded(body, frame, rank, world, dst=0, split=split)
        if split == "scales":
            order, owners = range(len(GEOMS)), [[r] for r in scale_plan([g[0] * g[1] for g in GEOMS], world)]
        else:
            order, owners, _ = split_plan([g[0] * g[1] for g in GEOMS], world, [g[0] for g in GEOMS])
        ok = sorted(body.computed) == [s for s, rs in enumerate(owners) if rank in rs]
        ok &= body.bands == [(s, *band_rows(GEOMS[s][0], len(owners[s]))[owners[s].index(rank)])
                             for s in order if rank in owners[s] and len(owners[s]) > 1]
        if split == "balanced" and world == 4:
            ok &= any(len(rs) > 1 for rs in owners)  # the test exercises real bands
        if rank == 0:
            ok &= len(out) == len(GEOMS)
            for s, m in enumerate(out):
                ok &= np.array_equal(m, _FakeBody().scale_maps(frame[None], s))
        else:
            ok &= out is None
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,split", [(2, "scales"), (3, "scales"), (3, "balanced"), (4, "balanced")])
def test_scale_sharded_gathers_lowres_maps(world, split):
    """Scale / band sharding on CPU ranks: each rank computes exactly its planned pieces, band
    neighbours exchange halo rows (src.dist.band_exchange over gloo), and rank 0 reassembles
    every scale's maps in row order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29900 + world * 13 + (split == "balanced") * 7 + os.getpid() % 200
    procs = [ctx.Process(target=_scale_worker, args=(r, world, port, q, split)) for r in range(world)]
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


def test_split_plan_cuts_the_largest_scale_into_bands():
    """split_plan (src/dist.py): C5's pyramid (hl x wl = 23x41, 46x82, 69x123, 92x164 at 1080p)
    over 1 / 2 / 4 / 8 ranks.  Two ranks keep whole scales (then the result stays bit-identical
    to one GPU); four and eight cut the 2.0 scale (and smaller ones) into row bands, lowering the
    modelled critical path well below the whole 2.0 scale (the longest-first bound)."""
    import sys
    sys.path.insert(0, PKG)
    from src.dist import band_rows, split_plan
    geo = [(23, 41), (46, 82), (69, 123), (92, 164)]
    costs = [h * w for h, w in geo]
    hls = [h for h, _ in geo]
    order, owners, load = split_plan(costs, 1, hls)
    assert owners == [[0]] * 4 and order == [3, 2, 1, 0]
    _, owners, load = split_plan(costs, 2, hls)
    assert all(len(o) == 1 for o in owners) and max(load) == costs[3]
    _, owners, load = split_plan(costs, 4, hls)
    assert len(owners[3]) >= 2 and max(load) < 0.8 * costs[3]
    _, owners, load = split_plan(costs, 8, hls)
    assert len(owners[3]) >= 4 and max(load) < 0.5 * costs[3]
    assert max(load) > sum(costs) / 8                 # never better than a perfect split
    for w in (3, 4, 5, 8):
        order, owners, load = split_plan(costs, w, hls)
        for s, rs in enumerate(owners):
            assert len(set(rs)) == len(rs) and all(0 <= r < w for r in rs)
            if len(rs) > 1:
                assert min(b - a for a, b in band_rows(hls[s], len(rs))) >= 8
    rows = band_rows(92, 5)
    assert rows[0][0] == 0 and rows[-1][1] == 92 and all(a[1] == b[0] for a, b in zip(rows, rows[1:]))


class _FakeHandle:
    def __init__(self):
        self.inits, self.peers = [], None

    @staticmethod
    def rccl_unique_id():
        return bytes(range(128))

    def rccl_init(self, uid, rank, world):
        self.inits.append((uid, rank, world))

    def set_band_peers(self, up, dn):
        self.peers = (up, dn)

    def rccl_wait(self, timeout_s):
        pass


class _FakeRcclBody(_FakeBody):
    """The device (RCCL) branch of body_scale_sharded: maps as tensors, bands through the
    library's own exchange (exchange == "rccl" with the peers set on the handle)."""

    def __init__(self):
        super().__init__()
        self.handle = _FakeHandle()

    def scale_maps(self, frame, s):
        return torch.from_numpy(super().scale_maps(frame, s))

    def band_maps(self, frame, s, r0, r1, exchange=None):
        assert exchange == "rccl" and len(self.handle.inits) == 1
        self.bands.append((s, r0, r1, self.handle.peers))
        return torch.from_numpy(_FakeBody.scale_maps(self, frame[None], s)[:, :, r0:r1].copy())

    def post_scales(self, maps, H, W):
        return [m.numpy() for m in maps]


def _rccl_worker(rank, world, port, q):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    from src import dist as sdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sdist.dist.get_backend = lambda group=None: "nccl"  # exercise the RCCL branch over gloo
        body = _FakeRcclBody()
        frame = torch.zeros((90, 160, 3), dtype=torch.uint8)
        out = sdist.body_scale_sharded(body, frame, rank, world, dst=0, split="balanced")
        order, owners, _ = sdist.split_plan([g[0] * g[1] for g in GEOMS], world, [g[0] for g in GEOMS])
        ok = body.handle.inits == [(bytes(range(128)), rank, world)]  # every rank, once
        want = []
        for s in order:
            rs = owners[s]
            if rank in rs and len(rs) > 1:
                b = rs.index(rank)
                want.append((s, *sdist.band_rows(GEOMS[s][0], len(rs))[b],
                             (rs[b - 1] if b else None, rs[b + 1] if b + 1 < len(rs) else None)))
        ok &= body.bands == want
        if rank == 0:
            for s, m in enumerate(out):
                ok &= np.array_equal(m, _FakeBody().scale_maps(np.zeros((1, 90, 160, 3), np.uint8), s))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_balanced_split_rccl_branch_four_ranks():
    """body_scale_sharded's device branch (RCCL on a node) with four ranks: the library's
    communicator is set up collectively on every rank (also those without a band), each band
    rank sets its neighbours before its band, and rank 0 reassembles every scale."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29950 + os.getpid() % 40
    procs = [ctx.Process(target=_rccl_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(4)}


class _FailingBandBody(_FakeBody):
    """Band pieces that fail on one rank after its first halo exchange (a library error, a bad
    callback): the ranks banded with it must not wait in their remaining exchanges."""

    def __init__(self, fail):
        super().__init__()
        self.fail = fail

    def band_maps(self, frame, s, r0, r1, exchange=None):
        if not self.fail:
            return super().band_maps(frame, s, r0, r1, exchange)
        xbuf = torch.zeros(4 * 64, dtype=torch.uint8)
        exchange(xbuf, 64, 40, None)
        raise RuntimeError("band failed on this rank")


def _failing_worker(rank, world, port, q, bad, abort_group=True, band_timeout=60.0):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    from src.dist import body_scale_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=__import__("datetime").timedelta(seconds=600))
    try:
        body_scale_sharded(_FailingBandBody(rank == bad), np.zeros((90, 160, 3), np.uint8), rank, world, split="balanced",
                           abort_group=abort_group, band_timeout=band_timeout)
        q.put((rank, "returned"))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "raised: %s" % type(e).__name__))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_failed_band_rank_does_not_hang_its_neighbours():
    """one band rank raising mid-band used to leave its neighbours blocked in the
    remaining halo exchanges until the backend timeout (10 min here).  With abort_group=True
    (the caller's opt-in for its WORLD group) body_scale_sharded destroys the group on the failing
    rank, so within seconds the failing rank re-raises its own
    error, its band neighbours raise, and no rank is left waiting."""
    import sys
    sys.path.insert(0, PKG)
    from src.dist import split_plan
    world = 4
    _, owners, _ = split_plan([g[0] * g[1] for g in GEOMS], world, [g[0] for g in GEOMS])
    banded = [rs for rs in owners if len(rs) > 1][0]
    bad = banded[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29990 + os.getpid() % 8
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, q, bad)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert not p.is_alive()
    assert res[bad] == "raised: RuntimeError", res
    for r in banded[1:]:
        assert res[r].startswith("raised"), res


def test_failed_band_rank_gloo_bounded_wait_keeps_world_group():
    """without abort_group the failing rank leaves the WORLD group alone, and its
    neighbours still do not hang: each gloo halo send / recv waits at most band_timeout seconds
    (band_exchange), so they raise in seconds, not after the group's 10-minute timeout."""
    import sys
    import time
    sys.path.insert(0, PKG)
    from src.dist import split_plan
    world = 4
    _, owners, _ = split_plan([g[0] * g[1] for g in GEOMS], world, [g[0] for g in GEOMS])
    banded = [rs for rs in owners if len(rs) > 1][0]
    bad = banded[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29930 + os.getpid() % 16
    t0 = time.time()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, q, bad, False, 3.0)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert not p.is_alive()
    assert res[bad] == "raised: RuntimeError", res
    for r in banded[1:]:
        assert res[r].startswith("raised"), res
    assert time.time() - t0 < 100


class _DeadlineHandle(_FakeHandle):
    """The library handle of a band rank whose neighbour failed: rccl_wait raises what the library
    reports after its deadline (or an interrupt arrives while waiting)."""

    def __init__(self, exc):
        super().__init__()
        self.exc, self.waits, self.aborts = exc, [], 0

    def rccl_wait(self, timeout_s):
        self.waits.append(timeout_s)
        raise self.exc

    def rccl_abort(self):
        self.aborts += 1


class _DeadlineBody(_FakeRcclBody):
    def band_maps(self, frame, s, r0, r1, exchange=None):
        assert exchange == "rccl"
        self.bands.append((s, r0, r1, self.handle.peers))
        return torch.zeros((1, 57, r1 - r0, GEOMS[s][1]))


@pytest.mark.parametrize("exc,aborts", [(TimeoutError("no progress within the deadline"), 1),
                                        (KeyboardInterrupt(), 0)])
def test_rccl_band_neighbour_bounded_wait(monkeypatch, exc, aborts):
    """on the RCCL path a failed rank's ncclCommAbort cannot cancel the recv kernels
    queued on its neighbours' streams.  Every band rank therefore waits for its exchanges with
    Handle.rccl_wait(band_timeout); when that reports the deadline (the library has then aborted
    the rank's own communicator so its kernels exit), body_scale_sharded drops the communicator
    and re-raises, leaving the torch process group alone.  An interrupt is not a band failure:
    nothing is aborted."""
    import sys
    sys.path.insert(0, PKG)
    from src import dist as sdist
    destroyed = []
    monkeypatch.setattr(sdist.dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(sdist.dist, "destroy_process_group", lambda group=None: destroyed.append(group))
    monkeypatch.setattr(sdist, "init_band_comm", lambda body, group=None: None)
    world = 4
    _, owners, _ = sdist.split_plan([g[0] * g[1] for g in GEOMS], world, [g[0] for g in GEOMS])
    rank = [rs for rs in owners if len(rs) > 1][0][1]  # a band with a neighbour above
    body = _DeadlineBody()
    body.handle = _DeadlineHandle(exc)
    with pytest.raises(type(exc)):
        sdist.body_scale_sharded(body, torch.zeros((90, 160, 3), dtype=torch.uint8), rank, world,
                                 band_timeout=0.25)
    # one bounded wait, after every banded piece of this rank was enqueued
    assert body.handle.waits == [0.25] and len(body.bands) == sum(rank in rs for rs in owners if len(rs) > 1)
    assert body.handle.aborts == aborts and destroyed == []


def test_abort_band_group_leaves_world_group_unless_asked(monkeypatch):
    """abort_band_group destroys a process group only on the gloo path and only when
    the caller asks (body_scale_sharded asks for an explicitly passed band subgroup, or with
    abort_group=True); the RCCL path never touches the torch process group."""
    import sys
    sys.path.insert(0, PKG)
    from src import dist as sdist
    destroyed = []
    monkeypatch.setattr(sdist.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(sdist.dist, "destroy_process_group", lambda group=None: destroyed.append(group))
    body = _DeadlineBody()
    body.handle = _DeadlineHandle(None)
    sdist.abort_band_group(body, None)
    sdist.abort_band_group(body, "sub", rccl=True, destroy_group=True)
    assert destroyed == [] and body.handle.aborts == 1
    sdist.abort_band_group(body, "sub", destroy_group=True)
    sdist.abort_band_group(body, None, destroy_group=True)
    assert destroyed == ["sub", None]
