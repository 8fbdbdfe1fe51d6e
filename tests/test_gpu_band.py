"""GPU: row bands of one scale (opose_body_band_maps) — the balanced C5 split (SURVEY.md §8(e):
"balance them, because 736x1312 is 53 % of FLOPs").

A band rank runs the trunk on its rows plus a 10-row margin past each cut (recomputed) and the
CPM stages (src/model.py:106-133) on its own output rows, with 3 halo rows exchanged before
every 3x3 / 7x7 stage layer.

Every conv sums a pixel in an order fixed by the layer and the whole frame (k slabs and kernel
family), whatever rows a band launch covers and whatever grid runs it, so:
* bands put together equal opose_body_scale_maps (the whole scale's network) bit for bit, for
  2, 3 and 5 bands -- the trunk margin and the halo exchange lose nothing;
* body_scale_sharded(split="balanced") with four and eight gloo ranks on cuda:0 (the 2.0 scale
  cut into 2 / 5 bands, the 1.5 scale into 2 at eight): every scale's gathered maps equal Body's
  own, and the (candidate, subset) arrays equal Body(frame)'s -- the north-star bar exactly."""
import os
import threading

import numpy as np
import pytest
import torch

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

SCALES = (0.5, 1.0, 1.5, 2.0)
HW = (368, 656)  # the 2.0 scale is C5's largest network: 736 x 1312 -> 92 x 164 maps


@pytest.fixture(scope="module")
def bodies():
    from src.body import Body
    from src.weights import seeded_state_dict
    sd = seeded_state_dict("body", 0)
    return [Body(sd, scale_search=SCALES) for _ in range(5)]


@pytest.fixture(scope="module")
def frame():
    return np.random.default_rng(41).integers(0, 256, HW + (3,), dtype=np.uint8)


def _run_bands(bodies, frame, s, rows):
    """Every band on its own handle and thread; the halo exchange copies device to device
    between neighbouring bands' xbufs (two barriers: both sides packed / both sides copied)."""
    nb = len(rows)
    bar = threading.Barrier(nb)
    xbufs = [None] * nb
    out = [None] * nb
    errs = []

    def exchange_for(b):
        def ex(xbuf, cap, n, stream):
            torch.cuda.ExternalStream(stream).synchronize()
            xbufs[b] = xbuf
            bar.wait()
            if b > 0:
                xbuf[2 * cap:2 * cap + n].copy_(xbufs[b - 1][cap:cap + n])   # above: its bottom rows
            if b + 1 < nb:
                xbuf[3 * cap:3 * cap + n].copy_(xbufs[b + 1][0:n])           # below: its top rows
            torch.cuda.synchronize()
            bar.wait()
        return ex

    def run(b):
        try:
            r0, r1 = rows[b]
            out[b] = bodies[b].band_maps(frame, s, r0, r1, exchange_for(b))
        except BaseException as e:
            errs.append(e)
            bar.abort()

    th = [threading.Thread(target=run, args=(b,)) for b in range(nb)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "band threads hung"
    if errs:
        raise errs[0]
    return np.concatenate(out, 2)


@pytest.mark.parametrize("s,nb", [(3, 2), (3, 3), (3, 5), (2, 2), (1, 2)])
def test_bands_equal_scale_maps(bodies, frame, s, nb):
    from src.dist import band_rows
    hl, wl, _, _ = bodies[0].scale_geom(*HW)[s]
    ref = bodies[0].scale_maps(frame, s)
    whole = bodies[0].band_maps(frame, s, 0, hl)
    assert whole.shape == (1, 57, hl, wl)
    assert np.array_equal(whole, ref)
    got = _run_bands(bodies, frame, s, band_rows(hl, nb))
    assert np.array_equal(got, ref)
    assert (got[:, 38:] >= 0).all()  # Mconv7_stage6_L2 keeps its ReLU (src/model.py:30-33)


def test_band_maps_argument_checks(bodies, frame):
    from src._native import OposeError
    hl = bodies[0].scale_geom(*HW)[3][0]
    with pytest.raises(OposeError):
        bodies[0].band_maps(frame, 3, 0, 2)           # fewer than 3 rows
    with pytest.raises(OposeError):
        bodies[0].band_maps(frame, 3, 10, hl + 1)     # past the map
    with pytest.raises(RuntimeError):
        bodies[0].band_maps(frame, 3, 0, 40)          # neighbours but no exchange


def _balanced_worker(rank, world, port, q):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from src.body import Body
    from src.dist import body_scale_sharded, split_plan
    from src.weights import c5_out_scale, seeded_state_dict
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=SCALES)
        img = np.random.default_rng(43).integers(0, 256, HW + (3,), dtype=np.uint8)
        geo = b.scale_geom(*HW)
        _, owners, _ = split_plan([g[0] * g[1] for g in geo], world, [g[0] for g in geo])
        banded = len(owners[3]) > 1
        got_maps = []
        out = body_scale_sharded(b, img, rank, world, split="balanced", maps_out=got_maps)
        msg = ""
        if rank == 0:
            (cand, subset), = out
            (rc, rs), = b.batch(img[None])
            ok = banded and len(cand) > 0
            for s, m in enumerate(got_maps):  # each scale's gathered maps: Body's own, bit for bit
                ref = b.scale_maps(img, s)
                if not np.array_equal(np.asarray(m), ref):
                    ok = False
                    msg += "scale %d owners %s max diff %.3g; " % (s, owners[s], float(np.abs(np.asarray(m) - ref).max()))
            msg += "banded=%s peaks %d/%d people %d/%d" % (banded, len(cand), len(rc), len(subset), len(rs))
            ok = ok and np.array_equal(cand, rc) and np.array_equal(subset, rs)
        else:
            ok = out is None
        q.put((rank, bool(ok), msg))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_balanced_split_matches_body(world):
    """4 ranks: the 2.0 scale in 2 bands; 8 ranks (C5's node): the 2.0 scale in 5 bands of 18-19
    rows (middle bands exchange with both neighbours) and the 1.5 scale in 2."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world * 37 + os.getpid() % 300
    procs = [ctx.Process(target=_balanced_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


def test_rccl_exchange_moves_the_halo_rows(bodies, frame):
    """The library's own halo exchange (exchange="rccl": ncclSend / ncclRecv on the handle's
    stream between the stage layers) on a one-rank communicator with the band's neighbours set
    to itself: RCCL pairs the sends and receives in order, so each band edge receives its own
    packed rows.  The same routing done by a Python callback gives the same maps bit for bit,
    so RCCL moved exactly the packed bytes, in stream order, at every one of the 27 exchanges."""
    from src._native import OposeError
    b, ref_body = bodies[0], bodies[1]
    with pytest.raises(OposeError):
        b.band_maps(frame, 3, 30, 60, "rccl")     # no communicator yet
    b.handle.rccl_init(b.handle.rccl_unique_id(), 0, 1)
    b.handle.set_band_peers(0, 0)
    got = b.band_maps(frame, 3, 30, 60, "rccl")

    def self_copy(xbuf, cap, n, stream):
        torch.cuda.ExternalStream(stream).synchronize()
        xbuf[2 * cap:2 * cap + n].copy_(xbuf[0:n])
        xbuf[3 * cap:3 * cap + n].copy_(xbuf[cap:cap + n])
        torch.cuda.synchronize()
    ref = ref_body.band_maps(frame, 3, 30, 60, self_copy)
    assert np.array_equal(got, ref)
    dev = b.band_maps(torch.from_numpy(frame).cuda(), 3, 30, 60, "rccl")
    b.handle.rccl_wait(30.0)  # the exchanges completed: the bounded wait returns, nothing aborted
    assert np.array_equal(dev.cpu().numpy(), ref)
    dev2 = b.band_maps(torch.from_numpy(frame).cuda(), 3, 30, 60, "rccl")  # the communicator is still up
    b.handle.rccl_wait(30.0)
    assert np.array_equal(dev2.cpu().numpy(), ref)
    b.handle.set_band_peers(None, None)


def test_body_lockstep_equals_per_scale_networks(frame):
    """A multi-scale Body's four networks in lockstep (default: one conv launch per layer for all
    scales, their work units scheduled together) against one network per scale on concurrent
    streams (OPOSE_LOCKSTEP=0): the same (candidate, subset) bit for bit."""
    from src.body import Body
    from src.weights import c5_out_scale, seeded_state_dict
    sd = seeded_state_dict("body", 0, out_scale=c5_out_scale())
    lock = Body(sd, scale_search=SCALES)
    old = os.environ.get("OPOSE_LOCKSTEP")
    os.environ["OPOSE_LOCKSTEP"] = "0"
    try:
        per = Body(sd, scale_search=SCALES)
    finally:
        if old is None:
            del os.environ["OPOSE_LOCKSTEP"]
        else:
            os.environ["OPOSE_LOCKSTEP"] = old
    (ca, sa), = lock.batch(frame[None])
    (cb, sb), = per.batch(frame[None])
    assert len(ca) > 0 and np.array_equal(ca, cb) and np.array_equal(sa, sb)
