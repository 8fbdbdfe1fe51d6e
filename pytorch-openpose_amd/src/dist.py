"""Frame-parallel multi-GPU Body inference: one process per GPU, RCCL gather of keypoints.

The reference has no multi-GPU pose path: frames are independent, so a video
batch shards across ranks with no data-path collective; the only exchange is the final gather
of the fixed-size per-frame records (include/opose.h, opose_body_record_bytes) — KB-scale, so
a single all_gather over xGMI (RCCL = torch.distributed 'nccl' on ROCm) per batch.

    import torch.distributed as dist
    dist.init_process_group("nccl")                  # torchrun, one rank per GPU
    body = Body(weights, device=local_rank)
    lo, hi = shard_bounds(len(frames), rank, world)
    rec = body.infer_records(frames_dev[lo:hi])      # async on the GPU
    allrec = gather_records(rec, len(frames), world)  # [n_frames, record_bytes], frame order
    results = body.decode_records(allrec)            # rank 0 (or every rank)
"""
from __future__ import annotations

import datetime
import functools
import itertools

import torch
import torch.distributed as dist


def shard_bounds(n_frames: int, rank: int, world: int):
    """Contiguous, balanced [lo, hi) frame range of `rank` (first n % world ranks get one more)."""
    base, extra = divmod(n_frames, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_records(rec: torch.Tensor, n_frames: int, world: int, group=None) -> torch.Tensor:
    """All-gather every rank's [n_local, record_bytes] uint8 records into frame order.

    Uneven shards are padded to the largest shard for the collective and trimmed after."""
    if world == 1:
        return rec
    per = [shard_bounds(n_frames, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in per)
    rb = rec.shape[1]
    if rec.shape[0] < cap:
        pad = torch.zeros((cap - rec.shape[0], rb), dtype=rec.dtype, device=rec.device)
        rec = torch.cat([rec, pad], 0)
    parts = all_gather_padded(rec, world, group)
    return torch.cat([p[:hi - lo] for p, (lo, hi) in zip(parts, per)], 0)


def all_gather_padded(rec: torch.Tensor, world: int, group=None):
    """The collective of gather_records: every rank's [cap, record_bytes] block, rank order.
    RCCL ('nccl'): one all_gather_into_tensor on the device tensors; gloo: through host memory."""
    rb = rec.shape[1]
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * rec.shape[0], rb), dtype=rec.dtype, device=rec.device)
        dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
        return list(out.view(world, rec.shape[0], rb))
    host = rec.cpu()
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host.contiguous(), group=group)
    return [p.to(rec.device) for p in parts]


# ---------------------------------------------------------------- single-frame scale sharding
# one 1080p frame at scale_search = [0.5, 1.0, 1.5, 2.0] (src/body.py:34-50).
# The four scale passes are independent until the float64 average of the full-resolution heat
# maps (src/body.py:48-49), so each rank runs the network for its scales and sends only the
# LOW-RES maps ([57, hl, wl] fp32, <= 3.4 MB per scale at 1080p) to one rank, which runs the
# whole multi-scale post path (opose_body_post_scales).  The 1080x1920x57 full-res maps never
# cross xGMI.

def scale_plan(costs, world: int):
    """Longest-processing-time assignment of scales to ranks: owner[s] for each scale.

    costs: per-scale work (the network is ~linear in hl*wl).  The largest scale dominates
    (2.0^2 / (0.25 + 1 + 2.25 + 4) = 53% at C5), so extra ranks beyond the scale count idle."""
    load = [0.0] * world
    owner = [0] * len(costs)
    for s in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        r = min(range(world), key=lambda k: (load[k], k))
        owner[s] = r
        load[r] += costs[s]
    return owner


# ---- balanced split: the largest scales cut into row bands (opose_body_band_maps)
# Scales are whole networks, so longest-first assignment leaves the 2.0 scale (53 % of the
# pyramid) alone on one rank.  A scale can instead be cut into nb row bands on nb ranks: each
# band rank runs the VGG trunk (TRUNK_FRAC of the FLOPs: 602 k of 2.007 M per network-input
# pixel, src/model.py:7-49 against 106-133) on its rows plus BAND_MARGIN rows past each cut
# (recomputed, not exchanged: the trunk's receptive field is small) and the CPM stages on its
# own rows, exchanging 3 halo rows with its neighbours before each 3x3 / 7x7 stage layer (the
# stages' receptive field, 84 rows at H/8, rules out recomputing theirs).
TRUNK_FRAC = 0.30
BAND_MARGIN = 10  # output rows (engine.cpp kBandTrunkMargin)
# per banded piece: a fraction of the scale's work (lower grid fill of the band's smaller
# layers) plus a fixed latency in output pixels (~0.5 ms: 54 pack / unpack launches, 27 halo
# callbacks, per-launch costs of the band's ~90 launches); fitted to one MI355X
# (profiles/r3_bench_configs.json C5_band_ms: 2.0 scale in 3 / 4 bands 4.89 / 4.10 ms against
# 8.17 whole, 1.5 in 3 bands 3.47 against 5.35, 1.0 in 2 bands 2.61 against 2.72)
BAND_OVERHEAD = 0.12
BAND_LATENCY_PX = 900
MIN_BAND_ROWS = 8


def band_rows(hl: int, nb: int):
    """Contiguous [r0, r1) output rows of each of nb bands of an hl-row map."""
    return [(hl * i // nb, hl * (i + 1) // nb) for i in range(nb)]


MAX_PLAN_COMBOS = 4096  # band-count combinations split_plan searches (the largest scales first)


def split_plan(costs, world: int, hls=None, trunk_frac: float = TRUNK_FRAC, overhead: float = BAND_OVERHEAD):
    """Balanced single-frame split of a scale pyramid over `world` ranks.

    costs[s]: work of scale s in output pixels (hl * wl); hls[s]: its output rows (bands keep
    >= MIN_BAND_ROWS).
    Returns (order, owners, load): owners[s] = ranks of scale s's bands, top to bottom (one rank:
    the whole scale); every rank runs its pieces in `order` (scales by decreasing piece cost, the
    same order everywhere, so the band groups' halo exchanges cannot wait on each other in a
    cycle); load[r] = modelled work of rank r.  Searches the band counts of the largest scales
    exhaustively -- as many scales as keep the search within MAX_PLAN_COMBOS combinations (all
    four of C5 up to 8 ranks: 8^4 = 4096); smaller scales stay whole -- pieces placed
    largest-first on the least loaded distinct ranks; ties keep fewer bands.  The plan is a pure
    function of its arguments and is cached, so a video's frames pay for the search once."""
    order, owners, load = _split_plan(tuple(costs), int(world), None if hls is None else tuple(hls),
                                      float(trunk_frac), float(overhead))
    return list(order), [list(o) for o in owners], list(load)


@functools.lru_cache(maxsize=256)
def _split_plan(costs, world, hls, trunk_frac, overhead):
    ns = len(costs)
    hls = hls if hls is not None else (10 ** 9,) * ns
    best = None
    choices = [[nb for nb in range(1, world + 1) if nb == 1 or hls[s] // nb >= MIN_BAND_ROWS] for s in range(ns)]
    combos = 1
    for s in sorted(range(ns), key=lambda i: (-costs[i], i)):  # band the largest scales first
        if combos * len(choices[s]) > MAX_PLAN_COMBOS:
            choices[s] = [1]
        combos *= len(choices[s])
    for nbs in itertools.product(*choices):
        piece = [costs[s] * (1.0 if nbs[s] == 1 else
                             trunk_frac * min(1.0, (hls[s] / nbs[s] + 2 * BAND_MARGIN) / hls[s])
                             + (1 - trunk_frac) / nbs[s] + overhead) + (BAND_LATENCY_PX if nbs[s] > 1 else 0)
                 for s in range(ns)]
        order = sorted(range(ns), key=lambda i: (-piece[i], i))
        load = [0.0] * world
        owners = [None] * ns
        for s in order:
            ranks = sorted(range(world), key=lambda k: (load[k], k))[:nbs[s]]
            owners[s] = sorted(ranks)
            for r in ranks:
                load[r] += piece[s]
        key = (round(max(load), 9), sum(nbs))
        if best is None or key < best[0]:
            best = (key, tuple(order), tuple(tuple(o) for o in owners), tuple(load))
    return best[1], best[2], best[3]


def band_exchange(rank_up, rank_dn, group=None, timeout: float | None = None):
    """Halo exchange of one band for Body.band_maps: send_up -> the band above (rank_up), send_dn
    -> the band below (rank_dn), their rows into recv_up / recv_dn.  RCCL ('nccl'): device
    P2P ops ordered on the library's stream; gloo: through host memory, synchronously, each
    send / recv waited for at most `timeout` seconds (None: the process group's own timeout), so
    the neighbour of a rank that failed mid-band raises instead of blocking in its next exchange
    (the library reports the callback's error as OPOSE_E_CALLBACK)."""
    wait_kw = {} if timeout is None else {"timeout": datetime.timedelta(seconds=timeout)}

    def ex(xbuf, cap, n, stream):
        pairs = [(r, o) for r, o in ((rank_up, 0), (rank_dn, 1)) if r is not None]
        if dist.get_backend(group) == "nccl":
            with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=xbuf.device)):
                ops = []
                for r, o in pairs:
                    ops.append(dist.P2POp(dist.isend, xbuf[o * cap:o * cap + n], r, group))
                    ops.append(dist.P2POp(dist.irecv, xbuf[(2 + o) * cap:(2 + o) * cap + n], r, group))
                for q in dist.batch_isend_irecv(ops):
                    q.wait()
            return
        if xbuf.is_cuda:
            torch.cuda.ExternalStream(stream, device=xbuf.device).synchronize()  # send halves packed
        recv = {o: torch.empty(n, dtype=torch.uint8) for _, o in pairs}
        reqs = []
        for r, o in pairs:
            reqs.append(dist.isend(xbuf[o * cap:o * cap + n].cpu(), r, group=group))
            reqs.append(dist.irecv(recv[o], r, group=group))
        for q in reqs:
            q.wait(**wait_kw)
        for _, o in pairs:
            xbuf[(2 + o) * cap:(2 + o) * cap + n].copy_(recv[o])
        if xbuf.is_cuda:
            torch.cuda.current_stream(xbuf.device).synchronize()  # before the library unpacks them
    return ex


def abort_band_group(body, group=None, rccl: bool = False, destroy_group: bool = False):
    """A band rank failed mid-frame: its neighbours are (or will be) blocked in one of the 27
    halo exchanges.
    RCCL: abort the library's communicator on this rank (its own queued send / recv exit).  The
    abort cannot reach the neighbours' queued kernels (xGMI P2P has no peer-failure signal); each
    neighbour bounds its own wait with Handle.rccl_wait (body_scale_sharded's band_timeout) and
    aborts its communicator when the deadline passes.  The torch process group is left alone.
    gloo: the exchange runs through the torch process group, so only destroying it releases the
    peers' pending send / recv.  That happens only when the caller opts in (destroy_group), and then
    to `group` -- the default (WORLD) group when group is None."""
    if rccl:
        try:
            body.handle.rccl_abort()
        except Exception:
            pass
        body._band_comm = None
        return
    if destroy_group:
        try:
            if dist.is_initialized():
                dist.destroy_process_group(group)
        except Exception:
            pass


def abort_band(body, group, rccl: bool, abort_group):
    """body_scale_sharded's failure path: abort_band_group, destroying a gloo group only for an
    explicitly passed `group` unless the caller decides (abort_group)."""
    abort_band_group(body, group, rccl, destroy_group=(group is not None) if abort_group is None else abort_group)


def init_band_comm(body, group=None):
    """The library's own RCCL communicator over the ranks of `group` (Body.band_maps with
    exchange="rccl": halo send/recv on the library's stream, no Python between the layers).
    Rank 0 makes the id; it travels by one broadcast on the group.  Collective: every rank of
    the group calls it (once per Body and group: a call with the same ranks returns at once, a
    call with another group of the same size builds a new communicator)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    members = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(world))
    if getattr(body, "_band_comm", None) == (rank, world, members):
        return
    obj = [body.handle.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    body.handle.rccl_init(obj[0], rank, world)
    body._band_comm = (rank, world, members)


def body_scale_sharded(body, frame, rank: int, world: int, dst: int = 0, group=None, split: str = "balanced",
                       maps_out=None, band_timeout: float = 60.0, abort_group=None):
    """Body(frame) with its scales split across ranks; returns [(candidate, subset)] on `dst`
    (None elsewhere).  frame: uint8 [H,W,3] / [1,H,W,3] numpy, or a torch cuda tensor (then the
    maps stay on the device and travel over RCCL; with gloo they go through host memory).

    split="scales": whole scales, longest first (scale_plan).
    split="balanced" (default): split_plan, which may cut the largest scales into row bands
    (Body.band_maps).
    Either way the result is identical to body.batch(frame) on one GPU, bit for bit: every conv
    sums each pixel in an order fixed by the layer and the scale's geometry (k slabs, DESIGN
    §4.1), so a band's rows and a scale on another rank equal the one-GPU network's maps, and the
    post path is the same code.
    A band rank whose piece fails aborts its band communicator (RCCL) before re-raising; on the
    RCCL path every band rank, once all its pieces are enqueued, waits for its exchanges for at
    most `band_timeout` seconds (one Handle.rccl_wait), so a neighbour of a failed rank aborts its
    own communicator and raises TimeoutError instead of waiting forever.  gloo: each halo send /
    recv is waited for at most `band_timeout` seconds, so the neighbours of a failed rank raise
    too; the failing rank also destroys the process group (releasing the peers' pending send /
    recv at once) when `abort_group` is true -- the default only for an explicitly passed
    `group`: the caller's WORLD group is left alone unless asked.  KeyboardInterrupt / SystemExit are not band failures and abort nothing.
    maps_out: a list that receives the gathered per-scale maps on `dst` (tests)."""
    import numpy as np
    dev = hasattr(frame, "data_ptr")
    if not dev:
        frame = np.asarray(frame)
        if frame.ndim == 3:
            frame = frame[None]
    else:
        if frame.dim() == 3:
            frame = frame[None]
    N, H, W, _ = frame.shape
    geoms = body.scale_geom(H, W)
    costs = [g[0] * g[1] for g in geoms]
    if split == "scales" or N != 1:
        order = list(range(len(geoms)))
        owners = [[r] for r in scale_plan(costs, world)]
    elif split == "balanced":
        order, owners, _ = split_plan(costs, world, [g[0] for g in geoms])
    else:
        raise ValueError("split must be 'balanced' or 'scales'")
    on_device = dev and dist.get_backend(group) == "nccl"
    local = frame if on_device else (frame.cpu().numpy() if dev else frame)
    if on_device and any(len(o) > 1 for o in owners):
        init_band_comm(body, group)  # collective: every rank, banded pieces or not
    pieces = {}  # (s, band) -> maps of this rank
    banded = False
    for s in order:
        if rank not in owners[s]:
            continue
        if len(owners[s]) == 1:
            m = body.scale_maps(local, s)
        else:
            b = owners[s].index(rank)
            r0, r1 = band_rows(geoms[s][0], len(owners[s]))[b]
            up = owners[s][b - 1] if b > 0 else None
            dn = owners[s][b + 1] if b + 1 < len(owners[s]) else None
            try:
                if on_device:  # RCCL: the library exchanges the halos itself, on its stream
                    body.handle.set_band_peers(up, dn)
                    m = body.band_maps(local[0], s, r0, r1, "rccl")
                    banded = True
                else:
                    m = body.band_maps(local[0], s, r0, r1, band_exchange(up, dn, group, band_timeout))
            except Exception:
                abort_band(body, group, on_device, abort_group)
                raise
        pieces[(s, owners[s].index(rank))] = m if on_device else torch.from_numpy(m)
    if banded:
        # every piece is enqueued: one bounded wait for all of this rank's halo exchanges (a
        # neighbour that failed -> the library aborts its communicator, TimeoutError here)
        try:
            body.handle.rccl_wait(band_timeout)
        except Exception:
            abort_band(body, group, on_device, abort_group)
            raise
    maps = [None] * len(geoms)
    reqs = []
    for s in range(len(geoms)):
        nb = len(owners[s])
        rows = band_rows(geoms[s][0], nb)
        parts = []
        for b, r in enumerate(owners[s]):
            if r == rank and (rank == dst or world == 1):
                parts.append(pieces[(s, b)])
            elif rank == r:
                reqs.append(dist.isend(pieces[(s, b)].contiguous(), dst, group=group))
            elif rank == dst:
                t = torch.empty((N, 57, rows[b][1] - rows[b][0], geoms[s][1]), dtype=torch.float32,
                                device=frame.device if on_device else "cpu")
                reqs.append(dist.irecv(t, r, group=group))
                parts.append(t)
        if rank == dst:
            maps[s] = parts
    for q in reqs:
        q.wait()
    if rank != dst:
        return None
    maps = [p[0] if len(p) == 1 else torch.cat(p, 2) for p in maps]
    if maps_out is not None:
        maps_out.extend(maps)
    if on_device:
        return body.post_scales(maps, H, W)
    return body.post_scales([m.numpy() for m in maps], H, W)
