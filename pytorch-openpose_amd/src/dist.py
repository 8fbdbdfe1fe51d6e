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


def body_scale_sharded(body, frame, rank: int, world: int, dst: int = 0, group=None):
    """Body(frame) with its scales split across ranks; returns [(candidate, subset)] on `dst`
    (None elsewhere).  frame: uint8 [H,W,3] / [1,H,W,3] numpy, or a torch cuda tensor (then the
    maps stay on the device and travel over RCCL; with gloo they go through host memory).

    Result: identical to body.batch(frame) on one GPU — each scale's network runs with the same
    shapes (so the same kernels and summation order) and the post path is the same code."""
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
    owner = scale_plan([g[0] * g[1] for g in geoms], world)
    on_device = dev and dist.get_backend(group) == "nccl"
    maps = [None] * len(geoms)
    for s, r in enumerate(owner):
        if r != rank:
            continue
        if on_device:
            maps[s] = body.scale_maps(frame, s)
        else:
            host = body.scale_maps(frame.cpu().numpy() if dev else frame, s)
            maps[s] = torch.from_numpy(host)
    if world > 1:
        reqs = []
        for s, r in enumerate(owner):
            if r == dst and rank == dst:
                continue
            if rank == r:
                reqs.append(dist.isend(maps[s].contiguous(), dst, group=group))
            elif rank == dst:
                hl, wl = geoms[s][0], geoms[s][1]
                maps[s] = torch.empty((N, 57, hl, wl), dtype=torch.float32,
                                      device=frame.device if on_device else "cpu")
                reqs.append(dist.irecv(maps[s], r, group=group))
        for q in reqs:
            q.wait()
    if rank != dst:
        return None
    if on_device:
        return body.post_scales(maps, H, W)
    return body.post_scales([m.numpy() for m in maps], H, W)
