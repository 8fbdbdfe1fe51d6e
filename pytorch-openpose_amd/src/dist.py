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
    backend = dist.get_backend(group)
    if backend == "nccl":
        out = torch.empty((world * cap, rb), dtype=rec.dtype, device=rec.device)
        dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
        parts = list(out.view(world, cap, rb))
    else:
        parts = [torch.empty_like(rec) for _ in range(world)]
        dist.all_gather(parts, rec.contiguous(), group=group)
    return torch.cat([p[:hi - lo] for p, (lo, hi) in zip(parts, per)], 0)
