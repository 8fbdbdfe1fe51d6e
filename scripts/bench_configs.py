"""Secondary measurements for BASELINE.json configs C2, C3 and C5 on one MI355X (bench.py is
the driver's C2/C4 throughput line).  Prints one JSON object; synthetic frames and seeded
weights (BENCH_OUT_SCALE calibration for the body net) as in bench.py.

C2  Body() on one 368x656 frame: host-in/host-out latency (PCIe included) and the
    device-resident batch-1 path (infer_records).
C3  Body()+Hand() per frame (src.pipeline.motion_data_every_frame, mode "bodyhand": hands of
    the selected person, 368x368-class crops, 4 hand scales) and Hand() alone on a 368x368 crop.
C5  1920x1080 frames with scale_search [0.5, 1.0, 1.5, 2.0] (averaged heat maps), device
    resident batches -> frames/s per GPU (C5 shards frames over 8 GPUs like C4).
f2  motion-matrix extraction (src/motion.py) over 256 decoded 368x656 frames, body and
    bodyhand modes: the GPU ingest against host batches.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
from src.body import Body  # noqa: E402
from src.hand import Hand  # noqa: E402
from src.pipeline import motion_data_every_frame  # noqa: E402
from src.weights import BENCH_OUT_SCALE, c5_out_scale, seeded_state_dict  # noqa: E402


def timed(fn, iters, warm=2):
    """Median wall time of fn() with the device drained after each call (device-tensor entry
    points return asynchronously, ordered on torch's current stream)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    return float(np.median(t)) * 1e3


SKIP = set(filter(None, os.environ.get("BC_SKIP", "").split(",")))  # stages to leave out (diagnosis)


def main():
    rng = np.random.default_rng(3)
    out = {}
    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
    hand = Hand(seeded_state_dict("hand", 0))
    img = rng.integers(0, 256, (368, 656, 3), dtype=np.uint8)

    # C2
    out["C2_body_latency_ms"] = timed(lambda: body(img), 20)
    dev = torch.device("cuda", 0)
    f1 = torch.from_numpy(img[None].copy()).to(dev)
    rec = torch.empty((1, body.handle.record_bytes()), dtype=torch.uint8, device=dev)

    def dev1():
        body.infer_records(f1, rec)
        body.handle.synchronize()
    out["C2_body_device_batch1_ms"] = timed(dev1, 20)

    # C3
    crop = rng.integers(0, 256, (368, 368, 3), dtype=np.uint8)
    if "c3" in SKIP:
        out["C3_hand_latency_ms"] = timed(lambda: hand(crop), 10)
        return c5(out, rng, dev)
    out["C3_hand_latency_ms"] = timed(lambda: hand(crop), 10)
    n_hands = []

    def pipe():
        pose = motion_data_every_frame(body, hand, img, "bodyhand")
        n_hands.append(int((pose[18:39, 2] > 0).any()) + int((pose[39:60, 2] > 0).any()))
    out["C3_bodyhand_frame_ms"] = timed(pipe, 10)
    out["C3_note"] = "hands found per frame (median over runs): %d" % int(np.median(n_hands))
    crop2 = rng.integers(0, 256, (256, 256, 3), dtype=np.uint8)
    out["C3_hand_two_crops_sequential_ms"] = timed(lambda: (hand(crop), hand(crop2)), 5)
    out["C3_hand_two_crops_batched_ms"] = timed(lambda: hand.batch_crops([crop, crop2]), 5)
    from src.pipeline import motion_data_frames
    T = 8
    vid = rng.integers(0, 256, (T, 368, 656, 3), dtype=np.uint8)
    hands = []

    def pipe_batch():
        poses = motion_data_frames(body, hand, vid)
        hands.append(int((poses[:, 18:39, 2] > 0).any(1).sum() + (poses[:, 39:60, 2] > 0).any(1).sum()))
    ms = timed(pipe_batch, 3, warm=1)
    out["C3_bodyhand_batched_8frames_ms_per_frame"] = ms / T
    out["C3_bodyhand_batched_hands_per_8frames"] = int(np.median(hands))

    # f2: motion-matrix extraction over a decoded video (src/motion.py extract_motion_data:
    # pinned double-buffered uploads, pipelined Body, poses of batch k-1 decoded while batch k
    # runs), frames already decoded in host memory (no video decoder in this image)
    from src.motion import extract_motion_data
    video = rng.integers(0, 256, (256, 368, 656, 3), dtype=np.uint8)
    for mode in ("body", "bodyhand"):
        extract_motion_data(video[:64], body, hand, mode=mode, batch=32)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        extract_motion_data(video, body, hand, mode=mode, batch=32)
        torch.cuda.synchronize()
        out[f"f2_motion_{mode}_frames_per_s"] = len(video) / (time.perf_counter() - t0)
        t0 = time.perf_counter()
        extract_motion_data(video[:96], body, hand, mode=mode, batch=32, device=False)
        out[f"f2_motion_{mode}_host_batches_frames_per_s"] = 96 / (time.perf_counter() - t0)

    # fast mode (srcmx/Batch_model.py Batch_body) on the C4 batch: 32 frames 368x656 per GPU
    from src.batch_model import Batch_body
    bb = Batch_body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE), peaks_per_part=256, max_people=128)
    f32 = torch.from_numpy(rng.integers(0, 256, (32, 368, 656, 3), dtype=np.uint8)).to(dev)
    recb = torch.empty((32, bb.handle.record_bytes()), dtype=torch.uint8, device=dev)

    def stepb():
        bb.infer_records(f32, recb)
        bb.handle.synchronize()
    ms = timed(stepb, 5, warm=2)
    out["fast_mode_batch_body_frames_per_s"] = 32 / (ms * 1e-3)
    out["fast_mode_status_nonzero"] = int((recb.view(torch.int32)[:, 0] != 0).sum().item())

    return c5(out, rng, dev)


def c5(out, rng, dev):
    # C5
    # C5_OUT_SCALE: the heat conv's per-channel affine measured at 1080p / 4 scales (~190 peaks,
    # ~10 people per frame; src/weights.py).  The network (value independent) is >97 % of this
    # config's time.
    cal = c5_out_scale()
    body5 = Body(seeded_state_dict("body", 0, out_scale=cal), scale_search=(0.5, 1.0, 1.5, 2.0))
    B = 4
    f5 = torch.from_numpy(rng.integers(0, 256, (B, 1080, 1920, 3), dtype=np.uint8)).to(dev)
    rec5 = torch.empty((B, body5.handle.record_bytes()), dtype=torch.uint8, device=dev)

    def step5():
        body5.infer_records(f5, rec5)
        body5.handle.synchronize()
    ms = timed(step5, 5, warm=1)
    out["C5_1080p_4scale_batch"] = B
    out["C5_1080p_4scale_ms_per_batch"] = ms
    out["C5_1080p_4scale_frames_per_s_per_gpu"] = B / (ms * 1e-3)
    # the same batches back to back with OPOSE_PIPELINE (each batch's post-processing overlaps
    # the next batch's network; the scales of a batch run concurrently on per-scale streams
    # forked from and joined into the network stream) -- the video-throughput reading of C5
    recs5 = [torch.empty_like(rec5) for _ in range(2)]
    for w in range(2):
        body5.infer_records(f5, recs5[w], pipeline=True)
    body5.handle.synchronize()
    T5 = 6
    t0 = time.perf_counter()
    for it in range(T5):
        body5.infer_records(f5, recs5[it % 2], pipeline=True)
    body5.handle.synchronize()
    torch.cuda.synchronize()
    out["C5_1080p_4scale_pipelined_frames_per_s_per_gpu"] = B * T5 / (time.perf_counter() - t0)
    st = rec5.view(torch.int32)[:, 0].cpu().numpy()
    out["C5_status_nonzero"] = int((st != 0).sum())
    out["C5_mean_peaks_people"] = rec5.view(torch.int32)[:, 1:3].float().mean(0).cpu().tolist()

    # the same C5 work with one network per scale on concurrent streams (OPOSE_LOCKSTEP=0; the
    # default runs the four scales' networks in lockstep, one conv launch per layer, DESIGN §4.3;
    # both give the same maps bit for bit)
    os.environ["OPOSE_LOCKSTEP"] = "0"
    try:
        body5l = Body(seeded_state_dict("body", 0, out_scale=cal), scale_search=(0.5, 1.0, 1.5, 2.0))
    finally:
        del os.environ["OPOSE_LOCKSTEP"]

    def step5l():
        body5l.infer_records(f5, rec5)
        body5l.handle.synchronize()
    ms = timed(step5l, 5, warm=1)
    out["C5_per_scale_streams_frames_per_s_per_gpu"] = B / (ms * 1e-3)

    def one5l():
        body5l.infer_records(f5[:1].contiguous(), rec5[:1])
        body5l.handle.synchronize()
    out["C5_per_scale_streams_single_frame_latency_ms"] = timed(one5l, 10, warm=2)
    del body5l

    # C5 single-frame latency: all four scales on one GPU vs the scale-sharded split
    # (src.dist.body_scale_sharded): per-scale network time and the multi-scale post on the
    # gathered low-res maps, measured here; the sharded latency is max over ranks of its scales'
    # network time + the gather of <= 3.4 MB low-res maps per scale + the post on rank 0.
    from src.dist import scale_plan
    f1 = f5[:1].contiguous()
    rec1 = rec5[:1]

    def one5():
        body5.infer_records(f1, rec1)
        body5.handle.synchronize()
    out["C5_single_frame_latency_ms"] = timed(one5, 10, warm=2)
    geoms = body5.scale_geom(1080, 1920)
    maps = [body5.scale_maps(f1, s) for s in range(len(geoms))]
    net_ms = [timed(lambda s=s: body5.scale_maps(f1, s, out=maps[s]), 10, warm=1) for s in range(len(geoms))]
    post_ms = timed(lambda: body5.post_scales(maps, 1080, 1920), 10, warm=1)
    out["C5_scale_net_ms"] = net_ms
    out["C5_scale_lowres_mb"] = [4 * 57 * g[0] * g[1] / 1e6 for g in geoms]
    out["C5_post_scales_ms"] = post_ms
    for world in (2, 4):
        own = scale_plan([g[0] * g[1] for g in geoms], world)
        load = [sum(t for t, r in zip(net_ms, own) if r == k) for k in range(world)]
        out["C5_sharded_w%d_model_ms_excl_gather" % world] = max(load) + post_ms
    # balanced split (src.dist.split_plan): the largest scales cut into row bands.  A band's time
    # is measured here with the library's own RCCL exchange on a one-rank communicator whose
    # neighbours are the rank itself (the 27 pack / send / recv / unpack steps per band run as on
    # a node; the bytes move within the GPU); the xGMI transfer is added as 27 x (10 us + 2 x the
    # halo bytes at 100 GB/s), the halo bytes being 3 rows x 256 channels x 6 B x (wl + 3).
    from src.dist import band_rows, split_plan
    body5.handle.rccl_init(body5.handle.rccl_unique_id(), 0, 1)
    body5.handle.set_band_peers(0, 0)
    costs, hls = [g[0] * g[1] for g in geoms], [g[0] for g in geoms]
    band_ms = {}
    for world in (2, 4, 8):
        order, owners, _ = split_plan(costs, world, hls)
        load = [0.0] * world
        for s in order:
            nb = len(owners[s])
            if nb == 1:
                t = net_ms[s]
            else:
                if (s, nb) not in band_ms:
                    xfer = 27 * (10e-3 + 2 * 3 * 256 * 6 * (geoms[s][1] + 3) / 100e9 * 1e3)
                    band_ms[(s, nb)] = max(
                        timed(lambda r=r: body5.band_maps(f1, s, r[0], r[1], "rccl"), 5, warm=1)
                        for r in band_rows(geoms[s][0], nb)) + xfer
                t = band_ms[(s, nb)]
            for r in owners[s]:
                load[r] += t
        out["C5_balanced_w%d_owners" % world] = owners
        out["C5_balanced_w%d_model_ms_excl_gather" % world] = max(load) + post_ms
    out["C5_band_ms"] = {"%d/%d" % k: v for k, v in band_ms.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
