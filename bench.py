"""Benchmark: Body() frames/s at 368x656 (BASELINE.json metric), 1..8 MI355X, one process per GPU.

Workload (a "step"): one video batch of B synthetic 368x656 uint8 BGR frames per GPU, already
resident in HBM, through the full Body() path on the GPU — uint8 cubic resize/pad/normalise,
the 92-conv VGG-19/CPM network, x8 cubic upsample + resize, Gaussian peak NMS, PAF scoring,
greedy matching, person assembly — producing one fixed-size keypoint record per frame; with
N > 1 ranks the records are gathered across ranks with RCCL (all_gather over xGMI) each step.
Frames shard across ranks (weak scaling: B frames per GPU).  Weights are seeded synthetic
(real .pth files are unavailable offline).

Prints ONE JSON line on rank 0 (driver contract) including:
* roofline: the 7x7-conv kernel class (68 % of network FLOPs), algorithmic (fp32) FLOPs per
  launch / mean launch time from HIP events recorded around those launches (on the stream
  each runs on) inside the timed region -- only those: events around every launch cost ~3 %
  of the step -- against the ceiling of the kernel that ran: the split-bf16 conv (default; six
  bf16 MFMA piece products per fp32 multiply-add -> bf16 peak / 6) or the fp32 MFMA conv
  (OPOSE_CONV=f32 -> fp32 MFMA peak);
* stage_ms_per_step / stage_roofline: a separate profiled pass after the timed region;
* steps overlap (OPOSE_PIPELINE): frames are resident and static, so step k+1's network runs
  on the library's second stream while step k's post-processing finishes (BENCH_PIPELINE=0:
  serial);
* cpu_baseline: the oracle (torch-CPU conv graph + NumPy/SciPy post-processing, proven
  identical to the reference on the golden fixtures) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "pytorch-openpose_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

H, W = 368, 656
PEAK_FP32_TFLOPS = 157.3  # MI355X fp32 matrix peak (MI355X_MICROARCH.md: spec 157.3, 155 measured)
PEAK_BF16_TFLOPS = 2500.0  # dense bf16 MFMA peak (no sparsity)
# The network runs on the split-bf16 conv kernel (csrc/conv_x6.hip) unless OPOSE_CONV=f32: one
# fp32-equivalent multiply-add = 6 bf16 MFMA piece products, so its ceiling in fp32-equivalent
# (algorithmic) FLOP/s is the bf16 peak / 6.
X6 = os.environ.get("OPOSE_CONV", "x6") != "f32"
PEAK_CONV_TFLOPS = PEAK_BF16_TFLOPS / 6 if X6 else PEAK_FP32_TFLOPS
CONV_KERNEL = "conv_x6" if X6 else "conv_igemm_f32"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--latency-iters", type=int, default=10)
    ap.add_argument("--detail", action="store_true", help="per-layer kernel times to stderr")
    return ap.parse_args()


# frames are resident and static for the whole run, so every step may overlap its network with
# the previous step's post-processing (OPOSE_PIPELINE; BENCH_PIPELINE=0 for the serial A/B)
PIPELINE = os.environ.get("BENCH_PIPELINE", "1") != "0"


def pmc_traffic():
    """HBM bytes per 7x7-conv launch from the committed rocprofv3 PMC summary (separate
    --pmc passes of this same bench; scripts/gpu_profile.sh + scripts/pmc_summary.py)."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return None
    # the 7x7 class runs as one or two kernel instantiations (conv_x6<MT, PT, false, 7, MODE>,
    # 128x256 for the grouped 128-channel convs, 256x128 for Mconv1); dispatch-weighted mean
    tag = ", false, 7," if X6 else ", true, 7, 0>"
    num = den = 0.0
    for name, v in rec.items():
        if CONV_KERNEL + "<" in name and tag in name and "hbm_bytes_per_launch" in v:
            w = v.get("trace_calls", 1) or 1
            num += w * v["hbm_bytes_per_launch"]
            den += w
    return num / den if den else None


# per-stage roofline (north_star: "achieved fraction of MFMA/HBM roofline reported per stage"):
# conv classes against the fp32 matrix peak; streaming kernels against HBM with the algorithmic
# bytes the engine records per launch (csrc/engine.cpp prof_begin); the pair-scoring, matching
# and assembly kernels are latency bound (a few hundred candidates per frame) -> no roofline.
PEAK_HBM_GBS = 8000.0
# gauss_nms is float64-VALU bound, not HBM bound: the reference's scipy filter is 2 separable
# 25-tap passes per pixel, 37 float64 operations each (12 symmetric pair adds, 13 multiplies,
# 12 accumulates; no FMA, scipy's order), on each of the 18 full-resolution part maps.  Peak:
# MI355X float64 vector rate, 78.6 TFLOP/s counting an FMA as 2 -> 39.3 T non-FMA ops/s (AMD
# spec figure; the tile skip of all-below-threshold footprints can make the algorithmic rate
# exceed it on sparse maps).
GAUSS_OPS_PER_PIXEL = 2 * 37
PEAK_F64_OPS = 39.3e12
LATENCY_STAGES = ("peaks_finalize", "paf_score", "limb_greedy", "assemble", "hand_cc")


def stage_roofline(prof):
    out = {}
    for k, v in sorted(prof.items()):
        if v["ms"] <= 0:
            continue
        if k.startswith("conv"):
            a = v["flops"] / (v["ms"] * 1e-3) / 1e12
            out[k] = {"bound": "mfma", "achieved": round(a, 2), "peak": round(PEAK_CONV_TFLOPS, 1),
                      "unit": "TFLOP/s", "frac": round(a / PEAK_CONV_TFLOPS, 4)}
        elif k == "gauss_nms" and v.get("bytes", 0) > 0:
            # bytes recorded per launch = 4 (f32 map) or 8 (f64 average) per map pixel
            px = v["bytes"] / (4 if v.get("f32", True) else 8)
            a = px * GAUSS_OPS_PER_PIXEL / (v["ms"] * 1e-3)
            out[k] = {"bound": "valu_f64", "achieved": round(a / 1e12, 2), "peak": PEAK_F64_OPS / 1e12,
                      "unit": "T float64 ops/s", "frac": round(a / PEAK_F64_OPS, 4)}
        elif k in LATENCY_STAGES or v.get("bytes", 0) <= 0:
            out[k] = {"bound": "latency", "achieved": None, "peak": None, "unit": None, "frac": None}
        else:
            a = v["bytes"] / (v["ms"] * 1e-3) / 1e9
            out[k] = {"bound": "hbm", "achieved": round(a, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                      "frac": round(a / PEAK_HBM_GBS, 4)}
    return out


def cpu_baseline(frames_np, seconds):
    """Oracle (test infrastructure, used only as the timed CPU baseline) on whole frames."""
    from oracle import body_post, network
    from src.weights import BENCH_OUT_SCALE
    # the box's CPU share for one GPU (OMP_NUM_THREADS is set to it there), not the whole machine
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sd = network.seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE)

    def net_fn(x):
        p, h = network.body_forward(torch.from_numpy(x), sd)
        return p.numpy(), h.numpy()

    t0 = time.perf_counter()
    n = 0
    while True:
        body_post.body_infer(frames_np[n % len(frames_np)], net_fn)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} frame(s) of 368x656 through oracle Body() (torch-CPU net + NumPy/SciPy post), "
                      f"{dt:.1f} s, torch threads={threads}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from src.body import Body
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict

    body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE), device=local)
    B = args.batch
    rng = np.random.default_rng(1 + rank)
    frames_np = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    frames = torch.from_numpy(frames_np).to(dev)
    rb = body.handle.record_bytes()
    rec = torch.empty((B, rb), dtype=torch.uint8, device=dev)
    lib_stream = torch.cuda.ExternalStream(body.handle.stream(), device=dev)
    from src.dist import gather_records

    def step():
        body.infer_records(frames, rec, pipeline=PIPELINE)
        if world > 1:
            # RCCL all_gather of the per-frame keypoint records, ordered after the library's
            # kernels on its stream (src/dist.py)
            with torch.cuda.stream(lib_stream):
                gather_records(rec, world * B, world)

    for _ in range(args.warmup):
        step()
    body.handle.synchronize()
    torch.cuda.synchronize()
    # sanity on the warm output (outside the timed region)
    statuses = rec.view(torch.int32)[:, 0].cpu().numpy()
    counts = rec.view(torch.int32)[:, 1:3].cpu().numpy()

    # timed region: HIP events only around the 7x7 conv launches (the roofline's kernel class,
    # on the stream each launch runs on); every-launch events cost ~3 % of the step
    if not os.environ.get("BENCH_NO_PROF"):
        body.handle.profile(3)
    body.handle.profile_reset()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    body.handle.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    prof_timed = body.handle.profile_read()
    body.handle.profile(False)
    # per-stage breakdown: a separate profiled pass after the timed region, every launch
    # bracketed by events (the pipelined overlap inflates the post-network kernels' own times)
    prof_steps = max(2, min(args.steps, 5))
    body.handle.profile(2 if args.detail else 1)
    body.handle.profile_reset()
    for _ in range(prof_steps):
        step()
    body.handle.synchronize()
    torch.cuda.synchronize()
    prof = body.handle.profile_read()
    body.handle.profile(False)
    if args.detail and rank == 0:
        det = sorted(((k, v) for k, v in prof.items() if k.startswith("layer/")), key=lambda kv: -kv[1]["ms"])
        for k, v in det:
            tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
            print(f"{k:70s} {v['ms'] / prof_steps:8.3f} ms/step {tf:7.1f} TF/s", file=sys.stderr)
        prof = {k: v for k, v in prof.items() if not k.startswith("layer/")}
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())

    # single-frame latency (C2: one frame, host in -> host out through Body.__call__)
    lat = []
    if rank == 0 and args.latency_iters > 0:
        one = frames_np[0]
        body(one)
        for _ in range(args.latency_iters):
            t1 = time.perf_counter()
            body(one)
            lat.append(time.perf_counter() - t1)

    if rank == 0:
        frames_total = world * B * args.steps
        c7 = prof_timed.get("conv7x7", {"count": 0, "ms": 0.0, "flops": 0.0})
        conv_all = {k: v for k, v in prof.items() if k.startswith("conv")}
        achieved = (c7["flops"] / (c7["ms"] * 1e-3) / 1e12) if c7["ms"] > 0 else 0.0
        stage_ms = {k: round(v["ms"] / prof_steps, 4) for k, v in sorted(prof.items())}
        net_flops = sum(v["flops"] for v in conv_all.values())
        net_ms = sum(v["ms"] for v in conv_all.values())
        out = {
            "metric": "frames/sec (body+PAF grouping) at 368x656",
            "value": frames_total / dt,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "conv_arithmetic": ("fp32-accurate split-bf16 MFMA: x = x0+x1+x2 (bf16, exact), 6 piece products, "
                                "fp32 accumulate (tests/test_gpu_x6.py)") if X6 else "fp32 MFMA",
            "data": "synthetic (uniform uint8 frames, seeded He-normal weights; real weights unavailable offline)",
            "config": {"workload": f"C2/C4: Body() on 368x656 frames, {B} frames per GPU per step, "
                                   f"RCCL all_gather of per-frame keypoint records when n_gpus > 1",
                       "frame": [H, W], "frames_per_gpu_per_step": B, "scale_search": [0.5],
                       "net_input": [184, 328], "parallelism": f"frame-sharded dp{world}",
                       "step_overlap": "network of step k+1 overlaps post-processing of step k (OPOSE_PIPELINE)"
                       if PIPELINE else "none"},
            "roofline": {"bound": "mfma", "kernel": CONV_KERNEL + " (7x7 CPM stages)",
                         "achieved": achieved, "peak": PEAK_CONV_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_CONV_TFLOPS,
                         "peak_basis": ("dense bf16 MFMA peak 2500 / 6 piece products per fp32-equivalent "
                                        "multiply-add (algorithmic fp32 FLOPs)") if X6 else "fp32 MFMA peak",
                         "per_launch_flops": c7["flops"] / max(1, c7["count"]),
                         "mean_launch_ms": c7["ms"] / max(1, c7["count"]), "traffic": pmc_traffic(),
                         "traffic_unit": "bytes per launch (FETCH_SIZE*2 + WRITE_SIZE)*1KiB, profiles/pmc_summary.json"},
            "network_tflops": net_flops / (net_ms * 1e-3) / 1e12 if net_ms > 0 else 0.0,
            "stage_breakdown": f"separate profiled pass of {prof_steps} steps after the timed region "
                               "(events around every launch); the timed region brackets only the 7x7 convs",
            "stage_ms_per_step": stage_ms,
            "stage_roofline": stage_roofline(prof),
            "latency_ms_single_frame": (float(np.median(lat)) * 1e3) if lat else None,
            "frames_status_nonzero": int((statuses != 0).sum()),
            "mean_peaks_per_frame": float(counts[:, 0].mean()),
            "mean_people_per_frame": float(counts[:, 1].mean()),
        }
        if not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(frames_np[:2], args.cpu_seconds)
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
