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
# the 7x7 CPM convs of the bench's batch run on the LDS-window kernel (conv_win.hip)
CONV_KERNEL = "conv_win_x6" if X6 else "conv_igemm_f32"


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
    ap.add_argument("--host-steps", type=int, default=None,
                    help="steps of the host-to-host pass (pinned frames in, records out over PCIe); default --steps")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo ranks gather synthetic host records (tests the launcher and the gather)")
    return ap.parse_args()


def launch_ranks(args):
    """`bench.py --gpus N` without torchrun's environment: start N ranks (one per GPU) under
    torch.distributed.run as a child process and exit with its status.  Nothing here touches the
    GPU, so the child ranks own their devices from the start."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# frames are resident and static for the whole run, so every step may overlap its network with
# the previous step's post-processing (OPOSE_PIPELINE; BENCH_PIPELINE=0 for the serial A/B)
PIPELINE = os.environ.get("BENCH_PIPELINE", "1") != "0"
# BENCH_DEFER=1 (OPOSE_PIPELINE_DEFER): step k's post-processing is enqueued by step k+1 once its
# network reaches conv3_1, so it overlaps the middle of that network instead of its first layers.
# Measured same box: 2,065 vs 2,078 frames/s (conv1_2 1.22 -> 0.65 ms, conv3_1 0.30 -> 0.82 ms:
# the post kernels cost their CU time wherever they overlap), so the default overlaps from the start
DEFER = PIPELINE and os.environ.get("BENCH_DEFER", "0") != "0"


def pmc_traffic():
    """HBM bytes per 7x7-conv launch from the committed rocprofv3 PMC summary (separate
    --pmc passes of this same bench; scripts/gpu_profile.sh + scripts/pmc_summary.py)."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return None
    # the 7x7 class: conv_win_x6<128, 256, 7, WMAX, stages> (one instantiation at the bench's
    # shape); dispatch-weighted mean over whatever 7x7 instantiations the profile holds
    tag = "<128, 256, 7," if X6 else ", true, 7, 0>"
    num = den = 0.0
    for name, v in rec.items():
        if CONV_KERNEL + "<" in name and tag in name and "hbm_bytes_per_launch" in v:
            w = v.get("trace_calls", 1) or 1
            num += w * v["hbm_bytes_per_launch"]
            den += w
    return num / den if den else None


def pmc_traffic_lib_match():
    """True when profiles/pmc_summary.json was collected from the libopose.so this run loads
    (scripts/pmc_summary.py records its md5), False when it is stale, None without a record."""
    import hashlib
    try:
        meta = json.load(open(os.path.join(REPO, "profiles", "pmc_summary.json"))).get("_meta", {})
        lib = os.environ.get("OPOSE_LIB") or os.path.join(REPO, "pytorch-openpose_amd", "lib", "libopose.so")
        return meta["libopose_md5"] == hashlib.md5(open(lib, "rb").read()).hexdigest()
    except (OSError, ValueError, KeyError):
        return None


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
LATENCY_STAGES = ("peaks_finalize", "limb_greedy", "assemble", "hand_cc")
# paf_score: one lane per (candidate pair, sample) evaluates the x8 PAF values at the final
# resize's 4 x 4 taps from a 5x5 low-res patch: dependent float32 VALU chains per
# sample, a few hundred KB of low-res PAF read per frame -- neither a byte nor a FLOP roofline
VALU_LATENCY_STAGES = ("paf_score",)


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
        elif k == "gauss_nms_resize" and v.get("flops", 0) > 0:
            # the same filter with the heat-map resize fused in (csrc/post.hip gauss_nms_resize):
            # flops recorded per launch = GAUSS_OPS_PER_PIXEL x full-resolution map pixels
            a = v["flops"] / (v["ms"] * 1e-3)
            out[k] = {"bound": "valu_f64", "achieved": round(a / 1e12, 2), "peak": PEAK_F64_OPS / 1e12,
                      "unit": "T float64 ops/s", "frac": round(a / PEAK_F64_OPS, 4)}
        elif k in VALU_LATENCY_STAGES:
            out[k] = {"bound": "valu_latency", "achieved": None, "peak": None, "unit": None, "frac": None,
                      "note": "per-sample cubic resample chains (DESIGN §4)"}
        elif k in LATENCY_STAGES or v.get("bytes", 0) <= 0:
            out[k] = {"bound": "latency", "achieved": None, "peak": None, "unit": None, "frac": None}
        else:
            a = v["bytes"] / (v["ms"] * 1e-3) / 1e9
            out[k] = {"bound": "hbm", "achieved": round(a, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                      "frac": round(a / PEAK_HBM_GBS, 4)}
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(frames_np, seconds):
    """Oracle (test infrastructure, used only as the timed CPU baseline) on whole frames.

    Three bounded legs: the headline (C2 368x656 frames at the box's CPU share of threads, over
    distinct frames), the same at 1 thread, and C1 (one 368x368 image, src/body.py on CPU)."""
    from oracle import body_post, network
    from src.weights import BENCH_OUT_SCALE
    # the box's CPU share for one GPU (OMP_NUM_THREADS is set to it there), not the whole machine
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    sd = network.seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE)

    def net_fn(x):
        p, h = network.body_forward(torch.from_numpy(x), sd)
        return p.numpy(), h.numpy()

    def timed(frames, secs, nthreads, min_frames=1):
        torch.set_num_threads(nthreads)
        t0 = time.perf_counter()
        n = 0
        while n < min_frames or time.perf_counter() - t0 < secs:
            body_post.body_infer(frames[n % len(frames)], net_fn)
            n += 1
        return n, time.perf_counter() - t0

    n, dt = timed(frames_np, seconds, threads)
    n1, dt1 = timed(frames_np, seconds / 3, 1)
    c1 = np.random.default_rng(7).integers(0, 256, (368, 368, 3), dtype=np.uint8)
    nc, dtc = timed([c1], seconds / 3, threads)
    torch.set_num_threads(threads)
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} frame(s) of 368x656 ({min(n, len(frames_np))} distinct) through oracle Body() "
                      f"(torch-CPU net + NumPy/SciPy post), {dt:.1f} s, torch threads={threads}",
            "cpu_model": cpu_model(),
            "one_thread": {"value": n1 / dt1, "unit": "frames/s", "cores": 1,
                           "sample": f"{n1} frame(s) of 368x656, {dt1:.1f} s"},
            "c1_368x368": {"value": nc / dtc, "unit": "frames/s", "cores": threads,
                           "sample": f"{nc} run(s) of one 368x368 image (C1), {dtc:.1f} s"}}


def dry_run(args, world, rank):
    """CPU rehearsal of the multi-rank bench: gloo ranks, synthetic host records encoded per
    frame, the same gather (src/dist.py) the GPU path runs over RCCL; checks frame order."""
    import torch.distributed as dist
    from src import _native
    from src.dist import gather_records
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    B, ppp, maxp = args.batch, 8, 4
    recs = []
    for f in range(B):
        fid = rank * B + f
        recs.append(_native.encode_record([[fid, 0, 1.0, 0]], [[0] + [-1] * 17 + [1.0, 1]], ppp, maxp))
    rec = torch.from_numpy(np.stack(recs))
    t0 = time.perf_counter()
    for _ in range(args.warmup + args.steps):
        out = gather_records(rec, world * B, world)
    dt = time.perf_counter() - t0
    ids = [int(_native.decode_record(r.numpy(), ppp, maxp)[1][0, 0]) for r in out]
    assert ids == list(range(world * B)), "gathered records out of frame order"
    if rank == 0:
        print(json.dumps({"metric": "frames/sec (body+PAF grouping) at 368x656", "dry_run": True,
                          "value": world * B * (args.warmup + args.steps) / dt, "unit": "frames/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "frames_total": world * B * args.steps, "gathered_frames": len(ids)}))
    if world > 1:
        dist.destroy_process_group()


def max_over_ranks(x, dev):
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def numa_info(ptr, dev):
    """NUMA node of the pinned host buffer at `ptr` (/proc/self/numa_maps) and of the GPU's PCI
    device, so that a box-dependent PCIe rate can be attributed."""
    out = {"buffer_numa": None, "gpu_numa": None}
    try:
        for line in open("/proc/self/numa_maps"):
            addr, rest = line.split(" ", 1)
            # numa_maps lists VMAs by start address only: take the last VMA starting at or below ptr
            if int(addr, 16) <= ptr:
                nodes = {k[1:]: int(v) for k, v in (f.split("=") for f in rest.split() if f[:1] == "N" and "=" in f)}
                out["buffer_numa"] = nodes or None
    except (OSError, ValueError):
        pass
    try:
        p = torch.cuda.get_device_properties(dev)
        bus = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        out["gpu_pci"] = bus
        out["gpu_numa"] = int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
    except (OSError, ValueError, AttributeError, TypeError):
        pass
    return out


def copy_rates(host, dbuf, rhost, rdev, reps=5):
    """Standalone pinned-copy rates of the host-to-host pass's own buffers (GB/s, event-timed on
    an otherwise idle stream): what one step's upload and download cost on this box's link."""
    st = torch.cuda.Stream(device=dbuf.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for name, dst, src in (("h2d", dbuf, host), ("d2h", rhost, rdev)):
        with torch.cuda.stream(st):
            dst.copy_(src, non_blocking=True)
            e0.record(st)
            for _ in range(reps):
                dst.copy_(src, non_blocking=True)
            e1.record(st)
        e1.synchronize()
        res[name + "_GBps"] = round(reps * src.numel() * src.element_size() / (e0.elapsed_time(e1) * 1e-3) / 1e9, 2)
    return res


def host_to_host(body, frames_np, steps, dev, rank, world, mode=None):
    """PCIe-inclusive rate (the reference's boundary, src/body.py:44-50): pinned host frames
    uploaded every step, records downloaded to pinned host memory every step.

    Each cross-stream wait stands for exactly one data dependency (round 6; round 5's pass had
    each upload wait for the whole previous step's post-processing and queued the download on
    the post stream, 8-11 % below the device-resident rate on the driver's boxes):
    * the upload of step k+2's frames into dbuf[k%2] runs on cps[k%2] once step k's network has
      read that buffer (Handle.signal_input -> opose_signal_input: an event behind the network
      part on its own stream, not behind the post-network kernels on the handle's stream);
    * mode "sync" (default with the pipelined overlap): the host waits for the upload's own
      event, then makes the call with wait=False (OPOSE_PIPELINE's contract: the frames are
      complete when the call is made), so no marker is recorded on a caller stream at call time.
      Streams beyond the box's hardware queues share them, and a marker queued behind the
      handle's post-processing in a shared queue held the next network back (scripts/h2h_ab.py,
      profiles/r6_h2h_*); mode "stream": the call is made on cps[k%2] (opose_wait_stream);
    * step k's records go down on a stream of their own after an event behind its post-processing
      (and the RCCL gather), so step k+1's post is not queued behind the copy; the handle's stream
      waits for that download before step k+2 rewrites rdev[k%2]."""
    mode = mode or ("sync" if PIPELINE else "stream")
    B = len(frames_np)
    host = torch.from_numpy(frames_np).pin_memory()
    rb = body.handle.record_bytes()
    dbuf = [torch.empty_like(host, device=dev) for _ in range(2)]
    rdev = [torch.empty((B, rb), dtype=torch.uint8, device=dev) for _ in range(2)]
    rhost = [torch.empty((world * B if world > 1 else B, rb), dtype=torch.uint8).pin_memory() for _ in range(2)]
    cps = [torch.cuda.Stream(device=dev) for _ in range(2)]
    dls = torch.cuda.Stream(device=dev)
    posted = [torch.cuda.Event() for _ in range(2)]
    uploaded = [torch.cuda.Event() for _ in range(2)]
    landed = [torch.cuda.Event() for _ in range(2)]
    lib_stream = body.handle.torch_stream()
    from src.dist import gather_records
    info = dict(numa_info(host.data_ptr(), dev), **copy_rates(host, dbuf[0], rhost[0][:B], rdev[0]))
    info["upload_bytes_per_step"] = host.numel()
    info["download_bytes_per_step"] = rhost[0].numel() if rank == 0 else 0
    info["mode"] = mode

    def upload(i):
        body.handle.signal_input(cps[i])  # the network that last read dbuf[i] is done with it
        with torch.cuda.stream(cps[i]):
            dbuf[i].copy_(host, non_blocking=True)
            uploaded[i].record(cps[i])

    def run(n):
        for i in range(2):
            upload(i)
        for k in range(n):
            i = k % 2
            if k >= 2:
                lib_stream.wait_event(landed[i])  # step k-2's download has read rdev[i]
            if mode == "sync":
                uploaded[i].synchronize()
                body.infer_records(dbuf[i], rdev[i], pipeline=True, wait=False)
            else:
                with torch.cuda.stream(cps[i]):  # the library waits for this buffer's upload only
                    body.infer_records(dbuf[i], rdev[i], pipeline=PIPELINE)
            with torch.cuda.stream(lib_stream):
                allrec = gather_records(rdev[i], world * B, world) if world > 1 else rdev[i]
                posted[i].record(lib_stream)
            if rank == 0:
                dls.wait_event(posted[i])
                with torch.cuda.stream(dls):
                    rhost[i].copy_(allrec, non_blocking=True)
                if world > 1:
                    allrec.record_stream(dls)
            landed[i].record(dls)
            if k + 2 < n:
                upload(i)
        body.handle.synchronize()
        torch.cuda.synchronize()

    run(2)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = max_over_ranks(dt, dev)
    return world * B * steps / dt, dt / steps * 1e3, info


def hand_c3(device, iters):
    """C3's Hand leg: Hand() (src/hand.py:25-75) on one 368x368 crop, 4 scales, host in -> host
    out; per-stage times and the conv roofline from a profiled pass of the same calls."""
    from src.hand import Hand
    from src.weights import seeded_state_dict
    hand = Hand(seeded_state_dict("hand", 0), device=device)
    crop = np.random.default_rng(5).integers(0, 256, (368, 368, 3), dtype=np.uint8)
    for _ in range(2):
        hand(crop)
    ts = []
    for _ in range(iters):
        t1 = time.perf_counter()
        hand(crop)
        ts.append(time.perf_counter() - t1)
    ms = float(np.median(ts)) * 1e3
    hand.handle.profile(1)
    hand.handle.profile_reset()
    for _ in range(3):
        hand(crop)
    prof = hand.handle.profile_read()
    hand.handle.profile(False)
    conv = {k: v for k, v in prof.items() if k.startswith("conv")}
    flops = sum(v["flops"] for v in conv.values()) / 3
    conv_ms = sum(v["ms"] for v in conv.values()) / 3
    return {"workload": "C3 Hand(): one 368x368 crop, scale_search [0.5, 1, 1.5, 2], host in -> host out",
            "latency_ms": ms, "conv_tflop_per_call": flops / 1e12,
            "conv_ms_per_call": conv_ms,
            # the four scales run in lockstep (one launch per layer covers every scale of the
            # reference's loop, src/hand.py:36-57): the rate is the call's conv FLOPs over its wall latency,
            # so the preprocessing, heat average and peak search count against it
            "conv_roofline": {"bound": "mfma", "achieved": flops / (ms * 1e-3) / 1e12, "peak": PEAK_CONV_TFLOPS,
                              "unit": "TFLOP/s", "frac": (flops / (ms * 1e-3) / 1e12) / PEAK_CONV_TFLOPS,
                              "basis": "conv FLOPs per call / host-to-host latency of the call"},
            "stage_ms_per_call": {k: round(v["ms"] / 3, 4) for k, v in sorted(prof.items())},
            "stage_roofline": stage_roofline({k: dict(v, ms=v["ms"] / 3, flops=v["flops"] / 3, bytes=v["bytes"] / 3)
                                              for k, v in prof.items()})}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, world, rank)
    # one rank per GPU; BENCH_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks
    # per GPU (device = local rank modulo the visible GPUs, records gathered through the host)
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()
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
    lib_stream = body.handle.torch_stream()
    torch.cuda.synchronize()
    from src.dist import gather_records

    def step():
        # the frames are resident and complete, and only the handle's own stream touches rec (the
        # gather below is queued on it): pipelined calls need no marker on torch's stream
        # (wait=False, include/opose.h OPOSE_PIPELINE)
        body.infer_records(frames, rec, pipeline="defer" if DEFER else PIPELINE, wait=not PIPELINE)
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
    if DEFER and world > 1:
        # each step gathered the records complete at that point (the previous step's, deferred):
        # the last step's post-processing is flushed and gathered here
        body.handle.flush()
        with torch.cuda.stream(lib_stream):
            gather_records(rec, world * B, world)
    body.handle.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    prof_timed = body.handle.profile_read()
    body.handle.profile(False)
    if world > 1:
        dt = max_over_ranks(dt, dev)
    # per-stage breakdown: separate profiled passes after the timed region, every launch
    # bracketed by events.  The reported map comes from a serial pass (no step overlap): under
    # the pipelined overlap the post-network kernels share the chip with the next network, which
    # inflates both sides' own times; the pipelined pass is reported beside it.
    prof_steps = max(2, min(args.steps, 5))

    def profiled_pass(pipelined):
        body.handle.profile(2 if args.detail else 1)
        body.handle.profile_reset()
        for _ in range(prof_steps):
            body.infer_records(frames, rec, pipeline=pipelined)
        body.handle.synchronize()
        torch.cuda.synchronize()
        p = body.handle.profile_read()
        body.handle.profile(False)
        return p

    prof_pipe = profiled_pass(PIPELINE) if PIPELINE else None
    prof = profiled_pass(False)
    if args.detail and rank == 0:
        det = sorted(((k, v) for k, v in prof.items() if k.startswith("layer/")), key=lambda kv: -kv[1]["ms"])
        for k, v in det:
            tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
            print(f"{k:70s} {v['ms'] / prof_steps:8.3f} ms/step {tf:7.1f} TF/s", file=sys.stderr)
        prof = {k: v for k, v in prof.items() if not k.startswith("layer/")}
        if prof_pipe:
            prof_pipe = {k: v for k, v in prof_pipe.items() if not k.startswith("layer/")}
    # host-to-host (PCIe-inclusive) pass: reported beside `value`, never as it
    h2h_value, h2h_ms, h2h_info = host_to_host(body, frames_np, args.host_steps or args.steps, dev, rank, world)

    c3 = hand_c3(local, args.latency_iters) if rank == 0 and args.latency_iters > 0 else None

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
                       "step_overlap": ("post-processing of step k enqueued by step k+1 once its network reaches "
                                        "conv3_1 (OPOSE_PIPELINE_DEFER)") if DEFER else
                                       "network of step k+1 overlaps post-processing of step k (OPOSE_PIPELINE)"
                       if PIPELINE else "none"},
            "frames_total": frames_total,
            "value_host_to_host": h2h_value,
            "value_host_to_host_ratio": h2h_value / (frames_total / dt),
            "host_to_host": dict(h2h_info, ms_per_step=h2h_ms, basis=(
                "pinned host frames uploaded each step on per-buffer copy streams once the previous "
                "network has read the buffer (opose_signal_input), records (and the RCCL gather when "
                "n_gpus > 1) downloaded to pinned host memory each step on a stream of their own; "
                "reference boundary src/body.py:44-50")),
            "roofline": {"bound": "mfma", "kernel": CONV_KERNEL + " (7x7 CPM stages)",
                         "achieved": achieved, "peak": PEAK_CONV_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_CONV_TFLOPS,
                         "peak_basis": ("dense bf16 MFMA peak 2500 / 6 piece products per fp32-equivalent "
                                        "multiply-add (algorithmic fp32 FLOPs)") if X6 else "fp32 MFMA peak",
                         "per_launch_flops": c7["flops"] / max(1, c7["count"]),
                         "mean_launch_ms": c7["ms"] / max(1, c7["count"]), "traffic": pmc_traffic(),
                         "traffic_unit": "bytes per launch (FETCH_SIZE*2 + WRITE_SIZE)*1KiB, profiles/pmc_summary.json",
                         "traffic_same_library": pmc_traffic_lib_match()},
            "network_tflops": net_flops / (net_ms * 1e-3) / 1e12 if net_ms > 0 else 0.0,
            "stage_breakdown": f"separate profiled passes of {prof_steps} steps after the timed region (events "
                               "around every launch): stage_ms_per_step / stage_roofline from a serial pass (no "
                               "step overlap), *_pipelined from a pass with the bench's overlap; the timed region "
                               "brackets only the 7x7 convs",
            "stage_ms_per_step": stage_ms,
            "stage_roofline": stage_roofline(prof),
            "stage_ms_per_step_pipelined": ({k: round(v["ms"] / prof_steps, 4) for k, v in sorted(prof_pipe.items())}
                                            if prof_pipe else None),
            "stage_roofline_pipelined": stage_roofline(prof_pipe) if prof_pipe else None,
            "latency_ms_single_frame": (float(np.median(lat)) * 1e3) if lat else None,
            "c3_hand": c3,
            "frames_status_nonzero": int((statuses != 0).sum()),
            "mean_peaks_per_frame": float(counts[:, 0].mean()),
            "mean_people_per_frame": float(counts[:, 1].mean()),
        }
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(frames_np[:8], args.cpu_seconds)
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
