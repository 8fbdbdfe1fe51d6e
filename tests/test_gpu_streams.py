"""GPU: ordering against torch's current stream (opose_wait_stream / opose_signal_stream) and the
host-copy span of strided views.

* Inputs produced asynchronously on a torch side stream (behind a spin kernel) are read only
  after that stream gets there: Body.infer_records, the model forward on a `.half()` input.
* A bottom-right crop view that ends exactly at a PROT_NONE guard page: the host -> device
  staging copy must not read past the view's last pixel (include/opose.h host pointers)."""
import ctypes
import mmap
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def body():
    from src.body import Body
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    return Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))


def _same(got, exp):
    assert len(got) == len(exp)
    for (c, s), (ec, es) in zip(got, exp):
        assert np.array_equal(c, ec) and np.array_equal(s, es)


def test_infer_records_waits_for_torch_stream(body):
    frames = np.random.default_rng(5).integers(0, 256, (2, 184, 328, 3), dtype=np.uint8)
    exp = body.batch(frames)
    src = torch.from_numpy(frames).cuda()
    dst = torch.zeros_like(src)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.cuda._sleep(50_000_000)  # the frames land only after this spin
        dst.copy_(src)
        rec = body.infer_records(dst)
        got = body.decode_records(rec)
    _same(got, exp)
    with torch.cuda.stream(side):  # pipelined: the network stream waits too
        torch.cuda._sleep(50_000_000)
        dst.zero_()
        dst.copy_(src)
        rec = body.infer_records(dst, pipeline=True)
    _same(body.decode_records(rec), exp)


def test_producer_on_the_handle_stream_then_pipelined(body):
    """Frames written on the handle's own stream (a caller that orders itself on
    handle.torch_stream(), as bench.py's gather does), then two back-to-back pipelined calls: the
    pipelined network stream must wait for that stream too, not only for torch's other streams."""
    frames = np.random.default_rng(12).integers(0, 256, (2, 184, 328, 3), dtype=np.uint8)
    exp = body.batch(frames)
    src = torch.from_numpy(frames).cuda()
    dst = torch.zeros_like(src)
    torch.cuda.synchronize()
    for _ in range(2):  # network stream created; back-to-back pipelined calls (no main_dirty)
        body.infer_records(dst, pipeline=True)
    body.handle.synchronize()
    with torch.cuda.stream(body.handle.torch_stream()):
        torch.cuda._sleep(50_000_000)  # the frames land only after this spin
        dst.zero_()
        dst.copy_(src)
        r1 = body.infer_records(dst, pipeline=True)
        r2 = body.infer_records(dst, pipeline=True)
    _same(body.decode_records(r1), exp)
    _same(body.decode_records(r2), exp)


def test_signal_input_orders_the_next_upload(body):
    """bench.py's host-to-host pattern (opose_signal_input): a pipelined call whose network is held
    back (its input stream spins first), then the next batch written into the SAME frame buffer on
    another stream ordered only by Handle.signal_input, then a second call on that stream.  The
    overwrite must wait for the first call's network to have read the buffer: each call's records
    are its own batch's."""
    fx = np.random.default_rng(21).integers(0, 256, (2, 184, 328, 3), dtype=np.uint8)
    fy = np.random.default_rng(22).integers(0, 256, (2, 184, 328, 3), dtype=np.uint8)
    ex, ey = body.batch(fx), body.batch(fy)
    sx, sy = torch.from_numpy(fx).cuda(), torch.from_numpy(fy).cuda()
    dst = sx.clone()
    rb = body.handle.record_bytes()
    r1 = torch.empty((2, rb), dtype=torch.uint8, device="cuda")
    r2 = torch.empty_like(r1)
    for _ in range(2):  # the network stream exists; back-to-back pipelined calls
        body.infer_records(dst, r1, pipeline=True)
    body.handle.synchronize()
    torch.cuda.synchronize()
    side, up = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.cuda._sleep(50_000_000)  # the first call's network starts only after this spin
        body.infer_records(dst, r1, pipeline=True)
    body.handle.signal_input(up)
    with torch.cuda.stream(up):
        dst.copy_(sy)  # must not land before the first network has read dst
        body.infer_records(dst, r2, pipeline=True)
    body.handle.synchronize()
    torch.cuda.synchronize()
    _same(body.decode_records(r1), ex)
    _same(body.decode_records(r2), ey)


def test_pipelined_multiscale_matches_serial():
    """Pipelined two-scale batches (each batch's scales run concurrently on per-scale streams
    forked from the network stream, its post-processing under the next batch's networks),
    alternating inputs and record buffers, against the serial host path."""
    from src.body import Body
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    body2 = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE), scale_search=(0.5, 1.0))
    rng = np.random.default_rng(13)
    batches = [rng.integers(0, 256, (2, 120, 200, 3), dtype=np.uint8) for _ in range(2)]
    exp = [body2.batch(b) for b in batches]
    dev = [torch.from_numpy(b).cuda() for b in batches]
    rb = body2.handle.record_bytes()
    recs = [torch.empty((2, rb), dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    for k in range(6):
        body2.infer_records(dev[k % 2], recs[k % 2], pipeline=True)
        if k % 2:
            body2.handle.synchronize()
            for i in range(2):
                _same(body2.decode_records(recs[i]), exp[i])


def test_hand_scale_streams_bit_identical():
    """Hand() with one network per scale (OPOSE_LOCKSTEP=0): the scales' networks on concurrent
    streams (default) and one after another (OPOSE_SCALE_STREAMS=0, read when the handle is
    created) give identical peaks -- and equal the default lockstep pyramid's."""
    from src.hand import Hand
    from src.weights import seeded_state_dict
    crop = np.random.default_rng(14).integers(0, 256, (150, 150, 3), dtype=np.uint8)
    sd = seeded_state_dict("hand", 0)

    def make(env):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            return Hand(sd)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    concurrent = make({"OPOSE_LOCKSTEP": "0"})(crop)
    serial = make({"OPOSE_LOCKSTEP": "0", "OPOSE_SCALE_STREAMS": "0"})(crop)
    lockstep = Hand(sd)(crop)
    for b in (serial, lockstep):
        assert concurrent.dtype == b.dtype and np.array_equal(concurrent, b)


def test_graph_replay_equals_eager():
    """Body() / Hand() calls replay a captured hipGraph from the third call with the same shapes
    on; a handle created with OPOSE_NO_GRAPH=1 runs every call eagerly.  Replays (a two-scale
    lockstep pyramid with its slab schedules, and a hand pyramid) equal the eager calls exactly."""
    from src.body import Body
    from src.hand import Hand
    from src.weights import seeded_state_dict
    rng = np.random.default_rng(15)
    img = rng.integers(0, 256, (184, 232, 3), dtype=np.uint8)
    crop = rng.integers(0, 256, (128, 128, 3), dtype=np.uint8)
    bsd, hsd = seeded_state_dict("body", 0), seeded_state_dict("hand", 0)

    def make(env):
        old = os.environ.get("OPOSE_NO_GRAPH")
        if env:
            os.environ["OPOSE_NO_GRAPH"] = "1"
        try:
            return Body(bsd, scale_search=(0.5, 1.0)), Hand(hsd)
        finally:
            if old is None:
                os.environ.pop("OPOSE_NO_GRAPH", None)
            else:
                os.environ["OPOSE_NO_GRAPH"] = old
    gb, gh = make(False)
    eb, eh = make(True)
    ref_b, ref_h = eb(img), eh(crop)
    for _ in range(4):
        cand, sub = gb(img)
        assert np.array_equal(cand, ref_b[0]) and np.array_equal(sub, ref_b[1])
        pk = gh(crop)
        assert pk.dtype == ref_h.dtype and np.array_equal(pk, ref_h)


def test_destroyed_handles_graphs_do_not_break_replays():
    """handles with captured graphs are destroyed while others keep replaying
    theirs (the round-4 crash: gpurun_out/c3d.log, a C5 handle's replay after another handle's
    teardown).  Cause, reproduced without libopose by scripts/graph_fork_repro.hip: torch's
    bundled HIP 7.0.2 runtime segfaults in hipGraphLaunch on forked graphs once other forked
    executables are destroyed.  The library keeps every capture a single chain (run_graphed refuses
    any other), so here: a lockstep two-scale Body, a one-scale Body, an OPOSE_LOCKSTEP=0 Body (its
    scales fork eagerly onto pooled streams) and a Hand each capture; three of them are deleted in
    turn, and the survivors replay 5x after each deletion with unchanged outputs; handles created
    afterwards (reusing the pooled streams) capture and replay the same results."""
    import gc
    from src.body import Body
    from src.hand import Hand
    from src.weights import seeded_state_dict
    rng = np.random.default_rng(25)
    img = rng.integers(0, 256, (184, 232, 3), dtype=np.uint8)
    crop = rng.integers(0, 256, (128, 128, 3), dtype=np.uint8)
    bsd, hsd = seeded_state_dict("body", 0), seeded_state_dict("hand", 0)

    def lockstep_off():
        os.environ["OPOSE_LOCKSTEP"] = "0"
        try:
            return Body(bsd, scale_search=(0.5, 1.0))
        finally:
            del os.environ["OPOSE_LOCKSTEP"]

    makers = {"pyr": lambda: Body(bsd, scale_search=(0.5, 1.0)), "one": lambda: Body(bsd),
              "eager_fork": lockstep_off, "hand": lambda: Hand(hsd)}
    inputs = {"pyr": img, "one": img, "eager_fork": img, "hand": crop}
    hs = {k: m() for k, m in makers.items()}
    ref = {}
    for k, h in hs.items():
        for _ in range(3):  # eager, capture, replay
            ref[k] = h(inputs[k])

    def same(k, out):
        if k == "hand":
            assert out.dtype == ref[k].dtype and np.array_equal(out, ref[k]), k
        else:
            assert np.array_equal(out[0], ref[k][0]) and np.array_equal(out[1], ref[k][1]), k

    for victim in ("eager_fork", "pyr", "hand"):
        del hs[victim]
        gc.collect()
        for _ in range(5):
            for k, h in hs.items():
                same(k, h(inputs[k]))
    assert ref["pyr"][0].shape == ref["eager_fork"][0].shape
    assert np.array_equal(ref["pyr"][0], ref["eager_fork"][0])  # lockstep == per-scale networks
    for k in ("pyr", "hand", "eager_fork"):
        h = makers[k]()
        for _ in range(5):
            same(k, h(inputs[k]))
            same("one", hs["one"](img))


def test_alternating_shapes_on_one_handle():
    """One Body and one Hand fed frames of alternating sizes, each size three times in a row
    (eager, capture, replay) and then again after other sizes: the larger sizes grow the workspace,
    which invalidates every captured graph (g_alloc_epoch), and the per-signature launch plans and
    slab schedules pile up.  Every call equals an eager (OPOSE_NO_GRAPH=1) handle's call on the
    same frame, bit for bit."""
    from src.body import Body
    from src.hand import Hand
    from src.weights import seeded_state_dict
    rng = np.random.default_rng(27)
    frames = [rng.integers(0, 256, s, dtype=np.uint8) for s in ((96, 128, 3), (184, 232, 3), (368, 656, 3))]
    crops = [rng.integers(0, 256, (s, s, 3), dtype=np.uint8) for s in (128, 256, 184)]
    bsd, hsd = seeded_state_dict("body", 0), seeded_state_dict("hand", 0)
    os.environ["OPOSE_NO_GRAPH"] = "1"
    try:
        eb, eh = Body(bsd), Hand(hsd)
    finally:
        del os.environ["OPOSE_NO_GRAPH"]
    ref_b = [eb(f) for f in frames]
    ref_h = [eh(c) for c in crops]
    gb, gh = Body(bsd), Hand(hsd)
    for i in (0, 1, 0, 2, 1, 0, 2):
        for _ in range(3):
            cand, sub = gb(frames[i])
            assert np.array_equal(cand, ref_b[i][0]) and np.array_equal(sub, ref_b[i][1]), i
            pk = gh(crops[i])
            assert pk.dtype == ref_h[i].dtype and np.array_equal(pk, ref_h[i]), i


def test_handles_on_concurrent_threads():
    """Serving threads with a handle each (ctypes drops the GIL, so the library calls overlap):
    a Body and a Hand thread plus a second Body thread on other frames, 6 calls each (eager,
    capture, replays: the captures are thread-local, the workspace epoch and the scale-stream pool
    are process-wide), all equal to the same handles' single-threaded results."""
    import threading
    from src.body import Body
    from src.hand import Hand
    from src.weights import seeded_state_dict
    rng = np.random.default_rng(29)
    img_a = rng.integers(0, 256, (184, 232, 3), dtype=np.uint8)
    img_b = rng.integers(0, 256, (96, 176, 3), dtype=np.uint8)
    crop = rng.integers(0, 256, (128, 128, 3), dtype=np.uint8)
    bsd, hsd = seeded_state_dict("body", 0), seeded_state_dict("hand", 0)
    jobs = {"body_a": (Body(bsd, scale_search=(0.5, 1.0)), img_a), "body_b": (Body(bsd), img_b),
            "hand": (Hand(hsd), crop)}
    ref = {k: h(x) for k, (h, x) in jobs.items()}
    outs = {k: [] for k in jobs}
    errors = []

    def run(k):
        h, x = jobs[k]
        try:
            for _ in range(6):
                outs[k].append(h(x))
        except Exception as e:  # reported in the main thread
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=run, args=(k,)) for k in jobs]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts) and not errors, errors
    for k, res in outs.items():
        assert len(res) == 6, k
        for out in res:
            if k == "hand":
                assert np.array_equal(out, ref[k]), k
            else:
                assert np.array_equal(out[0], ref[k][0]) and np.array_equal(out[1], ref[k][1]), k


def test_forward_waits_for_half_input(body):
    x = torch.from_numpy(np.random.default_rng(6).standard_normal((1, 3, 64, 96)).astype(np.float32))
    xh = x.half()
    paf_ref, heat_ref = body.model.forward(xh.float().numpy())
    src = xh.cuda()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.cuda._sleep(50_000_000)
        xd = src * 1  # produced on the side stream after the spin
        paf, heat = body.model.forward(xd)
        paf, heat = paf.cpu().numpy(), heat.cpu().numpy()
    assert np.array_equal(paf, paf_ref) and np.array_equal(heat, heat_ref)


def test_host_copy_stops_at_view_end(body):
    """The view's last byte is the last byte before a PROT_NONE page."""
    H, W, page = 96, 128, mmap.PAGESIZE
    full_w = W + 40
    nbytes = (H + 20) * full_w * 3
    span = (nbytes + page - 1) // page * page
    buf = mmap.mmap(-1, span + page, prot=mmap.PROT_READ | mmap.PROT_WRITE)
    libc = ctypes.CDLL(None)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(buf))
    assert libc.mprotect(ctypes.c_void_p(addr + span), page, 0) == 0  # guard page
    try:
        # image rows end exactly at the guard: place the (H+20) x full_w image at span - nbytes
        img = np.frombuffer(buf, np.uint8, count=nbytes, offset=span - nbytes).reshape(H + 20, full_w, 3)
        img[:] = np.random.default_rng(8).integers(0, 256, img.shape, dtype=np.uint8)
        view = img[20:, 40:]  # bottom-right crop: its last pixel is the buffer's last byte
        assert view.ctypes.data + (H - 1) * view.strides[0] + 3 * W == addr + span
        got = body(view)
        exp = body(np.ascontiguousarray(view))
        _same([got], [exp])
    finally:
        libc.mprotect(ctypes.c_void_p(addr + span), page, mmap.PROT_READ | mmap.PROT_WRITE)
        del img, view
        buf.close()
