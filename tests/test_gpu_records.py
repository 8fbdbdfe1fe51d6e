"""GPU: the device-resident batch path (Body.infer_records, opose_body_infer with
IN_DEVICE | OUT_DEVICE) that bench.py times, against the host-memory batch path (Body.batch:
the same batch through the same network tiles), serial and pipelined (OPOSE_PIPELINE: each
call's network overlaps the previous call's post-processing on a second stream; the x8 maps
alternate between two buffer sets).  Bar: identical candidates and
subsets (same kernels, same arithmetic; only the launch order across streams differs)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H, W, B = 184, 328, 3


@pytest.fixture(scope="module")
def body():
    from src.body import Body
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    return Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))


@pytest.fixture(scope="module")
def batches():
    rng = np.random.default_rng(21)
    return [rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8) for _ in range(3)]


@pytest.fixture(scope="module")
def expected(body, batches):
    return [body.batch(frames) for frames in batches]


def _check(body, rec, exp):
    got = body.decode_records(rec)
    assert len(got) == len(exp)
    for (c, s), (ec, es) in zip(got, exp):
        assert np.array_equal(c, ec) and np.array_equal(s, es)


def test_records_serial(body, batches, expected):
    for frames, exp in zip(batches, expected):
        rec = body.infer_records(torch.from_numpy(frames).cuda())
        body.handle.synchronize()
        _check(body, rec, exp)


def test_records_pipelined(body, batches, expected):
    dev = [torch.from_numpy(f).cuda() for f in batches]
    torch.cuda.synchronize()  # frames complete before the pipelined calls (OPOSE_PIPELINE contract)
    order = [0, 1, 2, 0, 1, 2, 1]
    # repeated: a race that needs the post kernels to overlap a particular network layer shows
    # up in a few frames per hundred or thousand (the opt-in screened NMS lost peaks this way;
    # limb_greedy's shared counter changed 2-3 subsets per 840 frames), so one pass is not
    # enough evidence (scripts/pipeline_stress.sh runs longer)
    for _ in range(16):
        recs = [body.infer_records(dev[i], pipeline=True) for i in order]
        body.handle.synchronize()
        for i, rec in zip(order, recs):
            _check(body, rec, expected[i])
    # pipelined calls around a host-path call (shares the network workspace on the main stream)
    r0 = body.infer_records(dev[2], pipeline=True)
    mid = body.batch(batches[1])
    r1 = body.infer_records(dev[0], pipeline=True)
    body.handle.synchronize()
    _check(body, r0, expected[2])
    _check(body, r1, expected[0])
    for (c, s), (ec, es) in zip(mid, expected[1]):
        assert np.array_equal(c, ec) and np.array_equal(s, es)


@pytest.mark.parametrize("mix", ["defer_only", "mixed"])
def test_records_pipelined_deferred(body, batches, expected, mix):
    """pipeline="defer" (OPOSE_PIPELINE_DEFER; opt-in, bench.py with BENCH_DEFER=1): each call's post-processing
    is enqueued by the next call once its network reaches conv3_1 (or by flush / synchronize /
    decode_records / any other entry point).  Every record equals the host path's, whether the
    deferred calls run back to back, alternate with plain pipelined calls, or are followed by a
    host-path call, a decode without an explicit flush, or a synchronize."""
    dev = [torch.from_numpy(f).cuda() for f in batches]
    torch.cuda.synchronize()
    order = [0, 1, 2, 0, 2, 1, 1]
    for _ in range(8):
        modes = ["defer" if (mix == "defer_only" or k % 2 == 0) else True for k in range(len(order))]
        recs = [body.infer_records(dev[i], pipeline=m) for i, m in zip(order, modes)]
        body.handle.synchronize()
        for i, rec in zip(order, recs):
            _check(body, rec, expected[i])
    r0 = body.infer_records(dev[1], pipeline="defer")
    mid = body.batch(batches[2])  # another entry point flushes the deferred post first
    r1 = body.infer_records(dev[0], pipeline="defer")
    _check(body, r0, expected[1])
    _check(body, r1, expected[0])  # decode_records flushes
    for (c, s), (ec, es) in zip(mid, expected[2]):
        assert np.array_equal(c, ec) and np.array_equal(s, es)


def test_bench_frame_post_exact_vs_oracle(body):
    """The bench's own configuration: a uniform-random 368x656 frame at scale 0.5 with the bench's
    calibrated weights (crowded: ~300 peaks and ~20 people per frame).  The device path bench.py
    times (infer_records) equals the GPU post-network path on the GPU network's maps, and that
    equals the oracle's post-network restatement (src/body.py:52-212) on the same maps,
    bit-exactly -- the post-processing half of the north-star bar at the benchmarked size."""
    from oracle import body_post
    from src.model import bodypose_model
    from src.util import transfer
    from src.weights import BENCH_OUT_SCALE, seeded_state_dict
    img = np.random.default_rng(33).integers(0, 256, (368, 656, 3), dtype=np.uint8)
    x, pad, padded_hw = body_post.preprocess(img, 0.5)
    m = bodypose_model()
    m.load_state_dict(transfer(m, seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE)))
    paf, heat = m(x)
    paf, heat = np.asarray(paf), np.asarray(heat)
    cand, subset = body.post(np.concatenate([paf, heat], 1), list(pad), 368, 656)[0]
    assert len(cand) > 100 and len(subset) > 5  # the crowded regime the bench measures
    ref_c, ref_s = body_post.post_from_lowres((368, 656), [(paf[0], heat[0], list(pad), tuple(padded_hw))])
    assert np.array_equal(cand, ref_c) and np.array_equal(subset, ref_s)
    rec = body.infer_records(torch.from_numpy(img[None]).cuda())
    body.handle.synchronize()
    (dc, ds), = body.decode_records(rec)
    assert np.array_equal(dc, cand) and np.array_equal(ds, subset)
