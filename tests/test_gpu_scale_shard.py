"""GPU: the scale-sharded single-frame path of config C5.

* opose_body_scale_geom matches the oracle's preprocess geometry (src/body.py:35-41);
* opose_body_scale_maps(s) equals the network on the oracle-preprocessed input of scale s;
* opose_body_post_scales on planted multi-scale pyramids matches the oracle's
  post_from_lowres (src/body.py:51-212), host and device inputs alike;
* scale_maps for every scale + post_scales == Body(frame) bit for bit, and the same through
  src.dist.body_scale_sharded with two ranks (gloo, both on cuda:0)."""
import os

import numpy as np
import pytest
import torch

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

SCALES = (0.5, 1.0, 1.5, 2.0)


@pytest.fixture(scope="module")
def body():
    from src.body import Body
    from src.weights import seeded_state_dict
    return Body(seeded_state_dict("body", 0), scale_search=SCALES)


def _same(a, b):
    ca, sa = a
    cb, sb = b
    assert ca.shape == cb.shape and sa.shape == sb.shape
    if ca.size:
        assert np.array_equal(ca[:, [0, 1, 3]], cb[:, [0, 1, 3]])
        np.testing.assert_allclose(ca[:, 2], cb[:, 2], rtol=1e-12, atol=0)
    assert np.array_equal(sa[:, :18], sb[:, :18]) and np.array_equal(sa[:, 19], sb[:, 19])
    np.testing.assert_allclose(sa[:, 18], sb[:, 18], rtol=1e-12)


def _identical(a, b):
    for (ca, sa), (cb, sb) in zip(a, b):
        assert np.array_equal(ca, cb) and np.array_equal(sa, sb)


def _pyramid(H, W, n_people, seed):
    """Planted low-res maps for each scale of SCALES: the same people, scaled per grid."""
    from oracle import planted
    from oracle.body_post import preprocess
    rng = np.random.default_rng(seed)
    geo = []
    for s in SCALES:
        _, pad, padded = preprocess(np.zeros((H, W, 3), np.uint8), s * 368 / H)
        geo.append((pad, padded))
    h1, w1 = geo[1][1][0] // 8, geo[1][1][1] // 8
    people, vis = planted.random_people(rng, n_people, h1, w1)
    lowres = []
    for pad, padded in geo:
        h, w = padded[0] // 8, padded[1] // 8
        ppl = people * np.array([w / w1, h / h1]) if people.size else people
        paf, heat = planted.render_body(h, w, ppl, vis, rng)
        lowres.append((paf, heat, pad, padded))
    return lowres


@pytest.mark.parametrize("hw", [(1080, 1920), (184, 328), (97, 53), (368, 656)])
def test_scale_geom_matches_oracle(body, hw):
    from oracle.body_post import preprocess
    H, W = hw
    for s, g in zip(SCALES, body.scale_geom(H, W)):
        _, pad, padded = preprocess(np.zeros((H, W, 3), np.uint8), s * 368 / H)
        assert g == (padded[0] // 8, padded[1] // 8, pad[2], pad[3])


def test_scale_maps_equal_network(body):
    from oracle.body_post import preprocess
    img = np.random.default_rng(5).integers(0, 256, (72, 96, 3), dtype=np.uint8)
    for s, sc in enumerate(SCALES):
        x, _, _ = preprocess(img, sc * 368 / img.shape[0])
        paf, heat = body.model(x)
        maps = body.scale_maps(img, s)
        assert maps.shape == (1, 57) + paf.shape[2:]
        assert np.array_equal(maps[:, :38], paf) and np.array_equal(maps[:, 38:], heat)


@pytest.mark.parametrize("hw,n,seed", [((184, 328), 3, 1), ((368, 656), 6, 2), ((120, 90), 1, 3)])
def test_post_scales_vs_oracle(body, hw, n, seed):
    from oracle.body_post import post_from_lowres
    H, W = hw
    lowres = _pyramid(H, W, n, seed)
    ref = post_from_lowres((H, W), lowres)
    maps = [np.concatenate([paf, heat], 0)[None] for paf, heat, _, _ in lowres]
    got = body.post_scales(maps, H, W)[0]
    _same(got, (np.asarray(ref[0], np.float64).reshape(-1, 4), np.asarray(ref[1], np.float64).reshape(-1, 20)))
    if n > 1:
        assert got[1].shape[0] >= 1
    dev = body.post_scales([torch.from_numpy(m).cuda() for m in maps], H, W)[0]
    _identical([got], [dev])


def test_post_scales_rejects_wrong_shapes(body):
    maps = [np.zeros((1, 57, 4, 4), np.float32)] * len(SCALES)
    with pytest.raises(ValueError):
        body.post_scales(maps, 184, 328)
    with pytest.raises(ValueError):
        body.post_scales(maps[:2], 184, 328)


def test_scale_maps_then_post_equals_body(body):
    img = np.random.default_rng(31).integers(0, 256, (90, 160, 3), dtype=np.uint8)
    maps = [body.scale_maps(img, s) for s in range(len(SCALES))]
    _identical(body.post_scales(maps, 90, 160), body.batch(img[None]))
    dev = torch.from_numpy(img).cuda()
    dmaps = [body.scale_maps(dev, s) for s in range(len(SCALES))]
    for a, b in zip(maps, dmaps):
        assert np.array_equal(a, b.cpu().numpy())
    _identical(body.post_scales(dmaps, 90, 160), body.batch(img[None]))


def _shard_worker(rank, world, port, q):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from src.body import Body
    from src.dist import body_scale_sharded
    from src.weights import seeded_state_dict
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = Body(seeded_state_dict("body", 0), scale_search=SCALES)
        img = np.random.default_rng(31).integers(0, 256, (90, 160, 3), dtype=np.uint8)
        out = body_scale_sharded(b, img, rank, world)
        if rank == 0:
            ref = b.batch(img[None])
            ok = all(np.array_equal(ca, cb) and np.array_equal(sa, sb) for (ca, sa), (cb, sb) in zip(out, ref))
        else:
            ok = out is None
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_scale_sharded_two_ranks_equals_single():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


# ---------------------------------------------------------------- C5 at its real size
@pytest.mark.parametrize("name", ["body_c5_700_1080x1920_p8.npz", "body_c5_701_1080x1920_p3.npz"])
def test_post_scales_c5_reference_golden(body, name):
    """C5 (BASELINE.json): 1080x1920 at scale_search [0.5, 1, 1.5, 2]; planted per-scale maps,
    expected output from the reference's own multi-scale Body (oracle/gen_golden.py c5):
    bit-exact, host and device inputs."""
    from conftest import GOLDEN
    d = np.load(os.path.join(GOLDEN, name))
    H, W = (int(v) for v in d["img_hw"])
    assert tuple(d["scales"]) == SCALES
    maps = [np.concatenate([d[f"paf{i}"], d[f"heat{i}"]], 0)[None] for i in range(len(SCALES))]
    geo = body.scale_geom(H, W)
    for i, (hl, wl, pd, pr) in enumerate(geo):
        assert maps[i].shape[2:] == (hl, wl) and [pd, pr] == list(d[f"pad{i}"][2:])
    cand, subset = body.post_scales(maps, H, W)[0]
    assert np.array_equal(cand, d["candidate"]) and np.array_equal(subset, d["subset"])
    dev = body.post_scales([torch.from_numpy(m).cuda() for m in maps], H, W)[0]
    assert np.array_equal(dev[0], d["candidate"]) and np.array_equal(dev[1], d["subset"])


def test_body_1080p_full_network_equals_scale_decomposition():
    """One 1080p frame through the whole four-scale network (C5 calibration of the seeded output
    convs, as scripts/bench_configs.py runs it): completes (status 0) and equals the per-scale
    split that body_scale_sharded distributes (scale_maps per scale + post_scales)."""
    from src.body import Body
    from src.weights import c5_out_scale, seeded_state_dict
    body = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=SCALES)
    img = np.random.default_rng(31).integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
    whole = body.batch(img[None])
    cand, subset = whole[0]
    assert cand.ndim == 2 and cand.shape[1] == 4 and subset.shape[1] == 20
    maps = [body.scale_maps(img[None], s) for s in range(len(SCALES))]
    _identical(body.post_scales(maps, 1080, 1920), whole)


def _with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("scales", [(0.5, 1.0), (1.0, 1.5, 2.0), SCALES], ids=["2scales", "3scales", "4scales"])
def test_heat_full_scales_equals_per_scale_launches(scales):
    """The one-launch multi-scale heat average (imgproc.hip heat_full_scales, default) against one
    launch per scale into the float64 accumulator (OPOSE_HEAT_SCALES=0, read at handle creation):
    every scale's resize summed in scale order from 0.0 either way, so the records are identical
    bit for bit.  Two planted 368 x 656 frames per call (N = 2); at 368 rows the 1.0 scale is
    identity-sized (x8 of the 46-row map is the frame)."""
    from oracle.body_post import preprocess
    from src.body import Body
    from src.weights import seeded_state_dict
    H, W = 368, 656
    lowres = [_pyramid(H, W, n, seed) for n, seed in ((5, 41), (2, 42))]
    idx = [SCALES.index(s) for s in scales]
    maps = [np.concatenate([np.concatenate([lr[i][0], lr[i][1]], 0)[None] for lr in lowres], 0) for i in idx]
    for k, s in enumerate(scales):
        _, _, padded = preprocess(np.zeros((H, W, 3), np.uint8), s * 368 / H)
        assert maps[k].shape[2:] == (padded[0] // 8, padded[1] // 8)
    outs = []
    for on in ("1", "0"):
        b = _with_env({"OPOSE_HEAT_SCALES": on}, lambda: Body(seeded_state_dict("body", 0), scale_search=scales))
        outs.append(b.post_scales(maps, H, W))
        del b
    assert len(outs[0]) == 2
    _identical(outs[0], outs[1])
    assert any(len(sub) for _, sub in outs[0])


def test_hand_heat_full_scales_equals_per_scale_launches():
    """The same for Hand(): its four scales' heat average in one launch (default) or per scale."""
    from src.hand import Hand
    from src.weights import seeded_state_dict
    crop = np.random.default_rng(43).integers(0, 256, (200, 200, 3), dtype=np.uint8)
    outs = []
    for on in ("1", "0"):
        hd = _with_env({"OPOSE_HEAT_SCALES": on}, lambda: Hand(seeded_state_dict("hand", 0)))
        outs.append(hd(crop))
        del hd
    assert outs[0].dtype == outs[1].dtype and np.array_equal(outs[0], outs[1])
