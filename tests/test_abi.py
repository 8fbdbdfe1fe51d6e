"""CPU: the C-ABI library builds, loads and exports every symbol include/opose.h declares.

No compute calls here (there is no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import numpy as np

from conftest import REPO

HEADER = os.path.join(REPO, "include", "opose.h")
LIB = os.path.join(REPO, "pytorch-openpose_amd", "lib", "libopose.so")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(opose_[a-z_0-9]+)\s*\(", src)))


def test_library_exists_and_loads():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    ctypes.CDLL(LIB)


def test_every_declared_symbol_is_exported():
    syms = declared_symbols()
    assert len(syms) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (opose_\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_python_binding_covers_header():
    import sys
    sys.path.insert(0, os.path.join(REPO, "pytorch-openpose_amd"))
    from src import _native
    assert sorted(_native.EXPORTED) == declared_symbols()


def test_default_params_are_reference_constants():
    from src import _native
    p = _native.default_params(_native.NET_BODY)
    assert (p.n_scales, p.scales[0], p.boxsize, p.stride, p.pad_value) == (1, 0.5, 368.0, 8, 128)
    assert (p.thre1, p.thre2) == (0.1, 0.05)                   # src/body.py:25-31
    q = _native.default_params(_native.NET_HAND)
    assert list(q.scales[:q.n_scales]) == [0.5, 1.0, 1.5, 2.0]  # src/hand.py:26
    assert q.thre_hand == 0.03


def test_record_layout_decode_roundtrip():
    from src import _native
    ppp, maxp = 4, 3
    rec = np.zeros(16 + 32 * 18 * ppp + 160 * maxp, np.uint8)
    hdr = rec[:16].view(np.int32)
    hdr[:3] = (0, 2, 1)
    cand = rec[16:16 + 32 * 18 * ppp].view(np.float64).reshape(-1, 4)
    cand[:2] = [[1, 2, 0.5, 0], [3, 4, 0.25, 1]]
    sub = rec[16 + 32 * 18 * ppp:].view(np.float64).reshape(-1, 20)
    sub[0] = -1
    sub[0, :2] = [0, 1]
    status, c, s = _native.decode_record(rec, ppp, maxp)
    assert status == 0 and c.shape == (2, 4) and s.shape == (1, 20) and s[0, 1] == 1
    hdr[1:3] = 0
    _, c, s = _native.decode_record(rec, ppp, maxp)
    assert c.shape == (0,) and s.shape == (0, 20)


def test_gaussian_weights_match_scipy():
    from scipy.ndimage._filters import _gaussian_kernel1d
    src = open(os.path.join(REPO, "pytorch-openpose_amd", "csrc", "post.hip")).read()
    body = src[src.index("kGauss[13] = {"):src.index("};", src.index("kGauss[13] = {"))]
    vals = [float.fromhex(t) for t in re.findall(r"0x[0-9a-fp.+-]+", body)]
    w = _gaussian_kernel1d(3, 0, 12)
    assert vals == [float(v) for v in w[12:]]


def test_seeded_weights_identical_to_oracle():
    from oracle.network import seeded_state_dict as oracle_sd
    from src.weights import seeded_state_dict
    a, b = seeded_state_dict("hand", 3), oracle_sd("hand", 3)
    assert list(a) == list(b)
    assert all(np.array_equal(a[k], b[k].numpy()) for k in a)
