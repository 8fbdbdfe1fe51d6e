"""CPU: properties of the built gfx950 code objects, checked on the ISA (no GPU needed).

* No VOP3P packed-FP32 arithmetic (`v_pk_add_f32`, `v_pk_mul_f32`, `v_pk_fma_f32`) anywhere in
  libopose.so: compiler-generated packed-FP32 code gave wrong low-element results when its kernel
  ran beside the pipelined network stream's kernels, so every kernel is built with
  `-target-feature -packed-fp32-ops` (pytorch-openpose_amd/Makefile NOPK).  A flag or toolchain
  change that brings them back fails here instead of in a rare pipelined frame.
* The split-bf16 convolution is on the matrix cores: the conv code object holds
  `v_mfma_f32_16x16x32_bf16`, and the float64 post-processing kernels hold no FMA contraction
  (`-ffp-contract=off`: bit parity with NumPy / SciPy needs one rounding per operation)."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "pytorch-openpose_amd", "lib", "libopose.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


@pytest.fixture(scope="module")
def device_asm(tmp_path_factory):
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump (ROCm) not available")
    assert os.path.exists(LIB), "build libopose.so first (make -C pytorch-openpose_amd)"
    d = tmp_path_factory.mktemp("bundles")
    so = os.path.join(d, "libopose.so")
    shutil.copy(LIB, so)
    # --offloading writes each offload bundle next to its input
    subprocess.run([OBJDUMP, "--offloading", so], check=True, capture_output=True, cwd=d)
    objs = sorted(f for f in os.listdir(d) if f.endswith("gfx950"))
    assert len(objs) >= 5, objs  # one per translation unit with device code
    return {f: subprocess.run([OBJDUMP, "-d", os.path.join(d, f)], check=True, capture_output=True,
                              text=True).stdout for f in objs}


def test_no_packed_fp32_arithmetic(device_asm):
    pat = re.compile(r"\bv_pk_(add|mul|fma)_f32\b")
    bad = {f: len(pat.findall(asm)) for f, asm in device_asm.items() if pat.search(asm)}
    assert not bad, f"packed-FP32 instructions in {bad}"


def test_conv_runs_on_bf16_matrix_cores(device_asm):
    n = sum(asm.count("v_mfma_f32_16x16x32_bf16") for asm in device_asm.values())
    assert n > 1000, n


def _functions(asm):
    """disassembly -> {symbol: body text}"""
    out, name = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            name = m.group(1)
            out[name] = []
        elif name:
            out[name].append(line)
    return {k: "\n".join(v) for k, v in out.items()}


def test_float64_filters_not_contracted(device_asm):
    """The Gaussian NMS kernels (scipy's filter order, one rounding per operation): float64 adds
    and multiplies, no FMA.  (paf_score / assemble_people hold v_fma_f64 only inside the IEEE
    division and square-root expansions, which round once.)"""
    fns = {}
    for asm in device_asm.values():
        fns.update(_functions(asm))
    gauss = {k: v for k, v in fns.items() if "gauss_nms" in k}
    assert len(gauss) >= 2, sorted(fns)[:20]
    for k, body in gauss.items():
        assert "v_mul_f64" in body and "v_add_f64" in body, k
        assert not re.search(r"v_fmac?_f64", body), k
