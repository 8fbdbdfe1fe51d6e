"""Error table of Winograd variants in split-bf16 arithmetic against the accuracy gate of
tests/test_gpu_x6.py (|err| <= 4e-6 * conv(|x|, |w|) per output, mean |err| <= 3x the fp32
kernel's), on the CPU: a numpy model of the MFMA arithmetic, not the kernels themselves.

Model: every operand a fp32 value carried as three exact bf16 pieces (x = x0 + x1 + x2); each
v_mfma_f32_16x16x32_bf16 adds the exact sum of 32 piece products, rounded to fp32, to an fp32
accumulator; the six piece products (i + j <= 2) in the kernels' order per 32-deep k chunk.
Transforms of the inputs and outputs run in fp32 (numpy float32 rounds every operation), weight
transforms in float64 rounded to fp32 once, as conv_wino.hip / x6_pack_weights_wino do.

    python scripts/wino_error_table.py [--cin 128] [--seeds 3]   (profiles/r6_wino_error_table.txt)
"""
import argparse

import numpy as np

PAIRS = [(0, 2), (0, 0), (0, 1), (1, 0), (2, 0), (1, 1)]


def bf16(x):
    """Round-to-nearest-even bf16 of float32 x, as float32."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def split3(x):
    x = np.asarray(x, np.float32)
    p0 = bf16(x)
    r = (x - p0).astype(np.float32)
    p1 = bf16(r)
    p2 = bf16((r - p1).astype(np.float32))
    return p0, p1, p2


def gemm_x6(A, B):
    """A [M, K] fp32, B [K, P] fp32 -> fp32 [M, P]: the split-bf16 MFMA loop (K padded to 32)."""
    K = A.shape[1]
    Kp = -(-K // 32) * 32
    A = np.pad(A, ((0, 0), (0, Kp - K)))
    B = np.pad(B, ((0, Kp - K), (0, 0)))
    a, b = split3(A), split3(B)
    acc = np.zeros((A.shape[0], B.shape[1]), np.float32)
    for k in range(0, Kp, 32):
        for i, j in PAIRS:
            s = a[i][:, k:k + 32].astype(np.float64) @ b[j][k:k + 32].astype(np.float64)
            acc = (acc + s.astype(np.float32)).astype(np.float32)
    return acc


def gemm_f32(A, B):
    """The fp32 MFMA kernel's model: exact 32-deep chunk sums of fp32 products, fp32 accumulate."""
    K = A.shape[1]
    acc = np.zeros((A.shape[0], B.shape[1]), np.float32)
    for k in range(0, K, 32):
        prods = (A[:, k:k + 32, None].astype(np.float32) * B[None, k:k + 32].astype(np.float32))
        acc = (acc + prods.astype(np.float64).sum(1).astype(np.float32)).astype(np.float32)
    return acc


def im2col(x, taps):
    """x [C, H+2, W+2] padded -> [(C, tap), H*W] for the (dy, dx) taps."""
    C, Hp, Wp = x.shape
    H, W = Hp - 2, Wp - 2
    return np.stack([x[:, dy:dy + H, dx:dx + W].reshape(C, -1) for dy, dx in taps], 1).reshape(C * len(taps), -1)


TAPS = [(dy, dx) for dy in range(3) for dx in range(3)]


def direct(x, w, gemm):
    Cout = w.shape[0]
    return gemm(w.reshape(Cout, -1), im2col(x, TAPS)).reshape(Cout, x.shape[1] - 2, x.shape[2] - 2)


# 1-D F(2,3) along x (conv_wino.hip): d0..d3 = in[x0-1 .. x0+2]
G23 = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]])


def wino_f23(x, w):
    Cout, C = w.shape[:2]
    H, W = x.shape[1] - 2, x.shape[2] - 2
    U = np.einsum("vk,mcyk->vmcy", G23, w.astype(np.float64)).astype(np.float32)  # [4, M, C, 3]
    d = [x[:, :, j:j + W:2] for j in range(4)]  # column j of each output pair's input window
    V = [d[0] - d[2], d[1] + d[2], d[2] - d[1], d[1] - d[3]]  # fp32
    M = []
    for v in range(4):
        Vv = np.stack([V[v][:, ky:ky + H] for ky in range(3)], 1).reshape(C * 3, -1)
        M.append(gemm_x6(U[v].reshape(Cout, -1), Vv).reshape(Cout, H, W // 2))
    out = np.empty((Cout, H, W), np.float32)
    out[:, :, 0::2] = (M[0] + M[1]) + M[2]
    out[:, :, 1::2] = (M[1] - M[2]) - M[3]
    return out


# 1-D F(4,3) along x, points 0, 1, -1, 2, -2 (+ infinity)
BT43 = np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0],
                 [0, -2, -1, 2, 1, 0], [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], np.float32)
G43 = np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6],
                [1 / 24, 1 / 12, 1 / 6], [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]])
AT43 = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]], np.float32)


def wino_f43(x, w):
    Cout, C = w.shape[:2]
    H, W = x.shape[1] - 2, x.shape[2] - 2
    U = np.einsum("vk,mcyk->vmcy", G43, w.astype(np.float64)).astype(np.float32)
    d = np.stack([x[:, :, j:j + W:4] for j in range(6)], 0)  # [6, C, H+2, W/4]
    V = np.zeros_like(d)
    for v in range(6):
        acc = np.zeros_like(d[0])
        for j in range(6):
            if BT43[v, j]:
                acc = (acc + np.float32(BT43[v, j]) * d[j]).astype(np.float32)
        V[v] = acc
    M = []
    for v in range(6):
        Vv = np.stack([V[v][:, ky:ky + H] for ky in range(3)], 1).reshape(C * 3, -1)
        M.append(gemm_x6(U[v].reshape(Cout, -1), Vv).reshape(Cout, H, W // 4))
    out = np.empty((Cout, H, W), np.float32)
    for r in range(4):
        acc = np.zeros_like(M[0])
        for v in range(6):
            if AT43[r, v]:
                acc = (acc + np.float32(AT43[r, v]) * M[v]).astype(np.float32)
        out[:, :, r::4] = acc
    return out


# 2-D F(2x2,3x3)
BT22 = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float32)
AT22 = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float32)


def wino_f22(x, w):
    Cout, C = w.shape[:2]
    H, W = x.shape[1] - 2, x.shape[2] - 2
    U = np.einsum("ay,mcyk,bk->abmc", G23, w.astype(np.float64), G23).astype(np.float32)  # [4,4,M,C]
    d = np.stack([np.stack([x[:, i:i + H:2, j:j + W:2] for j in range(4)], 0) for i in range(4)], 0)
    # V = BT d B, rows then columns, fp32
    t = np.einsum("ai,ij...->aj...", BT22, d).astype(np.float32)
    V = np.einsum("bj,aj...->ab...", BT22, t).astype(np.float32)
    M = np.empty((4, 4, Cout, H // 2, W // 2), np.float32)
    for a in range(4):
        for b in range(4):
            M[a, b] = gemm_x6(U[a, b], V[a, b].reshape(C, -1)).reshape(Cout, H // 2, W // 2)
    t = np.einsum("ra,ab...->rb...", AT22, M).astype(np.float32)
    Y = np.einsum("sb,rb...->rs...", AT22, t).astype(np.float32)
    out = np.empty((Cout, H, W), np.float32)
    for r in range(2):
        for s in range(2):
            out[:, r::2, s::2] = Y[r, s]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=128)
    ap.add_argument("--cout", type=int, default=32)
    ap.add_argument("--hw", type=int, default=16)
    ap.add_argument("--seeds", type=int, default=3)
    a = ap.parse_args()
    rows = {}
    for seed in range(a.seeds):
        rng = np.random.default_rng(seed)
        x = np.maximum(rng.standard_normal((a.cin, a.hw, a.hw)), 0).astype(np.float32)  # post-ReLU
        x = np.pad(x, ((0, 0), (1, 1), (1, 1)))
        w = (rng.standard_normal((a.cout, a.cin, 3, 3)) * np.sqrt(2 / (9 * a.cin))).astype(np.float32)
        ref = direct(x.astype(np.float64), w.astype(np.float64), lambda A, B: A @ B)
        mag = direct(np.abs(x).astype(np.float64), np.abs(w).astype(np.float64), lambda A, B: A @ B)
        for name, fn in (("fp32 MFMA direct", lambda: direct(x, w, gemm_f32)),
                         ("split-bf16 direct", lambda: direct(x, w, gemm_x6)),
                         ("split-bf16 F(2,3) 1-D", lambda: wino_f23(x, w)),
                         ("split-bf16 F(2x2,3x3)", lambda: wino_f22(x, w)),
                         ("split-bf16 F(4,3) 1-D", lambda: wino_f43(x, w))):
            err = np.abs(fn().astype(np.float64) - ref)
            r = rows.setdefault(name, [0.0, []])
            r[0] = max(r[0], float((err / np.maximum(mag, 1e-30)).max()))
            r[1].append(float(err.mean()))
    base = np.mean(rows["fp32 MFMA direct"][1])
    print(f"Cin {a.cin}, Cout {a.cout}, {a.hw}x{a.hw}, {a.seeds} seeds; gate: max <= 4e-6, mean ratio <= 3")
    print(f"{'variant':24s} {'max |err|/conv(|x|,|w|)':>24s} {'mean |err|':>12s} {'vs fp32':>8s}  gate")
    for name, (mx, means) in rows.items():
        m = float(np.mean(means))
        ok = mx <= 4e-6 and m <= 3 * base
        print(f"{name:24s} {mx:24.3e} {m:12.3e} {m / base:8.2f}  {'pass' if ok else 'FAIL'}")


if __name__ == "__main__":
    main()
