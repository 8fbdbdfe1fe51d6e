// conv_x6.hip — fp32-accurate implicit-GEMM convolution on the gfx950 bf16 matrix cores.
//
// Same GEMM view as conv.hip (out[m][p] = bias[m] + sum_k W[m][k] im2col[k][p], src/model.py
// make_layers / forward), but every fp32 operand is carried as three bfloat16 pieces
// (x = x0 + x1 + x2 exactly, see common.h X6) and each product is rebuilt from the six
// piece products whose weight is >= 2^-16 of the leading one:
//     a*b ~= a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0)
// The dropped terms (a1 b2 + a2 b1 + a2 b2) are below 2^-23 |a b|, the size of one fp32
// rounding, and every piece product is exact in the fp32 accumulator: the sum carries fp32
// rounding error like the v_mfma_f32_32x32x2_f32 kernel (tests/test_gpu_x6.py measures both
// against a float64 reference).  The bf16 matrix rate is 16x the fp32 MFMA's, so six piece
// products run at 2.7x the fp32 MFMA rate.
//
// * Operand units are 16 bytes = 8 consecutive k of one row (A) / pixel (B): the per-lane
//   fragment of v_mfma_f32_16x16x32_bf16 (lane l: row / pixel l & 15, k = 8 (l >> 4) .. +7), so
//   LDS tiles are [piece][group][row] unit arrays read with one ds_read_b128 per fragment.
// * Both tiles are filled by LDS-DMA: weights (pre-split, [chunk][piece][group][Mpad] units)
//   by buffer loads to LDS, the im2col pixels of a (piece, channel group, tap) by
//   buffer_load_dwordx4 ... lds with the zero padding from the buffer range check.
// * K chunk = 32 k = 4 channel groups of one tap (or 4 taps of a single group when Cin <= 8),
//   two LDS stages, one barrier per chunk.  Work units (tile, k slab): a tile of a group with
//   `slabs` slabs sums fixed chunk ranges, each from zero, and conv_x6_fixup folds the slab
//   partials in slab order (common.h X6Group::slabs, x6.h x6_unit_of).
// * The epilogue adds bias, applies ReLU and writes the output split again (X6) into a
//   group slice of a wider buffer (the CPM concat), or fp32 NCHW for the network outputs.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "x6.h"

namespace opose {


// Main loop: v_mfma_f32_16x16x32_bf16, one k-step (32 k) per chunk, refill-after-last-use
// fragment schedule pinned by sched_barrier (see below).  Measured and dropped:
// a two-wait loop, the 32x32x16 pipelined loop, and im2col fragments loaded straight into
// registers (same speed, LDS for the weights only).
template <int MT, int PT, bool SMALL, int KS>
__global__ __launch_bounds__(64 * x6_waves(MT, PT), 1) void conv_x6(X6Args a) {
    const int ks = KS ? KS : a.ks;
    const int taps = ks * ks;
    // waves along M: 8-wave tiles one per 64 rows; the 4-wave tiles 2 x 2
    constexpr int NW = x6_waves(MT, PT), NWM = NW == 8 ? MT / 64 : 2, NWP = NW / NWM;
    constexpr int WM = MT / NWM, WP = PT / NWP;
    constexpr int MB = 16;                       // MFMA block (rows = pixels)
    constexpr int TM = WM / MB, TN = WP / MB;
    constexpr int ACC_N = MB * MB / 64;          // accumulator registers per block
    using AccT = f32x4;
    constexpr int PJ = PT / 64;                  // 64-pixel runs per tile
    constexpr int A_U = 12 * MT, B_U = 12 * PT;  // 16-byte units per stage
    constexpr int A_PW = A_U / 64 / NW;          // A DMA instructions per wave per chunk
    constexpr int WPJ = NW / PJ;                 // waves sharing one pixel run
    constexpr int B_PW = 12 / WPJ;               // B DMA instructions per wave per chunk
    static_assert(NW % PJ == 0 && 12 % WPJ == 0 && A_U % (64 * NW) == 0, "x6 tile");

    constexpr int STAGE_U = A_U + B_U;
    __shared__ __attribute__((aligned(16))) uint4 lds[2 * STAGE_U];
    __shared__ float s_bias[MT];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nM = a.Mpad / MT;
    // geometry of the current tile's group (X6Group N, H, W, npix)
    int H = 0, W = 0, HW = 0, npix = 0, ylo = 0, yspan = 0;
    // pooled conv (a.pool): GEMM columns run over the 2x2 quads of the pooled grid, quad-major
    // (column q -> pooled pixel q >> 2, quadrant q & 3), so the epilogue pools 4 adjacent lanes
    int Wo = 0, HWo = 0;
    auto decode = [&](int p, int& n, int& r) __attribute__((always_inline)) {  // column -> frame, y*W+x
        if (a.pool) {
            const int q = p >> 2, d = p & 3;
            n = q / HWo;
            const int ro = q - n * HWo;
            const int yo = ro / Wo;
            r = (2 * yo + (d >> 1)) * W + 2 * (ro - yo * Wo) + (d & 1);
        } else {
            n = p / HW;
            r = p - n * HW;
        }
    };
    const int wm0 = (wave % NWM) * WM;
    const int wp0 = (wave / NWM) * WP;
    const int jw = wave % PJ;    // this wave's pixel run for the im2col DMA
    const int pg0 = wave / PJ;   // its first (piece, group) row; then every WPJ-th

    const int Gw = gridDim.x;
    const int b = blockIdx.x;
    const int q = Gw >> 3, rr = Gw & 7, xcd = b & 7;
    const int id = xcd * q + min(xcd, rr) + (b >> 3);
    const X6Work wk = x6_work_of(a, id);

    for (int k = wk.k0; k < wk.k1; ++k) {
        const int uid = wk.list ? wk.list[k] : k;
        const X6Unit un = x6_unit_of(a, uid);
        const int tile = un.tile, c_begin = un.c0, c_end = un.c1;
        const X6Group G = a.g[un.g];
        H = G.H;
        W = G.W;
        HW = H * W;
        ylo = G.yhi ? G.ylo : 0;  // rows the taps may read: [0, H), or a row band's halo too
        yspan = (G.yhi ? G.yhi : H) - ylo;
        npix = G.npix;
        Wo = W >> 1;
        HWo = (H >> 1) * Wo;
        const int mt = (tile - G.t0) % nM;
        const int pt = (tile - G.t0) / nM;
        const int p0 = pt * PT;
        const int m0 = mt * MT;

        __syncthreads();
        if (tid < MT) s_bias[tid] = (m0 + tid < G.cout) ? G.bias[m0 + tid] : 0.f;

        // the lane's im2col pixel (run jw): byte offset of its unit in group 0, plane 0
        // (a row band's view starts its buffer resource 3 rows + 3 units early, so the halo
        // taps above the band keep non-negative offsets)
        const uint32_t hshift = G.yhi ? 3u * G.in_l.rs + 3u : 0u;
        const uint8_t* in_base = G.in + (size_t)(G.in_l.o0 - hshift) * 16;
        int py, px;
        uint32_t pbase;
        {
            const int p = p0 + jw * 64 + lane;
            const bool v = p < npix;
            int n, r;
            decode(v ? p : 0, n, r);
            const int y = r / W;
            px = r - y * W;
            py = v ? y : -100000;
            pbase = (n * G.in_l.fs + (uint32_t)y * G.in_l.rs + (uint32_t)px + hshift) * 16u;
        }

        AccT acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < ACC_N; ++r) acc[i][j][r] = 0.f;

        auto tap_off = [&](int tap) __attribute__((always_inline)) -> uint32_t {
            const int ky = tap / ks;
            const int dy = ky - a.pad, dx = tap - ky * ks - a.pad;
            const int iy = py + dy, ix = px + dx;
            const bool ok = (unsigned)(iy - ylo) < (unsigned)yspan && (unsigned)ix < (unsigned)W;
            return ok ? pbase + (uint32_t)((dy * (int)G.in_l.rs + dx) * 16) : 0x80000000u;  // >= num_records -> 0
        };
        // im2col DMA of chunk c, unit u of this wave ((piece, group) row pg0 + u * WPJ) into stage buf;
        // voff / cb: the chunk's tap offset and channel block (b_prep).  One buffer resource per
        // piece plane; the group offset rides in soffset, the pixel + tap offset in voffset (the
        // engine keeps a plane below 2^31 bytes, so 0x80000000 stays out of range either way)
        struct BPrep {
            uint32_t voff;
            int cb;
        };
        auto b_prep = [&](int c) __attribute__((always_inline)) -> BPrep {
            BPrep r{0u, 0};
            if constexpr (!SMALL) {
                r.cb = c / taps;
                r.voff = tap_off(c - r.cb * taps);
            }
            return r;
        };
        const uint32_t grp_bytes = G.in_l.gs * 16u;
        auto dma_b_unit = [&](int c, const BPrep& bp, int buf, int u) __attribute__((always_inline)) {
            uint4* Bs = lds + buf * STAGE_U + A_U;
            const int pg = pg0 + u * WPJ;
            const int pc = pg >> 2, gi = pg & 3;
            int grp;
            uint32_t off;
            if constexpr (SMALL) {
                grp = 0;
                off = tap_off(min(c * 4 + gi, taps - 1));  // padded taps: weights are 0
            } else {
                grp = min(bp.cb * 4 + gi, a.cin_g - 1);  // padded groups: any valid data (weights 0)
                off = bp.voff;
            }
            const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(in_base + (size_t)pc * G.in_ps), (short)0, (int)0x80000000u, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(Bs + pg * PT + jw * 64), 16, off,
                                                     (int)((uint32_t)grp * grp_bytes), 0, 0);
        };
        auto dma_b = [&](int c, int buf) __attribute__((always_inline)) {
            const BPrep bp = b_prep(c);
#pragma unroll
            for (int u = 0; u < B_PW; ++u) dma_b_unit(c, bp, buf, u);
        };
        // weights: one buffer resource per chunk, the unit's row offset in soffset, lane * 16 in voffset
        const uint32_t lane16 = (uint32_t)lane * 16u;
        auto dma_a_unit = [&](int c, int buf, int u) __attribute__((always_inline)) {
            uint4* As = lds + buf * STAGE_U;
            const int unit0 = (wave * A_PW + u) * 64;
            const int pg = unit0 / MT, m = unit0 - pg * MT;
            const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(G.wt + (size_t)c * 12 * a.Mpad * 16), (short)0, (int)0x7fffffff, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(As + unit0), 16, lane16,
                                                     (int)((uint32_t)(pg * a.Mpad + m0 + m) * 16u), 0, 0);
        };
        auto dma_a = [&](int c, int buf) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < A_PW; ++u) dma_a_unit(c, buf, u);
        };

        i32x4 fa[1][3][TM], fb[1][3][TN];
        {
            // 16x16x32 MFMAs: a chunk (32 k) is one k-step.  Lane l holds row / pixel (l & 15) and
            // the k-group (l >> 4) of its 16-row block; the LDS layout is the same [piece][group][row]
            // unit array (ds_read_b128's 16-lane phases hit 4 rows of each of 4 groups: conflict free).
            // One fragment set: the 6 piece products run as blocks of TM*TN MFMAs in the order
            //   (0,2) (0,0) (0,1) | barrier | (1,0) (2,0) (1,1)
            // and each piece's registers are refilled with the next chunk's fragments right after
            // their last use in this chunk: R0 = A0, B2 (after block 2), R1 = B0, A2 (after block 4),
            // R2 = B1, A1 (in the next chunk's block 0).  The barrier sits after block 2: by then
            // every wave has read this chunk's stage (R2 waited before block 2) and the next stage
            // has landed (vmcnt(0)), so the next chunk's R0 / R1 reads and the DMA of the chunk
            // after it (into this stage) follow it, interleaved one per MFMA gap.
            constexpr int PA[6] = {0, 0, 0, 1, 2, 1};
            constexpr int PB[6] = {2, 0, 1, 0, 0, 1};
            constexpr int NB = TM * TN;           // MFMAs per block
            constexpr int TMN = TM + TN;          // reads per refill group
            constexpr int NDA = A_PW + B_PW;      // LDS-DMA instructions per chunk
            const int a16 = (lane >> 4) * MT + wm0 + (lane & 15);
            const int b16 = (lane >> 4) * PT + wp0 + (lane & 15);
            auto la = [&](int buf) __attribute__((always_inline)) {
                return (uint32_t)(uintptr_t)(lds_ptr_t)(lds + buf * STAGE_U + a16);
            };
            auto lb = [&](int buf) __attribute__((always_inline)) {
                return (uint32_t)(uintptr_t)(lds_ptr_t)(lds + buf * STAGE_U + A_U + b16);
            };
            // refill group g (0: A0 B2, 1: B0 A2, 2: B1 A1), read r of TMN
            auto rd = [&](int g, int r, uint32_t abase, uint32_t bbase) __attribute__((always_inline)) {
                const bool isA = g == 0 ? r < TM : r >= TN;
                const int k = g == 0 ? (r < TM ? r : r - TM) : (r < TN ? r : r - TN);
                const int pc = g == 0 ? (isA ? 0 : 2) : g == 1 ? (isA ? 2 : 0) : 1;
                if (isA)
                    asm volatile("ds_read_b128 %0, %1 offset:%2"
                                 : "=v"(fa[0][pc][k])
                                 : "v"(abase), "i"((pc * 4 * MT + 16 * k) * 16));
                else
                    asm volatile("ds_read_b128 %0, %1 offset:%2"
                                 : "=v"(fb[0][pc][k])
                                 : "v"(bbase), "i"((pc * 4 * PT + 16 * k) * 16));
            };
            auto mf = [&](int t, int q) __attribute__((always_inline)) {
                const int i = q / TN, j = q % TN;
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[0][PA[t]][i]),
                                                                    __builtin_bit_cast(bf16x8, fb[0][PB[t]][j]),
                                                                    acc[i][j], 0, 0, 0);
            };
            auto fence_all = [&]() __attribute__((always_inline)) {
#pragma unroll
                for (int pc = 0; pc < 3; ++pc) {
#pragma unroll
                    for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(fa[0][pc][i]));
#pragma unroll
                    for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(fb[0][pc][j]));
                }
            };
            dma_a(c_begin, 0);
            dma_b(c_begin, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            {
                const uint32_t a0 = la(0), b0 = lb(0);
#pragma unroll
                for (int r = 0; r < TMN; ++r) rd(0, r, a0, b0);
#pragma unroll
                for (int r = 0; r < TMN; ++r) rd(1, r, a0, b0);
                const int cn = min(c_begin + 1, c_end - 1);
                dma_a(cn, 1);
                dma_b(cn, 1);
            }
            for (int c = c_begin; c < c_end; ++c) {
                const int buf = (c - c_begin) & 1;
                const uint32_t a_cur = la(buf), b_cur = lb(buf);
                const uint32_t a_nxt = la(buf ^ 1), b_nxt = lb(buf ^ 1);
                const int c2 = min(c + 2, c_end - 1);  // past the end: a harmless reload of the last chunk
                const BPrep bp2 = b_prep(c2);
                // block 0 (needs R0): R2 of this chunk interleaved
                asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(TMN > 15 ? 15 : TMN) : "memory");
                fence_all();
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    mf(0, q);
#pragma unroll
                    for (int r = q * TMN / NB; r < (q + 1) * TMN / NB; ++r) rd(2, r, a_cur, b_cur);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // block 1 (needs R1)
                asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(TMN > 15 ? 15 : TMN) : "memory");
                fence_all();
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    mf(1, q);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // block 2 (needs R2)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                fence_all();
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    mf(2, q);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // this stage read by all; the next stage landed (explicit vmcnt(0): the compiler's
                // barrier fence does not reliably count LDS-DMA, see conv_win.hip)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                __builtin_amdgcn_sched_barrier(0);
                // blocks 3-5: R0 (block 3) and R1 (block 5) of the next chunk, DMA of chunk c2
                constexpr int D3 = NDA / 3, D4 = 2 * NDA / 3;
                auto dma_op = [&](int d) __attribute__((always_inline)) {
                    if (d < A_PW) dma_a_unit(c2, buf, d);
                    else dma_b_unit(c2, bp2, buf, d - A_PW);
                };
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    mf(3, q);
                    constexpr int N3 = TMN + D3;
#pragma unroll
                    for (int o = q * N3 / NB; o < (q + 1) * N3 / NB; ++o) {
                        if (o < TMN) rd(0, o, a_nxt, b_nxt);
                        else dma_op(o - TMN);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    mf(4, q);
                    constexpr int N4 = D4 - D3;
#pragma unroll
                    for (int o = q * N4 / NB; o < (q + 1) * N4 / NB; ++o) dma_op(D3 + o);
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    mf(5, q);
                    constexpr int N5 = TMN + NDA - D4;
#pragma unroll
                    for (int o = q * N5 / NB; o < (q + 1) * N5 / NB; ++o) {
                        if (o < TMN) rd(1, o, a_nxt, b_nxt);
                        else dma_op(D4 + o - TMN);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last (unused) reads landed
            fence_all();
        }

        // ---- epilogue
        // accumulator register r of block (i, j): rows (channels) ml0 + (r & 3) of quad r >> 2,
        // column (pixel) pl.  32x32: quad qd covers rows 32i + 8qd + 4hk .. +3, pixel 32j + l31;
        // 16x16: rows 16i + 4(l >> 4) .. +3, pixel 16j + (l & 15).
        const bool whole = un.whole;
        const int cout8 = (G.cout + 7) & ~7;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int pl = wp0 + j * 16 + (lane & 15);
            const int p = p0 + pl;
            auto quad_row = [&](int i, int qd) __attribute__((always_inline)) {
                (void)qd;
                return wm0 + i * 16 + 4 * (lane >> 4);
            };
            if (!whole) {
                static_assert(ACC_N == 4, "slab quads: one 16x16 accumulator block per lane quad");
                const __amdgpu_buffer_rsrc_t srs = slab_rsrc(a.partial);
                const uint32_t sbase = (uint32_t)uid * (uint32_t)(MT * PT * 4);
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    store_slab_quad(srs, sbase + (uint32_t)((quad_row(i, 0) / 4) * PT + pl) * 16u, acc[i][j]);
                continue;
            }
            if (a.pool) {
                // 2x2 max over the quad's 4 lanes, then bias + ReLU (both monotone: identical to
                // pooling the biased, rectified values), one lane per quad stores the pooled pixel.
                // X6 output; the slabs of a multi-slab pooled tile are pooled by conv_x6_fixup.
                const int q = p >> 2;
                const int n = q / HWo;
                const int remo = q - n * HWo;
                const int yo = remo / Wo, xo = remo - yo * Wo;
                const bool lead = (lane & 3) == 0 && p < npix;
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int qd = 0; qd < ACC_N / 4; ++qd) {
                        const int ml = quad_row(i, qd);
                        const int mq = m0 + ml;
                        float v[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            float m = acc[i][j][4 * qd + t];
                            m = fmaxf(m, __shfl_xor(m, 1));
                            m = fmaxf(m, __shfl_xor(m, 2));
                            v[t] = m + s_bias[ml + t];
                            if (G.relu) v[t] = fmaxf(v[t], 0.f);
                        }
                        if (lead && mq < cout8) {
                            const int grp = mq >> 3, half = (mq >> 2) & 1;
                            store4_x6(static_cast<uint8_t*>(G.out) + (size_t)x6_unit(G.out_l, n, grp, yo, xo) * 16 +
                                          half * 8,
                                      G.out_ps, v);
                        }
                    }
                continue;
            }
            if (p >= npix) continue;
            const int n = p / HW;
            const int rem = p - n * HW;
            const int y = rem / W, x = rem - y * W;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int qd = 0; qd < ACC_N / 4; ++qd) {
                    const int ml = quad_row(i, qd);  // first of 4 consecutive channels (half a group)
                    const int mq = m0 + ml;
                    float v[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        v[t] = acc[i][j][4 * qd + t] + s_bias[ml + t];
                        if (G.relu) v[t] = fmaxf(v[t], 0.f);
                    }
                    if (G.out_f32) {
                        float* ob = static_cast<float*>(G.out) + ((size_t)n * G.out_c + G.out_off) * HW + rem;
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int m = mq + t;
                            if (m < G.cout) ob[(size_t)m * HW] = v[t];
                        }
                    } else if (mq < cout8) {
                        const int grp = mq >> 3, half = (mq >> 2) & 1;
                        store4_x6(static_cast<uint8_t*>(G.out) + (size_t)x6_unit(G.out_l, n, grp, y, x) * 16 + half * 8,
                                  G.out_ps, v);
                        if (G.out2)
                            store4_x6(static_cast<uint8_t*>(G.out2) + (size_t)x6_unit(G.out2_l, n, grp, y, x) * 16 +
                                          half * 8,
                                      G.out2_ps, v);
                    }
                }
        }
    }
}

// whole X6 unit (8 channels of one pixel): three 16-byte piece stores
__device__ __forceinline__ void store8_x6(uint8_t* unit, uint32_t ps, const float (&v)[8]) {
    uint32_t h[3][8];
#pragma unroll
    for (int t = 0; t < 8; ++t) split3(v[t], h[0][t], h[1][t], h[2][t]);
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
        uint4 w;
        w.x = h[pc][0] | (h[pc][1] << 16);
        w.y = h[pc][2] | (h[pc][3] << 16);
        w.z = h[pc][4] | (h[pc][5] << 16);
        w.w = h[pc][6] | (h[pc][7] << 16);
        *reinterpret_cast<uint4*>(unit + (size_t)pc * ps) = w;
    }
}

// Slab fixup: grid (tiles, MT*PT/8/256); each thread finishes one X6 unit (8 channels of one
// pixel) of a multi-slab tile: the slab partials folded in slab order, ((s0 + s1) + s2) + ...
// (the order is the group's, not the grid's).  Pixels run fastest across the lanes, so every
// slab load is a coalesced 1 KB run of channel quads (x6.h) and every store a whole 16-byte
// unit; two slabs' loads are in flight per round trip.
template <int MT, int PT>
__global__ __launch_bounds__(256) void conv_x6_fixup(X6Args a) {
    const int nM = a.Mpad / MT;
    const int tile = blockIdx.x;
    const X6Group G = a.g[x6_group_of(a, tile)];
    const int S = G.slabs;
    if (S == 1) return;  // written by the conv
    const int w0 = G.u0 + (tile - G.t0) * S, w1 = w0 + S - 1;  // the tile's slab partials
    const int mt = (tile - G.t0) % nM;
    const int pt = (tile - G.t0) / nM;
    const int HW = G.H * G.W;
    const int e = blockIdx.y * 256 + threadIdx.x;  // < MT/8 * PT
    const int pl = e % PT, ml0 = (e / PT) * 8;
    const int mg = mt * MT + ml0;  // first channel of the unit
    const int p = pt * PT + pl;
    if (p >= G.npix) return;
    const int cout8 = (G.cout + 7) & ~7;
    if (mg >= (G.out_f32 ? G.cout : cout8)) return;
    // the unit's two channel quads (x6.h slab layout): quads ml0/4 and ml0/4 + 1 of column c
    auto slab = [&](int w, int c) __attribute__((always_inline)) {
        return reinterpret_cast<const f32x4*>(a.partial + (size_t)w * (MT * PT)) + (size_t)(ml0 / 4) * PT + c;
    };
    // column c's 8 sums, slab partials folded in slab order
    auto fold = [&](int c, float (&v)[8]) __attribute__((always_inline)) {
        {
            const f32x4* s = slab(w0, c);
            const f32x4 lo = s[0], hi = s[PT];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                v[t] = lo[t];
                v[4 + t] = hi[t];
            }
        }
        int w = w0 + 1;
        for (; w < w1; w += 2) {
            const f32x4 *s0 = slab(w, c), *s1 = slab(w + 1, c);
            const f32x4 a0 = s0[0], a1 = s0[PT], b0 = s1[0], b1 = s1[PT];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                v[t] = (v[t] + a0[t]) + b0[t];
                v[4 + t] = (v[4 + t] + a1[t]) + b1[t];
            }
        }
        if (w == w1) {
            const f32x4* s = slab(w, c);
            const f32x4 lo = s[0], hi = s[PT];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                v[t] += lo[t];
                v[4 + t] += hi[t];
            }
        }
    };
    float v[8];
    if (a.pool) {
        // pooled conv (columns quad-major, the conv's pooled epilogue): the quad's lead thread folds
        // its 4 columns, takes their max, then bias + ReLU, and stores the pooled unit
        if (pl & 3) return;
        fold(pl, v);
#pragma unroll
        for (int c = 1; c < 4; ++c) {
            float u[8];
            fold(pl + c, u);
#pragma unroll
            for (int t = 0; t < 8; ++t) v[t] = fmaxf(v[t], u[t]);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int m = mg + t;
            v[t] += m < G.cout ? G.bias[m] : 0.f;
            if (G.relu) v[t] = fmaxf(v[t], 0.f);
        }
        const int Wo = G.W / 2, HWo = (G.H / 2) * Wo;
        const int q = p >> 2, n = q / HWo, remo = q - n * HWo;
        const int yo = remo / Wo, xo = remo - yo * Wo;
        store8_x6(static_cast<uint8_t*>(G.out) + (size_t)x6_unit(G.out_l, n, mg >> 3, yo, xo) * 16, G.out_ps, v);
        return;
    }
    fold(pl, v);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const int m = mg + t;
        v[t] += m < G.cout ? G.bias[m] : 0.f;
        if (G.relu) v[t] = fmaxf(v[t], 0.f);
    }
    const int n = p / HW;
    const int rem = p - n * HW;
    if (G.out_f32) {
        float* ob = static_cast<float*>(G.out) + ((size_t)n * G.out_c + G.out_off) * HW + rem;
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (mg + t < G.cout) ob[(size_t)(mg + t) * HW] = v[t];
        return;
    }
    const int grp = mg >> 3;
    const int y = rem / G.W, x = rem - y * G.W;
    store8_x6(static_cast<uint8_t*>(G.out) + (size_t)x6_unit(G.out_l, n, grp, y, x) * 16, G.out_ps, v);
    if (G.out2) store8_x6(static_cast<uint8_t*>(G.out2) + (size_t)x6_unit(G.out2_l, n, grp, y, x) * 16, G.out2_ps, v);
}

static int grid_for(size_t total) {
    size_t b = (total + 255) / 256;
    return (int)(b > 8192 ? 8192 : (b ? b : 1));
}

// Zero the padding units of X6P buffers (common.h) of one geometry: per (piece, group) plane the
// 3N + 4 rows outside the frames' pixel rows and the 3 units before each of the N*H pixel rows.
// One launch for up to 8 buffers (blockIdx.y), one thread per padding unit.
struct PadBufs {
    uint4* p[8];
    int planes[8];
};

__global__ __launch_bounds__(256) void x6p_clear_pads_kernel(PadBufs b, size_t plane, int N, int H, int W, int P) {
    const int pad_rows = 3 * N + 4;
    const size_t per_plane = (size_t)pad_rows * P + (size_t)N * H * (P - W);
    uint4* buf = b.p[blockIdx.y];
    const size_t total = per_plane * b.planes[blockIdx.y];
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const size_t pl = e / per_plane;
        size_t u = e - pl * per_plane;
        size_t unit;
        if (u < (size_t)pad_rows * P) {  // whole padding rows: 3 before frame 0, 3 after each frame, 1 extra
            const int pr = (int)(u / P), c = (int)(u - (size_t)pr * P);
            const int row = pr < 3 ? pr : 3 + ((pr - 3) / 3) * (H + 3) + H + (pr - 3) % 3;
            unit = (size_t)(pr >= 3 * N + 3 ? 3 + N * (H + 3) + (pr - 3 * N - 3) : row) * P + c;
        } else {  // the P - W zero units of a pixel row: 3 before its pixels, the rest after them
            u -= (size_t)pad_rows * P;
            const int pw = P - W;
            const int pr = (int)(u / pw), c = (int)(u - (size_t)pr * pw);
            const int n = pr / H, y = pr - n * H;
            unit = (size_t)(3 + n * (H + 3) + y) * P + (c < 3 ? c : c + W);
        }
        buf[pl * plane + unit] = z;
    }
}

void launch_x6p_clear_pads(uint8_t* const* bufs, const int* planes, int nbufs, int N, int H, int W, hipStream_t st) {
    if (nbufs < 1 || nbufs > 8) throw std::invalid_argument("x6p_clear_pads: 1..8 buffers");
    const int P = x6p_pitch(W);
    const size_t plane = (size_t)(N * (H + 3) + 4) * P;
    PadBufs b{};
    int most = 0;
    for (int i = 0; i < nbufs; ++i) {
        b.p[i] = reinterpret_cast<uint4*>(bufs[i]);
        b.planes[i] = planes[i];
        most = std::max(most, planes[i]);
    }
    const size_t pads = ((size_t)(3 * N + 4) * P + (size_t)N * H * (P - W)) * most;
    hipLaunchKernelGGL(x6p_clear_pads_kernel, dim3(std::min(grid_for(pads), 2048), nbufs), dim3(256), 0, st, b, plane,
                       N, H, W, P);
}

// Halo rows of a row band (engine.cpp band_halo): 3 consecutive rows of groups [g0, g0 + ng) of
// each piece plane of a one-frame X6P buffer <-> a packed [piece][group][3 P] unit block.
// blockIdx.y = direction d (0: the band's top edge, 1: its bottom edge), skipped unless bit d of
// mask; row[d]: the padded row (3 + y) of the block's first row.
__global__ __launch_bounds__(256) void x6p_halo_kernel(uint8_t* __restrict__ x6p, uint32_t ps, uint32_t gs, int g0,
                                                       int ng, int P, int row0, int row1, uint4* __restrict__ blk0,
                                                       uint4* __restrict__ blk1, int mask, int unpack) {
    const int d = blockIdx.y;
    if (!((mask >> d) & 1)) return;
    uint4* blk = d ? blk1 : blk0;
    const uint32_t row = (uint32_t)(d ? row1 : row0), per = 3u * (uint32_t)P, total = 3u * (uint32_t)ng * per;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const uint32_t pg = e / per, u = e - pg * per, pc = pg / (uint32_t)ng, g = pg - pc * (uint32_t)ng;
        uint4* x = reinterpret_cast<uint4*>(x6p + (size_t)pc * ps) + (size_t)(g0 + g) * gs + (size_t)row * P + u;
        if (unpack) *x = blk[e];
        else blk[e] = *x;
    }
}

void launch_x6p_halo(uint8_t* x6p, uint32_t ps, uint32_t gs, int g0, int ng, int P, int row0, int row1, void* blk0,
                     void* blk1, int mask, bool unpack, hipStream_t st) {
    if (!mask) return;
    const size_t total = (size_t)9 * ng * P;
    hipLaunchKernelGGL(x6p_halo_kernel, dim3(std::min(grid_for(total), 1024), 2), dim3(256), 0, st, x6p, ps, gs, g0,
                       ng, P, row0, row1, static_cast<uint4*>(blk0), static_cast<uint4*>(blk1), mask, unpack ? 1 : 0);
}

// fp32 NCHW channels [coff, coff + C) of cstride -> X6 groups [goff, goff + ceil(C/8)) of cg
// (channels >= C of the last group are written as 0)
__global__ __launch_bounds__(256) void to_x6_kernel(const float* __restrict__ in, int cstride, int coff, int C, int N,
                                                   int HW, uint8_t* __restrict__ out, int cg, int goff, uint32_t ps) {
    const int G8 = (C + 7) / 8;
    const size_t total = (size_t)N * G8 * HW;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int pix = (int)(e % HW);
        const size_t t = e / HW;
        const int gq = (int)(t % G8);
        const int n = (int)(t / G8);
        uint32_t h[3][8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int c = gq * 8 + k;
            const float x = c < C ? in[((size_t)n * cstride + coff + c) * HW + pix] : 0.f;
            split3(x, h[0][k], h[1][k], h[2][k]);
        }
        uint8_t* o = out + ((size_t)(n * cg + goff + gq) * HW + pix) * 16;
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
            uint4 w;
            w.x = h[pc][0] | (h[pc][1] << 16);
            w.y = h[pc][2] | (h[pc][3] << 16);
            w.z = h[pc][4] | (h[pc][5] << 16);
            w.w = h[pc][6] | (h[pc][7] << 16);
            *reinterpret_cast<uint4*>(o + (size_t)pc * ps) = w;
        }
    }
}

// X6 groups -> fp32 NCHW channels [coff, coff + C) of cstride
__global__ __launch_bounds__(256) void from_x6_kernel(const uint8_t* __restrict__ in, int cg, int goff, uint32_t ps,
                                                     int C, int N, int HW, float* __restrict__ out, int cstride,
                                                     int coff) {
    const int G8 = (C + 7) / 8;
    const size_t total = (size_t)N * G8 * HW;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int pix = (int)(e % HW);
        const size_t t = e / HW;
        const int gq = (int)(t % G8);
        const int n = (int)(t / G8);
        const uint8_t* s = in + ((size_t)(n * cg + goff + gq) * HW + pix) * 16;
        const uint4 w0 = *reinterpret_cast<const uint4*>(s);
        const uint4 w1 = *reinterpret_cast<const uint4*>(s + ps);
        const uint4 w2 = *reinterpret_cast<const uint4*>(s + 2 * (size_t)ps);
        const uint32_t a0[4] = {w0.x, w0.y, w0.z, w0.w}, a1[4] = {w1.x, w1.y, w1.z, w1.w},
                       a2[4] = {w2.x, w2.y, w2.z, w2.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int c = gq * 8 + k;
            if (c >= C) break;
            const int sh = (k & 1) * 16;
            const float x = join3((a0[k >> 1] >> sh) & 0xffffu, (a1[k >> 1] >> sh) & 0xffffu,
                                  (a2[k >> 1] >> sh) & 0xffffu);
            out[((size_t)n * cstride + coff + c) * HW + pix] = x;
        }
    }
}

// MaxPool2d(2, 2) floor mode (src/model.py:10-13) on X6: exact max of the rebuilt fp32 values
__global__ __launch_bounds__(256) void maxpool_x6_kernel(const uint8_t* __restrict__ in, uint32_t ips,
                                                        uint8_t* __restrict__ out, uint32_t ops, int NG, int H, int W) {
    const int Ho = H >> 1, Wo = W >> 1;
    const size_t total = (size_t)NG * Ho * Wo;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(e % Wo);
        const size_t t = e / Wo;
        const int y = (int)(t % Ho);
        const size_t ng = t / Ho;
        float m[8];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint8_t* s = in + ((ng * H + 2 * y + (d >> 1)) * W + 2 * x + (d & 1)) * 16;
            const uint4 w0 = *reinterpret_cast<const uint4*>(s);
            const uint4 w1 = *reinterpret_cast<const uint4*>(s + ips);
            const uint4 w2 = *reinterpret_cast<const uint4*>(s + 2 * (size_t)ips);
            const uint32_t a0[4] = {w0.x, w0.y, w0.z, w0.w}, a1[4] = {w1.x, w1.y, w1.z, w1.w},
                           a2[4] = {w2.x, w2.y, w2.z, w2.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int sh = (k & 1) * 16;
                const float v = join3((a0[k >> 1] >> sh) & 0xffffu, (a1[k >> 1] >> sh) & 0xffffu,
                                      (a2[k >> 1] >> sh) & 0xffffu);
                m[k] = d == 0 ? v : fmaxf(m[k], v);
            }
        }
        uint32_t h[3][8];
#pragma unroll
        for (int k = 0; k < 8; ++k) split3(m[k], h[0][k], h[1][k], h[2][k]);
        uint8_t* o = out + e * 16;
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
            uint4 w;
            w.x = h[pc][0] | (h[pc][1] << 16);
            w.y = h[pc][2] | (h[pc][3] << 16);
            w.z = h[pc][4] | (h[pc][5] << 16);
            w.w = h[pc][6] | (h[pc][7] << 16);
            *reinterpret_cast<uint4*>(o + (size_t)pc * ops) = w;
        }
    }
}

// ------------------------------------------------------------------ host side
// weights [cout][cin][ks][ks] (fp32, physical input channel order) -> X6 chunks
void x6_pack_weights(const float* w, int cout, int cin, int ks, int Mpad, int* nK_out, std::vector<uint16_t>& out) {
    const int taps = ks * ks;
    const int cin_g = (cin + 7) / 8;
    const bool small = cin_g == 1;
    const int nK = small ? (taps + 3) / 4 : ((cin_g + 3) / 4) * taps;
    *nK_out = nK;
    out.assign((size_t)nK * 12 * Mpad * 8, 0);
    auto rne = [](float x) -> uint32_t {
        uint32_t u;
        std::memcpy(&u, &x, 4);
        u += 0x7fffu + ((u >> 16) & 1u);
        return u >> 16;
    };
    auto f = [](uint32_t h) {
        const uint32_t u = h << 16;
        float x;
        std::memcpy(&x, &u, 4);
        return x;
    };
    for (int c = 0; c < nK; ++c)
        for (int gi = 0; gi < 4; ++gi) {
            int tap, grp;
            if (small) {
                tap = c * 4 + gi;
                grp = 0;
            } else {
                tap = c % taps;
                grp = (c / taps) * 4 + gi;
            }
            for (int m = 0; m < cout; ++m)
                for (int e = 0; e < 8; ++e) {
                    const int ch = grp * 8 + e;
                    if (tap >= taps || ch >= cin) continue;
                    const float x = w[((size_t)m * cin + ch) * taps + tap];
                    const uint32_t h0 = rne(x);
                    const float r = x - f(h0);
                    const uint32_t h1 = rne(r);
                    const uint32_t h2 = rne(r - f(h1));
                    const uint32_t hs[3] = {h0, h1, h2};
                    for (int pc = 0; pc < 3; ++pc)
                        out[(((size_t)c * 12 + pc * 4 + gi) * Mpad + m) * 8 + e] = (uint16_t)hs[pc];
                }
        }
}

// number the groups' tiles and work units (X6Group::t0 / u0, X6Args::tiles / units) for an
// MT x PT tile; slabs 0 counts as 1
X6Args x6_number_tiles(const X6Args& a0, int mt, int pt) {
    X6Args a = a0;
    if (a.ngroups < 1 || a.ngroups > kX6Groups || a.Mpad % mt) throw std::invalid_argument("conv_x6: bad groups");
    int t = 0, u = 0;
    for (int g = 0; g < a.ngroups; ++g) {
        X6Group& G = a.g[g];
        if (G.npix <= 0) throw std::invalid_argument("conv_x6: empty group");
        if (G.slabs < 1) G.slabs = 1;
        if (G.slabs > a.nK) throw std::invalid_argument("conv_x6: bad slab count");
        const int tg = (a.Mpad / mt) * ((G.npix + pt - 1) / pt);
        G.t0 = t;
        G.u0 = u;
        t += tg;
        u += tg * G.slabs;
    }
    a.tiles = t;
    a.units = u;
    return a;
}

template <int MT, int PT>
static void launch_x6_tile(const X6Args& a0, hipStream_t st) {
    const X6Args a = x6_number_tiles(a0, MT, PT);
    if (a.sk_grid < 1 || a.sk_grid > a.units) throw std::invalid_argument("conv_x6: bad grid");
    if ((size_t)a.units * MT * PT * 4 >= 0x7fffffffull) throw std::invalid_argument("conv_x6: too many slabs");
    const dim3 blk(64 * x6_waves(MT, PT));
    if (a.small != 0)
        hipLaunchKernelGGL((conv_x6<MT, PT, true, 0>), dim3(a.sk_grid), blk, 0, st, a);
    else if (a.ks == 7)
        hipLaunchKernelGGL((conv_x6<MT, PT, false, 7>), dim3(a.sk_grid), blk, 0, st, a);
    else if (a.ks == 3)
        hipLaunchKernelGGL((conv_x6<MT, PT, false, 3>), dim3(a.sk_grid), blk, 0, st, a);
    else if (a.ks == 1)
        hipLaunchKernelGGL((conv_x6<MT, PT, false, 1>), dim3(a.sk_grid), blk, 0, st, a);
    else
        hipLaunchKernelGGL((conv_x6<MT, PT, false, 0>), dim3(a.sk_grid), blk, 0, st, a);
    if (a.units != a.tiles)
        hipLaunchKernelGGL((conv_x6_fixup<MT, PT>), dim3(a.tiles, MT * PT / 8 / 256), dim3(256), 0, st, a);
}

void launch_conv_x6_fixup(const X6Args& a, int mt, int pt, hipStream_t st) {
    if (mt != 128 || pt != 256) throw std::invalid_argument("conv_x6_fixup: tile");
    hipLaunchKernelGGL((conv_x6_fixup<128, 256>), dim3(a.tiles, 128 * 256 / 8 / 256), dim3(256), 0, st, a);
}

void launch_conv_x6(const X6Args& a, int mt, int pt, hipStream_t st) {
    if (mt == 128 && pt == 128) launch_x6_tile<128, 128>(a, st);
    else if (mt == 128 && pt == 256) launch_x6_tile<128, 256>(a, st);
    else if (mt == 256 && pt == 128) launch_x6_tile<256, 128>(a, st);
    else if (mt == 128 && pt == 64) launch_x6_tile<128, 64>(a, st);
    else if (mt == 64 && pt == 128) launch_x6_tile<64, 128>(a, st);
    else if (mt == 64 && pt == 64) launch_x6_tile<64, 64>(a, st);
    else throw std::invalid_argument("unsupported x6 conv tile");
}


void launch_to_x6(const float* in, int cstride, int coff, int C, int N, int HW, uint8_t* out, int cg, int goff,
                  uint32_t ps, hipStream_t st) {
    hipLaunchKernelGGL(to_x6_kernel, dim3(grid_for((size_t)N * ((C + 7) / 8) * HW)), dim3(256), 0, st, in, cstride,
                       coff, C, N, HW, out, cg, goff, ps);
}

void launch_from_x6(const uint8_t* in, int cg, int goff, uint32_t ps, int C, int N, int HW, float* out, int cstride,
                    int coff, hipStream_t st) {
    hipLaunchKernelGGL(from_x6_kernel, dim3(grid_for((size_t)N * ((C + 7) / 8) * HW)), dim3(256), 0, st, in, cg,
                       goff, ps, C, N, HW, out, cstride, coff);
}

// The first conv (conv1_1: Cin = 3, 3x3, 64 outputs, ReLU; src/model.py:37 / :141) directly on
// the fp32 network input: one thread per output pixel holds its 27 inputs and produces all 64
// channels with fp32 FMAs (packed pairs), weights read as LDS broadcasts, X6 output.  The
// implicit GEMM would pad K = 27 to 3 chunks of 32 and spend the launch on tile prologues; this
// kernel is bound by its 384-byte-per-pixel X6 store.
typedef float f32x2 __attribute__((ext_vector_type(2)));
// F32OUT: the 64 channels as fp32 units of 8 channels (32 bytes, [N][8][H*W] units) for
// conv3_pool_win_x6<true>, which splits them itself: 256 instead of 384 bytes per pixel.
// segment of a multi-segment launch owning block (or tile) b: the last one whose b0 <= b
__device__ __forceinline__ int conv1_seg_of(const Conv1Segs& S, int b) {
    int k = 0;
    while (k + 1 < S.n && b >= S.s[k + 1].b0) ++k;
    return k;
}

template <int CIN, bool F32OUT>
__global__ __launch_bounds__(256) void conv_first_x6_kernel(Conv1Segs S, const float* __restrict__ wt, int Mpad,
                                                            const float* __restrict__ bias) {
    const int sk = conv1_seg_of(S, blockIdx.x);  // this block's segment (a pyramid scale)
    const float* __restrict__ x = static_cast<const float*>(S.s[sk].in);
    const int N = S.s[sk].N, H = S.s[sk].H, W = S.s[sk].W;
    uint8_t* __restrict__ out = S.s[sk].out;
    const uint32_t ops = S.s[sk].ops;
    const int lblock = blockIdx.x - S.s[sk].b0;
    const int lgrid = (sk + 1 < S.n ? S.s[sk + 1].b0 : (int)gridDim.x) - S.s[sk].b0;
    // weights (K x 64, K order (channel, tap)) and bias staged once per workgroup: the inner loop
    // reads them as LDS broadcasts instead of waiting on a global load per tap (0.395 -> 0.338 ms
    // per 32-frame step; two pixels per thread made the compiler hold a group's 54 weight reads
    // and the gather addresses at once, 420 VGPRs, and ran 3x slower)
    constexpr int K = CIN * 9;
    __shared__ __attribute__((aligned(16))) float s_w[K * 64];
    __shared__ __attribute__((aligned(16))) float s_b[64];
    for (int i = threadIdx.x; i < K * 64; i += blockDim.x) s_w[i] = wt[(size_t)(i >> 6) * Mpad + (i & 63)];
    if (threadIdx.x < 64) s_b[threadIdx.x] = bias[threadIdx.x];
    __syncthreads();
    const int HW = H * W;
    const size_t total = (size_t)N * HW;
    for (size_t e = (size_t)lblock * blockDim.x + threadIdx.x; e < total; e += (size_t)lgrid * blockDim.x) {
        const int n = (int)(e / HW);
        const int r = (int)(e - (size_t)n * HW);
        const int y = r / W, xx = r - (r / W) * W;
        float in[CIN * 9];
#pragma unroll
        for (int c = 0; c < CIN; ++c)
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int iy = y + t / 3 - 1, ix = xx + t % 3 - 1;
                const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
                in[c * 9 + t] = ok ? x[((size_t)n * CIN + c) * HW + iy * W + ix] : 0.f;
            }
        uint8_t* o = out + ((size_t)n * 8 * HW + r) * 16;
#pragma unroll 1
        for (int g = 0; g < 8; ++g) {
            f32x2 acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const f32x2 xv = {in[k], in[k]};
                const float4 w0 = *reinterpret_cast<const float4*>(s_w + k * 64 + g * 8);
                const float4 w1 = *reinterpret_cast<const float4*>(s_w + k * 64 + g * 8 + 4);
                acc[0] = __builtin_elementwise_fma(xv, f32x2{w0.x, w0.y}, acc[0]);
                acc[1] = __builtin_elementwise_fma(xv, f32x2{w0.z, w0.w}, acc[1]);
                acc[2] = __builtin_elementwise_fma(xv, f32x2{w1.x, w1.y}, acc[2]);
                acc[3] = __builtin_elementwise_fma(xv, f32x2{w1.z, w1.w}, acc[3]);
            }
            float v[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[2 * q] = fmaxf(acc[q].x + s_b[g * 8 + 2 * q], 0.f);
                v[2 * q + 1] = fmaxf(acc[q].y + s_b[g * 8 + 2 * q + 1], 0.f);
            }
            if constexpr (F32OUT) {
                float4* u = reinterpret_cast<float4*>(out + (((size_t)n * 8 + g) * HW + r) * 32);
                u[0] = make_float4(v[0], v[1], v[2], v[3]);
                u[1] = make_float4(v[4], v[5], v[6], v[7]);
                continue;
            }
            uint32_t hp[3][8];
#pragma unroll
            for (int k = 0; k < 8; ++k) split3(v[k], hp[0][k], hp[1][k], hp[2][k]);
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) {
                uint4 w4;
                w4.x = hp[pc][0] | (hp[pc][1] << 16);
                w4.y = hp[pc][2] | (hp[pc][3] << 16);
                w4.z = hp[pc][4] | (hp[pc][5] << 16);
                w4.w = hp[pc][6] | (hp[pc][7] << 16);
                *reinterpret_cast<uint4*>(o + (size_t)g * HW * 16 + (size_t)pc * ops) = w4;
            }
        }
    }
}

void launch_conv_first_x6_segs(Conv1Segs S, const float* wt, int Mpad, const float* bias, bool f32_out,
                               hipStream_t st) {
    if (S.n < 1 || S.n > kConv1Segs) throw std::invalid_argument("conv_first_x6: segment count");
    int grid = 0;
    for (int k = 0; k < S.n; ++k) {
        S.s[k].b0 = grid;
        grid += grid_for((size_t)S.s[k].N * S.s[k].H * S.s[k].W);
    }
    if (f32_out)
        hipLaunchKernelGGL((conv_first_x6_kernel<3, true>), dim3(grid), dim3(256), 0, st, S, wt, Mpad, bias);
    else
        hipLaunchKernelGGL((conv_first_x6_kernel<3, false>), dim3(grid), dim3(256), 0, st, S, wt, Mpad, bias);
}

void launch_conv_first_x6(const float* x, int N, int Cin, int H, int W, const float* wt, int Mpad, const float* bias,
                          uint8_t* out, uint32_t ops, bool f32_out, hipStream_t st) {
    if (Cin != 3) throw std::invalid_argument("conv_first_x6: Cin must be 3");
    Conv1Segs S{};
    S.n = 1;
    S.s[0] = Conv1Seg{x, out, 0u, ops, N, H, W, 0};
    launch_conv_first_x6_segs(S, wt, Mpad, bias, f32_out, st);
}

// ---------------------------------------------------------------- windowed conv1_2 (+ pool)
// conv1_2 (64 -> 64 channels, 3x3, pad 1) + MaxPool2d(2, 2) from conv1_1's X6 tensor, with the
// im2col operand replaced by a window (src/model.py:35-37 / :145-147).  conv_x6 streams each
// input unit through L2 -> LDS once per tap (9x) and, at M = 64, once per 64 output channels:
// 442 KB of im2col + 221 KB of weights per 64 x 128 tile, 10 GB per bench step.  Here a
// workgroup owns an 8 x 16 tile of conv1_2 outputs (4 x 8 pooled pixels) of one frame and, per
// channel block (4 groups = 32 channels), DMAs the 10 x 18 input window once (69 KB per tile for
// both blocks) and reads the nine taps' B fragments from it at the tap's offset:
//  * window [piece][group][row (pitch 24 units)][col]: the pitch (== 8 mod 16 units) and the
//    group pitch (== 0 mod 16) put every ds_read_b128 lane group on 16 distinct bank quads;
//    the pad columns 18..23 and the frame border load zeros through the buffer
//    range check (conv1_2's zero padding);
//  * 18 k-chunks (2 channel blocks x 9 taps) in the weight layout of conv_x6 (one chunk = 12
//    (piece, group) rows of 64 units), two weight stages by LDS-DMA, one barrier per chunk;
//    4 waves, each 64 channels x 32 GEMM columns (one pooled row of 8 pixels x their 4
//    quadrants): every A fragment read serves two column blocks (8 waves of 16 columns read
//    245 KB of LDS per chunk and CU, more than the MFMAs take at 128 B/clk); the six piece
//    products in conv_x6's order: bit-identical to the conv_x6 pooled launch;
//  * the fragments of chunk c + 1 are read during chunk c's MFMAs (two register sets); the second
//    block's window is DMA'd over the first block's buffer behind chunk 8's MFMAs;
//  * 70 KB of LDS: two workgroups per CU cover each other's DMA waits, barriers and epilogues.
namespace {
constexpr int V_TH = 8, V_TW = 16;                 // conv1_2 outputs per tile
constexpr int V_WR = V_TH + 2, V_WC = V_TW + 2;    // window 10 x 18
constexpr int V_RP = 24;                           // window row pitch (units)
constexpr int V_GP = V_WR * V_RP;                  // 240 units per channel group
constexpr int V_PP = 4 * V_GP;                     // 960 units per piece (one channel block)
constexpr int V_WIN = 3 * V_PP;                    // 2880 units
constexpr int V_DMA = V_WIN / 64;                  // 45 window DMA instructions
constexpr int V_NW = 4;                            // waves: 64 channels x 32 GEMM columns each
static_assert(V_RP % 16 == 8 && V_GP % 16 == 0 && V_RP >= V_WC && V_PP % 64 == 0, "conv1_2 window pitches");
struct WinSmem {
    uint4 win[V_WIN];
    uint4 a[2][12 * 64];
    float b[64];
};
}  // namespace

// F32IN: the input is conv_first_x6<.., true>'s fp32 units; each thread loads its window units
// into registers and writes their three bf16 pieces (split3, as the X6 epilogue would have) into
// the same LDS window (block 1's when every wave is past block 0's reads; the other workgroup on
// the CU covers the load latency).
template <bool F32IN>
__global__ __launch_bounds__(256, 2) void conv3_pool_win_x6_kernel(Conv1Segs S, const uint8_t* __restrict__ wt,
                                                                   const float* __restrict__ bias) {
    __shared__ WinSmem sm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int t;
    {
        const int Gw = gridDim.x, b = blockIdx.x;
        const int q = Gw >> 3, rr = Gw & 7, xcd = b & 7;
        t = xcd * q + min(xcd, rr) + (b >> 3);  // XCD-contiguous tiles (guide T1)
    }
    const int sk = conv1_seg_of(S, t);  // the tile's segment (a pyramid scale)
    const uint8_t* __restrict__ in = static_cast<const uint8_t*>(S.s[sk].in);
    uint8_t* __restrict__ out = S.s[sk].out;
    const uint32_t ips = S.s[sk].ips, ops = S.s[sk].ops;
    const int H = S.s[sk].H, W = S.s[sk].W;
    t -= S.s[sk].b0;
    const int ntx = (W + V_TW - 1) / V_TW, nty = (H + V_TH - 1) / V_TH;
    int n, y0, x0;
    {
        const int tx = t % ntx, rest = t / ntx;
        x0 = tx * V_TW;
        y0 = (rest % nty) * V_TH;
        n = rest / nty;
    }
    const size_t HW = (size_t)H * W;
    // window of channel block cb: instruction i (wave-strided) fills units [64 i, 64 i + 64)
    auto dma_win = [&](int cb) __attribute__((always_inline)) {
        for (int i = wave; i < V_DMA; i += V_NW) {
            const int pc = (64 * i) / V_PP;
            const int u = 64 * i - pc * V_PP + lane;
            const int gl = u / V_GP, r = u - gl * V_GP;
            const int wr = r / V_RP, wc = r - wr * V_RP;
            const int iy = y0 - 1 + wr, ix = x0 - 1 + wc;
            const bool ok = wc < V_WC && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
            const uint32_t off = ok ? (uint32_t)(((size_t)(n * 8 + cb * 4 + gl) * HW + (size_t)iy * W + ix) * 16)
                                    : 0x80000000u;  // >= num_records -> 0
            const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(in + (size_t)pc * ips), (short)0, (int)0x80000000u, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(sm.win + 64 * i), 16, off, 0, 0, 0);
        }
    };
    // fp32 input: window slot u = tid + 256 k of block cb (k < 4, u < V_PP), 8 channels each, in
    // named registers (an array here made the compiler put the fragment arrays in scratch, where
    // the asm ds_reads' results were copied before they landed)
    static_assert((V_PP + 255) / 256 == 4, "four window slots per thread");
    f32x4 w0a, w0b, w1a, w1b, w2a, w2b, w3a, w3b;
    auto load_slot = [&](int k, int cb, f32x4& a, f32x4& b) __attribute__((always_inline)) {
        const int u = tid + 256 * k;
        const int gl = u / V_GP, r = u - gl * V_GP;
        const int wr = r / V_RP, wc = r - wr * V_RP;
        const int iy = y0 - 1 + wr, ix = x0 - 1 + wc;
        const bool ok = u < V_PP && wc < V_WC && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        // unconditional loads (a padding slot reads its frame's first pixel), then a select
        const size_t off = ok ? ((size_t)(n * 8 + cb * 4 + gl) * HW + (size_t)iy * W + ix) * 32
                              : (size_t)n * 8 * HW * 32;
        const f32x4* src = reinterpret_cast<const f32x4*>(in + off);
        const f32x4 a0 = src[0], a1 = src[1];
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        a = ok ? a0 : z;
        b = ok ? a1 : z;
    };
    auto load_win32 = [&](int cb) __attribute__((always_inline)) {
        load_slot(0, cb, w0a, w0b);
        load_slot(1, cb, w1a, w1b);
        load_slot(2, cb, w2a, w2b);
        load_slot(3, cb, w3a, w3b);
    };
    auto store_slot = [&](int k, const f32x4& a, const f32x4& b) __attribute__((always_inline)) {
        const int u = tid + 256 * k;
        if (u >= V_PP) return;
        uint32_t hp[3][8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            split3(a[e], hp[0][e], hp[1][e], hp[2][e]);
            split3(b[e], hp[0][4 + e], hp[1][4 + e], hp[2][4 + e]);
        }
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
            i32x4 w4;
            w4[0] = (int)(hp[pc][0] | (hp[pc][1] << 16));
            w4[1] = (int)(hp[pc][2] | (hp[pc][3] << 16));
            w4[2] = (int)(hp[pc][4] | (hp[pc][5] << 16));
            w4[3] = (int)(hp[pc][6] | (hp[pc][7] << 16));
            // the window is only read by inline-asm ds_reads the compiler cannot see, so it is
            // written by asm too (waited for with an explicit lgkmcnt before the barrier that
            // publishes it)
            const uint32_t wa = (uint32_t)(uintptr_t)(lds_ptr_t)(sm.win + pc * V_PP + u);
            asm volatile("ds_write_b128 %0, %1\n\ts_nop 1" ::"v"(wa), "v"(w4) : "memory");
        }
    };
    auto store_win32 = [&]() __attribute__((always_inline)) {
        store_slot(0, w0a, w0b);
        store_slot(1, w1a, w1b);
        store_slot(2, w2a, w2b);
        store_slot(3, w3a, w3b);
    };
    auto dma_a = [&](int c, int st) __attribute__((always_inline)) {
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(wt + (size_t)c * 12 * 64 * 16), (short)0, (int)0x7fffffff, 0x00020000);
#pragma unroll
        for (int row = wave; row < 12; row += V_NW)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(sm.a[st] + row * 64), 16,
                                                     (uint32_t)lane * 16u, row * 64 * 16, 0, 0);
    };
    if constexpr (F32IN) {
        load_win32(0);
        store_win32();
    } else {
        dma_win(0);
    }
    dma_a(0, 0);
    dma_a(1, 1);
    if (tid < 64) sm.b[tid] = bias[tid];
    // this wave's 32 GEMM columns = pooled row `wave`, pooled cols 4 nb + (q >> 2) for column
    // blocks nb = 0, 1, quad-major; lane column q = lane & 15, k-group gi = lane >> 4
    const int q = lane & 15, gi = lane >> 4;
    const int d = q & 3;
    const int ty = 2 * wave + (d >> 1);
    constexpr int PA[6] = {0, 0, 0, 1, 2, 1};
    constexpr int PB[6] = {2, 0, 1, 0, 0, 1};
    f32x4 acc[2][4];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) acc[nb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
    i32x4 fb[2][2][3], fa[2][4][3];
    auto read_frags = [&](int c, int set) __attribute__((always_inline)) {
        const int tap = c % 9;
        const int dy = tap / 3, dx = tap - dy * 3;
        const uint32_t aw = (uint32_t)(uintptr_t)(lds_ptr_t)(sm.a[c & 1] + gi * 64 + q);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int tx = 2 * (4 * nb + (q >> 2)) + (d & 1);
            const uint32_t bw = (uint32_t)(uintptr_t)(lds_ptr_t)(sm.win + gi * V_GP + (ty + dy) * V_RP + (tx + dx));
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fb[set][nb][pc]) : "v"(bw), "i"(pc * V_PP * 16));
        }
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
                asm volatile("ds_read_b128 %0, %1 offset:%2"
                             : "=v"(fa[set][mb][pc])
                             : "v"(aw), "i"((pc * 4 * 64 + mb * 16) * 16));
    };
    auto fence_set = [&](int set) __attribute__((always_inline)) {
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) asm volatile("" : "+v"(fb[set][nb][pc]));
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) asm volatile("" : "+v"(fa[set][mb][pc]));
    };
    auto mfma_chunk = [&](int set) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tt = 0; tt < 6; ++tt)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int mb = 0; mb < 4; ++mb)
                    acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, fa[set][mb][PA[tt]]), __builtin_bit_cast(bf16x8, fb[set][nb][PB[tt]]),
                        acc[nb][mb], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // window block 0, weight chunks 0 and 1
    __syncthreads();
    read_frags(0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence_set(0);
    // chunk c's fragments are in register set c & 1 and its weights in stage c & 1; the reads of
    // chunk c + 1 are issued before chunk c's MFMAs and waited for after them
    // (three loops, each fully unrolled: as one loop with chunk 8's window switch inside, the
    // fp32-input instantiation was too large for the unroller, and a rolled loop keeps the
    // fragment register sets in scratch)
    auto chunk = [&](int c) __attribute__((always_inline)) {
        const int set = c & 1;
        if (c + 1 < 18) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // weight chunk c + 1 (issued at c - 1)
            __syncthreads();  // ... landed everywhere; every wave is past chunk c's reads
            if (c + 2 < 18) dma_a(c + 2, c & 1);
            read_frags(c + 1, set ^ 1);
        }
        mfma_chunk(set);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        fence_set(set ^ 1);
    };
#pragma unroll
    for (int c = 0; c < 8; ++c) chunk(c);
    {
        // every wave is past chunk 7 (chunk 8's fragments in registers): block 1's window
        // replaces block 0's and weight chunk 10 goes into chunk 8's stage, behind chunk 8's
        // MFMAs
        __syncthreads();
        if constexpr (F32IN) {
            load_win32(1);
            store_win32();
        } else {
            dma_win(1);
        }
        dma_a(10, 0);
        mfma_chunk(0);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __syncthreads();
        read_frags(9, 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        fence_set(1);
    }
#pragma unroll
    for (int c = 9; c < 18; ++c) chunk(c);
    // pooled epilogue: lane holds channels 16 mb + 4 gi + (0..3) of column q of block nb
    const int Wo = W >> 1, Ho = H >> 1;
    const size_t HWo = (size_t)Ho * Wo;
    const int py = (y0 >> 1) + wave;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        const int px = (x0 >> 1) + 4 * nb + (q >> 2);
        const bool lead = (lane & 3) == 0 && px < Wo && py < Ho;
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            const int m = mb * 16 + 4 * gi;
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float mx = acc[nb][mb][j];
                mx = fmaxf(mx, __shfl_xor(mx, 1));
                mx = fmaxf(mx, __shfl_xor(mx, 2));
                v[j] = fmaxf(mx + sm.b[m + j], 0.f);
            }
            if (lead)
                store4_x6(out + (((size_t)n * 8 + (m >> 3)) * HWo + (size_t)py * Wo + px) * 16 + ((m >> 2) & 1) * 8,
                          ops, v);
        }
    }
}

void launch_conv3_pool_win_x6_segs(Conv1Segs S, const uint8_t* wt, const float* bias, bool f32_in, hipStream_t st) {
    if (S.n < 1 || S.n > kConv1Segs) throw std::invalid_argument("conv3_pool_win_x6: segment count");
    int tiles = 0;
    for (int k = 0; k < S.n; ++k) {
        const Conv1Seg& g = S.s[k];
        if (g.H < 2 || g.W < 2 || (size_t)g.N * 8 * g.H * g.W * 16 >= 0x80000000ull)
            throw std::invalid_argument("conv3_pool_win_x6: frame shape out of range");
        S.s[k].b0 = tiles;
        tiles += g.N * ((g.H + V_TH - 1) / V_TH) * ((g.W + V_TW - 1) / V_TW);
    }
    if (f32_in)
        hipLaunchKernelGGL(conv3_pool_win_x6_kernel<true>, dim3(tiles), dim3(64 * V_NW), 0, st, S, wt, bias);
    else
        hipLaunchKernelGGL(conv3_pool_win_x6_kernel<false>, dim3(tiles), dim3(64 * V_NW), 0, st, S, wt, bias);
}

void launch_conv3_pool_win_x6(const uint8_t* in, uint32_t ips, int N, int H, int W, const uint8_t* wt,
                              const float* bias, uint8_t* out, uint32_t ops, bool f32_in, hipStream_t st) {
    Conv1Segs S{};
    S.n = 1;
    S.s[0] = Conv1Seg{in, out, ips, ops, N, H, W, 0};
    launch_conv3_pool_win_x6_segs(S, wt, bias, f32_in, st);
}

void launch_maxpool_x6(const uint8_t* in, uint32_t ips, uint8_t* out, uint32_t ops, int NG, int H, int W,
                       hipStream_t st) {
    hipLaunchKernelGGL(maxpool_x6_kernel, dim3(grid_for((size_t)NG * (H / 2) * (W / 2))), dim3(256), 0, st, in, ips,
                       out, ops, NG, H, W);
}

}  // namespace opose
