// conv_win.hip — the 7x7 CPM convolutions (src/model.py:71-85 Mconv1-5 of stages 2-6, body and
// hand) as split-bf16 implicit GEMMs whose im2col operand comes from an input window in LDS.
//
// conv_x6 streams the im2col tile of every 32-deep k chunk through L2 into LDS by LDS-DMA: at
// 7x7 each input unit travels 49 times, 2/3 of the kernel's DMA instructions and LDS-DMA bytes.
// Here the input is the padded X6P layout (common.h): every tap of a pixel is the unit at a
// constant shift dy*P + dx, and the units of a run of PT consecutive pixels (across rows and
// frames) plus its 3-row halo form one contiguous range of each (piece, group) plane.  So a
// workgroup DMAs, per input channel group, that window (3 pieces x L <= WMAX units, once per 49
// taps) and reads the B fragment of (group, tap) for pixel p at window position wpos(p) + dy*P +
// dx with ds_read_b128.
//  * K order (pair order): k = (pair q, channel c of its group), pair q = (group q / 49, tap
//    q % 49), chunk = 4 consecutive pairs = the four 8-k groups of a 16x16x32 MFMA k-step; the
//    weights are packed in this order (x6_pack_weights_pairs).  A chunk may span two channel
//    groups: two window buffers, group g in buffer g & 1, the window of group g + 2 DMA'd right
//    after the barrier of the last chunk that reads group g (>= 10 chunks before its first use).
//  * Everything else is conv_x6's MODE-2 loop: 128 x 256 tile, 8 waves of 64 x 64, weights by
//    LDS-DMA into two stages, six piece products per chunk in the order
//    (0,2) (0,0) (0,1) | barrier | (1,0) (2,0) (1,1), fragments refilled after their last use.
//  * Work units (tile, k slab): a group's tiles sum their chunks in `slabs` fixed ranges
//    (common.h X6Group), so the order of every pixel's sum is set by the layer and the segment,
//    not by the grid; a workgroup runs a list of units (data parallel: one whole tile), a slab
//    of a multi-slab tile leaves a partial that conv_x6_fixup folds in slab order.  A slab may
//    start inside a channel group (its first two windows are loaded in the prologue).  The host
//    falls back to conv_x6 when a window would exceed WMAX.
//  * The groups of a launch (X6Group: CPM branches, pyramid scales) each carry their own
//    geometry; a tile's window and pixels come from its group.
//  * The same kernel runs the batched 3x3 convs on padded inputs (trunk conv3_x / conv4_x and
//    the stage-1 CPM convs, src/model.py:41-62): a window per group serves 9 taps.
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "x6.h"

namespace opose {

template <int MT, int PT, int KS, int WMAX, int NST>
__global__ __launch_bounds__(64 * x6_waves(MT, PT), 1) void conv_win_x6(X6Args a) {
    constexpr int TAPS = KS * KS, PAD = KS / 2;
    constexpr int NW = x6_waves(MT, PT), NWM = NW == 8 ? MT / 64 : 2, NWP = NW / NWM;
    constexpr int WM = MT / NWM, WP = PT / NWP;
    constexpr int TM = WM / 16, TN = WP / 16;
    constexpr int A_U = 12 * MT;                 // 16-byte units per weight stage
    constexpr int A_PW = A_U / 64 / NW;          // weight DMA instructions per wave per chunk
    constexpr int WBUF = 3 * WMAX;               // units per window buffer (3 pieces)
    // TAPS >= 9: a group ends at most once per chunk, and the window of group g + 2 (issued after
    // the last chunk of group g) lands at least one barrier before its first read
    static_assert(A_U % (64 * NW) == 0 && A_PW == 3 && WMAX % 64 == 0 && TAPS >= 9, "conv_win_x6 tile");
    // NST weight stages: the DMA of chunk c + NST goes into chunk c's stage right after chunk c's
    // barrier, so a stage has NST - 1 chunks to land
    static_assert(NST == 2 || NST == 3, "conv_win_x6 stages");
    constexpr int WOFF = NST * A_U;              // window buffers after the weight stages
    static_assert(TM * TN >= 3, "block 4 hosts the offset steps");

    __shared__ __attribute__((aligned(16))) uint4 lds[NST * A_U + 2 * WBUF];
    __shared__ float s_bias[MT];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nM = a.Mpad / MT;
    const int wm0 = (wave % NWM) * WM;
    const int wp0 = (wave / NWM) * WP;
    // two waves per SIMD: the younger half issues first when both are ready (guide T5, static form)
    if (NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);

    // this workgroup's work units (tile, k slab), XCD-contiguous ids (guide T1); a grid of one
    // workgroup per whole tile is the data-parallel case
    const int Gw = gridDim.x;
    int id;
    {
        const int b = blockIdx.x, q = Gw >> 3, rr = Gw & 7, xcd = b & 7;
        id = xcd * q + min(xcd, rr) + (b >> 3);
    }
    const X6Work wk = x6_work_of(a, id);
    for (int k = wk.k0; k < wk.k1; ++k) {
    const int uid = wk.list ? wk.list[k] : k;
    const X6Unit un = x6_unit_of(a, uid);
    const int tile = un.tile, c_begin = un.c0, c_end = un.c1;
    const X6Group G = a.g[un.g];
    const int H = G.H, W = G.W, HW = H * W, npix = G.npix;
    const int mt = (tile - G.t0) % nM;
    const int ptl = (tile - G.t0) / nM;
    const int p0 = ptl * PT, m0 = mt * MT;
    __syncthreads();  // the previous piece's LDS reads are done
    if (tid < MT) s_bias[tid] = (m0 + tid < G.cout) ? G.bias[m0 + tid] : 0.f;

    // ---- window geometry (wave-uniform): padded rows R of the tile's first / last pixel
    const int P = (int)G.in_l.rs;
    auto prow = [&](int p) __attribute__((always_inline)) {
        const int n = p / HW, y = (p - n * HW) / W;
        return 3 + n * (H + 3) + y;
    };
    const int p_last = min(p0 + PT, npix) - 1;
    const int R0 = prow(p0), R1 = prow(p_last);
    const int ws = (R0 - PAD) * P;                                // window start (unit of the plane)
    const int L = (R1 - R0 + 2 * PAD + 1) * P + PAD;              // units the taps can touch
    const int NQ = (L + 63) >> 6;                                 // DMA instructions per piece
    const uint32_t plane0 = G.in_l.o0 - 3u * (uint32_t)P - 3u;    // plane start of the slice's group 0
    const int cin_g = a.cin_g;

    // window of input group g -> buffer g & 1 (units [ws, ws + 64 NQ) of each piece plane)
    auto dma_win = [&](int g) __attribute__((always_inline)) {
        const uint32_t src = (plane0 + (uint32_t)g * G.in_l.gs + (uint32_t)ws) * 16u;
        uint4* dst = lds + WOFF + (g & 1) * WBUF;
        for (int i = wave; i < 3 * NQ; i += NW) {
            const int pc = i / NQ, j = i - pc * NQ;
            const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(G.in + (size_t)pc * G.in_ps), (short)0, (int)G.in_ps, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(dst + pc * WMAX + 64 * j), 16,
                                                     src + (uint32_t)(64 * j + lane) * 16u, 0, 0, 0);
        }
    };
    // weights: one buffer resource per chunk, the unit's row offset in soffset, lane * 16 in voffset
    const uint32_t lane16 = (uint32_t)lane * 16u;
    auto dma_a_unit = [&](int c, int buf, int u) __attribute__((always_inline)) {
        uint4* As = lds + buf * A_U;
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

    // ---- per-lane B fragment addresses: lane (k-group gi = lane >> 4, pixel lane & 15 of block j)
    const int gi = lane >> 4;
    uint32_t bbase[TN];  // LDS byte address of the lane's pixel unit (window buffer 0, piece 0)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int p = min(p0 + wp0 + 16 * j + (lane & 15), npix - 1);  // past the end: any window unit
        const int n = p / HW, r = p - n * HW, y = r / W, x = r - y * W;
        const int wpos = (3 + n * (H + 3) + y) * P + 3 + x - ws;
        bbase[j] = (uint32_t)(uintptr_t)(lds_ptr_t)(lds + WOFF + wpos);
    }
    // pair of this lane's k-group in a chunk: q = 4c + gi -> (group g, tap t), advanced by 4 per
    // chunk.  Chunk c + 1's fragment offsets are needed at chunk c's top; they are computed one
    // chunk ahead in OFF_STEPS pieces, one per MFMA gap of block 4, off the chunk's critical path
    // (computed at the chunk's top, their VALU chain delayed block 0: 7x7 launch 0.357 -> 0.353 ms)
    int pg_g = (4 * c_begin + gi) / TAPS, pg_t = (4 * c_begin + gi) % TAPS;  // chunk c_begin
    int s_dy = 0, s_dx = 0;
    uint32_t off_n = 0;
    constexpr int OFF_STEPS = 3;
    auto off_step = [&](int k) __attribute__((always_inline)) {
        if (k == 0) {
            s_dy = pg_t / KS;
            s_dx = pg_t - s_dy * KS - PAD;
            s_dy -= PAD;
        } else if (k == 1) {  // padded pairs past the last group: its data (weights 0)
            off_n = (uint32_t)((min(pg_g, cin_g - 1) & 1) * WBUF * 16 + (s_dy * P + s_dx) * 16);
        } else {  // advance to the next chunk's pair (branch-free)
            const int w = pg_t + 4 >= TAPS ? 1 : 0;
            pg_t = pg_t + 4 - w * TAPS;
            pg_g += w;
        }
    };
    auto off_all = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < OFF_STEPS; ++k) off_step(k);
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    i32x4 fa[3][TM], fb[3][TN];
    constexpr int PA[6] = {0, 0, 0, 1, 2, 1};
    constexpr int PB[6] = {2, 0, 1, 0, 0, 1};
    constexpr int NB = TM * TN;
    constexpr int TMN = TM + TN;
    const int a16 = (lane >> 4) * MT + wm0 + (lane & 15);
    auto la = [&](int buf) __attribute__((always_inline)) {
        return (uint32_t)(uintptr_t)(lds_ptr_t)(lds + buf * A_U + a16);
    };
    // refill group g (0: A0 B2, 1: B0 A2, 2: B1 A1), read r of TMN; B addresses of the chunk in bq
    auto rd = [&](int g, int r, uint32_t abase, const uint32_t (&bq)[TN]) __attribute__((always_inline)) {
        const bool isA = g == 0 ? r < TM : r >= TN;
        const int k = g == 0 ? (r < TM ? r : r - TM) : (r < TN ? r : r - TN);
        const int pc = g == 0 ? (isA ? 0 : 2) : g == 1 ? (isA ? 2 : 0) : 1;
        if (isA)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[pc][k]) : "v"(abase), "i"((pc * 4 * MT + 16 * k) * 16));
        else
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fb[pc][k]) : "v"(bq[k]), "i"(pc * WMAX * 16));
    };
    auto mf = [&](int t, int q) __attribute__((always_inline)) {
        const int i = q / TN, j = q % TN;
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[PA[t]][i]),
                                                            __builtin_bit_cast(bf16x8, fb[PB[t]][j]), acc[i][j], 0,
                                                            0, 0);
    };
    auto fence_all = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
#pragma unroll
            for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(fa[pc][i]));
#pragma unroll
            for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(fb[pc][j]));
        }
    };

    // ---- prologue: windows of the first two groups the range reads, weight stages of its first
    // two chunks
    const int g_first = (4 * c_begin) / TAPS;
    dma_win(g_first);
    if (g_first + 1 < cin_g) dma_win(g_first + 1);
#pragma unroll
    for (int st = 0; st < NST; ++st) dma_a(min(c_begin + st, c_end - 1), st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // both windows and every stage landed everywhere
    uint32_t bcur[TN], bnxt[TN];
    {
        off_all();  // chunk c_begin
#pragma unroll
        for (int j = 0; j < TN; ++j) bnxt[j] = bbase[j] + off_n;  // chunk 0
        off_all();  // chunk c_begin + 1, read at the first chunk's top
        const uint32_t a0 = la(0);
#pragma unroll
        for (int r = 0; r < TMN; ++r) rd(0, r, a0, bnxt);
#pragma unroll
        for (int r = 0; r < TMN; ++r) rd(1, r, a0, bnxt);
    }
    // group whose last chunk comes next, and that chunk: its buffer is refilled after that barrier
    int end_g = g_first;
    int end_c = (g_first * TAPS + TAPS - 1) / 4;
    int buf = 0;  // stage of chunk c
    for (int c = c_begin; c < c_end; ++c) {
        const int nbuf = buf + 1 == NST ? 0 : buf + 1;
        const uint32_t a_cur = la(buf), a_nxt = la(nbuf);
        const int c2 = min(c + NST, c_end - 1);  // past the end: a harmless reload of the last chunk
#pragma unroll
        for (int j = 0; j < TN; ++j) bcur[j] = bnxt[j];
#pragma unroll
        for (int j = 0; j < TN; ++j) bnxt[j] = bbase[j] + off_n;  // chunk c + 1 (computed in chunk c - 1)
        // block 0 (needs R0): R2 of this chunk interleaved
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(TMN > 15 ? 15 : TMN) : "memory");
        fence_all();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            mf(0, q);
#pragma unroll
            for (int r = q * TMN / NB; r < (q + 1) * TMN / NB; ++r) rd(2, r, a_cur, bcur);
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
        // this weight stage and every fragment of chunk c read by all; the next stage (and any
        // window DMA'd since the previous barrier) landed -- with 3 stages the A_PW DMA
        // instructions of the chunk after it (issued last) may still be in flight.  The vmcnt is
        // explicit: the compiler does not count LDS-DMA as LDS writes at a workgroup barrier (it
        // emitted a bare s_barrier here), and the fragment reads are inline asm it cannot see
        if constexpr (NST == 3)
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(A_PW) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
        if (c == end_c) {  // group end_g is read for the last time: its buffer takes group end_g + 2
            if (end_g + 2 < cin_g) dma_win(end_g + 2);
            ++end_g;
            end_c = (end_g * TAPS + TAPS - 1) / 4;
        }
        __builtin_amdgcn_sched_barrier(0);
        // blocks 3-5: R0 (block 3) and R1 (block 5) of the next chunk, weight DMA of chunk c2
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            mf(3, q);
            constexpr int N3 = TMN + 1;
#pragma unroll
            for (int o = q * N3 / NB; o < (q + 1) * N3 / NB; ++o) {
                if (o < TMN) rd(0, o, a_nxt, bnxt);
                else dma_a_unit(c2, buf, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            mf(4, q);
            constexpr int N4 = A_PW - 2;
#pragma unroll
            for (int o = q * N4 / NB; o < (q + 1) * N4 / NB; ++o) dma_a_unit(c2, buf, 1 + o);
            if (q < OFF_STEPS) off_step(q);  // chunk c + 2's offsets
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            mf(5, q);
            constexpr int N5 = TMN + 1;
#pragma unroll
            for (int o = q * N5 / NB; o < (q + 1) * N5 / NB; ++o) {
                if (o < TMN) rd(1, o, a_nxt, bnxt);
                else dma_a_unit(c2, buf, A_PW - 1);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        buf = nbuf;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the last (unused) reads / loads landed
    fence_all();

    // ---- epilogue: a slab of a multi-slab tile leaves an fp32 partial (folded in slab order by
    // conv_x6_fixup); a whole tile adds bias + ReLU and writes X6 / X6P slices or fp32 NCHW
    if (!un.whole) {
        const __amdgpu_buffer_rsrc_t srs = slab_rsrc(a.partial);
        const uint32_t sbase = (uint32_t)uid * (uint32_t)(MT * PT * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int pl = wp0 + j * 16 + (lane & 15);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int q = (wm0 + i * 16) / 4 + (lane >> 4);
                store_slab_quad(srs, sbase + (uint32_t)(q * PT + pl) * 16u, acc[i][j]);
            }
        }
        continue;
    }
    const int cout8 = (G.cout + 7) & ~7;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int p = p0 + wp0 + j * 16 + (lane & 15);
        if (p >= npix) continue;
        const int n = p / HW;
        const int rem = p - n * HW;
        const int y = rem / W, x = rem - y * W;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int ml = wm0 + i * 16 + 4 * (lane >> 4);  // first of 4 consecutive channels
            const int mq = m0 + ml;
            float v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                v[t] = acc[i][j][t] + s_bias[ml + t];
                if (G.relu) v[t] = fmaxf(v[t], 0.f);
            }
            if (G.out_f32) {
                float* ob = static_cast<float*>(G.out) + ((size_t)n * G.out_c + G.out_off) * HW + rem;
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (mq + t < G.cout) ob[(size_t)(mq + t) * HW] = v[t];
            } else if (mq < cout8) {
                const int grp = mq >> 3, half = (mq >> 2) & 1;
                store4_x6(static_cast<uint8_t*>(G.out) + (size_t)x6_unit(G.out_l, n, grp, y, x) * 16 + half * 8,
                          G.out_ps, v);
                if (G.out2)
                    store4_x6(static_cast<uint8_t*>(G.out2) + (size_t)x6_unit(G.out2_l, n, grp, y, x) * 16 + half * 8,
                              G.out2_ps, v);
            }
        }
    }
    }  // pieces
}

// weights [cout][cin][ks][ks] (fp32, physical input channel order) -> X6 chunks in pair order:
// chunk c, k-group gi = pair q = 4c + gi = (group q / taps, tap q % taps); pairs past the last
// group are zero.  Same unit format as x6_pack_weights ([chunk][piece][4][Mpad][8] bf16).
void x6_pack_weights_pairs(const float* w, int cout, int cin, int ks, int Mpad, int* nK_out,
                           std::vector<uint16_t>& out) {
    const int taps = ks * ks;
    const int cin_g = (cin + 7) / 8;
    const int nK = (cin_g * taps + 3) / 4;
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
            const int q = 4 * c + gi, grp = q / taps, tap = q % taps;
            if (grp >= cin_g) continue;
            for (int m = 0; m < cout; ++m)
                for (int e = 0; e < 8; ++e) {
                    const int ch = grp * 8 + e;
                    if (ch >= cin) continue;
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

// window capacities (units per (piece, group)): LDS = 3 weight stages (72 KB) + 2 x 3 x 832 units
// (78 KB; the bench's 23 x 41 frames at P = 44: <= 707 units), or 2 stages + 2 x 3 x 1088 units
constexpr int kWinSmall = 832, kWinLarge = 1088;
constexpr int kWinStagesSmall = 3;  // weight stages of the small-window kernels (2: 2,021 vs 2,048 frames/s)

// largest window (units) a tile of PT pixels needs on an N x H x W batch for a KS x KS conv
int conv_win_units(int N, int H, int W, int ks, int pt) {
    const int HW = H * W, P = x6p_pitch(W), npix = N * HW, pad = ks / 2;
    int worst = 0;
    for (int p0 = 0; p0 < npix; p0 += pt) {
        const int p1 = std::min(p0 + pt, npix) - 1;
        auto prow = [&](int p) { return 3 + (p / HW) * (H + 3) + (p % HW) / W; };
        worst = std::max(worst, (prow(p1) - prow(p0) + 2 * pad + 1) * P + pad);
    }
    return worst;
}

bool conv_win_fits(int N, int H, int W, int ks) {
    return (ks == 3 || ks == 7) && x6p_pitch(W) <= 1024 && conv_win_units(N, H, W, ks, 256) <= kWinLarge;
}

bool conv_win_fits_rows(int W, int ks) {
    // a run starting at column x spans (x + 255) / W + 1 rows: at most (W + 254) / W + 1
    const int pad = ks / 2, span = (W + 254) / W;
    return (ks == 3 || ks == 7) && x6p_pitch(W) <= 1024 && (span + 2 * pad + 1) * x6p_pitch(W) + pad <= kWinLarge;
}

void launch_conv_win_x6(const X6Args& a0, hipStream_t st) {
    if ((a0.ks != 3 && a0.ks != 7) || a0.small || a0.pool || a0.Mpad % 128)
        throw std::invalid_argument("conv_win_x6: unsupported layer");
    const X6Args a = x6_number_tiles(a0, 128, 256);
    int need = 0;
    for (int g = 0; g < a.ngroups; ++g) {
        const X6Group& G = a.g[g];
        if (G.in_l.rs != (uint32_t)x6p_pitch(G.W) || G.in_l.fs != (uint32_t)(G.H + 3) * G.in_l.rs)
            throw std::invalid_argument("conv_win_x6: input is not X6P");
        need = std::max(need, conv_win_units(G.N, G.H, G.W, a.ks, 256));
    }
    if (a.sk_grid < 1 || a.sk_grid > a.units) throw std::invalid_argument("conv_win_x6: bad grid");
    if ((size_t)a.units * 128 * 256 * 4 >= 0x7fffffffull) throw std::invalid_argument("conv_win_x6: too many slabs");
    const dim3 grid(a.sk_grid), blk(512);
    if (need <= kWinSmall) {  // room for a third weight stage (48 + 72 + 24 KB of LDS)
        if (a.ks == 7) hipLaunchKernelGGL((conv_win_x6<128, 256, 7, kWinSmall, kWinStagesSmall>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((conv_win_x6<128, 256, 3, kWinSmall, kWinStagesSmall>), grid, blk, 0, st, a);
    } else if (need <= kWinLarge) {
        if (a.ks == 7) hipLaunchKernelGGL((conv_win_x6<128, 256, 7, kWinLarge, 2>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((conv_win_x6<128, 256, 3, kWinLarge, 2>), grid, blk, 0, st, a);
    } else {
        throw std::invalid_argument("conv_win_x6: window exceeds LDS");
    }
    if (a.units != a.tiles) launch_conv_x6_fixup(a, 128, 256, st);
}

}  // namespace opose
