// conv_wino.hip — 3x3 convolutions on padded (X6P) inputs as a one-dimensional Winograd
// F(2,3) along x, in split-bf16 arithmetic (the trunk's conv3_1 .. conv4_4_CPM and the stage-1
// CPM convs, src/model.py:41-62; the hand's 3x3 layers, src/model.py:136-195).
//
// An output pair (x0, x0 + 1), x0 even, of one row y from the input row pixels d_j = in[x0-1+j]:
//   V_0 = d0 - d2,  V_1 = d1 + d2,  V_2 = d2 - d1,  V_3 = d1 - d3       (input transform, fp32)
//   M_v[m] = sum over (c, ky) of U_v[m][c][ky] * V_v[c][row y + ky - 1]   (four GEMMs, K = 3 Cin)
//   y0 = (M_0 + M_1) + M_2,  y1 = (M_1 - M_2) - M_3                      (output transform)
// with U_v = sum_kx G[v][kx] w[m][c][ky][kx], G = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1]
// (float64, rounded to fp32 once, x6_pack_weights_wino).  Two outputs take 4 x 3 Cin products
// instead of 2 x 9 Cin: 2/3 of the direct conv's MFMAs.
//
// Arithmetic: V is formed in fp32 from the exact fp32 inputs (x = x0 + x1 + x2 of the X6 pieces)
// and split into three bf16 pieces again, so every GEMM is the six-piece-product split-bf16
// product of conv_x6 (fp32-class; tests/test_gpu_x6.py::test_wino_conv_fp32_accuracy).  The
// output pair is anchored at even x of the frame, so a pixel's value does not depend on the
// launch, the batch, the grid or a row band (engine.cpp seg_kernel).
//
// Workgroup: 128 output channels x 128 tiles (output pairs) = 256 output pixels, 4 waves (one
// per SIMD, 512 registers each), wave w owns tiles [32 w, 32 w + 32) of all 128 channels:
// 4 transforms x 8 x 2 accumulator blocks of 16 x 16 (256 registers).  K order: pairs q =
// (channel group q / 3, kernel row q % 3), chunk c = pairs 4c .. 4c+3; each chunk runs four
// steps v = 0..3 (the v-th GEMM on that chunk's 32 k), a step = 96 v_mfma_f32_16x16x32_bf16 per
// wave in the six piece products (0,2) (0,0) (0,1) | barrier | (1,0) (2,0) (1,1).
//  * A (U_v of the chunk): LDS-DMA weight stages, two, refilled after their last read as in
//    conv_win_x6.
//  * B (V_v): computed by each wave from the X6 input window in LDS during the previous step
//    (two 16-tile fragments: 6 ds_read_b128, join, transform, split), into the other of two
//    register sets.  The input window of channel group g (3 pieces, the tiles' rows +- 1) lives
//    in buffer g % 3; a chunk reads at most two groups, so three buffers let the next group's
//    window land while the current two are read -- except where a chunk starts four new groups'
//    period (c % 3 == 0): there both its groups are new, and the step's B is formed after an
//    extra barrier at its start (one step in twelve).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "x6.h"

namespace opose {

namespace {
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
// round-to-nearest-even bf16 of (lo, hi), packed lo | hi << 16 (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}
}  // namespace

constexpr int kWinoMT = 128, kWinoTT = 128;

// tile slot t of a group -> frame n, row y, column pair tx; false for padding slots
struct WinoTile {
    int n, y, tx;
    bool ok;
};
__device__ __forceinline__ WinoTile wino_tile(const X6Group& G, int t, int TW) {
    const int HT = G.H * TW;
    WinoTile r;
    int lt;
    if (G.tpf) {
        r.n = t / G.tpf;
        lt = t - r.n * G.tpf;
    } else {
        r.n = t / HT;
        lt = t - r.n * HT;
    }
    r.ok = t < G.npix && lt < HT && r.n < G.N;
    r.y = lt / TW;
    r.tx = lt - r.y * TW;
    return r;
}

template <int WMAX, int NW>
__global__ __launch_bounds__(64 * NW, 1) void conv_wino_x6(X6Args a) {
    // NW = 4: one wave per SIMD, 128 tiles, wave w = all 128 channels x tiles [32 w, 32 w + 32);
    // NW = 8: two per SIMD, 64 tiles, wave w = channels [64 (w & 1), +64) x tiles [16 (w >> 1), +16)
    constexpr int MT = kWinoMT, TM = 32 / NW, TN = NW == 8 ? 1 : 2, TT = 64 * TN, NT = 64 * NW;
    constexpr int A_U = 12 * MT;           // 16-byte units per weight stage
    constexpr int A_PW = A_U / 64 / NW;    // weight DMA instructions per wave per step
    constexpr int WH = WMAX / 2;           // 16-byte units per (column parity, channel half) sub-plane
    constexpr int WF = 4 * WH;             // units per fp32 window buffer
    constexpr int WOFF = 2 * A_U;          // three window buffers after the two weight stages
    constexpr int SOFF = WOFF + 3 * WF;    // X6 staging buffer (3 pieces) after them
    constexpr int NU = (WMAX + NT - 1) / NT; // window units per thread
    static_assert(A_PW * 64 * NW == A_U && WMAX % 64 == 0, "conv_wino_x6 tile");

    __shared__ __attribute__((aligned(16))) uint4 lds[2 * A_U + 3 * WF + 3 * WMAX];
    __shared__ float s_bias[MT];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nM = a.Mpad / MT;
    int id;
    {  // XCD-contiguous tile ids (guide T1): blocks b and b + 8 share an XCD
        const int b = blockIdx.x, Gw = gridDim.x, q = Gw >> 3, rr = Gw & 7, xcd = b & 7;
        id = xcd * q + min(xcd, rr) + (b >> 3);
    }
    const X6Group G = a.g[x6_group_of(a, id)];
    const int H = G.H, W = G.W, TW = (W + 1) >> 1;
    const int mt = (id - G.t0) % nM;
    const int t0 = ((id - G.t0) / nM) * TT, m0 = mt * MT;
    if (tid < MT) s_bias[tid] = (m0 + tid < G.cout) ? G.bias[m0 + tid] : 0.f;

    // ---- window geometry: padded rows of the first and last real tile of the workgroup
    const int P = (int)G.in_l.rs;
    const WinoTile f = wino_tile(G, t0, TW);
    int tl = min(t0 + TT, G.npix) - 1;
    if (G.tpf) tl = min(tl, f.n * G.tpf + H * TW - 1);
    else tl = min(tl, G.N * H * TW - 1);
    const WinoTile l = wino_tile(G, tl, TW);
    const int R0 = 3 + f.n * (H + 3) + f.y, R1 = 3 + l.n * (H + 3) + l.y;
    const int L = (R1 - R0 + 3) * P + 2;          // units the row-pair taps can touch
    const int NQ = (L + 63) >> 6;                 // staging DMA instructions per piece
    // byte offset of the window of group 0 (unit (R0 - 1) * P of the slice's first plane)
    const uint32_t win0 = (G.in_l.o0 - 3u * (uint32_t)P - 3u + (uint32_t)((R0 - 1) * P)) * 16u;
    const int cin_g = a.cin_g;
    const uint32_t lane16 = (uint32_t)lane * 16u;

    // ---- input windows, fp32: window unit u of group g (8 channels) at buffer g % 3, sub-plane
    // (u & 1) * 2 + half, index u >> 1 -- the 16 consecutive tiles of a B fragment read 16
    // consecutive 16-byte units.  A group's X6 window is DMA'd into the staging buffer after one
    // step's barrier, and joined (x0 + x1 + x2, exact) into its fp32 buffer after the next.
    // One buffer resource over the three piece planes; the DMA instruction list of a wave is walked
    // incrementally (piece sp, 64-unit block sj).
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)G.in, (short)0,
                                                                         (int)min(3ull * G.in_ps, 0xffffffffull), 0x00020000);
    int sp = 0, sj = 0;
    uint32_t sbase = 0;  // byte offset of the staged group's window
    auto stage_begin = [&](int g) __attribute__((always_inline)) {
        sbase = win0 + (uint32_t)g * G.in_l.gs * 16u;
        sp = 0;
        sj = wave;  // instruction i = wave + NW k of the 3 NQ: (piece, block) = divmod(i, NQ)
        while (sj >= NQ && sp < 3) {
            sj -= NQ;
            ++sp;
        }
    };
    auto stage_one = [&]() __attribute__((always_inline)) {  // one DMA instruction, if any left
        if (sp < 3) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_ptr_t)(lds + SOFF + sp * WMAX + 64 * sj), 16,
                                                     lane16, (int)(sbase + (uint32_t)sp * G.in_ps + (uint32_t)sj * 1024u),
                                                     0, 0);
            sj += NW;
            while (sj >= NQ && sp < 3) {
                sj -= NQ;
                ++sp;
            }
        }
    };
    auto conv_stage = [&](int g) __attribute__((always_inline)) {
        uint4* wb = lds + WOFF + (g % 3) * WF;
#pragma unroll
        for (int k = 0; k < NU; ++k) {
            const int u = tid + NT * k;
            if (u >= L) continue;
            const uint4 q0 = lds[SOFF + u], q1 = lds[SOFF + WMAX + u], q2 = lds[SOFF + 2 * WMAX + u];
            const uint32_t p0[4] = {q0.x, q0.y, q0.z, q0.w}, p1[4] = {q1.x, q1.y, q1.z, q1.w},
                           p2[4] = {q2.x, q2.y, q2.z, q2.w};
            float x[8];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                x[2 * w] = (lo_f(p0[w]) + lo_f(p1[w])) + lo_f(p2[w]);
                x[2 * w + 1] = (hi_f(p0[w]) + hi_f(p1[w])) + hi_f(p2[w]);
            }
            uint4* d = wb + (u & 1) * 2 * WH + (u >> 1);
            d[0] = uint4{__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
            d[WH] = uint4{__float_as_uint(x[4]), __float_as_uint(x[5]), __float_as_uint(x[6]), __float_as_uint(x[7])};
        }
    };
    // weights of step s = (chunk, v): units [s][piece][4 k-groups][Mpad]; this wave's A_PW DMA
    // instructions per step read fixed rows (soffset woff[u]) of the step's block (wstride apart)
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)G.wt, (short)0, (int)0x7fffffff,
                                                                        0x00020000);
    const uint32_t wstride = (uint32_t)(12 * a.Mpad * 16);
    uint32_t woff[A_PW];
#pragma unroll
    for (int u = 0; u < A_PW; ++u) {
        const int unit0 = (wave * A_PW + u) * 64, pg = unit0 / MT, m = unit0 - pg * MT;
        woff[u] = (uint32_t)(pg * a.Mpad + m0 + m) * 16u;
    }
    auto dma_a_unit = [&](uint32_t so, int buf, int u) __attribute__((always_inline)) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(lds + buf * A_U + (wave * A_PW + u) * 64), 16, lane16,
                                                 (int)(so + woff[u]), 0, 0);
    };

    // ---- per-lane B addressing: pair q = 4c + gi of chunk c -> (group pg, kernel row pk); the
    // window unit of d_0 of fragment j's tile at row pk is u0 = lbase[j] + pk P, its inputs d_k
    // sit at parity (u0 + k) & 1, index (u0 + k) >> 1: even (d_0, d_2) at ae, odd (d_1, d_3) at ao
    const int gi = lane >> 4;
    const int wm0 = NW == 8 ? 64 * (wave & 1) : 0, wt0 = NW == 8 ? 16 * (wave >> 1) : 32 * wave;
    int lbase[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int t = min(t0 + wt0 + 16 * j + (lane & 15), tl);  // padding slots: any real tile
        const WinoTile w = wino_tile(G, t, TW);
        lbase[j] = (3 + w.n * (H + 3) + w.y - R0) * P + 2 * w.tx + 2;
    }
    const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_ptr_t)(lds + WOFF);
    int pg = gi / 3, pk = gi - 3 * (gi / 3);  // chunk 0
    uint32_t ae[2][TN], ao[2][TN];  // [chunk parity][fragment]
    auto addr_of = [&](int par) __attribute__((always_inline)) {
        const int g = min(pg, cin_g - 1);  // pairs past the last group: weights 0
        const uint32_t b = lds0 + (uint32_t)((g % 3) * WF * 16);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int u0 = lbase[j] + pk * P, e = u0 & 1, i0 = u0 >> 1;
            ae[par][j] = b + (uint32_t)((e * 2 * WH + i0) * 16);
            ao[par][j] = b + (uint32_t)(((1 - e) * 2 * WH + i0 + e) * 16);
        }
    };
    auto advance = [&]() __attribute__((always_inline)) {  // q += 4
        pg += 1;
        pk += 1;
        if (pk >= 3) {
            pk -= 3;
            pg += 1;
        }
    };

    f32x4 acc[4][TM][TN];
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[v][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    i32x4 fa[2][TM];     // two A slots: this step's A1 and A0, then A2 in the A1 slot (below)
    i32x4 fb[2][3][TN];  // two B register sets: this step's B and the next step's
    i32x4 raw[2][2];     // (input a / b, channel half) of the B fragment being formed, fp32
    const int a16 = gi * MT + wm0 + (lane & 15);
    auto la = [&](int buf) __attribute__((always_inline)) {
        return (uint32_t)(uintptr_t)(lds_ptr_t)(lds + buf * A_U + a16);
    };
    // A piece pc of the stage at abase into slot sl
    auto rda = [&](int sl, int pc, int i, uint32_t abase) __attribute__((always_inline)) {
        if (pc == 0)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[sl][i]) : "v"(abase), "i"((0 * 4 * MT + 16 * i) * 16));
        else if (pc == 1)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[sl][i]) : "v"(abase), "i"((1 * 4 * MT + 16 * i) * 16));
        else
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[sl][i]) : "v"(abase), "i"((2 * 4 * MT + 16 * i) * 16));
    };
#define OPOSE_WINO_RD(S, ADDR, OFF)                                                                              \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(raw[S][0]) : "v"(ADDR), "i"(OFF));                     \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(raw[S][1]) : "v"(ADDR), "i"((OFF) + WH * 16))
    // inputs of V_v into raw[0] (d_ka) / raw[1] (d_kb): v0 (d0, d2), v1 (d1, d2), v2 (d2, d1), v3 (d1, d3)
    auto rd_in = [&](int par, int j, int v) __attribute__((always_inline)) {
        const uint32_t e = ae[par][j], o = ao[par][j];
        if (v == 0) {
            OPOSE_WINO_RD(0, e, 0); OPOSE_WINO_RD(1, e, 16);
        } else if (v == 1) {
            OPOSE_WINO_RD(0, o, 0); OPOSE_WINO_RD(1, e, 16);
        } else if (v == 2) {
            OPOSE_WINO_RD(0, e, 16); OPOSE_WINO_RD(1, o, 0);
        } else {
            OPOSE_WINO_RD(0, o, 0); OPOSE_WINO_RD(1, o, 16);
        }
    };
#undef OPOSE_WINO_RD
    // dword w (channels 2w, 2w+1) of V_v from raw[][], split into the three pieces of set `dst`
    auto form = [&](int v, int dst, int j, int w) __attribute__((always_inline)) {
        const int h = w >> 1, e = (w & 1) * 2;
        const float alo = __int_as_float(raw[0][h][e]), ahi = __int_as_float(raw[0][h][e + 1]);
        const float blo = __int_as_float(raw[1][h][e]), bhi = __int_as_float(raw[1][h][e + 1]);
        const float vlo = v == 1 ? alo + blo : alo - blo, vhi = v == 1 ? ahi + bhi : ahi - bhi;
        const uint32_t p0 = pk_bf16(vlo, vhi);
        const float elo = vlo - lo_f(p0), ehi = vhi - hi_f(p0);
        const uint32_t p1 = pk_bf16(elo, ehi);
        const uint32_t p2 = pk_bf16(elo - lo_f(p1), ehi - hi_f(p1));
        fb[dst][0][j][w] = (int)p0;
        fb[dst][1][j][w] = (int)p1;
        fb[dst][2][j][w] = (int)p2;
    };
    // MFMA of A slot sl and B piece pb (set `set`) for transform v, accumulator block qq
    auto mf = [&](int v, int sl, int set, int pb, int qq) __attribute__((always_inline)) {
        const int i = qq / TN, j = qq % TN;
        acc[v][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[sl][i]),
                                                               __builtin_bit_cast(bf16x8, fb[set][pb][j]),
                                                               acc[v][i][j], 0, 0, 0);
    };
    auto fence_a = [&](int sl) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(fa[sl][i]));
    };
    auto fence_raw = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int h = 0; h < 2; ++h) asm volatile("" : "+v"(raw[k][h]));
    };

    // ---- window schedule.  Every window read of a step (the next step's B inputs) comes before
    // its barrier, except the B of a four-group period's first step, read after the barrier of the
    // step before it.  Group g is DMA'd into the staging buffer after the barrier of step X(g) =
    // max(L(g - 3) - 1, X(g - 1) + 2), L(g) = 4 ((3g + 2) / 4) + 2 the step that last reads group
    // g, and converted into buffer g % 3 in step X(g) + 1 after its barrier: after every read of
    // group g - 3, and visible from step X(g) + 3 on, before the first read of group g (checked
    // for 1..69 groups)
    int next_g = min(3, cin_g), xlast = -1000, pend = -1;
    int lr = 4 * ((3 * (next_g - 3) + 2) >> 2) + 2;  // L(next_g - 3)

    // ---- prologue: windows of groups 0..2, weight stages of steps 0 and 1, A1 and B of step 0
    const int nS = 4 * a.nK;
#pragma unroll
    for (int u = 0; u < A_PW; ++u) dma_a_unit(0, 0, u);
#pragma unroll
    for (int u = 0; u < A_PW; ++u) dma_a_unit((uint32_t)min(1, nS - 1) * wstride, 1, u);
    for (int g = 0; g < next_g; ++g) {
        stage_begin(g);
        while (sp < 3) stage_one();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        conv_stage(g);
        __syncthreads();
    }
    addr_of(0);
    {
        const uint32_t a0 = la(0);
#pragma unroll
        for (int i = 0; i < TM; ++i) rda(0, 1, i, a0);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            rd_in(0, j, 0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            fence_raw();
#pragma unroll
            for (int w = 0; w < 4; ++w) form(0, 0, j, w);
        }
    }

    // One step: transform v (static); slot X holds this step's A1 (read in the previous step's
    // block 5), slot Y takes its A0 now and the next step's A1 in block 5, X takes A2 after block 1.
    // Piece products in the order (1,0) (1,1) (0,2) | barrier | (0,0) (0,1) (2,0).  The next step's
    // B: inputs read before the barrier, formed in blocks 1 (fragment 0) and 3-4 (fragment 1), or,
    // for a four-group period's first step, read and formed in block 5.  After the barrier, spread
    // over the MFMAs: the fp32 conversion of the window staged a step earlier (start of block 3),
    // the weight DMA of step s + 2 (block 3), the staging DMA of a window (blocks 4-5).
    // par: parity of this chunk's address set; c3 = c % 3.
    auto step = [&](const int v, const int X, const int Y, const int cur, const int nxt, const int c, const int s,
                    const int par, const int c3) __attribute__((always_inline)) {
        const int bufA = s & 1;
        const uint32_t a_cur = la(bufA), a_nxt = la(bufA ^ 1);
        const int s2 = min(s + 2, nS - 1);  // past the end: a harmless reload of the last step
        const bool last = c + 1 >= a.nK;
        const bool nbp = v == 3 && !last && c3 == 2;  // next B after the barrier (period start)
        const bool pre = v < 3 || (!last && c3 != 2);  // next B before it
        const int pn = v < 3 ? par : par ^ 1, vn = (v + 1) & 3;
#pragma unroll
        for (int i = 0; i < TM; ++i) rda(Y, 0, i, a_cur);  // A0 of this step
        if (pre) rd_in(pn, 0, vn);
        if (pre) asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(TM + 4) : "memory");  // A1 (slot X) landed
        else asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(TM) : "memory");
        fence_a(X);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int qq = 0; qq < TM * TN; ++qq) {
            mf(v, X, cur, 0, qq);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // A0 and fragment 0's inputs
        fence_a(Y);
        fence_raw();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int qq = 0; qq < TM * TN; ++qq) {
            mf(v, X, cur, 1, qq);
            if (pre && qq % (TM * TN / 4) == TM * TN / 4 - 1) form(vn, nxt, 0, qq / (TM * TN / 4));
        }
        // A2 into slot X (A1's last use was block 1); fragment 1's inputs
#pragma unroll
        for (int i = 0; i < TM; ++i) rda(X, 2, i, a_cur);
        if (TN > 1 && pre) rd_in(pn, 1, TN > 1 ? vn : 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int qq = 0; qq < TM * TN; ++qq) {
            mf(v, Y, cur, 2, qq);
        }
        // barrier: this step's stage read by all (A0, A2), the window reads of the step done; the
        // next stage and a staged window have landed.  The vmcnt is explicit: the compiler does not
        // count LDS-DMA as LDS writes at a barrier, and the fragment reads are inline asm
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        fence_a(X);
        fence_raw();
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
        const bool conv = pend >= 0 && xlast == s - 1;
        const int cg = pend;
        if (conv) pend = -1;
        const bool stg = next_g < cin_g && s >= lr - 1 && s >= xlast + 2;
        if (stg) {
            stage_begin(next_g);
            pend = next_g;
            xlast = s;
            ++next_g;
            lr = 4 * ((3 * (next_g - 3) + 2) >> 2) + 2;
        }
        const uint32_t wso = (uint32_t)s2 * wstride;
#pragma unroll
        for (int qq = 0; qq < TM * TN; ++qq) {
            mf(v, Y, cur, 0, qq);
            if (conv && qq == 0) conv_stage(cg);
            if (qq >= TM * TN / 2 - A_PW / 2 && qq < TM * TN / 2 - A_PW / 2 + A_PW)
                dma_a_unit(wso, bufA, qq - (TM * TN / 2 - A_PW / 2));
            if (TN > 1 && pre && qq % (TM * TN / 2) == TM * TN / 2 - 1) form(vn, nxt, TN - 1, qq / (TM * TN / 2));
        }
#pragma unroll
        for (int qq = 0; qq < TM * TN; ++qq) {
            mf(v, Y, cur, 1, qq);
            if (stg && qq == 0)
                for (int k = 0; k < 5; ++k) stage_one();
            if (TN > 1 && pre && qq % (TM * TN / 2) == TM * TN / 2 - 1) form(vn, nxt, TN - 1, 2 + qq / (TM * TN / 2));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) rda(Y, 1, i, a_nxt);  // the next step's A1 (slot Y: A0 done)
        if (nbp) rd_in(pn, 0, vn);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int qq = 0; qq < TM * TN; ++qq) {
            mf(v, X, cur, 0, qq);
            if (stg && qq == 0)
                while (sp < 3) stage_one();
            if (nbp && qq == TM * TN / 4 - 1) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                fence_raw();
#pragma unroll
                for (int w = 0; w < 4; ++w) form(vn, nxt, 0, w);
                if (TN > 1) rd_in(pn, TN - 1, vn);
            }
            if (TN > 1 && nbp && qq == TM * TN / 2 + 1) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                fence_raw();
#pragma unroll
                for (int w = 0; w < 4; ++w) form(vn, nxt, TN - 1, w);
            }
        }
    };

    // chunks in pairs: the address sets of chunk c (parity c & 1) and c + 1 alternate statically
    int c3 = 0;
    for (int c = 0; c < a.nK; c += 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int cc = c + h;
            if (cc >= a.nK) break;
            advance();
            addr_of(h ^ 1);  // chunk cc + 1 (read by this chunk's last step)
            step(0, 0, 1, 0, 1, cc, 4 * cc + 0, h, c3);
            step(1, 1, 0, 1, 0, cc, 4 * cc + 1, h, c3);
            step(2, 0, 1, 0, 1, cc, 4 * cc + 2, h, c3);
            step(3, 1, 0, 1, 0, cc, 4 * cc + 3, h, c3);
            c3 = c3 == 2 ? 0 : c3 + 1;
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // ---- epilogue: output transform, bias + ReLU, two pixels per tile
    const int cout8 = (G.cout + 7) & ~7;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const WinoTile w = wino_tile(G, t0 + wt0 + 16 * j + (lane & 15), TW);
        if (!w.ok) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int ml = wm0 + i * 16 + 4 * gi;  // first of 4 consecutive channels
            const int mq = m0 + ml;
            float y[2][4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float M0 = acc[0][i][j][r], M1 = acc[1][i][j][r], M2 = acc[2][i][j][r], M3 = acc[3][i][j][r];
                y[0][r] = (M0 + M1) + M2 + s_bias[ml + r];
                y[1][r] = (M1 - M2) - M3 + s_bias[ml + r];
                if (G.relu) {
                    y[0][r] = fmaxf(y[0][r], 0.f);
                    y[1][r] = fmaxf(y[1][r], 0.f);
                }
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int x = 2 * w.tx + e;
                if (x >= W) continue;
                if (G.out_f32) {
                    float* ob = static_cast<float*>(G.out) + ((size_t)w.n * G.out_c + G.out_off) * (H * W) + w.y * W + x;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (mq + r < G.cout) ob[(size_t)(mq + r) * H * W] = y[e][r];
                } else if (mq < cout8) {
                    const int grp = mq >> 3, half = (mq >> 2) & 1;
                    store4_x6(static_cast<uint8_t*>(G.out) + (size_t)x6_unit(G.out_l, w.n, grp, w.y, x) * 16 + half * 8,
                              G.out_ps, y[e]);
                    if (G.out2)
                        store4_x6(static_cast<uint8_t*>(G.out2) + (size_t)x6_unit(G.out2_l, w.n, grp, w.y, x) * 16 +
                                      half * 8,
                                  G.out2_ps, y[e]);
                }
            }
        }
    }
}

// weights [cout][cin][3][3] (fp32, physical channel order) -> U_v in pair order: step s = 4c + v,
// k-group gi = pair q = 4c + gi = (group q / 3, kernel row q % 3); same unit format as
// x6_pack_weights ([step][piece][4][Mpad][8] bf16)
void x6_pack_weights_wino(const float* w, int cout, int cin, int Mpad, int* nK_out, std::vector<uint16_t>& out) {
    const int cin_g = (cin + 7) / 8;
    const int nK = (cin_g * 3 + 3) / 4;
    *nK_out = nK;
    out.assign((size_t)nK * 4 * 12 * Mpad * 8, 0);
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
    static const double Gm[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    for (int c = 0; c < nK; ++c)
        for (int v = 0; v < 4; ++v)
            for (int gi = 0; gi < 4; ++gi) {
                const int q = 4 * c + gi, grp = q / 3, ky = q % 3;
                if (grp >= cin_g) continue;
                for (int m = 0; m < cout; ++m)
                    for (int e = 0; e < 8; ++e) {
                        const int ch = grp * 8 + e;
                        if (ch >= cin) continue;
                        const float* wr = w + (((size_t)m * cin + ch) * 3 + ky) * 3;
                        const float x = (float)(Gm[v][0] * (double)wr[0] + Gm[v][1] * (double)wr[1] + Gm[v][2] * (double)wr[2]);
                        const uint32_t h0 = rne(x);
                        const float r = x - f(h0);
                        const uint32_t h1 = rne(r);
                        const uint32_t h2 = rne(r - f(h1));
                        const uint32_t hs[3] = {h0, h1, h2};
                        for (int pc = 0; pc < 3; ++pc)
                            out[((((size_t)(4 * c + v) * 3 + pc) * 4 + gi) * Mpad + m) * 8 + e] = (uint16_t)hs[pc];
                    }
            }
}

// window units of a tile block, and the whole launch's worst case: tiles numbered across frames
// (tpf == 0) or in frame-aligned blocks of 128 (tpf = slots per frame)
static int wino_block_units(int N, int H, int W, int tpf, int t0) {
    const int TW = (W + 1) / 2, HT = H * TW, P = x6p_pitch(W);
    const int nslots = tpf ? N * tpf : N * HT;
    auto rowof = [&](int t) {
        const int n = tpf ? t / tpf : t / HT, lt = tpf ? t - n * tpf : t - n * HT;
        return 3 + n * (H + 3) + lt / TW;
    };
    int tl = std::min(t0 + kWinoTT, nslots) - 1;
    if (tpf) tl = std::min(tl, (t0 / tpf) * tpf + HT - 1);
    else tl = std::min(tl, N * HT - 1);
    return (rowof(tl) - rowof(t0) + 3) * P + 2;
}

int wino_units(int N, int H, int W, int tpf) {
    const int TW = (W + 1) / 2, HT = H * TW;
    const int nslots = tpf ? N * tpf : N * HT;
    int worst = 0;
    for (int t0 = 0; t0 < nslots; t0 += kWinoTT) {
        if (tpf && t0 % tpf >= HT) continue;
        worst = std::max(worst, wino_block_units(N, H, W, tpf, t0));
    }
    return worst;
}

constexpr int kWinoWin = 768;  // window units per group: 3 fp32 buffers (72 KB) + X6 staging (36 KB) + 2 x 24 KB of weights

// tile slots per frame for a batch: 0 (numbered across frames) when those windows fit, else
// frame-aligned blocks of 128; -1 when neither fits.  A function of (N, H, W) only; for one frame
// the bound does not depend on H beyond the rows a block can span (a row band and its frame agree).
int wino_tpf(int N, int H, int W) {
    const int TW = (W + 1) / 2, HT = H * TW;
    if (x6p_pitch(W) > 1024) return -1;
    if (N == 1) {
        // a block spans at most ceil((TW - 1 + 128) / TW) rows of any frame height
        const int rows = (TW - 1 + kWinoTT + TW - 1) / TW;
        return (rows + 2) * x6p_pitch(W) + 2 <= kWinoWin ? 0 : -1;
    }
    if (wino_units(N, H, W, 0) <= kWinoWin) return 0;
    const int tpf = (HT + kWinoTT - 1) / kWinoTT * kWinoTT;
    return wino_units(N, H, W, tpf) <= kWinoWin ? tpf : -1;
}

// one wave per SIMD and 128 tiles per workgroup (default: conv3_2 of the bench 0.64 ms), or
// OPOSE_WINO_WAVES=8: two waves per SIMD and 64 tiles (0.79 ms; the window kernel: 0.54 ms)
static int wino_waves() {
    static const int nw = [] {
        const char* e = getenv("OPOSE_WINO_WAVES");
        return e && e[0] == '8' ? 8 : 4;
    }();
    return nw;
}
static int wino_tt() { return wino_waves() == 4 ? 128 : 64; }

void launch_conv_wino_x6(const X6Args& a0, hipStream_t st) {
    if (a0.ks != 3 || a0.pool || a0.Mpad % kWinoMT) throw std::invalid_argument("conv_wino_x6: unsupported layer");
    X6Args a = a0;
    int t = 0;
    for (int g = 0; g < a.ngroups; ++g) {
        X6Group& G = a.g[g];
        if (G.in_l.rs != (uint32_t)x6p_pitch(G.W) || G.in_l.fs != (uint32_t)(G.H + 3) * G.in_l.rs)
            throw std::invalid_argument("conv_wino_x6: input is not X6P");
        if (G.slabs > 1) throw std::invalid_argument("conv_wino_x6: whole tiles only");
        const int TW = (G.W + 1) / 2;
        G.npix = G.tpf ? G.N * G.tpf : G.N * G.H * TW;  // tile slots
        if (wino_units(G.N, G.H, G.W, G.tpf) > kWinoWin) throw std::invalid_argument("conv_wino_x6: window exceeds LDS");
        G.slabs = 1;
        G.t0 = t;
        G.u0 = t;
        t += (a.Mpad / kWinoMT) * ((G.npix + wino_tt() - 1) / wino_tt());
    }
    a.tiles = a.units = t;
    a.sk_grid = t;
    a.sched = nullptr;
    if (wino_waves() == 4) hipLaunchKernelGGL((conv_wino_x6<kWinoWin, 4>), dim3(t), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_wino_x6<kWinoWin, 8>), dim3(t), dim3(512), 0, st, a);
}

}  // namespace opose
