// conv1x1_chain.hip — the two 1x1 convs that end a CPM stage, in one launch.
//
// Every stage of both networks ends in a pair of 1x1 convs (src/model.py:55-56, 61-62 conv5_4 ->
// conv5_5 of body stage 1; :76-77, 86-87 Mconv6 -> Mconv7 of stages 2-6; the hand's conv6_1 ->
// conv6_2 and Mconv6 -> Mconv7, :185-214):
//     Y = W2 relu(W1 X + b1) + b2        (X: 128 channels, W1: M1 = 128 or 512 rows, Y <= 64)
// Run as two launches, the M1-channel intermediate goes to HBM as X6 (6 bytes a value) and comes
// straight back: 2/3 of the pair's traffic for a few GFLOP.  Here a workgroup owns 64 pixels:
// for each 128-row slice of W1 it forms that slice of the intermediate in registers (bias, ReLU,
// split into bf16 pieces exactly as conv_x6's epilogue does), parks it in LDS as the B operand of
// the second GEMM, and accumulates W2's matching 128 columns into Y.  Only X is read and Y written.
//
// Arithmetic: the same split-bf16 products (6 per multiply-add) in the same order as conv_x6's
// whole-tile 1x1 launches -- chunks of 4 channel groups in ascending order, the piece products
// (0,2) (0,0) (0,1) (1,0) (2,0) (1,1) per chunk, bias added after the sum -- so Y equals the
// two-launch result bit for bit whenever conv_x6 ran both convs on whole tiles
// (tests/test_gpu_x6.py).
//
// Operands come straight from global memory into registers by buffer loads (16-byte fragments:
// X is re-read by the 4 waves from L2, the weights are L2/MALL resident; X of chunk c + 1 is in
// flight while chunk c's MFMAs run); the op is bound by HBM traffic, not by the matrix cores.
#include <stdexcept>

#include "common.h"
#include "kernels.h"
#include "x6.h"

namespace opose {

namespace {
constexpr int kChainPT = 64;  // pixels per workgroup

__device__ __forceinline__ int chain_group_of(const X6ChainArgs& a, int tile) {
    int g = 0;
    for (int i = 1; i < a.ngroups; ++i) g = tile >= a.g[i].t0 ? i : g;
    return g;
}
}  // namespace

__global__ __launch_bounds__(256) void conv1x1_chain_x6(X6ChainArgs a) {
    constexpr int PT = kChainPT;
    constexpr int PA[6] = {0, 0, 0, 1, 2, 1};
    constexpr int PB[6] = {2, 0, 1, 0, 0, 1};
    // intermediate slice: [piece][16 groups][64 pixels] units
    __shared__ __attribute__((aligned(16))) uint4 hs[3 * 16 * PT];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile = blockIdx.x;
    const X6ChainGroup G = a.g[chain_group_of(a, tile)];
    const int p0 = (tile - G.t0) * PT;
    const int HW = G.H * G.W;
    const int gi = lane >> 4, l16 = lane & 15;
    const int M1 = a.m1;
    constexpr int NK1 = 4;  // k chunks of the first conv: 128 input channels (the launcher checks)

    // Fragments by buffer loads: per lane a fixed byte offset (pixel / row and k-group), per k chunk
    // a uniform soffset -- no per-chunk 64-bit addresses in VGPRs.
    // X: the lane's pixel of each 16-pixel block, its k-group's unit, one resource per piece plane
    uint32_t xo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int p = min(p0 + 16 * j + l16, G.npix - 1);  // past the end: any pixel (not stored)
        const int n = p / HW, r = p - n * HW, y = r / G.W, x = r - y * G.W;
        xo[j] = (x6_unit(G.in_l, n, gi, y, x)) * 16u;
    }
    __amdgpu_buffer_rsrc_t xr[3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc)
        xr[pc] = __builtin_amdgcn_make_buffer_rsrc((void*)(G.in + (size_t)pc * G.in_ps), (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc((void*)G.w1, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t w2r = __builtin_amdgcn_make_buffer_rsrc((void*)G.w2, (short)0, 0x7fffffff, 0x00020000);
    auto bld = [](__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) __attribute__((always_inline)) {
        return __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vo, (int)so, 0));
    };
    auto mfma = [](const i32x4& x, const i32x4& y, f32x4 c) __attribute__((always_inline)) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x), __builtin_bit_cast(bf16x8, y), c,
                                                       0, 0, 0);
    };

    f32x4 acc2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int mc = 0; mc < M1 / 128; ++mc) {
        // ---- first conv, rows mc*128 + 32 wave .. +31 (2 blocks) x 64 pixels (4 blocks); the
        // fragments of k chunk c + 1 are loaded while chunk c's MFMAs run
        f32x4 acc1[2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int row1 = mc * 128 + 32 * wave + l16;
        // (X fragments double buffered: they come from HBM; the weight fragments hit L2)
        i32x4 fa[3][2], fb[2][3][4];
        auto load_x = [&](int c, int b) __attribute__((always_inline)) {
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
#pragma unroll
                for (int j = 0; j < 4; ++j) fb[b][pc][j] = bld(xr[pc], xo[j], (uint32_t)(4 * c) * G.in_l.gs * 16u);
        };
        const uint32_t wo = (uint32_t)(gi * M1 + row1) * 16u;  // + (pc * 4 M1 + 16 i) * 16
        load_x(0, 0);
#pragma unroll
        for (int c = 0; c < NK1; ++c) {
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    fa[pc][i] = bld(w1r, wo + (uint32_t)(pc * 4 * M1 + 16 * i) * 16u, (uint32_t)(c * 12 * M1) * 16u);
            if (c + 1 < NK1) load_x(c + 1, (c + 1) & 1);
#pragma unroll
            for (int t = 0; t < 6; ++t)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc1[i][j] = mfma(fa[PA[t]][i], fb[c & 1][PB[t]][j], acc1[i][j]);
        }
        // the second conv's weight fragments for this slice (4 k chunks), in flight during the
        // epilogue below
        i32x4 fw[4][3];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
                fw[s][pc] = bld(w2r, (uint32_t)((pc * 4 + gi) * 64 + 16 * wave + l16) * 16u,
                                (uint32_t)((mc * 4 + s) * 12 * 64) * 16u);
        // bias + ReLU, split, into LDS as the second GEMM's B operand (conv_x6's X6 epilogue)
        __syncthreads();  // the previous slice's reads are done
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int rl = 32 * wave + 16 * i + 4 * gi;  // first of 4 consecutive rows of the slice
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) v[t] = fmaxf(acc1[i][j][t] + G.b1[mc * 128 + rl + t], 0.f);
                uint32_t h[3][4];
#pragma unroll
                for (int t = 0; t < 4; ++t) split3(v[t], h[0][t], h[1][t], h[2][t]);
                const int px = 16 * j + l16;
#pragma unroll
                for (int pc = 0; pc < 3; ++pc) {
                    uint2 w;
                    w.x = h[pc][0] | (h[pc][1] << 16);
                    w.y = h[pc][2] | (h[pc][3] << 16);
                    *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(&hs[(pc * 16 + (rl >> 3)) * PT + px]) +
                                              ((rl >> 2) & 1) * 8) = w;
                }
            }
        }
        __syncthreads();
        // ---- second conv: rows 16 wave .. +15 of Y, k = this slice's 128 channels (4 chunks)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            i32x4 fh[3][4];
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    fh[pc][j] = *reinterpret_cast<const i32x4*>(&hs[(pc * 16 + 4 * s + gi) * PT + 16 * j + l16]);
#pragma unroll
            for (int t = 0; t < 6; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc2[j] = mfma(fw[s][PA[t]], fh[PB[t]][j], acc2[j]);
        }
    }

    // ---- epilogue: bias (+ ReLU), X6 slice or fp32 NCHW channels
    const int cout8 = (G.cout2 + 7) & ~7;
    const int mq = 16 * wave + 4 * gi;  // first of 4 consecutive output channels
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int p = p0 + 16 * j + l16;
        if (p >= G.npix) continue;
        const int n = p / HW, rem = p - n * HW, y = rem / G.W, x = rem - y * G.W;
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            v[t] = acc2[j][t] + (mq + t < G.cout2 ? G.b2[mq + t] : 0.f);
            if (G.relu2) v[t] = fmaxf(v[t], 0.f);
        }
        if (G.out_f32) {
            float* ob = static_cast<float*>(G.out) + ((size_t)n * G.out_c + G.out_off) * HW + rem;
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (mq + t < G.cout2) ob[(size_t)(mq + t) * HW] = v[t];
        } else if (mq < cout8) {
            store4_x6(static_cast<uint8_t*>(G.out) + (size_t)x6_unit(G.out_l, n, mq >> 3, y, x) * 16 + ((mq >> 2) & 1) * 8,
                      G.out_ps, v);
        }
    }
}

void launch_conv1x1_chain_x6(const X6ChainArgs& a0, hipStream_t st) {
    X6ChainArgs a = a0;
    if (a.ngroups < 1 || a.ngroups > kX6Groups || a.cin_g != 16 || a.m1 % 128 || a.m1 < 128)
        throw std::invalid_argument("conv1x1_chain_x6: unsupported shape");
    int t = 0;
    for (int g = 0; g < a.ngroups; ++g) {
        if (a.g[g].npix <= 0 || a.g[g].cout2 > 64) throw std::invalid_argument("conv1x1_chain_x6: bad group");
        a.g[g].t0 = t;
        t += (a.g[g].npix + kChainPT - 1) / kChainPT;
    }
    a.tiles = t;
    hipLaunchKernelGGL(conv1x1_chain_x6, dim3(a.tiles), dim3(256), 0, st, a);
}

}  // namespace opose
