// imgproc.hip — pre-processing and the heat-map resize chain (HBM-bound kernels).
//
// Reference steps replaced (hitmaxiang/pytorch-openpose):
//  * src/body.py:38-41  cv2.resize(oriImg, fx=fy=scale, INTER_CUBIC) on uint8 BGR,
//                       util.padRightDownCorner (src/util.py:12-32), float32(x)/256 - 0.5,
//                       HWC -> NCHW                       => preprocess_u8
//  * src/body.py:55-56  cv2.resize(map, fx=fy=8, INTER_CUBIC) + crop of the padding
//                                                         => cubic_resize_rows<0> (writes only the crop)
//  * src/body.py:57,67  cv2.resize(map, (W, H)) + heatmap_avg += map / n_scales (float64)
//                                                         => heat_full_accum
// Compiled with -ffp-contract=off (see cubic.h).
#include <stdexcept>

#include "common.h"
#include "cubic.h"
#include "kernels.h"

namespace opose {

// uint8 cubic resize (fixed point, coefficients x2048, (v + 2^21) >> 22) + pad + normalise.
__global__ __launch_bounds__(256) void preprocess_u8(const uint8_t* __restrict__ src, int64_t frame_stride,
                                                     int64_t row_stride, int H, int W, int Hs, int Ws,
                                                     double scale_y, double scale_x, int Hp, int Wp,
                                                     float pad_val, float* __restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int n = blockIdx.z;
    if (x >= Wp) return;
    const size_t plane = (size_t)Hp * Wp;
    float* o = out + (size_t)n * 3 * plane + (size_t)y * Wp + x;
    if (y >= Hs || x >= Ws) {
        o[0] = pad_val;
        o[plane] = pad_val;
        o[2 * plane] = pad_val;
        return;
    }
    const CubicTap ty = cubic_tap(y, scale_y, H);
    const CubicTap tx = cubic_tap(x, scale_x, W);
    int ia[4], ib[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ia[j] = coef_short(tx.c[j]);
        ib[j] = coef_short(ty.c[j]);
    }
    const uint8_t* f = src + (size_t)n * frame_stride;
    int acc[3] = {0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint8_t* row = f + (size_t)ty.i[r] * row_stride;
        int h[3] = {0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint8_t* px = row + 3 * tx.i[j];
            h[0] += px[0] * ia[j];
            h[1] += px[1] * ia[j];
            h[2] += px[2] * ia[j];
        }
        acc[0] += h[0] * ib[r];
        acc[1] += h[1] * ib[r];
        acc[2] += h[2] * ib[r];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        int v = (acc[c] + (1 << 21)) >> 22;
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        o[(size_t)c * plane] = (float)v / 256.f - 0.5f;
    }
}

// cubic resize of mid [N][Cm][Hs][Ws] channels [coff, coff+P) to [H][W], then
// avg[n][p] (+)= (double)(v / nscales)   (float32 divide, float64 accumulate).
// T = float when there is a single scale: the average is then exactly the float32 resize
// output (0.0 + (double)v), so the float64 map can be stored at half the bytes.
template <typename T>
__global__ __launch_bounds__(256) void heat_full_accum(const float* __restrict__ mid, int Cm, int coff, int P, int Hs,
                                                       int Ws, int H, int W, double scale_y, double scale_x,
                                                       float nscales, int accumulate, T* __restrict__ avg) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int np = blockIdx.z;
    if (x >= W) return;
    const int n = np / P, p = np - n * P;
    const CubicTap ty = cubic_tap(y, scale_y, Hs);
    const CubicTap tx = cubic_tap(x, scale_x, Ws);
    const float* plane = mid + ((size_t)n * Cm + coff + p) * Hs * Ws;
    float v = (Hs == H && Ws == W) ? plane[(size_t)y * Ws + x] : cubic_sample_f32(plane, Ws, ty, tx);
    v = v / nscales;
    T* d = avg + ((size_t)np * H + y) * W + x;
    if constexpr (sizeof(T) == 4) *d = 0.f + v;  // == (float)(0.0 + (double)v), incl. the sign of zero
    else *d = accumulate ? *d + (double)v : 0.0 + (double)v;
}

// Row-staged cubic resize (the fast path of upsample8 / heat_full_accum, same arithmetic):
// a workgroup owns RT output rows x 256 output columns of one plane.  OpenCV's horizontal pass
// h[r][x] = ((p0*a0 + p1*a1) + p2*a2) + p3*a3 is computed once per (source row, output column)
// into LDS, then every output row combines its 4 staged rows vertically -- instead of
// recomputing 4 horizontal sums (16 scattered loads) per output pixel.  Bit-identical to
// cubic_sample_f32: the same expressions in the same order.
// MODE 0: out[nc] = v (x8 upsample into mid), 1: float heat map 0.f + v/ns,
// 2: float64 heat average (+)= (double)(v/ns).
constexpr int RS_RT = 16;      // output rows per workgroup
constexpr int RS_MAXR = 44;    // staged source rows (RT * scale + 5 <= 44  <=>  scale <= 2.4)
constexpr int RS_CHUNK = 8;    // staged rows loaded per round

// MAXR: LDS rows actually staged (8 for x8, 16 for x2): small tiles keep many workgroups
// resident, which this HBM-bound kernel needs
template <int MODE, int MAXR>
__global__ __launch_bounds__(256) void cubic_resize_rows(const float* __restrict__ in, int in_cstride, int in_coff,
                                                         int C, int hi, int wi, int ho, int wo, double sy, double sx,
                                                         float nscales, int accumulate, void* __restrict__ out,
                                                         int torch) {
    __shared__ float hs[MAXR][256];
    __shared__ CubicTap s_ty[RS_RT];  // the vertical taps of this workgroup's rows, computed once
    const int tid = threadIdx.x;
    const int x = blockIdx.x * 256 + tid;
    const int y0 = blockIdx.y * RS_RT;
    const int y1 = min(y0 + RS_RT, ho);
    const int nc = blockIdx.z;
    const int n = nc / C, c = nc - n * C;
    const float* plane = in + ((size_t)n * in_cstride + in_coff + c) * hi * wi;
    // staged source rows: the clamped tap rows of the first and last output row bound them
    const int r_lo = cubic_tap_any(y0, sy, hi, torch).i[0];
    const int r_hi = cubic_tap_any(y1 - 1, sy, hi, torch).i[3];
    const bool live = x < wo;
    if (tid < y1 - y0) s_ty[tid] = cubic_tap_any(y0 + tid, sy, hi, torch);
    if (live) {
        const CubicTap tx = cubic_tap_any(x, sx, wi, torch);
        // RS_CHUNK rows per round with every load issued before the first use (rows past r_hi
        // re-read r_hi and are not stored): a row-at-a-time loop waited out one memory round
        // trip per staged row
        for (int k0 = 0; k0 < MAXR && r_lo + k0 <= r_hi; k0 += RS_CHUNK) {
            float p[RS_CHUNK][4];
#pragma unroll
            for (int k = 0; k < RS_CHUNK; ++k) {
                const float* row = plane + (size_t)min(r_lo + k0 + k, r_hi) * wi;
#pragma unroll
                for (int j = 0; j < 4; ++j) p[k][j] = row[tx.i[j]];
            }
#pragma unroll
            for (int k = 0; k < RS_CHUNK; ++k) {
                float v = p[k][0] * tx.c[0];
                v = v + p[k][1] * tx.c[1];
                v = v + p[k][2] * tx.c[2];
                v = v + p[k][3] * tx.c[3];
                if (k0 + k < MAXR && r_lo + k0 + k <= r_hi) hs[k0 + k][tid] = v;
            }
        }
    }
    __syncthreads();
    if (!live) return;
    const bool div = nscales != 1.f;  // x / 1.0f == x exactly: skip the IEEE division sequence
    for (int y = y0; y < y1; ++y) {
        const CubicTap ty = s_ty[y - y0];
        float o = hs[ty.i[0] - r_lo][tid] * ty.c[0];
        o = o + hs[ty.i[1] - r_lo][tid] * ty.c[1];
        o = o + hs[ty.i[2] - r_lo][tid] * ty.c[2];
        o = o + hs[ty.i[3] - r_lo][tid] * ty.c[3];
        const size_t e = ((size_t)nc * ho + y) * wo + x;
        if constexpr (MODE == 0) {
            reinterpret_cast<float*>(out)[e] = o;
        } else if constexpr (MODE == 1) {
            reinterpret_cast<float*>(out)[e] = 0.f + (div ? o / nscales : o);
        } else {
            double* d = reinterpret_cast<double*>(out) + e;
            const float v = div ? o / nscales : o;
            *d = accumulate ? *d + (double)v : 0.0 + (double)v;
        }
    }
}

// All scales of a pyramid in one pass (src/body.py:51-67 and src/hand.py:43-56: for every m,
// heatmap_avg += cv2.resize(x8 map, (W, H)) / len(multiplier)): per scale the row-staged resize
// above, into a float64 register accumulator per output row, added in scale order from 0.0 --
// the float64 sums launch_heat_full's per-scale launches store and re-read, with one write of the
// average instead of a read-modify-write per scale.  A scale whose x8 map already has the output
// size is read directly (cv2.resize copies).
template <int MAXR>
__global__ __launch_bounds__(256) void heat_full_scales(HeatScales S, int P, int H, int W, double* __restrict__ avg) {
    __shared__ float hs[MAXR][256];
    __shared__ CubicTap s_ty[RS_RT];
    const int tid = threadIdx.x;
    const int x = blockIdx.x * 256 + tid;
    const int y0 = blockIdx.y * RS_RT;
    const int y1 = min(y0 + RS_RT, H);
    const int nc = blockIdx.z;
    const int n = nc / P, c = nc - n * P;
    const bool live = x < W;
    double acc[RS_RT];
#pragma unroll
    for (int r = 0; r < RS_RT; ++r) acc[r] = 0.0;
    for (int s = 0; s < S.n; ++s) {
        const HeatScale& g = S.s[s];
        const float* plane = g.mid + ((size_t)n * g.Cm + g.coff + c) * g.Hs * g.Ws;
        const bool div = S.ns != 1.f;
        if (g.Hs == H && g.Ws == W) {  // identity: the map itself
            if (live) {
#pragma unroll
                for (int r = 0; r < RS_RT; ++r)
                    if (y0 + r < y1) {
                        const float o = plane[(size_t)(y0 + r) * W + x];
                        const float v = div ? o / S.ns : o;
                        acc[r] = acc[r] + (double)v;
                    }
            }
            continue;
        }
        const int r_lo = cubic_tap(y0, g.sy, g.Hs).i[0];
        const int r_hi = cubic_tap(y1 - 1, g.sy, g.Hs).i[3];
        __syncthreads();  // the previous scale's staged rows are consumed
        if (tid < y1 - y0) s_ty[tid] = cubic_tap(y0 + tid, g.sy, g.Hs);
        if (live) {
            const CubicTap tx = cubic_tap(x, g.sx, g.Ws);
            for (int k0 = 0; k0 < MAXR && r_lo + k0 <= r_hi; k0 += RS_CHUNK) {
                float q[RS_CHUNK][4];
#pragma unroll
                for (int k = 0; k < RS_CHUNK; ++k) {
                    const float* row = plane + (size_t)min(r_lo + k0 + k, r_hi) * g.Ws;
#pragma unroll
                    for (int j = 0; j < 4; ++j) q[k][j] = row[tx.i[j]];
                }
#pragma unroll
                for (int k = 0; k < RS_CHUNK; ++k) {
                    float v = q[k][0] * tx.c[0];
                    v = v + q[k][1] * tx.c[1];
                    v = v + q[k][2] * tx.c[2];
                    v = v + q[k][3] * tx.c[3];
                    if (k0 + k < MAXR && r_lo + k0 + k <= r_hi) hs[k0 + k][tid] = v;
                }
            }
        }
        __syncthreads();
        if (live) {
#pragma unroll
            for (int r = 0; r < RS_RT; ++r)
                if (y0 + r < y1) {
                    const CubicTap ty = s_ty[r];
                    float o = hs[ty.i[0] - r_lo][tid] * ty.c[0];
                    o = o + hs[ty.i[1] - r_lo][tid] * ty.c[1];
                    o = o + hs[ty.i[2] - r_lo][tid] * ty.c[2];
                    o = o + hs[ty.i[3] - r_lo][tid] * ty.c[3];
                    const float v = div ? o / S.ns : o;
                    acc[r] = acc[r] + (double)v;
                }
        }
    }
    if (!live) return;
#pragma unroll
    for (int r = 0; r < RS_RT; ++r)
        if (y0 + r < y1) avg[((size_t)nc * H + y0 + r) * W + x] = acc[r];
}

// staged rows needed by one workgroup for a source step `scale` (destination -> source)
static bool rows_fit(double scale) { return RS_RT * scale + 5.0 <= (double)RS_MAXR; }

template <int MODE>
static void launch_resize_rows(dim3 grid, hipStream_t st, const float* in, int cstride, int coff, int C, int hi,
                               int wi, int ho, int wo, double sy, double sx, float ns, int acc, void* out,
                               int torch = 0) {
    const double need = RS_RT * sy + 5.0;
    if (need <= 8.0)
        hipLaunchKernelGGL((cubic_resize_rows<MODE, 8>), grid, dim3(256), 0, st, in, cstride, coff, C, hi, wi, ho, wo,
                           sy, sx, ns, acc, out, torch);
    else if (need <= 16.0)
        hipLaunchKernelGGL((cubic_resize_rows<MODE, 16>), grid, dim3(256), 0, st, in, cstride, coff, C, hi, wi, ho,
                           wo, sy, sx, ns, acc, out, torch);
    else
        hipLaunchKernelGGL((cubic_resize_rows<MODE, RS_MAXR>), grid, dim3(256), 0, st, in, cstride, coff, C, hi, wi,
                           ho, wo, sy, sx, ns, acc, out, torch);
}

void launch_preprocess(const uint8_t* src, int64_t frame_stride, int64_t row_stride, int N, int H, int W, int Hs,
                       int Ws, double sy, double sx, int Hp, int Wp, float pad_val, float* out, hipStream_t st) {
    dim3 grid((Wp + 255) / 256, Hp, N);
    hipLaunchKernelGGL(preprocess_u8, grid, dim3(256), 0, st, src, frame_stride, row_stride, H, W, Hs, Ws, sy, sx, Hp,
                       Wp, pad_val, out);
}

void launch_upsample8(const float* in, int in_cstride, int in_coff, int C, int N, int hl, int wl, int Hs, int Ws,
                      float* out, hipStream_t st) {
    dim3 grid((Ws + 255) / 256, (Hs + RS_RT - 1) / RS_RT, N * C);
    launch_resize_rows<0>(grid, st, in, in_cstride, in_coff, C, hl, wl, Hs, Ws, 0.125, 0.125, 1.f, 0, (void*)out);
}

void launch_heat_full(const float* mid, int Cm, int coff, int P, int N, int Hs, int Ws, int H, int W, double sy,
                      double sx, int nscales, int accumulate, double* avg, hipStream_t st) {
    if (!(Hs == H && Ws == W) && rows_fit(sy)) {
        dim3 grid((W + 255) / 256, (H + RS_RT - 1) / RS_RT, N * P);
        launch_resize_rows<2>(grid, st, mid, Cm, coff, P, Hs, Ws, H, W, sy, sx, (float)nscales, accumulate, (void*)avg);
        return;
    }
    dim3 grid((W + 255) / 256, H, N * P);
    hipLaunchKernelGGL(heat_full_accum<double>, grid, dim3(256), 0, st, mid, Cm, coff, P, Hs, Ws, H, W, sy, sx,
                       (float)nscales, accumulate, avg);
}

bool heat_full_scales_fits(const HeatScales& S, int H, int W) {
    for (int s = 0; s < S.n; ++s)
        if (!((S.s[s].Hs == H && S.s[s].Ws == W) || rows_fit(S.s[s].sy))) return false;
    return S.n >= 1 && S.n <= kHeatScales;
}

void launch_heat_full_scales(const HeatScales& S, int N, int P, int H, int W, double* avg, hipStream_t st) {
    if (!heat_full_scales_fits(S, H, W)) throw std::invalid_argument("heat_full_scales: scale out of range");
    dim3 grid((W + 255) / 256, (H + RS_RT - 1) / RS_RT, N * P);
    hipLaunchKernelGGL(heat_full_scales<RS_MAXR>, grid, dim3(256), 0, st, S, P, H, W, avg);
}

void launch_heat_full_f32(const float* mid, int Cm, int coff, int P, int N, int Hs, int Ws, int H, int W, double sy,
                          double sx, float* avg, hipStream_t st) {
    if (!(Hs == H && Ws == W) && rows_fit(sy)) {
        dim3 grid((W + 255) / 256, (H + RS_RT - 1) / RS_RT, N * P);
        launch_resize_rows<1>(grid, st, mid, Cm, coff, P, Hs, Ws, H, W, sy, sx, 1.f, 0, (void*)avg);
        return;
    }
    dim3 grid((W + 255) / 256, H, N * P);
    hipLaunchKernelGGL(heat_full_accum<float>, grid, dim3(256), 0, st, mid, Cm, coff, P, Hs, Ws, H, W, sy, sx, 1.f, 0,
                       avg);
}

// ---------------------------------------------------------------- Batch_body fast mode
// transforms.ToTensor (uint8 / 255.f) -> F.interpolate(bicubic, scale_factor) -> - 0.5 ->
// F.pad(0) on the right / bottom (srcmx/Batch_model.py:147-150): torch bicubic taps in float,
// rows first, x0*c0 + x1*c1 + x2*c2 + x3*c3.
__global__ __launch_bounds__(256) void preprocess_torch_u8(const uint8_t* __restrict__ src, int64_t frame_stride,
                                                           int64_t row_stride, int H, int W, int nh, int nw,
                                                           float scale_y, float scale_x, int Hp, int Wp,
                                                           float* __restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int n = blockIdx.z;
    if (x >= Wp) return;
    const size_t plane = (size_t)Hp * Wp;
    float* o = out + (size_t)n * 3 * plane + (size_t)y * Wp + x;
    if (y >= nh || x >= nw) {
        o[0] = 0.f;
        o[plane] = 0.f;
        o[2 * plane] = 0.f;
        return;
    }
    const CubicTap ty = cubic_tap_torch(y, scale_y, H);
    const CubicTap tx = cubic_tap_torch(x, scale_x, W);
    const uint8_t* f = src + (size_t)n * frame_stride;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint8_t* row = f + (size_t)ty.i[r] * row_stride;
            float v = (float)row[3 * tx.i[0] + c] / 255.f * tx.c[0];
            v = v + (float)row[3 * tx.i[1] + c] / 255.f * tx.c[1];
            v = v + (float)row[3 * tx.i[2] + c] / 255.f * tx.c[2];
            v = v + (float)row[3 * tx.i[3] + c] / 255.f * tx.c[3];
            h[r] = v;
        }
        float v = h[0] * ty.c[0];
        v = v + h[1] * ty.c[1];
        v = v + h[2] * ty.c[2];
        v = v + h[3] * ty.c[3];
        o[(size_t)c * plane] = v - 0.5f;
    }
}

void launch_preprocess_torch(const uint8_t* src, int64_t frame_stride, int64_t row_stride, int N, int H, int W, int nh,
                             int nw, float scale_y, float scale_x, int Hp, int Wp, float* out, hipStream_t st) {
    dim3 grid((Wp + 255) / 256, Hp, N);
    hipLaunchKernelGGL(preprocess_torch_u8, grid, dim3(256), 0, st, src, frame_stride, row_stride, H, W, nh, nw,
                       scale_y, scale_x, Hp, Wp, out);
}

// torch bicubic x8 of channels [in_coff, in_coff + C) cropped to nh x nw (scale 1/8 exactly)
void launch_upsample8_torch(const float* in, int in_cstride, int in_coff, int C, int N, int hl, int wl, int nh, int nw,
                            float* out, hipStream_t st) {
    dim3 grid((nw + 255) / 256, (nh + RS_RT - 1) / RS_RT, N * C);
    launch_resize_rows<0>(grid, st, in, in_cstride, in_coff, C, hl, wl, nh, nw, 0.125, 0.125, 1.f, 0, (void*)out, 1);
}

// torch bicubic to H x W (size given: scale = float(nh) / float(H)); float map out
void launch_resize_torch_f32(const float* mid, int Cm, int coff, int P, int N, int nh, int nw, int H, int W,
                             float* out, hipStream_t st) {
    const float sy = (float)nh / (float)H, sx = (float)nw / (float)W;
    if (!rows_fit(sy)) throw std::invalid_argument("fast mode: downscale too strong for the staged resize");
    dim3 grid((W + 255) / 256, (H + RS_RT - 1) / RS_RT, N * P);
    launch_resize_rows<1>(grid, st, mid, Cm, coff, P, nh, nw, H, W, (double)sy, (double)sx, 1.f, 0, (void*)out, 1);
}

}  // namespace opose
