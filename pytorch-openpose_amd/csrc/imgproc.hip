// imgproc.hip — pre-processing and the heat-map resize chain (HBM-bound kernels).
//
// Reference steps replaced (hitmaxiang/pytorch-openpose):
//  * src/body.py:38-41  cv2.resize(oriImg, fx=fy=scale, INTER_CUBIC) on uint8 BGR,
//                       util.padRightDownCorner (src/util.py:12-32), float32(x)/256 - 0.5,
//                       HWC -> NCHW                       => preprocess_u8
//  * src/body.py:55-56  cv2.resize(map, fx=fy=8, INTER_CUBIC) + crop of the padding
//                                                         => upsample8  (writes only the crop)
//  * src/body.py:57,67  cv2.resize(map, (W, H)) + heatmap_avg += map / n_scales (float64)
//                                                         => heat_full_accum
// Compiled with -ffp-contract=off (see cubic.h).
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

// x8 cubic upsample of the low-res network maps, cropped to Hs x Ws (float32).
// in: [N][in_cstride][hl][wl] channels [in_coff, in_coff + C); out: [N][C][Hs][Ws]
__global__ __launch_bounds__(256) void upsample8(const float* __restrict__ in, int in_cstride, int in_coff, int C,
                                                 int hl, int wl, int Hs, int Ws, float* __restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int nc = blockIdx.z;
    if (x >= Ws) return;
    const int n = nc / C, c = nc - n * C;
    const CubicTap ty = cubic_tap(y, 0.125, hl);
    const CubicTap tx = cubic_tap(x, 0.125, wl);
    const float* plane = in + ((size_t)n * in_cstride + in_coff + c) * hl * wl;
    out[((size_t)nc * Hs + y) * Ws + x] = cubic_sample_f32(plane, wl, ty, tx);
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

void launch_preprocess(const uint8_t* src, int64_t frame_stride, int64_t row_stride, int N, int H, int W, int Hs,
                       int Ws, double sy, double sx, int Hp, int Wp, float pad_val, float* out, hipStream_t st) {
    dim3 grid((Wp + 255) / 256, Hp, N);
    hipLaunchKernelGGL(preprocess_u8, grid, dim3(256), 0, st, src, frame_stride, row_stride, H, W, Hs, Ws, sy, sx, Hp,
                       Wp, pad_val, out);
}

void launch_upsample8(const float* in, int in_cstride, int in_coff, int C, int N, int hl, int wl, int Hs, int Ws,
                      float* out, hipStream_t st) {
    dim3 grid((Ws + 255) / 256, Hs, N * C);
    hipLaunchKernelGGL(upsample8, grid, dim3(256), 0, st, in, in_cstride, in_coff, C, hl, wl, Hs, Ws, out);
}

void launch_heat_full(const float* mid, int Cm, int coff, int P, int N, int Hs, int Ws, int H, int W, double sy,
                      double sx, int nscales, int accumulate, double* avg, hipStream_t st) {
    dim3 grid((W + 255) / 256, H, N * P);
    hipLaunchKernelGGL(heat_full_accum<double>, grid, dim3(256), 0, st, mid, Cm, coff, P, Hs, Ws, H, W, sy, sx,
                       (float)nscales, accumulate, avg);
}

void launch_heat_full_f32(const float* mid, int Cm, int coff, int P, int N, int Hs, int Ws, int H, int W, double sy,
                          double sx, float* avg, hipStream_t st) {
    dim3 grid((W + 255) / 256, H, N * P);
    hipLaunchKernelGGL(heat_full_accum<float>, grid, dim3(256), 0, st, mid, Cm, coff, P, Hs, Ws, H, W, sy, sx, 1.f, 0,
                       avg);
}

}  // namespace opose
