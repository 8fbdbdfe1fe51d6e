// cubic.h — OpenCV INTER_CUBIC arithmetic (resizeGeneric_ scalar path), device side.
//
// The reference resizes with cv2.resize(..., INTER_CUBIC) at src/body.py:38,55,57,61,63 and
// src/hand.py:38,53,55.  Everything here must be compiled with -ffp-contract=off: the
// coefficients and sums are float32 expressions evaluated in source order without FMA,
// exactly as the oracle (oracle/cv_resize.py) restates them.
#pragma once
#include <hip/hip_runtime.h>

namespace opose {

struct CubicTap {
    int i[4];      // clamped source taps (replicate border)
    float c[4];    // float32 coefficients
};

// interpolateCubic(x) with A = -0.75 (float32)
__device__ __forceinline__ void cubic_coeffs(float x, float* c) {
    const float A = -0.75f;
    const float x1 = x + 1.f;
    c[0] = ((A * x1 - (5.f * A)) * x1 + (8.f * A)) * x1 - (4.f * A);
    c[1] = (((A + 2.f) * x - (A + 3.f)) * x) * x + 1.f;
    const float om = 1.f - x;
    c[2] = (((A + 2.f) * om - (A + 3.f)) * om) * om + 1.f;
    c[3] = ((1.f - c[0]) - c[1]) - c[2];
}

// destination index d -> taps/coefficients; scale = source step (1 / inv_scale)
__device__ __forceinline__ CubicTap cubic_tap(int d, double scale, int ssize) {
    CubicTap t;
    float f = (float)(((double)d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f = f - (float)s;
    cubic_coeffs(f, t.c);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int v = s - 1 + j;
        t.i[j] = v < 0 ? 0 : (v >= ssize ? ssize - 1 : v);
    }
    return t;
}

// PyTorch upsample_bicubic2d (align_corners=False, A = -0.75; aten UpSample.h): source
// coordinate scale * (d + 0.5) - 0.5 in float (scale = float(1 / scale_factor), or
// float(in) / float(out) when a size is given), index clamped to the last row, lambda clamped
// to [0, 1], each of the four coefficients from its own polynomial (no 1 - sum), taps clamped.
// Used by the Batch_body fast mode (srcmx/Batch_model.py:147-168).
__device__ __forceinline__ CubicTap cubic_tap_torch(int d, float scale, int ssize) {
    CubicTap t;
    const float A = -0.75f;
    const float real = scale * ((float)d + 0.5f) - 0.5f;
    int idx = (int)floorf(real);
    idx = idx < ssize - 1 ? idx : ssize - 1;
    float lam = real - (float)idx;
    lam = fminf(fmaxf(lam, 0.f), 1.f);
    const float x1 = lam + 1.f;
    t.c[0] = ((A * x1 - 5.f * A) * x1 + 8.f * A) * x1 - 4.f * A;
    t.c[1] = ((A + 2.f) * lam - (A + 3.f)) * lam * lam + 1.f;
    const float x2 = 1.f - lam;
    t.c[2] = ((A + 2.f) * x2 - (A + 3.f)) * x2 * x2 + 1.f;
    const float x3 = x2 + 1.f;
    t.c[3] = ((A * x3 - 5.f * A) * x3 + 8.f * A) * x3 - 4.f * A;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int v = idx - 1 + j;
        t.i[j] = v < 0 ? 0 : (v >= ssize ? ssize - 1 : v);
    }
    return t;
}

// taps of either convention (torch: scale holds the exact float scale)
__device__ __forceinline__ CubicTap cubic_tap_any(int d, double scale, int ssize, bool torch) {
    return torch ? cubic_tap_torch(d, (float)scale, ssize) : cubic_tap(d, scale, ssize);
}

// float32 image: horizontal then vertical pass, ((p0+p1)+p2)+p3 each.
// plane: row-major [rows][ld] (ld = row stride in floats)
__device__ __forceinline__ float cubic_sample_f32(const float* __restrict__ plane, int ld, const CubicTap& ty,
                                                  const CubicTap& tx) {
    float h[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float* row = plane + (size_t)ty.i[r] * ld;
        float v = row[tx.i[0]] * tx.c[0];
        v = v + row[tx.i[1]] * tx.c[1];
        v = v + row[tx.i[2]] * tx.c[2];
        v = v + row[tx.i[3]] * tx.c[3];
        h[r] = v;
    }
    float o = h[0] * ty.c[0];
    o = o + h[1] * ty.c[1];
    o = o + h[2] * ty.c[2];
    o = o + h[3] * ty.c[3];
    return o;
}

__device__ __forceinline__ int coef_short(float c) {
    float v = rintf(c * 2048.f);
    v = fminf(fmaxf(v, -32768.f), 32767.f);
    return (int)v;
}

}  // namespace opose
