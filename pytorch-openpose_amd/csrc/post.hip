#include <cstdlib>
#include <stdexcept>
// post.hip — the post-network Body path as wavefront-parallel kernels.
//
// Reference (hitmaxiang/pytorch-openpose src/body.py), all float64 like the reference:
//  * :70-94   gaussian_filter(sigma=3) (scipy, mode 'reflect', radius 12) + 4-neighbour
//             '>=' NMS + '> thre1' + np.nonzero (row-major)      => gauss_nms + peaks_finalize
//  * :109-141 PAF line integral over 10 linspace samples per (i, j) pair of each limb
//                                                                => paf_score
//  * :143-155 stable sort by score (desc) + greedy matching      => limb_greedy
//  * :157-208 person assembly (found 0/1/2, merge '+1' quirk, IndexError when a third row
//             matches) + pruning                                  => assemble_people
// Compiled with -ffp-contract=off: every float64 expression is evaluated in the
// reference's order with one rounding per operation (bit-exact with NumPy/SciPy).
#include "common.h"
#include "cubic.h"
#include "kernels.h"

namespace opose {

// scipy.ndimage._filters._gaussian_kernel1d(3, 0, 12): centre .. tail (symmetric)
__constant__ double kGauss[13] = {
    0x1.105a329f98197p-3, 0x1.01a25f86eb137p-3, 0x1.b42a57d56c0bep-4, 0x1.4a614d1afd337p-4,
    0x1.bfde9c12bec92p-5, 0x1.0fa58939b528fp-5, 0x1.26defcaeb0202p-6, 0x1.1e6bccad344bap-7,
    0x1.f1e9915139406p-9, 0x1.8345966f69518p-10, 0x1.0d8a5ad43c165p-11, 0x1.4fbe39149e277p-13,
    0x1.763a210dfb306p-15};

// src/body.py:97-103
__constant__ int kLimbA[19] = {1, 1, 2, 3, 5, 6, 1, 8, 9, 1, 11, 12, 1, 0, 14, 0, 15, 2, 5};
__constant__ int kLimbB[19] = {2, 5, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 0, 14, 16, 15, 17, 16, 17};
__constant__ int kPafX[19] = {12, 20, 14, 16, 22, 24, 0, 2, 4, 6, 8, 10, 28, 30, 34, 32, 36, 18, 26};

// scipy 'reflect' (d c b a | a b c d | d c b a), periodic with period 2n
__device__ __forceinline__ int reflect_idx(int i, int n) {
    const int p = 2 * n;
    i %= p;
    if (i < 0) i += p;
    return i < n ? i : p - 1 - i;
}

// Gaussian tile (the hand threshold, gauss_threshold; the body NMS uses the wide tile below):
// TW x TH outputs of one map (+ the 1-pixel NMS ring).  scipy order: axis 0
// (vertical) then axis 1, symmetric taps summed centre-first then |j| = 12 .. 1, float64, no FMA.
//  * vertical pass straight from global memory: a thread owns one column of the tile's
//    13-pixel-haloed footprint and half its rows, sliding a 41-entry register window down the
//    column (one load per input, coalesced across threads), result -> LDS v[VR][VW];
//  * horizontal pass: a thread owns one row and 10 columns of v, register window of 34;
//  * NMS on the smoothed tile.
// 64 x 32 outputs per tile: 2.6 filter evaluations per output pixel (halo included) instead
// of 3.1 for 32 x 32 tiles, and no staged input tile (42 KB of LDS, 3 workgroups per CU).
constexpr int TW = 64, TH = 32;
constexpr int VW = TW + 26;   // vertical-pass columns: 13-pixel halo (12 filter + 1 ring) each side
constexpr int VR = TH + 2;    // smoothed rows incl. the NMS ring
constexpr int GW = TW + 2;    // smoothed cols incl. the NMS ring
constexpr int VH = VR / 2;    // rows per thread in the vertical pass (two halves)
constexpr int HC = 10;        // cols per thread in the horizontal pass (7 x 10 >= GW)

struct GaussTile {
    double v[VR][VW];
    double g[VR][GW];
};

__device__ __forceinline__ double gauss_skip_below(double thre) {
    return thre > 0.0 ? thre * (1.0 - 1e-9) : -__builtin_inf();  // no skipping for thre <= 0
}

// Returns false (and leaves t unset) when every input pixel of the footprint is below
// `skip_below`: the filter is a convex combination (weights > 0, sum 1), so no smoothed value of
// the tile can then exceed the caller's threshold (skip_below = thre * (1 - 1e-9) covers the
// float64 rounding of the 2 x 25-tap sums, < 1e-14 relative); NaN inputs count as below, as a
// NaN in a pixel's support makes its comparison false in the reference too.
template <typename T>
__device__ __forceinline__ bool gauss_tile(const T* __restrict__ m, int H, int W, int x0, int y0, GaussTile& t,
                                           double skip_below) {
    const int tid = threadIdx.x;
    bool hot = false;
    const bool vt = tid < 2 * VW;  // axis 0: thread -> (column c, half h)
    const int c = tid % VW, h = tid / VW;
    double win[VH + 24];
    if (vt) {
        const T* col = m + reflect_idx(x0 - 13 + c, W);
        const int r0 = y0 - 13 + h * VH;  // image row of window entry 0
#pragma unroll
        for (int i = 0; i < VH + 24; ++i) win[i] = (double)col[(size_t)reflect_idx(r0 + i, H) * W];
#pragma unroll
        for (int i = 0; i < VH + 24; ++i) hot |= win[i] >= skip_below;
    }
    if (!__syncthreads_or(hot)) return false;
    if (vt) {
#pragma unroll
        for (int i = 0; i < VH; ++i) {
            double acc = win[i + 12] * kGauss[0];
#pragma unroll
            for (int j = 12; j >= 1; --j) acc = acc + (win[i + 12 - j] + win[i + 12 + j]) * kGauss[j];
            t.v[h * VH + i][c] = acc;
        }
    }
    __syncthreads();
    if (tid < VR * 7) {  // axis 1: thread -> (row r, 10-column run)
        const int r = tid % VR, c0 = (tid / VR) * HC;
        double win[HC + 24];
#pragma unroll
        for (int i = 0; i < HC + 24; ++i) win[i] = (c0 + i < VW) ? t.v[r][c0 + i] : 0.0;
#pragma unroll
        for (int i = 0; i < HC; ++i) {
            if (c0 + i < GW) {
                double acc = win[i + 12] * kGauss[0];
#pragma unroll
                for (int j = 12; j >= 1; --j) acc = acc + (win[i + 12 - j] + win[i + 12 + j]) * kGauss[j];
                t.g[r][c0 + i] = acc;
            }
        }
    }
    __syncthreads();
    return true;
}

// tile id -> (x tile, y tile, map) with an XCD-contiguous order (guide T1): horizontally and
// vertically adjacent tiles, which re-read each other's 13-pixel halos, share an L2.
__device__ __forceinline__ void gauss_tile_coords_of(int H, int W, int total, int b, int& x0, int& y0, int& np) {
    const int ntx = (W + TW - 1) / TW, nty = (H + TH - 1) / TH;
    const int q = total >> 3, rr = total & 7, xcd = b & 7;
    const int id = xcd * q + min(xcd, rr) + (b >> 3);
    const int tx = id % ntx, rest = id / ntx;
    const int ty = rest % nty;
    np = rest / nty;
    x0 = tx * TW;
    y0 = ty * TH;
}
__device__ __forceinline__ void gauss_tile_coords(int H, int W, int& x0, int& y0, int& np) {
    gauss_tile_coords_of(H, W, gridDim.x, blockIdx.x, x0, y0, np);
}

// ---------------------------------------------------------------- Gaussian NMS (body peaks)
// avg: [N*P][H][W] (float32 single scale / float64 average); one workgroup per tile of 102 x 30
// outputs, so that both passes keep all 256 threads busy and the halo costs 2.43 filter
// evaluations per output pixel (2.59 for gauss_tile's 64 x 32; 0.42 vs 1.15 ms per bench step):
//  * vertical pass: thread = (column c of the 128-column footprint, half h of the 32 smoothed
//    rows), a 40-entry float64 register window sliding down the column straight from global
//    memory (coalesced rows); interior tiles step a pointer, border tiles reflect without
//    divisions whenever the footprint lies within one reflection of the map (every tile of any
//    map of at least 115 x 43);
//  * horizontal pass: thread = (row r, 13-column run): its 37 inputs into registers, a barrier,
//    then the 13 outputs written in place over the row (one LDS plane: 33 KB, 4 workgroups/CU);
//    row stride 129 doubles: the 32 rows of a lane group fall in distinct bank pairs;
//  * 4-neighbour NMS on the smoothed tile, then the reference's `> thre` (src/body.py:70-94).
// scipy order throughout (axis 0 then axis 1; centre tap, then |j| = 12 .. 1 pairs), float64,
// no FMA: bit-exact with scipy.ndimage.gaussian_filter(sigma=3).
constexpr int WTW = 102, WTH = 30;      // outputs per tile
constexpr int WVW = WTW + 26;           // 128 footprint / vertical-pass columns
constexpr int WVR = WTH + 2;            // 32 smoothed rows incl. the NMS ring
constexpr int WVH = WVR / 2;            // 16 rows per vertical thread
constexpr int WGW = WTW + 2;            // 104 smoothed columns incl. the ring
constexpr int WHC = WGW / 8;            // 13 columns per horizontal thread (8 runs x 32 rows)
static_assert(WVW * 2 == 256 && WVR * 8 == 256 && WHC * 8 == WGW, "wide Gaussian tile");

__device__ __forceinline__ int reflect_near(int i, int n) {  // valid for -n <= i < 2n
    return i < 0 ? -1 - i : (i >= n ? 2 * n - 1 - i : i);
}

// MODE 0: footprint inside the map (no reflection: one pointer step per row); 1: within one
// reflection of it (no divisions); 2: anything else (periodic reflect_idx)
template <typename T, int MODE>
__device__ __forceinline__ void gauss_wide_load(const T* __restrict__ m, int H, int W, int x0, int y0, int c, int h,
                                                double (&win)[WVH + 24]) {
    const int xi = x0 - 13 + c, r0 = y0 - 13 + h * WVH;
    if constexpr (MODE == 0) {
        const T* p = m + (size_t)r0 * W + xi;
#pragma unroll
        for (int i = 0; i < WVH + 24; ++i, p += W) win[i] = (double)*p;
    } else {
        const T* col = m + (MODE == 1 ? reflect_near(xi, W) : reflect_idx(xi, W));
#pragma unroll
        for (int i = 0; i < WVH + 24; ++i) {
            const int ry = MODE == 1 ? reflect_near(r0 + i, H) : reflect_idx(r0 + i, H);
            win[i] = (double)col[(size_t)ry * W];
        }
    }
}

// smoothing + NMS of one wide tile from the vertical pass's register window (every thread of
// the workgroup calls it; sv may alias a staging buffer the window was built from: the first
// barrier below comes after every window is complete).  score_at(y, x) = map_ori[y, x].
template <typename ScoreAt>
__device__ __forceinline__ void gauss_wide_tail(double (&win)[WVH + 24], double (*sv)[WVW + 1], int H, int W, int x0,
                                                int y0, int np, double thre, int cap, int* __restrict__ cnt,
                                                int* __restrict__ list, double* __restrict__ list_score,
                                                ScoreAt score_at) {
    const int tid = threadIdx.x;
    const int c = tid & (WVW - 1), h = tid >> 7;
    bool hot = false;
    const double skip_below = gauss_skip_below(thre);
#pragma unroll
    for (int i = 0; i < WVH + 24; ++i) hot |= win[i] >= skip_below;
    if (!__syncthreads_or(hot)) return;  // no smoothed value can pass `> thre` (see gauss_tile)
#pragma unroll
    for (int i = 0; i < WVH; ++i) {
        double acc = win[i + 12] * kGauss[0];
#pragma unroll
        for (int j = 12; j >= 1; --j) acc = acc + (win[i + 12 - j] + win[i + 12 + j]) * kGauss[j];
        sv[h * WVH + i][c] = acc;
    }
    __syncthreads();
    {
        const int r = tid & (WVR - 1), c0 = (tid >> 5) * WHC;
        double hw[WHC + 24];
#pragma unroll
        for (int i = 0; i < WHC + 24; ++i) hw[i] = sv[r][c0 + i];
        __syncthreads();  // every thread holds its inputs: outputs go in place
#pragma unroll
        for (int i = 0; i < WHC; ++i) {
            double acc = hw[i + 12] * kGauss[0];
#pragma unroll
            for (int j = 12; j >= 1; --j) acc = acc + (hw[i + 12 - j] + hw[i + 12 + j]) * kGauss[j];
            sv[r][c0 + i] = acc;
        }
    }
    __syncthreads();
    for (int e = tid; e < WTW * WTH; e += 256) {
        const int r = e / WTW, cc = e - r * WTW;
        const int y = y0 + r, x = x0 + cc;
        if (y >= H || x >= W) continue;
        const double v = sv[r + 1][cc + 1];
        const double up = y > 0 ? sv[r][cc + 1] : 0.0;
        const double dn = y < H - 1 ? sv[r + 2][cc + 1] : 0.0;
        const double lf = x > 0 ? sv[r + 1][cc] : 0.0;
        const double rt = x < W - 1 ? sv[r + 1][cc + 2] : 0.0;
        if (v >= up && v >= dn && v >= lf && v >= rt && v > thre) {
            const int slot = atomicAdd(cnt + np, 1);
            if (slot < cap) {
                list[(size_t)np * cap + slot] = y * W + x;
                list_score[(size_t)np * cap + slot] = score_at(y, x);
            }
        }
    }
}

// wide tile id -> (x0, y0, map) in XCD-contiguous ranges (guide T1)
__device__ __forceinline__ void gauss_wide_coords(int H, int W, int& x0, int& y0, int& np) {
    const int ntx = (W + WTW - 1) / WTW, nty = (H + WTH - 1) / WTH;
    const int total = gridDim.x, b = blockIdx.x;
    const int q = total >> 3, rr = total & 7, xcd = b & 7;
    const int id = xcd * q + min(xcd, rr) + (b >> 3);
    const int tx = id % ntx, rest = id / ntx;
    x0 = tx * WTW;
    y0 = (rest % nty) * WTH;
    np = rest / nty;
}

template <typename T>
__global__ __launch_bounds__(256) void gauss_nms_wide(const T* __restrict__ avg, int H, int W, double thre, int cap,
                                                      int* __restrict__ cnt, int* __restrict__ list,
                                                      double* __restrict__ list_score) {
    __shared__ double sv[WVR][WVW + 1];
    int x0, y0, np;
    gauss_wide_coords(H, W, x0, y0, np);
    const T* m = avg + (size_t)np * H * W;
    const int tid = threadIdx.x;
    const int c = tid & (WVW - 1), h = tid >> 7;
    double win[WVH + 24];
    if (x0 >= 13 && x0 + WTW + 13 <= W && y0 >= 13 && y0 + WTH + 13 <= H)
        gauss_wide_load<T, 0>(m, H, W, x0, y0, c, h, win);
    else if (x0 - 13 >= -W && x0 + WTW + 13 <= 2 * W && y0 - 13 >= -H && y0 + WTH + 13 <= 2 * H)
        gauss_wide_load<T, 1>(m, H, W, x0, y0, c, h, win);
    else
        gauss_wide_load<T, 2>(m, H, W, x0, y0, c, h, win);
    gauss_wide_tail(win, sv, H, W, x0, y0, np, thre, cap, cnt, list, list_score,
                    [&](int y, int x) { return (double)m[(size_t)y * W + x]; });
}

// Single-scale Body path with heat_full's cubic resize (src/body.py:57) fused in: the NMS window
// is resized from the x8 map (mid) inside the tile, so the full-resolution float32 map is neither
// written nor re-read (8 bytes per pixel and part), and a tile whose sources are all too small to
// produce a peak is dropped before any arithmetic (on the bench's maps ~60 % of the tiles: a
// part's peaks sit in a few places of the frame).  The footprint's source rows are resized
// horizontally once into LDS (aliasing the smoothing plane), then each vertical-pass thread
// combines its 40 window rows from them -- cubic_resize_rows<1>'s arithmetic in its order, so the
// window holds exactly the values launch_heat_full_f32 would have stored (0.f + v).  The score of
// a peak (map_ori[y, x]) is resampled from mid with cubic_sample_f32 (bit-identical, rare).
constexpr int GR_FOOT = WVR + 24;  // 56 footprint rows
constexpr int GR_MAXR = 40;        // staged source rows: 55 * sy + 6 <= 40
static_assert(GR_MAXR * WVW * 4 <= WVR * (WVW + 1) * 8, "staged rows fit in the smoothing plane");

__global__ __launch_bounds__(256) void gauss_nms_resize(const float* __restrict__ mid, int Cm, int coff, int P, int Hs,
                                                        int Ws, int H, int W, double sy, double sx, double thre,
                                                        int cap, int* __restrict__ cnt, int* __restrict__ list,
                                                        double* __restrict__ list_score) {
    __shared__ double sv[WVR][WVW + 1];
    __shared__ CubicTap s_ty[GR_FOOT];
    __shared__ int s_lo, s_hi;
    float (*hs)[WVW] = reinterpret_cast<float (*)[WVW]>(&sv[0][0]);
    int x0, y0, np;
    gauss_wide_coords(H, W, x0, y0, np);
    const int n = np / P, p = np - n * P;
    const float* plane = mid + ((size_t)n * Cm + coff + p) * Hs * Ws;
    const int tid = threadIdx.x;
    const int c = tid & (WVW - 1), h = tid >> 7;
    if (tid == 0) {
        s_lo = 0x7fffffff;
        s_hi = -1;
    }
    __syncthreads();
    if (tid < GR_FOOT) {  // vertical taps of the footprint rows (reflected like scipy)
        const CubicTap ty = cubic_tap(reflect_idx(y0 - 13 + tid, H), sy, Hs);
        s_ty[tid] = ty;
        atomicMin(&s_lo, ty.i[0]);
        atomicMax(&s_hi, ty.i[3]);
    }
    __syncthreads();
    const int lo = s_lo, hi = s_hi;
    {
        const CubicTap tx = cubic_tap(reflect_idx(x0 - 13 + c, W), sx, Ws);
        // Cold-tile skip, decided on the source before any arithmetic: every resized value of the
        // footprint is sum_i ty.c[i] * sum_j tx.c[j] * q_ij over the source values q this loop
        // reads, and the cubic (A = -0.75) weights of one axis sum to at most 1.375 in absolute
        // value (t = 0.5), so |resized| <= 1.890625 * max|q| (float32 rounding: < 1e-6 relative;
        // 1.9 covers it).  The smoothing is a convex combination of the resized footprint, so
        // when 1.9 * max|q| is below the threshold no output of the tile can pass `> thre`:
        // nothing to resize, filter or report (the exact criterion gauss_wide_tail applies to
        // the resized values, taken earlier and more conservatively).  NaN sources count as
        // below, as in gauss_wide_tail (a NaN only ever removes peaks).
        // One pass over the source: the horizontal resize of every footprint row goes to LDS
        // while the same loads feed the bound (a cold tile then returns without a second read
        // of its sources; a hot one has its rows staged already)
        float mx = 0.f;
        for (int r0 = lo + h; r0 <= hi; r0 += 16) {  // 8 rows per round, loads issued first
            float q[8][4];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float* row = plane + (size_t)min(r0 + 2 * k, hi) * Ws;
#pragma unroll
                for (int j = 0; j < 4; ++j) q[k][j] = row[tx.i[j]];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
#pragma unroll
                for (int j = 0; j < 4; ++j) mx = fmaxf(mx, fabsf(q[k][j]));
                float v = q[k][0] * tx.c[0];
                v = v + q[k][1] * tx.c[1];
                v = v + q[k][2] * tx.c[2];
                v = v + q[k][3] * tx.c[3];
                if (r0 + 2 * k <= hi) hs[r0 + 2 * k - lo][c] = v;
            }
        }
        // (the vote is also the barrier before the vertical pass reads hs)
        if (!__syncthreads_or(1.9 * (double)mx >= gauss_skip_below(thre))) return;
    }
    double win[WVH + 24];
#pragma unroll
    for (int i = 0; i < WVH + 24; ++i) {
        const CubicTap ty = s_ty[h * WVH + i];
        float o = hs[ty.i[0] - lo][c] * ty.c[0];
        o = o + hs[ty.i[1] - lo][c] * ty.c[1];
        o = o + hs[ty.i[2] - lo][c] * ty.c[2];
        o = o + hs[ty.i[3] - lo][c] * ty.c[3];
        win[i] = (double)(0.f + o);
    }
    gauss_wide_tail(win, sv, H, W, x0, y0, np, thre, cap, cnt, list, list_score, [&](int y, int x) {
        return (double)(0.f + cubic_sample_f32(plane, Ws, cubic_tap(y, sy, Hs), cubic_tap(x, sx, Ws)));
    });
}

bool gauss_nms_resize_fits(int Hs, int Ws, int H, int W, double sy) {
    return !(Hs == H && Ws == W) && 55.0 * sy + 6.0 <= (double)GR_MAXR;
}

void launch_gauss_nms_resize(const float* mid, int Cm, int coff, int P, int N, int Hs, int Ws, int H, int W, double sy,
                             double sx, double thre, int cap, int* cnt, int* list, double* list_score,
                             hipStream_t st) {
    if (!gauss_nms_resize_fits(Hs, Ws, H, W, sy)) throw std::invalid_argument("gauss_nms_resize: scale out of range");
    const int tiles = ((W + WTW - 1) / WTW) * ((H + WTH - 1) / WTH) * N * P;
    hipLaunchKernelGGL(gauss_nms_resize, dim3(tiles), dim3(256), 0, st, mid, Cm, coff, P, Hs, Ws, H, W, sy, sx, thre,
                       cap, cnt, list, list_score);
}

// Hand: binary = gaussian_filter(map) > thre (src/hand.py:62-63) as union-find seeds, labelled
// within each 64 x 32 tile: lab[i] = the first pixel (raster order) of i's component inside
// the tile where set, -1 elsewhere; cnt[np] += #set.
__global__ __launch_bounds__(256) void gauss_threshold(const double* __restrict__ avg, int H, int W, double thre,
                                                       int* __restrict__ lab, int* __restrict__ cnt,
                                                       double* __restrict__ sums) {
    __shared__ GaussTile t;
    __shared__ int s_n;
    int x0, y0, np;
    gauss_tile_coords(H, W, x0, y0, np);
    if (threadIdx.x == 0) s_n = 0;
    if (!gauss_tile(avg + (size_t)np * H * W, H, W, x0, y0, t, gauss_skip_below(thre))) {
        for (int e = threadIdx.x; e < TW * TH; e += 256) {  // nothing passes `> thre`
            const int r = e / TW, c = e - r * TW;
            const int y = y0 + r, x = x0 + c;
            if (y < H && x < W) lab[(size_t)np * H * W + y * W + x] = -1;
        }
        return;
    }
    int mine = 0;
    // The tile's own 8-connected components, in LDS (the vertical-pass plane is free now): a
    // wave = one 64-pixel tile row; each set pixel starts at the first pixel of its run (parent
    // < itself), runs are linked to the runs above them (one union per run contact, as in
    // cc_union), then every pixel stores the global index of its local root -- the component's
    // first pixel in raster order within the tile.  cc_border joins components across tiles.
    static_assert(TW == 64 && sizeof(t.v) >= sizeof(int) * TW * TH, "tile labels");
    int* sl = reinterpret_cast<int*>(&t.v[0][0]);
    const int lane = threadIdx.x & 63;
    for (int e = threadIdx.x; e < TW * TH; e += 256) {
        const int r = e / TW, c = e - r * TW;
        const bool on = y0 + r < H && x0 + c < W && t.g[r + 1][c + 1] > thre;
        const unsigned long long unset = ~__ballot(on) & ((1ull << lane) - 1);  // unset lanes below
        const int start = unset ? 64 - __clzll((long long)unset) : 0;          // first lane of the run
        sl[e] = on ? e - (lane - start) : -1;
        mine += on;
    }
    __syncthreads();
    const volatile int* vsl = sl;  // re-read: other lanes relink roots concurrently
    auto find = [&](int x) __attribute__((always_inline)) {
        int p = vsl[x];
        while (p != x) {
            x = p;
            p = vsl[x];
        }
        return x;
    };
    auto unite = [&](int a, int b) __attribute__((always_inline)) {
        for (;;) {
            a = find(a);
            b = find(b);
            if (a == b) return;
            if (a < b) {
                const int tmp = a;
                a = b;
                b = tmp;
            }
            const int old = atomicMin(sl + a, b);  // link root a (larger) under b
            if (old == a) return;
            a = old;
        }
    };
    for (int e = threadIdx.x + TW; e < TW * TH; e += 256) {
        if (sl[e] < 0) continue;
        const int c = e & (TW - 1), u = e - TW;
        const bool left = c > 0 && sl[e - 1] >= 0;
        const bool ul = c > 0 && sl[u - 1] >= 0, up = sl[u] >= 0, ur = c + 1 < TW && sl[u + 1] >= 0;
        if (!left) {
            if (ul) unite(e, u - 1);
            if (up && !ul) unite(e, u);
        }
        if (ur && !up) unite(e, u + 1);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < TW * TH; e += 256) {
        const int r = e / TW, c = e - r * TW;
        const int y = y0 + r, x = x0 + c;
        if (y >= H || x >= W) continue;
        int g = -1;
        if (sl[e] >= 0) {
            const int root = find(e);
            g = (y0 + root / TW) * W + x0 + (root & (TW - 1));
            // every component's root is one of its tiles' local roots: the sums cc_compress_sum
            // accumulates start from these zeros (no memset of the whole map)
            if (root == e) sums[(size_t)np * H * W + g] = 0.0;
        }
        lab[(size_t)np * H * W + y * W + x] = g;
    }
    if (mine) atomicAdd(&s_n, mine);
    __syncthreads();
    if (threadIdx.x == 0 && s_n) atomicAdd(cnt + np, s_n);
}

// tiles of gauss_threshold (per map); cc_border's grid
void gauss_threshold_tiles(int H, int W, int* ntx, int* nty) {
    *ntx = (W + TW - 1) / TW;
    *nty = (H + TH - 1) / TH;
}

// ---------------------------------------------------------------- Batch_body fast mode
// srcmx/utilmx.py:251-255 (float32)
__constant__ float kBlur5[5][5] = {{0.00078633f, 0.00655965f, 0.01330373f, 0.00655965f, 0.00078633f},
                                   {0.00655965f, 0.05472157f, 0.11098164f, 0.05472157f, 0.00655965f},
                                   {0.01330373f, 0.11098164f, 0.22508352f, 0.11098164f, 0.01330373f},
                                   {0.00655965f, 0.05472157f, 0.11098164f, 0.05472157f, 0.00655965f},
                                   {0.00078633f, 0.00655965f, 0.01330373f, 0.00655965f, 0.00078633f}};

// torch 'reflect' padding: edge not repeated (d c b | a b c d | c b a)
__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    const int p = 2 * n - 2;
    i %= p;
    if (i < 0) i += p;
    return i < n ? i : p - i;
}

constexpr int BT = 32;            // output tile (BT x BT)
constexpr int BI = BT + 6;        // input tile: 2 (blur) + 1 (NMS ring) each side

// heat [NP][H][W] float; one workgroup per BT x BT tile of one part map (1-D XCD-ordered grid)
__global__ __launch_bounds__(256) void blur5_nms(const float* __restrict__ heat, int H, int W, double thre, int cap,
                                                 int* __restrict__ cnt, int* __restrict__ list,
                                                 double* __restrict__ list_score) {
    __shared__ float s_in[BI][BI];
    __shared__ float s_b[BT + 2][BT + 2];
    const int ntx = (W + BT - 1) / BT, nty = (H + BT - 1) / BT;
    const int total = gridDim.x, b = blockIdx.x;
    const int q = total >> 3, rr = total & 7, xcd = b & 7;
    const int id = xcd * q + min(xcd, rr) + (b >> 3);
    const int tx = id % ntx, rest = id / ntx;
    const int ty = rest % nty, np = rest / nty;
    const int x0 = tx * BT, y0 = ty * BT;
    const float* m = heat + (size_t)np * H * W;
    for (int e = threadIdx.x; e < BI * BI; e += 256) {
        const int r = e / BI, c = e - r * BI;
        s_in[r][c] = m[(size_t)reflect101(y0 - 3 + r, H) * W + reflect101(x0 - 3 + c, W)];
    }
    __syncthreads();
    // blurred values for the tile plus a 1-pixel ring (rows / cols y0-1 .. y0+BT)
    for (int e = threadIdx.x; e < (BT + 2) * (BT + 2); e += 256) {
        const int r = e / (BT + 2), c = e - r * (BT + 2);
        float acc = 0.f;
#pragma unroll
        for (int dy = 0; dy < 5; ++dy)
#pragma unroll
            for (int dx = 0; dx < 5; ++dx) acc = acc + s_in[r + dy][c + dx] * kBlur5[dy][dx];
        s_b[r][c] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < BT * BT; e += 256) {
        const int r = e / BT, c = e - r * BT;
        const int y = y0 + r, x = x0 + c;
        if (y >= H || x >= W) continue;
        const float v = s_b[r + 1][c + 1];
        const float up = y > 0 ? s_b[r][c + 1] : 0.f;     // findpeaks_torch pads with zeros
        const float dn = y < H - 1 ? s_b[r + 2][c + 1] : 0.f;
        const float lf = x > 0 ? s_b[r + 1][c] : 0.f;
        const float rt = x < W - 1 ? s_b[r + 1][c + 2] : 0.f;
        if (v > (float)thre && v >= up && v >= dn && v >= lf && v >= rt) {
            const int slot = atomicAdd(cnt + np, 1);
            if (slot < cap) {
                list[(size_t)np * cap + slot] = y * W + x;
                list_score[(size_t)np * cap + slot] = (double)v;  // the blurred value (Batch_model.py:191)
            }
        }
    }
}

// Batch_hand fast mode (srcmx/Batch_model.py:327-354): blurred = 5x5 Gaussian of the x8 map
// (float32); binary = blurred > thre seeds the union-find labelling (run starts, as
// gauss_threshold); the blurred map (as float64) is what components are summed and searched
// on.  64 x 16 tiles: one wave = one 64-pixel row segment.
constexpr int SW = 64, SH = 16;
__global__ __launch_bounds__(256) void blur5_seed(const float* __restrict__ heat, int H, int W, double thre,
                                                  double* __restrict__ blurred, int* __restrict__ lab,
                                                  int* __restrict__ cnt) {
    __shared__ float s_in[SH + 4][SW + 4];
    __shared__ int s_n;
    const int ntx = (W + SW - 1) / SW, nty = (H + SH - 1) / SH;
    const int total = gridDim.x, b = blockIdx.x;
    const int q = total >> 3, rr = total & 7, xcd = b & 7;
    const int id = xcd * q + min(xcd, rr) + (b >> 3);
    const int tx = id % ntx, rest = id / ntx;
    const int ty = rest % nty, np = rest / nty;
    const int x0 = tx * SW, y0 = ty * SH;
    const float* m = heat + (size_t)np * H * W;
    if (threadIdx.x == 0) s_n = 0;
    for (int e = threadIdx.x; e < (SH + 4) * (SW + 4); e += 256) {
        const int r = e / (SW + 4), c = e - r * (SW + 4);
        s_in[r][c] = m[(size_t)reflect101(y0 - 2 + r, H) * W + reflect101(x0 - 2 + c, W)];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    int mine = 0;
    for (int e = threadIdx.x; e < SW * SH; e += 256) {
        const int r = e / SW, c = e - r * SW;
        const int y = y0 + r, x = x0 + c;
        const bool in = y < H && x < W;
        float acc = 0.f;
#pragma unroll
        for (int dy = 0; dy < 5; ++dy)
#pragma unroll
            for (int dx = 0; dx < 5; ++dx) acc = acc + s_in[r + dy][c + dx] * kBlur5[dy][dx];
        const bool on = in && acc > (float)thre;
        const unsigned long long unset = ~__ballot(on) & ((1ull << lane) - 1);
        const int start = unset ? 64 - __clzll((long long)unset) : 0;
        if (!in) continue;
        const size_t i = (size_t)y * W + x;
        blurred[(size_t)np * H * W + i] = (double)acc;
        lab[(size_t)np * H * W + i] = on ? (int)i - (lane - start) : -1;
        mine += on;
    }
    if (mine) atomicAdd(&s_n, mine);
    __syncthreads();
    if (threadIdx.x == 0 && s_n) atomicAdd(cnt + np, s_n);
}

// One workgroup per (frame, part): order the part's peaks row-major (np.nonzero), assign the
// global running ids (the counts of the parts before it), write candidate rows (x, y, score, id)
// into the record.  (One workgroup per frame walking the 18 parts took 40 us for a single frame:
// 18 dependent global round trips.)
__global__ __launch_bounds__(128) void peaks_finalize(const int* __restrict__ cnt, const int* __restrict__ list,
                                                      const double* __restrict__ list_score, int H, int W, RecordLayout L,
                                                      uint8_t* __restrict__ records, int* __restrict__ peak_pos,
                                                      int* __restrict__ part_cnt) {
    const int n = blockIdx.x / 18, p = blockIdx.x - n * 18;
    const int cap = L.peaks_per_part;
    __shared__ int s_c, s_start;
    __shared__ int s_v[1024];
    if (threadIdx.x < 64) {  // one wave: clamped counts, this part's start, the header (part 0)
        const int q = threadIdx.x;
        const int raw = q < 18 ? cnt[n * 18 + q] : 0;
        const int c = raw > cap ? cap : raw;
        int before = q < p ? c : 0;
        int total = c;
        bool over = raw > cap;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            before += __shfl_xor(before, off);
            total += __shfl_xor(total, off);
        }
        const bool any_over = __ballot(over) != 0ull;
        if (q == p) s_c = c;
        if (q == 0) {
            s_start = before;
            if (p == 0) {
                int32_t* hdr = reinterpret_cast<int32_t*>(records + (size_t)n * L.bytes);
                hdr[0] = any_over ? -5 : 0;
                hdr[1] = total;
                hdr[2] = 0;
                hdr[3] = 0;
            }
        }
    }
    __syncthreads();
    const int c = s_c;
    const int* lp = list + ((size_t)n * 18 + p) * cap;
    const bool staged = c <= 1024;
    if (staged)
        for (int i = threadIdx.x; i < c; i += blockDim.x) s_v[i] = lp[i];
    __syncthreads();
    double* cand = reinterpret_cast<double*>(records + (size_t)n * L.bytes + L.cand_off);
    for (int i = threadIdx.x; i < c; i += blockDim.x) {
        const int v = staged ? s_v[i] : lp[i];
        int rank = 0;
        for (int j = 0; j < c; ++j) rank += (staged ? s_v[j] : lp[j]) < v;
        const int y = v / W, x = v - y * W;
        const int id = s_start + rank;
        double* row = cand + (size_t)id * 4;
        row[0] = (double)x;
        row[1] = (double)y;
        row[2] = list_score[((size_t)n * 18 + p) * cap + i];
        row[3] = (double)id;
        peak_pos[((size_t)n * 18 + p) * cap + rank] = v;
    }
    if (threadIdx.x == 0) part_cnt[n * 18 + p] = c;
}

// value of the x8 map (cv2.resize(fx=fy=8, INTER_CUBIC) of an hl x wl plane, cropped) at (y8, x8):
// cubic_resize_rows<0>'s horizontal-then-vertical sums, so bit-identical to the staged map
__device__ __forceinline__ float x8_at(const float* __restrict__ low, int hl, int wl, int y8, int x8) {
    return cubic_sample_f32(low, wl, cubic_tap(y8, 0.125, hl), cubic_tap(x8, 0.125, wl));
}

// source floor of cubic_tap (its taps are floor - 1 .. floor + 2, clamped)
__device__ __forceinline__ int cubic_floor(int d, double scale) {
    return (int)floorf((float)(((double)d + 0.5) * scale - 0.5));
}

// the final resize (taps ty / tx over the x8 map) at one point of the PAF pair (chx, chx + 1), the
// x8 values evaluated from the low-res planes lx / ly.  The 4 x 4 x8 samples read a 5 x 5
// low-res patch: 4 consecutive x8 rows (columns) have source floors f0 or f0 + 1, so tap m of x8
// row r is patch row (f_r - f0) + m of the patch whose row k holds low-res row clamp(f0 - 1 + k)
// -- the clamped tap's row.  The patch is loaded once, every horizontal sum computed once per
// (patch row, x8 column), and each value is cubic_resize_rows<0>'s sum, then cubic_sample_f32's
// over those, in their order: bit-identical to resampling the staged x8 map.
__device__ __forceinline__ void resize_x8_pair(const float* __restrict__ lx, const float* __restrict__ ly, int hl,
                                               int wl, const CubicTap& ty, const CubicTap& tx, float& ox, float& oy) {
    float cxc[4][4];  // the x8 columns' horizontal coefficients
    bool bx[4], by[4];  // x8 column / row j's floor is f0 + 1
    const int fx0 = cubic_floor(tx.i[0], 0.125), fy0 = cubic_floor(ty.i[0], 0.125);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const CubicTap t = cubic_tap(tx.i[j], 0.125, wl);
#pragma unroll
        for (int n = 0; n < 4; ++n) cxc[j][n] = t.c[n];
        bx[j] = cubic_floor(tx.i[j], 0.125) != fx0;
        by[j] = cubic_floor(ty.i[j], 0.125) != fy0;
    }
    int cc[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) cc[d] = min(max(fx0 - 1 + d, 0), wl - 1);
#pragma unroll 1
    for (int ch = 0; ch < 2; ++ch) {  // one channel at a time: half the live registers
        const float* plane = ch ? ly : lx;
        float hs[4][5];  // [x8 column j][patch row k]
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const float* row = plane + (size_t)min(max(fy0 - 1 + k, 0), hl - 1) * wl;
            float p[5];
#pragma unroll
            for (int d = 0; d < 5; ++d) p[d] = row[cc[d]];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool b = bx[j];
                float v = (b ? p[1] : p[0]) * cxc[j][0];
                v = v + (b ? p[2] : p[1]) * cxc[j][1];
                v = v + (b ? p[3] : p[2]) * cxc[j][2];
                v = v + (b ? p[4] : p[3]) * cxc[j][3];
                hs[j][k] = v;
            }
        }
        float o = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const CubicTap ry = cubic_tap(ty.i[r], 0.125, hl);  // the x8 row's vertical coefficients
            const bool b = by[r];
            float x8[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float u = (b ? hs[j][1] : hs[j][0]) * ry.c[0];
                u = u + (b ? hs[j][2] : hs[j][1]) * ry.c[1];
                u = u + (b ? hs[j][3] : hs[j][2]) * ry.c[2];
                u = u + (b ? hs[j][4] : hs[j][3]) * ry.c[3];
                x8[j] = u;
            }
            float v = x8[0] * tx.c[0];
            v = v + x8[1] * tx.c[1];
            v = v + x8[2] * tx.c[2];
            v = v + x8[3] * tx.c[3];
            o = r == 0 ? v * ty.c[0] : o + v * ty.c[r];
        }
        if (ch) oy = o;
        else ox = o;
    }
}

// grid (frames * 19 limbs, blocks per limb); pair (i, j) -> score[n][k][i*nB + j]
// (-inf when criterion1/criterion2 fail; src/body.py:137-141).  A thread per (pair, sample): the
// ten samples of a pair are evaluated by ten lanes (each a cubic resample chain of dependent
// loads), then summed in sample order by the pair's first lane -- the reference's float64 order.
constexpr int PS_PAIRS = 25;  // pairs per 256-thread pass (250 lanes)
__global__ __launch_bounds__(256) void paf_score(PafScales S, const int* __restrict__ peak_pos,
                                                 const int* __restrict__ part_cnt, int cap, double thre2,
                                                 double* __restrict__ score) {
    const int nk = blockIdx.x;
    const int n = nk / 19, k = nk - n * 19;
    const int pa = kLimbA[k], pb = kLimbB[k];
    const int nA = part_cnt[n * 18 + pa], nB = part_cnt[n * 18 + pb];
    const int total = nA * nB;
    const int chx = kPafX[k];  // y component is channel chx + 1 (src/body.py:101-103)
    const int* posA = peak_pos + ((size_t)n * 18 + pa) * cap;
    const int* posB = peak_pos + ((size_t)n * 18 + pb) * cap;
    double* out = score + (size_t)nk * cap * cap;
    __shared__ double s_sm[PS_PAIRS * 10];
    const int q = threadIdx.x / 10, t = threadIdx.x - q * 10;  // pair slot, sample
    for (int e0 = blockIdx.y * PS_PAIRS; e0 < total; e0 += gridDim.y * PS_PAIRS) {
        const int e = e0 + q;
        const bool live = q < PS_PAIRS && e < total;
        double ux = 0.0, uy = 0.0, norm = 1.0;
        if (live) {
            const int i = e / nB, j = e - i * nB;
            const int va = posA[i], vb = posB[j];
            const int ya = va / S.W, xa = va - ya * S.W;
            const int yb = vb / S.W, xb = vb - yb * S.W;
            const long long vx = xb - xa, vy = yb - ya;
            norm = sqrt((double)(vx * vx + vy * vy)) + 1e-10;
            ux = (double)vx / norm;
            uy = (double)vy / norm;
            const double stx = ((double)xb - (double)xa) / 9.0;
            const double sty = ((double)yb - (double)ya) / 9.0;
            const double fx = t == 9 ? (double)xb : (double)t * stx + (double)xa;
            const double fy = t == 9 ? (double)yb : (double)t * sty + (double)ya;
            const int X = (int)rint(fx), Y = (int)rint(fy);
            // paf_avg[Y, X, ch] = sum over scales of float32(resize(x8 map) / n_scales),
            // accumulated in float64 (src/body.py:61-68); only the sampled pixels are
            // ever evaluated, the full-resolution PAF maps are never materialised.
            double px = 0.0, py = 0.0;
            for (int s = 0; s < S.n; ++s) {
                const size_t plane = (size_t)S.hs[s] * S.ws[s];
                const float* mx = S.mid[s] + ((size_t)n * S.cm + chx) * plane;
                float vx_, vy_;
                if (S.low[s]) {  // x8 values from the low-res PAF channels (L2-resident)
                    const size_t lp = (size_t)S.hl[s] * S.wl[s];
                    const float* lx = S.low[s] + ((size_t)n * S.lcm + chx) * lp;
                    if (S.hs[s] == S.H && S.ws[s] == S.W) {
                        vx_ = x8_at(lx, S.hl[s], S.wl[s], Y, X);
                        vy_ = x8_at(lx + lp, S.hl[s], S.wl[s], Y, X);
                    } else {
                        const CubicTap ty = cubic_tap(Y, S.sy[s], S.hs[s]);
                        const CubicTap tx = cubic_tap(X, S.sx[s], S.ws[s]);
                        resize_x8_pair(lx, lx + lp, S.hl[s], S.wl[s], ty, tx, vx_, vy_);
                    }
                } else if (S.hs[s] == S.H && S.ws[s] == S.W) {
                    vx_ = mx[(size_t)Y * S.ws[s] + X];
                    vy_ = mx[plane + (size_t)Y * S.ws[s] + X];
                } else {
                    const CubicTap ty = cubic_tap_any(Y, S.sy[s], S.hs[s], S.torch);
                    const CubicTap tx = cubic_tap_any(X, S.sx[s], S.ws[s], S.torch);
                    vx_ = cubic_sample_f32(mx, S.ws[s], ty, tx);
                    vy_ = cubic_sample_f32(mx + plane, S.ws[s], ty, tx);
                }
                px = px + (double)(vx_ / (float)S.n);
                py = py + (double)(vy_ / (float)S.n);
            }
            s_sm[q * 10 + t] = px * ux + py * uy;
        }
        __syncthreads();
        if (live && t == 0) {
            double acc = 0.0;
            int above = 0;
            for (int u = 0; u < 10; ++u) {
                const double sm = s_sm[q * 10 + u];
                acc = acc + sm;
                above += sm > thre2;
            }
            const double prior = 0.5 * (double)S.H / norm - 1.0;
            const double sc = acc / 10.0 + (prior > 0.0 ? 0.0 : prior);
            out[e] = (above > 8 && sc > 0.0) ? sc : -INFINITY;
        }
        __syncthreads();
    }
}

// One workgroup per (frame, limb): greedy matching in the order of a stable descending
// sort (ties -> smaller i*nB+j first), stopping at min(nA, nB) (src/body.py:143-151).
__global__ __launch_bounds__(256) void limb_greedy(const double* __restrict__ score, const int* __restrict__ part_cnt,
                                                   int cap, Conn* __restrict__ conn, int* __restrict__ conn_cnt) {
    const int nk = blockIdx.x;
    const int n = nk / 19, k = nk - n * 19;
    const int nA = part_cnt[n * 18 + kLimbA[k]], nB = part_cnt[n * 18 + kLimbB[k]];
    extern __shared__ unsigned char s_used[];  // [cap] A flags, [cap] B flags
    __shared__ double s_bs[4];
    __shared__ int s_bi[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (nA == 0 || nB == 0) {
        if (tid == 0) conn_cnt[nk] = -1;  // special_k (src/body.py:153-155)
        return;
    }
    for (int i = tid; i < 2 * cap; i += 256) s_used[i] = 0;
    __syncthreads();
    const double* sc = score + (size_t)nk * cap * cap;
    const int total = nA * nB, limit = nA < nB ? nA : nB;
    Conn* out = conn + (size_t)nk * cap;
    // the first GR_REG * 256 pairs stay in registers (score, i, j) for all rounds; a used pair is
    // retired to -inf in place (each round re-read every score from global memory before)
    constexpr int GR_REG = 8;
    double rv[GR_REG];
    int ri[GR_REG], rj[GR_REG];
#pragma unroll
    for (int r = 0; r < GR_REG; ++r) {
        const int e = tid + 256 * r;
        ri[r] = e < total ? e / nB : 0;
        rj[r] = e < total ? e - ri[r] * nB : 0;
        rv[r] = e < total ? sc[e] : -INFINITY;
    }
    int count = 0;
    for (;;) {
        double best = -INFINITY;
        int bidx = 0x7fffffff;
#pragma unroll
        for (int r = 0; r < GR_REG; ++r) {  // e increases per thread, so ties keep the smaller index
            if (rv[r] > best) {
                best = rv[r];
                bidx = tid + 256 * r;
            }
        }
        for (int e = tid + 256 * GR_REG; e < total; e += 256) {
            const int i = e / nB, j = e - i * nB;
            if (s_used[i] | s_used[cap + j]) continue;
            const double v = sc[e];
            if (v > best) {
                best = v;
                bidx = e;
            }
        }
        for (int off = 32; off >= 1; off >>= 1) {
            const double ob = __shfl_xor(best, off);
            const int oi = __shfl_xor(bidx, off);
            if (ob > best || (ob == best && oi < bidx)) {
                best = ob;
                bidx = oi;
            }
        }
        if (lane == 0) {
            s_bs[wave] = best;
            s_bi[wave] = bidx;
        }
        __syncthreads();
        best = s_bs[0];
        bidx = s_bi[0];
        for (int w = 1; w < 4; ++w)
            if (s_bs[w] > best || (s_bs[w] == best && s_bi[w] < bidx)) {
                best = s_bs[w];
                bidx = s_bi[w];
            }
        if (bidx == 0x7fffffff || best == -INFINITY) break;
        const int i = bidx / nB, j = bidx - i * nB;
#pragma unroll
        for (int r = 0; r < GR_REG; ++r)
            if (ri[r] == i || rj[r] == j) rv[r] = -INFINITY;
        if (tid == 0) {
            out[count].i = i;
            out[count].j = j;
            out[count].s = best;
            s_used[i] = 1;
            s_used[cap + j] = 1;
        }
        __syncthreads();
        // the count lives in every thread's registers: a shared counter bumped by thread 0 could
        // be read after the bump by a slower wave, which then left the loop a round early
        if (++count >= limit) break;
    }
    if (tid == 0) conn_cnt[nk] = count;
}

// One wavefront per frame: sequential person assembly with lane-parallel row scans.  Every
// limb's connections (score, both candidates' scores, candidate indices) are staged into LDS in
// one parallel pass when they fit `stage` entries (the serial loop then reads LDS only, and the
// dependent global loads -- count, connection, candidate score -- are paid once per frame instead
// of once per limb); otherwise limb by limb.
__global__ __launch_bounds__(64) void assemble_people(const Conn* __restrict__ conn, const int* __restrict__ conn_cnt,
                                                      const int* __restrict__ part_cnt, RecordLayout L,
                                                      uint8_t* __restrict__ records, int stage) {
    // [max_people][20] subset rows, then the staged connections
    extern __shared__ double smem[];
    const int n = blockIdx.x;
    const int lane = threadIdx.x;
    const int cap = L.peaks_per_part, maxp = L.max_people;
    double* s_sub = smem;
    double* s_cs = smem + (size_t)maxp * 20;
    double* s_sa = s_cs + stage;
    double* s_sb = s_sa + stage;
    int* s_ci = reinterpret_cast<int*>(s_sb + stage);
    uint8_t* rec = records + (size_t)n * L.bytes;
    int32_t* hdr = reinterpret_cast<int32_t*>(rec);
    const double* cand = reinterpret_cast<const double*>(rec + L.cand_off);
    double* outsub = reinterpret_cast<double*>(rec + L.subset_off);
    __shared__ int s_start[18], s_nc[19], s_off[20];
    if (lane < 18) {
        int acc = 0;
        for (int p = 0; p < lane; ++p) acc += part_cnt[n * 18 + p];
        s_start[lane] = acc;
    }
    if (lane < 19) s_nc[lane] = conn_cnt[n * 19 + lane];
    __syncthreads();
    if (lane == 0) {
        int acc = 0;
        for (int k = 0; k < 19; ++k) {
            s_off[k] = acc;
            acc += max(s_nc[k], 0);
        }
        s_off[19] = acc;
    }
    __syncthreads();
    // stage connection c of limb k at entry e
    auto stage_one = [&](int k, int c, int e) __attribute__((always_inline)) {
        const Conn cc = conn[((size_t)n * 19 + k) * cap + c];
        const int ga = s_start[kLimbA[k]] + cc.i, gb = s_start[kLimbB[k]] + cc.j;
        s_cs[e] = cc.s;
        s_sa[e] = cand[(size_t)ga * 4 + 2];
        s_sb[e] = cand[(size_t)gb * 4 + 2];
        s_ci[2 * e] = ga;
        s_ci[2 * e + 1] = gb;
    };
    const bool all = s_off[19] <= stage;
    if (all) {
        for (int e = lane; e < s_off[19]; e += 64) {
            int k = 0;
            while (k < 18 && e >= s_off[k + 1]) ++k;
            stage_one(k, e - s_off[k], e);
        }
        __syncthreads();
    }
    int status = hdr[0];
    int nrows = 0;
    for (int k = 0; k < 19 && status == 0; ++k) {
        const int nc = s_nc[k];
        if (nc < 0) continue;
        const int ia = kLimbA[k], ib = kLimbB[k];
        int base = s_off[k];
        if (!all) {
            base = 0;
            for (int c = lane; c < nc; c += 64) stage_one(k, c, c);
            __syncthreads();
        }
        for (int c0 = 0; c0 < nc; ++c0) {
            const int c = base + c0;
            const double idA = (double)s_ci[2 * c];
            const double idB = (double)s_ci[2 * c + 1];
            const double s = s_cs[c];
            int found = 0, j1 = -1, j2 = -1;
            for (int r0 = 0; r0 < nrows; r0 += 64) {
                const int r = r0 + lane;
                const bool hit = r < nrows && (s_sub[r * 20 + ia] == idA || s_sub[r * 20 + ib] == idB);
                unsigned long long b = __ballot(hit);
                while (b && found < 3) {
                    const int bit = __ffsll((long long)b) - 1;
                    b &= b - 1;
                    if (found == 0) j1 = r0 + bit;
                    else if (found == 1) j2 = r0 + bit;
                    ++found;
                }
            }
            if (found > 2) {  // subset_idx[2] = j -> IndexError (src/body.py:173)
                status = -6;
                break;
            }
            if (found == 1) {
                if (lane == 0 && s_sub[j1 * 20 + ib] != idB) {
                    s_sub[j1 * 20 + ib] = idB;
                    s_sub[j1 * 20 + 19] = s_sub[j1 * 20 + 19] + 1.0;
                    s_sub[j1 * 20 + 18] = s_sub[j1 * 20 + 18] + (s_sb[c] + s);
                }
            } else if (found == 2) {
                const bool both = lane < 18 && s_sub[j1 * 20 + lane] >= 0.0 && s_sub[j2 * 20 + lane] >= 0.0;
                if (__ballot(both) == 0ull) {  // disjoint: merge j2 into j1, drop j2
                    if (lane < 18) s_sub[j1 * 20 + lane] = s_sub[j1 * 20 + lane] + (s_sub[j2 * 20 + lane] + 1.0);
                    if (lane == 18 || lane == 19) s_sub[j1 * 20 + lane] = s_sub[j1 * 20 + lane] + s_sub[j2 * 20 + lane];
                    __syncthreads();
                    if (lane == 0) s_sub[j1 * 20 + 18] = s_sub[j1 * 20 + 18] + s;
                    __syncthreads();
                    for (int r = j2; r < nrows - 1; ++r) {
                        double v = lane < 20 ? s_sub[(r + 1) * 20 + lane] : 0.0;
                        __syncthreads();
                        if (lane < 20) s_sub[r * 20 + lane] = v;
                        __syncthreads();
                    }
                    --nrows;
                } else if (lane == 0) {
                    s_sub[j1 * 20 + ib] = idB;
                    s_sub[j1 * 20 + 19] = s_sub[j1 * 20 + 19] + 1.0;
                    s_sub[j1 * 20 + 18] = s_sub[j1 * 20 + 18] + (s_sb[c] + s);
                }
            } else if (k < 17) {
                if (nrows >= maxp) {
                    status = -5;
                    break;
                }
                if (lane < 20) {
                    double v = -1.0;
                    if (lane == ia) v = idA;
                    if (lane == ib) v = idB;
                    if (lane == 19) v = 2.0;
                    if (lane == 18) v = (s_sa[c] + s_sb[c]) + s;
                    s_sub[nrows * 20 + lane] = v;
                }
                ++nrows;
            }
            __syncthreads();
        }
        if (!all) __syncthreads();  // the staged connections are re-filled by the next limb
    }
    // prune (src/body.py:203-208) and emit in order
    int kept = 0;
    if (status == 0) {
        for (int r = 0; r < nrows; ++r) {
            const double cntp = s_sub[r * 20 + 19], tot = s_sub[r * 20 + 18];
            const bool drop = cntp < 4.0 || tot / cntp < 0.4;
            if (!drop) {
                if (lane < 20) outsub[(size_t)kept * 20 + lane] = s_sub[r * 20 + lane];
                ++kept;
            }
        }
    }
    if (lane == 0) {
        hdr[0] = status;
        hdr[2] = kept;
    }
}

// ------------------------------------------------------------------ launchers
void launch_gauss_nms(const void* avg, bool f32, int NP, int H, int W, double thre, int cap, int* cnt, int* list,
                      double* list_score, hipStream_t st) {
    const dim3 grid(((W + WTW - 1) / WTW) * ((H + WTH - 1) / WTH) * NP);
    if (f32)
        hipLaunchKernelGGL(gauss_nms_wide<float>, grid, dim3(256), 0, st, (const float*)avg, H, W, thre, cap, cnt,
                           list, list_score);
    else
        hipLaunchKernelGGL(gauss_nms_wide<double>, grid, dim3(256), 0, st, (const double*)avg, H, W, thre, cap, cnt,
                           list, list_score);
}

void launch_blur5_nms(const float* heat, int NP, int H, int W, double thre, int cap, int* cnt, int* list,
                      double* list_score, hipStream_t st) {
    dim3 grid(((W + BT - 1) / BT) * ((H + BT - 1) / BT) * NP);
    hipLaunchKernelGGL(blur5_nms, grid, dim3(256), 0, st, heat, H, W, thre, cap, cnt, list, list_score);
}

void launch_blur5_seed(const float* heat, int NP, int H, int W, double thre, double* blurred, int* lab, int* cnt,
                       hipStream_t st) {
    dim3 grid(((W + SW - 1) / SW) * ((H + SH - 1) / SH) * NP);
    hipLaunchKernelGGL(blur5_seed, grid, dim3(256), 0, st, heat, H, W, thre, blurred, lab, cnt);
}

void launch_gauss_threshold(const double* avg, int NP, int H, int W, double thre, int* lab, int* cnt, double* sums,
                            hipStream_t st) {
    dim3 grid(((W + TW - 1) / TW) * ((H + TH - 1) / TH) * NP);
    hipLaunchKernelGGL(gauss_threshold, grid, dim3(256), 0, st, avg, H, W, thre, lab, cnt, sums);
}

void launch_peaks_finalize(const int* cnt, const int* list, const double* list_score, int N, int H, int W,
                           const RecordLayout& L, uint8_t* records, int* peak_pos, int* part_cnt, hipStream_t st) {
    hipLaunchKernelGGL(peaks_finalize, dim3(N * 18), dim3(128), 0, st, cnt, list, list_score, H, W, L, records,
                       peak_pos, part_cnt);
}


void launch_paf_score(const PafScales& S, const int* peak_pos, const int* part_cnt, int N, int cap, double thre2,
                      double* score, hipStream_t st) {
    int by = (cap * cap + PS_PAIRS - 1) / PS_PAIRS;
    if (by > 64) by = 64;
    hipLaunchKernelGGL(paf_score, dim3(N * 19, by), dim3(256), 0, st, S, peak_pos, part_cnt, cap, thre2, score);
}

void launch_limb_greedy(const double* score, const int* part_cnt, int N, int cap, Conn* conn, int* conn_cnt,
                        hipStream_t st) {
    hipLaunchKernelGGL(limb_greedy, dim3(N * 19), dim3(256), 2 * cap, st, score, part_cnt, cap, conn, conn_cnt);
}

void launch_assemble(const Conn* conn, const int* conn_cnt, const int* part_cnt, int N, const RecordLayout& L,
                     uint8_t* records, hipStream_t st) {
    // staged connection entries: every limb's (19 x peaks_per_part) when that fits 64 KB with the
    // subset rows, at least one limb's
    constexpr size_t kEntry = 3 * sizeof(double) + 2 * sizeof(int);
    const size_t sub = sizeof(double) * 20 * L.max_people;
    const size_t fit = sub < 64 * 1024 ? (64 * 1024 - sub) / kEntry : 0;
    const int stage = (int)std::max<size_t>((size_t)L.peaks_per_part, std::min<size_t>(19 * (size_t)L.peaks_per_part, fit));
    const size_t shm = sub + (size_t)stage * kEntry;
    if (shm > 64 * 1024) {  // grown capacities (up to 256 people / 1024 peaks per part: 80 KB)
        static size_t granted = 0;
        if (shm > granted) {
            OPOSE_HIP_CHECK(hipFuncSetAttribute((const void*)assemble_people,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
            granted = shm;
        }
    }
    hipLaunchKernelGGL(assemble_people, dim3(N), dim3(64), shm, st, conn, conn_cnt, part_cnt, L, records, stage);
}

}  // namespace opose
