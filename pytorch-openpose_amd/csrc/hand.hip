// hand.hip — Hand() post-network path: 8-connected components + component selection.
//
// Reference: hitmaxiang/pytorch-openpose src/hand.py:59-75 (per part):
//   binary = gaussian_filter(map_ori, 3) > thre          (gauss_threshold in post.hip)
//   label(binary, connectivity=2)                         => gauss_threshold (per 64x32 tile, in LDS)
//                                                            + cc_border / cc_compress_sum
//   best = argmax_i sum(map_ori[label == i]) + 1          => cc_compress_sum / hand_select_*
//   map_ori[label != best] = 0; (y, x) = util.npmax(map_ori) (first row-major max)
//
// Labels: every component is represented by its minimum linear pixel index (union-find with
// atomicMin linking larger roots under smaller ones).  skimage / scipy number components in
// raster order of their first pixel, which is exactly the order of those minima, so
// "first component with the maximal sum" is "smallest root with the maximal sum".
// Component sums: per wave one float64 atomic per distinct root (order differs from numpy's
// pairwise sum: only an exact tie within ~1e-16 relative between two components could
// resolve differently).
#include "common.h"
#include "kernels.h"

namespace opose {

__device__ __forceinline__ int uf_find(const int* L, int x) {
    int p = L[x];
    while (p != x) {
        x = p;
        p = L[x];
    }
    return x;
}

__device__ __forceinline__ void uf_union(int* L, int a, int b) {
    for (;;) {
        a = uf_find(L, a);
        b = uf_find(L, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        // link root a (larger) under b; succeeds iff a was still a root
        const int old = atomicMin(L + a, b);
        if (old == a) return;
        a = old;
    }
}

// lab: [NP][H*W] seeds (-1, or the start of the pixel's run within its 64-pixel row segment,
// see gauss_threshold).  8-connectivity with one union per run contact instead of four per
// pixel: a run is already one tree, so a pixel whose left neighbour is set only links an
// up-right pixel that starts a new run above (its left neighbour covers up-left and up);
// a run start links the first pixel of each run above it; runs crossing a 64-pixel segment
// boundary are joined at the boundary.
__global__ __launch_bounds__(256) void cc_union(int* __restrict__ lab, int H, int W) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int np = blockIdx.z;
    if (x >= W) return;
    int* L = lab + (size_t)np * H * W;
    const int i = y * W + x;
    if (L[i] < 0) return;
    const bool left = x > 0 && L[i - 1] >= 0;
    if (left && (x & 63) == 0) uf_union(L, i, i - 1);  // run continues across the segment edge
    if (y > 0) {
        const int u = i - W;
        const bool ul = x > 0 && L[u - 1] >= 0, up = L[u] >= 0, ur = x + 1 < W && L[u + 1] >= 0;
        if (!left) {
            if (ul) uf_union(L, i, u - 1);
            if (up && !ul) uf_union(L, i, u);
        }
        if (ur && !up) uf_union(L, i, u + 1);
    }
}

// Seeds already labelled per 64 x 32 tile (gauss_threshold: every set pixel points at its
// tile-local root): join components across tile edges.  One thread per pixel of a tile's top row
// (links to the three pixels above it) and of its left column (links to the three pixels left of
// it) -- every 8-adjacent pair of set pixels in different tiles is one of these.
constexpr int kSeedTW = 64, kSeedTH = 32;

__global__ __launch_bounds__(128) void cc_border(int* __restrict__ lab, int H, int W, int ntx) {
    const int tx = blockIdx.x % ntx, ty = blockIdx.x / ntx, np = blockIdx.y;
    const int x0 = tx * kSeedTW, y0 = ty * kSeedTH;
    int* L = lab + (size_t)np * H * W;
    const int t = threadIdx.x;
    if (t < kSeedTW) {  // top row: (y0 - 1, x - 1 .. x + 1)
        const int x = x0 + t, y = y0;
        if (y0 == 0 || x >= W || y >= H) return;
        const int i = y * W + x;
        if (L[i] < 0) return;
        for (int dx = -1; dx <= 1; ++dx) {
            const int xx = x + dx;
            if (xx >= 0 && xx < W && L[i - W + dx] >= 0) uf_union(L, i, i - W + dx);
        }
    } else if (t < kSeedTW + kSeedTH) {  // left column: (y - 1 .. y + 1, x0 - 1)
        const int x = x0, y = y0 + t - kSeedTW;
        if (x0 == 0 || y >= H) return;
        const int i = y * W + x;
        if (L[i] < 0) return;
        for (int dy = -1; dy <= 1; ++dy) {
            const int yy = y + dy;
            if (yy >= 0 && yy < H && L[i + dy * W - 1] >= 0) uf_union(L, i, i + dy * W - 1);
        }
    }
}

// flatten to roots and accumulate component sums of the raw (unsmoothed) heat
__global__ __launch_bounds__(256) void cc_compress_sum(int* __restrict__ lab, const double* __restrict__ ori, int H,
                                                       int W, double* __restrict__ sums) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int np = blockIdx.z;
    const size_t off = (size_t)np * H * W;
    int* L = lab + off;
    const int i = y * W + x;
    int r = -1;
    double v = 0.0;
    if (x < W && L[i] >= 0) {
        r = uf_find(L, i);
        L[i] = r;
        v = ori[off + i];
    }
    // one atomic per distinct root per wave (a component covers long runs of pixels: per-pixel
    // float64 atomics on one address serialised the whole map)
    bool active = r >= 0;
    while (__any(active)) {
        const unsigned long long m = __ballot(active);
        const int src = __ffsll((long long)m) - 1;
        const int rr = __shfl(r, src);
        const bool mine = active && r == rr;
        double sv = mine ? v : 0.0;
        for (int o = 32; o >= 1; o >>= 1) sv += __shfl_xor(sv, o);
        if ((int)(threadIdx.x & 63) == src) atomicAdd(sums + off + rr, sv);
        active = active && !mine;
    }
}

// Selection (src/hand.py:66-75), spread over SEL_NB workgroups per (crop, part):
// pass 1: the component with the largest sum (ties: smallest root = lowest label);
// pass 2: the first row-major maximum of {map_ori inside it, 0 elsewhere} (util.npmax).
// Each pass: per-slice (value, index) partials, then a one-wave reduction.  The (greater
// value, else smaller index) rule is associative, so the result is order independent.
constexpr int SEL_NB = 32;

__device__ __forceinline__ void better(double& v, int& i, double ov, int oi) {
    if (ov > v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
    }
}

template <int PASS>
__global__ __launch_bounds__(256) void hand_select_part(const int* __restrict__ lab, const double* __restrict__ ori,
                                                        const double* __restrict__ sums, const int* __restrict__ cnt,
                                                        const int* __restrict__ best, int n,
                                                        double* __restrict__ part_v, int* __restrict__ part_i) {
    const int b = blockIdx.x, np = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (cnt[np] == 0) return;
    const size_t off = (size_t)np * n;
    const int chunk = (n + SEL_NB - 1) / SEL_NB;
    const int i0 = b * chunk, i1 = min(n, i0 + chunk);
    const int bc = PASS == 2 ? best[np] : 0;
    double v = -INFINITY;
    int idx = 0x7fffffff;
    for (int i = i0 + tid; i < i1; i += 256) {  // ascending per thread: ties keep the smaller
        const int l = lab[off + i];
        if (PASS == 1) {
            if (l == i && sums[off + i] > v) {
                v = sums[off + i];
                idx = i;
            }
        } else {
            const double x = l == bc ? ori[off + i] : 0.0;
            if (x > v) {
                v = x;
                idx = i;
            }
        }
    }
    for (int o = 32; o >= 1; o >>= 1) better(v, idx, __shfl_xor(v, o), __shfl_xor(idx, o));
    __shared__ double s_v[4];
    __shared__ int s_i[4];
    if (lane == 0) {
        s_v[wave] = v;
        s_i[wave] = idx;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; ++w) better(v, idx, s_v[w], s_i[w]);
        part_v[np * SEL_NB + b] = v;
        part_i[np * SEL_NB + b] = idx;
    }
}

// one wave per (crop, part): reduce the SEL_NB partials
template <int PASS>
__global__ __launch_bounds__(64) void hand_select_reduce(const int* __restrict__ cnt, const double* __restrict__ part_v,
                                                         const int* __restrict__ part_i, int W, int* __restrict__ best,
                                                         double* __restrict__ peaks, int* __restrict__ found) {
    const int np = blockIdx.x, lane = threadIdx.x;
    if (cnt[np] == 0) {  // nothing above threshold: the reference's [0, 0, 0] row
        if (PASS == 2 && lane == 0) {
            peaks[np * 3 + 0] = 0.0;
            peaks[np * 3 + 1] = 0.0;
            peaks[np * 3 + 2] = 0.0;
            found[np] = 0;
        }
        return;
    }
    double v = lane < SEL_NB ? part_v[np * SEL_NB + lane] : -INFINITY;
    int idx = lane < SEL_NB ? part_i[np * SEL_NB + lane] : 0x7fffffff;
    for (int o = 32; o >= 1; o >>= 1) better(v, idx, __shfl_xor(v, o), __shfl_xor(idx, o));
    if (lane != 0) return;
    if (PASS == 1) {
        best[np] = idx;
    } else {
        peaks[np * 3 + 0] = (double)(idx % W);
        peaks[np * 3 + 1] = (double)(idx / W);
        peaks[np * 3 + 2] = v;
        found[np] = 1;
    }
}

size_t hand_cc_workspace_bytes(int NP) { return (size_t)NP * SEL_NB * (sizeof(double) + sizeof(int)) + NP * 4; }

void launch_hand_cc(double* avg, int NP, int H, int W, int* lab, double* sums, const int* cnt, double* peaks,
                    int* found, void* ws, bool tile_seeds, hipStream_t st) {
    dim3 grid((W + 255) / 256, H, NP);
    if (tile_seeds) {
        int ntx, nty;
        gauss_threshold_tiles(H, W, &ntx, &nty);
        hipLaunchKernelGGL(cc_border, dim3(ntx * nty, NP), dim3(128), 0, st, lab, H, W, ntx);
    } else {
        hipLaunchKernelGGL(cc_union, grid, dim3(256), 0, st, lab, H, W);
    }
    if (!tile_seeds)  // tile seeds: gauss_threshold zeroed the sums at every possible root
        OPOSE_HIP_CHECK(hipMemsetAsync(sums, 0, sizeof(double) * (size_t)NP * H * W, st));
    hipLaunchKernelGGL(cc_compress_sum, grid, dim3(256), 0, st, lab, avg, H, W, sums);
    double* part_v = static_cast<double*>(ws);
    int* part_i = reinterpret_cast<int*>(part_v + (size_t)NP * SEL_NB);
    int* best = part_i + (size_t)NP * SEL_NB;
    const int n = H * W;
    hipLaunchKernelGGL(hand_select_part<1>, dim3(SEL_NB, NP), dim3(256), 0, st, lab, avg, sums, cnt, best, n, part_v,
                       part_i);
    hipLaunchKernelGGL(hand_select_reduce<1>, dim3(NP), dim3(64), 0, st, cnt, part_v, part_i, W, best, peaks, found);
    hipLaunchKernelGGL(hand_select_part<2>, dim3(SEL_NB, NP), dim3(256), 0, st, lab, avg, sums, cnt, best, n, part_v,
                       part_i);
    hipLaunchKernelGGL(hand_select_reduce<2>, dim3(NP), dim3(64), 0, st, cnt, part_v, part_i, W, best, peaks, found);
}

}  // namespace opose
