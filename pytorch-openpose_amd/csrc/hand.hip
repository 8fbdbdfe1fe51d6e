// hand.hip — Hand() post-network path: 8-connected components + component selection.
//
// Reference: hitmaxiang/pytorch-openpose src/hand.py:59-75 (per part):
//   binary = gaussian_filter(map_ori, 3) > thre          (gauss_threshold in post.hip)
//   label(binary, connectivity=2)                         => cc_union / cc_compress
//   best = argmax_i sum(map_ori[label == i]) + 1          => cc_sums / hand_select
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

// lab: [NP][H*W] seeds (index or -1); 8-connectivity: link to left, up-left, up, up-right
__global__ __launch_bounds__(256) void cc_union(int* __restrict__ lab, int H, int W) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int np = blockIdx.z;
    if (x >= W) return;
    int* L = lab + (size_t)np * H * W;
    const int i = y * W + x;
    if (L[i] < 0) return;
    if (x > 0 && L[i - 1] >= 0) uf_union(L, i, i - 1);
    if (y > 0) {
        const int u = i - W;
        if (x > 0 && L[u - 1] >= 0) uf_union(L, i, u - 1);
        if (L[u] >= 0) uf_union(L, i, u);
        if (x + 1 < W && L[u + 1] >= 0) uf_union(L, i, u + 1);
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

// one workgroup per (crop, part): pick the component, then the first row-major maximum of
// {map_ori inside it, 0 elsewhere}; writes peaks[np] = (x, y, value), found[np]
__global__ __launch_bounds__(256) void hand_select(const int* __restrict__ lab, const double* __restrict__ ori,
                                                   const double* __restrict__ sums, const int* __restrict__ cnt,
                                                   int H, int W, double* __restrict__ peaks, int* __restrict__ found) {
    const int np = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t off = (size_t)np * H * W;
    const int n = H * W;
    __shared__ double s_v[4];
    __shared__ int s_i[4];
    if (cnt[np] == 0) {  // nothing above threshold: the reference's [0, 0, 0] row
        if (tid == 0) {
            peaks[np * 3 + 0] = 0.0;
            peaks[np * 3 + 1] = 0.0;
            peaks[np * 3 + 2] = 0.0;
            found[np] = 0;
        }
        return;
    }
    auto reduce = [&](double& v, int& idx) {
        for (int o = 32; o >= 1; o >>= 1) {
            const double ov = __shfl_xor(v, o);
            const int oi = __shfl_xor(idx, o);
            if (ov > v || (ov == v && oi < idx)) {
                v = ov;
                idx = oi;
            }
        }
        if (lane == 0) {
            s_v[wave] = v;
            s_i[wave] = idx;
        }
        __syncthreads();
        v = s_v[0];
        idx = s_i[0];
        for (int w = 1; w < 4; ++w)
            if (s_v[w] > v || (s_v[w] == v && s_i[w] < idx)) {
                v = s_v[w];
                idx = s_i[w];
            }
        __syncthreads();
    };
    // 1) component with the largest sum (ties: smallest root = lowest label)
    double bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < n; i += 256) {
        if (lab[off + i] == i) {
            const double v = sums[off + i];
            if (v > bv) {  // ascending i per thread: ties keep the smaller root
                bv = v;
                bi = i;
            }
        }
    }
    reduce(bv, bi);
    const int best = bi;
    // 2) first maximum of the masked map (everything outside the component reads 0.0)
    double mv = -INFINITY;
    int mi = 0x7fffffff;
    for (int i = tid; i < n; i += 256) {
        const double v = lab[off + i] == best ? ori[off + i] : 0.0;
        if (v > mv) {
            mv = v;
            mi = i;
        }
    }
    reduce(mv, mi);
    if (tid == 0) {
        peaks[np * 3 + 0] = (double)(mi % W);
        peaks[np * 3 + 1] = (double)(mi / W);
        peaks[np * 3 + 2] = mv;
        found[np] = 1;
    }
}

void launch_hand_cc(double* avg, int NP, int H, int W, int* lab, double* sums, const int* cnt, double* peaks,
                    int* found, hipStream_t st) {
    dim3 grid((W + 255) / 256, H, NP);
    hipLaunchKernelGGL(cc_union, grid, dim3(256), 0, st, lab, H, W);
    OPOSE_HIP_CHECK(hipMemsetAsync(sums, 0, sizeof(double) * (size_t)NP * H * W, st));
    hipLaunchKernelGGL(cc_compress_sum, grid, dim3(256), 0, st, lab, avg, H, W, sums);
    hipLaunchKernelGGL(hand_select, dim3(NP), dim3(256), 0, st, lab, avg, sums, cnt, H, W, peaks, found);
}

}  // namespace opose
