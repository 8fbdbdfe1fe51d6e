// conv.hip — implicit-GEMM convolution on the gfx950 fp32 matrix cores.
//
// Replaces the nn.Conv2d(+ReLU) / nn.MaxPool2d / torch.cat graph of
// hitmaxiang/pytorch-openpose src/model.py:7-22 (make_layers), :106-133 (body forward),
// :197-214 (hand forward).
//
// GEMM view of a stride-1 'same' convolution over a batch of NCHW frames:
//   out[m][p] = bias[m] + sum_k  W[m][k] * im2col[k][p]
//   m = output channel, p = (frame, y, x) flattened, k = (c, ky, kx) in OIHW order.
// * A = weights, pre-transposed once at load time to Wt[Kpad][Mpad] (zero padded), so a
//   KC x MT tile is MT contiguous floats per k row (16-B vector loads, ds_write_b128).
// * B = im2col gathered on the fly from the NCHW activation (L2-resident at these sizes):
//   every wave loads whole k rows for 64 consecutive pixels -> coalesced along x; the
//   k -> (c, ky, kx) decode is wave-uniform (scalar loads of a per-layer table).
// * v_mfma_f32_32x32x2_f32: exact fp32 (bitwise an fmaf chain), 64 FLOP/clk/SIMD.  A
//   256-thread workgroup = 2x2 waves, each wave owns (MT/2)x(PT/2) outputs =
//   (MT/64)x(PT/64) 32x32 accumulators; K is consumed in chunks of 32 through a
//   double-buffered LDS tile with register staging (one barrier per chunk).
// * split-K (gridDim.z) writes fp32 partial slabs that a second kernel sums in a fixed
//   order (deterministic), fusing bias + ReLU there.
// * epilogue fuses bias + ReLU and writes into a channel slice of a wider buffer, so the
//   reference's torch.cat([L1, L2, trunk]) (src/model.py:112-128) never materialises.
#include "common.h"
#include "kernels.h"

namespace opose {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));  // native vector (HIP's float4 class defeats SROA)
typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int KC = 32;   // k rows per chunk
constexpr int NT = 256;  // threads per workgroup

template <int MT, int PT>
__global__ __launch_bounds__(NT, 2) void conv_igemm_f32(ConvArgs a, const int* __restrict__ ktab) {
    constexpr int WM = MT / 2, WP = PT / 2;
    constexpr int TM = WM / 32, TN = WP / 32;
    constexpr int A_F4 = MT * KC / 4 / NT;  // float4 A loads per thread per chunk
    constexpr int PJ = PT / 64;             // pixel columns per lane
    constexpr int RW = KC / 4;              // k rows loaded per wave per chunk
    constexpr int A_SZ = KC * MT, B_SZ = KC * PT;

    __shared__ __attribute__((aligned(16))) float lds[2 * (A_SZ + B_SZ) + MT];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int l31 = lane & 31, hk = lane >> 5;

    const int zg = blockIdx.z;
    const int g = zg / a.splits;
    const int split = zg - g * a.splits;
    const ConvGroup G = g == 0 ? a.g[0] : a.g[1];  // no dynamic kernarg indexing

    const int p0 = blockIdx.x * PT;
    const int m0 = blockIdx.y * MT;
    const int HW = a.H * a.W;
    float* s_bias = lds + 2 * (A_SZ + B_SZ);
    if (tid < MT) s_bias[tid] = (m0 + tid < G.cout) ? G.bias[m0 + tid] : 0.f;

    // ---- per-lane pixel state for the im2col gather.  The activation is read through a
    // buffer resource: an invalid (zero-padding) tap gets voffset 0xffffffff, which the
    // hardware range check turns into 0.0f -> the gather is branch free.
    const float* in_base = G.in + (size_t)G.in_coff * HW;
    const int32_t* ib32 = reinterpret_cast<const int32_t*>(&in_base);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)in_base, (short)0, (int)0xffffff00u, 0x00020000);
    (void)ib32;
    uint32_t poff[PJ];  // element offset of the lane's pixel (channel 0 of its frame)
    int py[PJ], px[PJ];
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
        int p = p0 + j * 64 + lane;
        const bool v = p < a.npix;
        int pc = v ? p : 0;
        int n = pc / HW;
        int r = pc - n * HW;
        py[j] = v ? r / a.W : -100000;  // out-of-range row => every tap invalid
        px[j] = r - (r / a.W) * a.W;
        poff[j] = (uint32_t)(n * G.in_cstride * HW + r);
    }

    const int nchunks = a.Kpad / KC;
    const int c_begin = split * a.chunks_per_split;
    const int c_end = min(nchunks, c_begin + a.chunks_per_split);

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    f32x4 ra[A_F4];
    float rb[RW][PJ];

    auto load_chunk = [&](int c) __attribute__((always_inline)) {
        const int k0 = c * KC;
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            int idx = tid + i * NT;
            int row = idx / (MT / 4);
            int c4 = idx - row * (MT / 4);
            ra[i] = *reinterpret_cast<const f32x4*>(G.wt + (size_t)(k0 + row) * a.Mpad + m0 + c4 * 4);
        }
        const int kw0 = __builtin_amdgcn_readfirstlane(k0 + wave * RW);
        const i32x8 codes = *reinterpret_cast<const i32x8*>(ktab + kw0);  // wave-uniform
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int code = codes[r];  // (c << 8) | (ky << 4) | kx ; K padding rows carry zero weights
            const int cch = code >> 8;
            const int dy = ((code >> 4) & 15) - a.pad;
            const int dx = (code & 15) - a.pad;
            const int delta = cch * HW + dy * a.W + dx;
#pragma unroll
            for (int j = 0; j < PJ; ++j) {
                const int iy = py[j] + dy, ix = px[j] + dx;
                const bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
                const uint32_t off = ok ? (poff[j] + (uint32_t)delta) * 4u : 0xffffffffu;
                rb[r][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
            }
        }
    };

    auto store_chunk = [&](int buf) __attribute__((always_inline)) {
        float* As = lds + buf * (A_SZ + B_SZ);
        float* Bs = As + A_SZ;
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            int idx = tid + i * NT;
            int row = idx / (MT / 4);
            int c4 = idx - row * (MT / 4);
            *reinterpret_cast<f32x4*>(As + row * MT + c4 * 4) = ra[i];
        }
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
            for (int j = 0; j < PJ; ++j) Bs[(wave * RW + r) * PT + j * 64 + lane] = rb[r][j];
    };

    const int wm0 = (wave & 1) * WM;
    const int wp0 = (wave >> 1) * WP;

    if (c_begin < c_end) {
        load_chunk(c_begin);
        store_chunk(0);
        __syncthreads();
        for (int c = c_begin; c < c_end; ++c) {
            const int buf = (c - c_begin) & 1;
            const bool more = c + 1 < c_end;
            if (more) load_chunk(c + 1);
            const float* As = lds + buf * (A_SZ + B_SZ) + wm0 + l31;
            const float* Bs = lds + buf * (A_SZ + B_SZ) + A_SZ + wp0 + l31;
            // fragments of k-step ks+1 are read while the MFMAs of k-step ks run
            float av[2][TM], bv[2][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) av[0][i] = As[hk * MT + i * 32];
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[0][j] = Bs[hk * PT + j * 32];
#pragma unroll
            for (int ks = 0; ks < KC / 2; ++ks) {
                const int cur = ks & 1, nxt = cur ^ 1;
                if (ks + 1 < KC / 2) {
                    const int kr = 2 * (ks + 1) + hk;
#pragma unroll
                    for (int i = 0; i < TM; ++i) av[nxt][i] = As[kr * MT + i * 32];
#pragma unroll
                    for (int j = 0; j < TN; ++j) bv[nxt][j] = Bs[kr * PT + j * 32];
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur][i], bv[cur][j], acc[i][j], 0, 0, 0);
            }
            if (more) store_chunk(buf ^ 1);
            __syncthreads();
        }
    }

    // ---- epilogue
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int p = p0 + wp0 + j * 32 + l31;
        if (p >= a.npix) continue;
        if (a.splits > 1) {
            float* slab = a.partial + ((size_t)(g * a.splits + split) * a.Mpad) * a.npix + p;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hk;
                    slab[(size_t)m * a.npix] = acc[i][j][r];
                }
            continue;
        }
        const int n = p / HW;
        const int rem = p - n * HW;
        float* ob = G.out + ((size_t)n * G.out_cstride + G.out_coff) * HW + rem;
        float* ob2 = G.out2 ? G.out2 + ((size_t)n * G.out2_cstride + G.out2_coff) * HW + rem : nullptr;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hk;
                if (m < G.cout) {
                    float v = acc[i][j][r] + s_bias[m - m0];
                    if (G.relu) v = fmaxf(v, 0.f);
                    ob[(size_t)m * HW] = v;
                    if (ob2) ob2[(size_t)m * HW] = v;
                }
            }
    }
}

// Deterministic split-K combine: slabs summed in split order, then bias + ReLU.
__global__ __launch_bounds__(256) void conv_splitk_reduce(ConvArgs a) {
    const int g = blockIdx.y;
    const ConvGroup G = g == 0 ? a.g[0] : a.g[1];
    const int HW = a.H * a.W;
    const size_t total = (size_t)G.cout * a.npix;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int m = (int)(e / a.npix);
        const int p = (int)(e - (size_t)m * a.npix);
        const float* s = a.partial + ((size_t)g * a.splits * a.Mpad + m) * a.npix + p;
        float v = s[0];
        for (int k = 1; k < a.splits; ++k) v += s[(size_t)k * a.Mpad * a.npix];
        v += G.bias[m];
        if (G.relu) v = fmaxf(v, 0.f);
        const int n = p / HW;
        const int rem = p - n * HW;
        G.out[((size_t)n * G.out_cstride + G.out_coff + m) * HW + rem] = v;
        if (G.out2) G.out2[((size_t)n * G.out2_cstride + G.out2_coff + m) * HW + rem] = v;
    }
}

// MaxPool2d(2, 2), floor mode (src/model.py:10-13); NCHW, C channels contiguous planes.
__global__ __launch_bounds__(256) void maxpool2x2(const float* __restrict__ in, float* __restrict__ out,
                                                  int NC, int H, int W) {
    const int Ho = H >> 1, Wo = W >> 1;
    const size_t total = (size_t)NC * Ho * Wo;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(e % Wo);
        const size_t t = e / Wo;
        const int y = (int)(t % Ho);
        const size_t nc = t / Ho;
        const float* s = in + (nc * H + 2 * y) * W + 2 * x;
        out[e] = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[W], s[W + 1]));
    }
}

// ------------------------------------------------------------------ host launchers
template <int MT, int PT>
static void launch_tile(const ConvArgs& a, int ngroups, const int* ktab, hipStream_t st) {
    dim3 grid((a.npix + PT - 1) / PT, a.Mpad / MT, ngroups * a.splits);
    hipLaunchKernelGGL((conv_igemm_f32<MT, PT>), grid, dim3(NT), 0, st, a, ktab);
}

void launch_conv(const ConvArgs& a, int ngroups, const int* ktab, int mt, int pt, hipStream_t st) {
    if (mt == 128 && pt == 128) launch_tile<128, 128>(a, ngroups, ktab, st);
    else if (mt == 128 && pt == 64) launch_tile<128, 64>(a, ngroups, ktab, st);
    else if (mt == 64 && pt == 128) launch_tile<64, 128>(a, ngroups, ktab, st);
    else launch_tile<64, 64>(a, ngroups, ktab, st);
    if (a.splits > 1) {
        size_t total = 0;
        for (int g = 0; g < ngroups; ++g) total = total > (size_t)a.g[g].cout * a.npix ? total : (size_t)a.g[g].cout * a.npix;
        int blocks = (int)((total + 255) / 256);
        if (blocks > 2048) blocks = 2048;
        hipLaunchKernelGGL(conv_splitk_reduce, dim3(blocks, ngroups), dim3(256), 0, st, a);
    }
}

void launch_maxpool(const float* in, float* out, int NC, int H, int W, hipStream_t st) {
    size_t total = (size_t)NC * (H / 2) * (W / 2);
    int blocks = (int)((total + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(maxpool2x2, dim3(blocks), dim3(256), 0, st, in, out, NC, H, W);
}

}  // namespace opose
