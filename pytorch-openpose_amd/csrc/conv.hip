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
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int KC = 32;   // k rows per chunk
constexpr int NT = 256;  // threads per workgroup

// TAP: K ordered (tap, channel) with Cin padded to a multiple of KC -> one bounds check per
// pixel per chunk and a wave-uniform channel stride (all layers with Cin >= 32); otherwise K is
// the OIHW flattening decoded through `ktab` (conv1_1: K = 27).
// KS: compile-time kernel size (1, 3, 7) so the tap decode folds; 0 = runtime a.ks.
template <int MT, int PT, bool TAP, int KS>
__global__ __launch_bounds__(NT, 2) void conv_igemm_f32(ConvArgs a, const int* __restrict__ ktab) {
    const int ks = KS ? KS : a.ks;
    constexpr int WM = MT / 2, WP = PT / 2;
    constexpr int TM = WM / 32, TN = WP / 32;
    constexpr int PJ = PT / 64;             // pixel columns per lane
    constexpr int RW = KC / 4;              // k rows gathered per wave per chunk
    constexpr int A_SZ = KC * MT, B_SZ = KC * PT;
    constexpr int A_PW = A_SZ / 256 / 4;    // 1-KiB A pieces per wave per chunk

    // [2 stages][A tile KC x MT | B tile KC x PT] + bias; both tiles are filled by LDS-DMA
    // (buffer/global_load ... lds): no register staging, no ds_write pass.
    __shared__ __attribute__((aligned(16))) float lds[2 * (A_SZ + B_SZ) + MT];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l31 = lane & 31, hk = lane >> 5;

    // XCD-aware tile order (guide T1, bijective form): the dispatcher deals workgroups
    // round-robin over the 8 XCDs, so give XCD x a contiguous run of tiles instead — the
    // M-tiles of one pixel tile and neighbouring pixel tiles (which share im2col halo rows)
    // then share that XCD's L2.  Speed only: any placement is correct.
    const int nM = a.Mpad / MT, nP = (a.npix + PT - 1) / PT;
    const int total = gridDim.x;
    const int b = blockIdx.x;
    const int q = total >> 3, rr = total & 7, xcd = b & 7;
    const int id = xcd * q + min(xcd, rr) + (b >> 3);
    const int mt = id % nM;
    const int rest = id / nM;
    const int pt = rest % nP;
    const int zg = rest / nP;
    const int g = zg / a.splits;
    const int split = zg - g * a.splits;
    const ConvGroup G = g == 0 ? a.g[0] : a.g[1];  // no dynamic kernarg indexing

    const int p0 = pt * PT;
    const int m0 = mt * MT;
    const int HW = a.H * a.W;
    float* s_bias = lds + 2 * (A_SZ + B_SZ);
    if (tid < MT) s_bias[tid] = (m0 + tid < G.cout) ? G.bias[m0 + tid] : 0.f;

    // ---- per-lane pixel state for the im2col gather.  The activation is read through a
    // buffer resource: an invalid (zero-padding) tap gets a byte offset >= num_records, which
    // the hardware range check turns into 0.0f -> the gather is branch free.
    const float* in_base = G.in + (size_t)G.in_coff * HW;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)in_base, (short)0, (int)0x80000000u, 0x00020000);
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

    const uint32_t HW4 = (uint32_t)HW * 4u;
    // per-chunk gather state (computed once per chunk)
    uint32_t base[PJ];
    int ch0 = 0;

    auto chunk_setup = [&](int c) __attribute__((always_inline)) {
        if constexpr (TAP) {
            const int cpt = a.Kpad / (KC * ks * ks);  // chunks per tap (wave-uniform scalars)
            const int tap = c / cpt;
            ch0 = (c - tap * cpt) * KC + wave * RW;
            const int ky = tap / ks;
            const int dy = ky - a.pad, dx = tap - ky * ks - a.pad;
            const int shift = dy * a.W + dx;
#pragma unroll
            for (int j = 0; j < PJ; ++j) {
                const int iy = py[j] + dy, ix = px[j] + dx;
                const bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
                // invalid taps start at 3 GiB: every row offset stays >= 2 GiB = num_records -> 0.0f
                base[j] = ok ? (poff[j] + (uint32_t)shift) * 4u : 0xC0000000u;
            }
        }
    };
    // issue the LDS-DMA of B row r (this wave's) of chunk c into stage `buf`
    auto dma_b_row = [&](int c, int buf, int r) __attribute__((always_inline)) {
        if (a.ablate & 1) return;
        float* Bs = lds + buf * (A_SZ + B_SZ) + A_SZ + (wave * RW + r) * PT;
        if constexpr (TAP) {
            const int ch = min(ch0 + r, a.Cin - 1);  // padded channels: any valid address (weights are 0)
            const uint32_t choff = (uint32_t)ch * HW4;
#pragma unroll
            for (int j = 0; j < PJ; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(Bs + j * 64), 4, base[j] + choff, 0, 0, 0);
        } else {
            const int code = ktab[c * KC + wave * RW + r];  // (c << 8) | (ky << 4) | kx
            const int cch = code >> 8;
            const int dy = ((code >> 4) & 15) - a.pad;
            const int dx = (code & 15) - a.pad;
            const int delta = cch * HW + dy * a.W + dx;
#pragma unroll
            for (int j = 0; j < PJ; ++j) {
                const int iy = py[j] + dy, ix = px[j] + dx;
                const bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
                const uint32_t off = ok ? (poff[j] + (uint32_t)delta) * 4u : 0xC0000000u;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(Bs + j * 64), 4, off, 0, 0, 0);
            }
        }
    };
    auto dma_a = [&](int c, int buf) __attribute__((always_inline)) {
        if (a.ablate & 2) return;
        const int k0 = c * KC;
        float* As = lds + buf * (A_SZ + B_SZ);
#pragma unroll
        for (int i = 0; i < A_PW; ++i) {
            const int piece = wave * A_PW + i;
            const int f = piece * 256 + lane * 4;
            const int row = f / MT, col = f - row * MT;
            __builtin_amdgcn_global_load_lds((const void*)(G.wt + (size_t)(k0 + row) * a.Mpad + m0 + col),
                                             (lds_ptr_t)(As + piece * 256), 16, 0, 0);
        }
    };

    const int wm0 = (wave & 1) * WM;
    const int wp0 = (wave >> 1) * WP;

    if (c_begin < c_end) {
        chunk_setup(c_begin);
        dma_a(c_begin, 0);
#pragma unroll
        for (int r = 0; r < RW; ++r) dma_b_row(c_begin, 0, r);
        __syncthreads();  // s_waitcnt vmcnt(0) + barrier: stage 0 landed for every wave
        for (int c = c_begin; c < c_end; ++c) {
            const int buf = (c - c_begin) & 1;
            const bool more = c + 1 < c_end;
            if (more) {
                chunk_setup(c + 1);
                dma_a(c + 1, buf ^ 1);
            }
            const float* As = lds + buf * (A_SZ + B_SZ) + wm0 + l31;
            const float* Bs = lds + buf * (A_SZ + B_SZ) + A_SZ + wp0 + l31;
            // fragments of k-step ks+1 are read while the MFMAs of k-step ks run; the next
            // chunk's B rows are issued one per k-step, between this chunk's MFMAs
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
                if (ks < RW && more) dma_b_row(c + 1, buf ^ 1, ks);
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur][i], bv[cur][j], acc[i][j], 0, 0, 0);
                if (ks + 1 < KC / 2) {
                    // keep the next step's LDS reads ahead of this step's MFMAs
                    __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
                }
            }
            __syncthreads();  // next stage landed everywhere; this stage free for reuse
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

// fills a buffer with a cheap hash in [-1, 1) (timing runs must not run on zeros: DVFS)
__global__ void fill_hash(float* p, size_t n, uint32_t seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        p[i] = (float)(h & 0xffffff) / 8388608.f - 1.f;
    }
}

void launch_fill_hash(float* p, size_t n, uint32_t seed, hipStream_t st) {
    hipLaunchKernelGGL(fill_hash, dim3(2048), dim3(256), 0, st, p, n, seed);
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
    dim3 grid(((a.npix + PT - 1) / PT) * (a.Mpad / MT) * ngroups * a.splits);
    if (!a.tap_major)
        hipLaunchKernelGGL((conv_igemm_f32<MT, PT, false, 0>), grid, dim3(NT), 0, st, a, ktab);
    else if (a.ks == 7)
        hipLaunchKernelGGL((conv_igemm_f32<MT, PT, true, 7>), grid, dim3(NT), 0, st, a, ktab);
    else if (a.ks == 3)
        hipLaunchKernelGGL((conv_igemm_f32<MT, PT, true, 3>), grid, dim3(NT), 0, st, a, ktab);
    else if (a.ks == 1)
        hipLaunchKernelGGL((conv_igemm_f32<MT, PT, true, 1>), grid, dim3(NT), 0, st, a, ktab);
    else
        hipLaunchKernelGGL((conv_igemm_f32<MT, PT, true, 0>), grid, dim3(NT), 0, st, a, ktab);
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
