// common.h — shared host/device definitions for libopose (MI355X / gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

namespace opose {

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define OPOSE_HIP_CHECK(expr)                                                               \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            throw ::opose::HipError(std::string(#expr) + ": " + hipGetErrorString(_e) +     \
                                    " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")"); \
    } while (0)

// ---------------------------------------------------------------- convolution
// One "group" = one independent conv sharing the launch's shape (two CPM branches).
struct ConvGroup {
    const float* in;   // NCHW buffer; channels [in_coff, in_coff + Cin) of in_cstride
    const float* wt;   // [Kpad][Mpad] transposed, zero padded weights
    const float* bias; // [cout]
    float* out;        // NCHW buffer; channels [out_coff, out_coff + cout) of out_cstride
    float* out2;       // optional duplicate destination (nullptr = none)
    int in_cstride, in_coff;
    int out_cstride, out_coff;
    int out2_cstride, out2_coff;
    int cout;
    int relu;
};

struct ConvArgs {
    ConvGroup g[2];
    int N, H, W;        // batch and spatial size (stride-1 'same' conv)
    int Cin, ks, pad;   // input channels, kernel size, padding
    int K, Kpad, Mpad;  // K = Cin*ks*ks
    int npix;           // N*H*W
    int tap_major;      // K ordered (tap, channel) with Cin padded to 32 (else OIHW + ktab)
    int ngroups;        // 1 or 2 GEMM groups sharing the launch
    int sk_grid;        // stream-K workgroups (== tiles: plain data-parallel grid)
    float* partial;     // stream-K partial slabs [2 * sk_grid][MT * PT] (summed by conv_sk_fixup)
};

// ---------------------------------------------------------------- split-bf16 ("x6") convolution
// Activation format X6: every fp32 value x is stored as three bfloat16 pieces x0 + x1 + x2 == x
// (exact: round-to-nearest bf16 of x, of the remainder, of the remainder's remainder -> 24
// significant bits = the whole fp32 significand).  8 channels of a pixel form one 16-byte unit;
// the three piece planes follow each other at `ps` bytes.  Within a plane a unit is addressed by
// an X6Layout: unit(n, g, y, x) = o0 + n * fs + g * gs + y * rs + x (g = group relative to the
// slice, o0 includes the slice's first group).  Two layouts are used:
//  * dense  [N][Cg][H*W]:  fs = Cg*H*W, gs = H*W, rs = W, o0 = goff*H*W (trunk activations);
//  * padded (X6P, the low-resolution CPM stage buffers): per group one tall image of the N
//    frames stacked with 3 zero rows above, between and below them and kX6PPad zero units
//    between consecutive rows (row pitch P = W + kX6PPad, pixel (n, y, x) at row 3 + n*(H+3) + y,
//    column 3 + x: the 3 zero units before a row's pixels also pad the previous row), plus one zero row
//    at the end: every tap of a 7x7 / 3x3 / 1x1 'same' conv is a constant shift dy*P + dx of the
//    pixel's unit, and the window of a run of consecutive pixels is contiguous across rows and
//    frames (conv_win_x6).  fs = (H+3)*P, gs = (N*(H+3)+4)*P, rs = P, o0 = goff*gs + 3*P + 3.  The
//    zero units are never written.
struct X6Layout {
    uint32_t fs, gs, rs, o0;
};

// Zero units per X6P row: 3 (the 7x7 taps' reach).  16 (P - W a multiple of 16 units, so a B
// fragment's 16 pixels stay on 16 distinct LDS bank slots across a row end) cut the modelled
// bank-conflict cycles of the window kernel's B reads from 51 % to 18.5 % but made every window
// 30 % longer: the bench's 7x7 launch 0.365 -> 0.376 ms, same box.
constexpr int kX6PPad = 3;
__host__ __device__ inline int x6p_pitch(int W) { return W + kX6PPad; }

struct X6Group {
    const uint8_t* in;     // X6 buffer (plane 0)
    const uint8_t* wt;     // [nK][3 pieces][4 groups][Mpad] units of 8 bf16
    const float* bias;     // [cout]
    void* out;             // X6 buffer, or fp32 NCHW when out_f32
    void* out2;            // optional duplicate destination, X6 (nullptr = none)
    uint32_t in_ps, out_ps, out2_ps;  // piece strides (bytes) of the X6 buffers
    X6Layout in_l, out_l, out2_l;     // unit addressing of the X6 slices
    int out_c, out_off;    // fp32 output: channels per frame / first channel
    int cout, relu, out_f32;
    int N, H, W;           // this group's frames (stride-1 'same' conv; pooled: the input's H, W)
    int npix;              // GEMM columns: N*H*W (pooled: N*(H/2)*(W/2)*4, quad-major)
    int ylo, yhi;          // conv_x6 taps read rows [ylo, yhi) (yhi == 0: [0, H)); a row band's
                           // view (engine.cpp Band) also reads its halo rows
    // k slabs: every tile of this group sums its nK chunks as `slabs` fixed ranges [s nK / slabs,
    // (s + 1) nK / slabs), each accumulated from zero, folded in slab order by conv_x6_fixup
    // (slabs == 1: one run over all chunks, written by the conv itself).  The count is a function
    // of the layer and the segment's logical geometry only (engine.cpp slab_count), never of the
    // launch's grid, groups or row band: a pixel sums in the same order whatever launch computes it.
    int slabs;
    int tpf;               // conv_wino_x6: tile slots per frame (frame-aligned blocks of 128), 0: tiles
                           // numbered across frames (set by the launcher; npix = tile slots)
    int t0;                // first tile of the group in the launch's tile space (set by the launcher)
    int u0;                // first work unit (tile, slab) of the group (set by the launcher)
};

// One launch runs up to kX6Groups GEMMs of the same conv shape (ks, Cin, Mpad): the two CPM
// branches of a stage, and the scales of a pyramid (Hand()'s four, C5's) -- a "segment" per
// (scale, branch), each with its own geometry and buffers.  Tiles are numbered group after
// group (t0), so one data-parallel or stream-K grid covers all of them.
constexpr int kX6Groups = 8;

struct X6Args {
    X6Group g[kX6Groups];
    int ks, pad;
    int cin_g;      // channel groups of the conv's input (Cin padded to 8)
    int small;      // 1: one group (Cin <= 8), chunks of 4 taps; 0: chunks of (4 groups, 1 tap)
    int nK;         // chunks of 32 k
    int Mpad, ngroups;
    int sk_grid;    // workgroups
    int tiles;      // tiles of all groups (set by the launcher)
    int units;      // work units (tile, slab) of all groups (set by the launcher)
    // unit lists: sched[w] .. sched[w + 1] index sched[sk_grid + 1 + i], the units workgroup w runs
    // (the host's longest-first schedule); nullptr: workgroup w runs units [w U / G, (w + 1) U / G)
    const int* sched;
    float* partial; // slab partials [units][MT * PT] (groups with slabs > 1)
    int pool;       // 1: 2x2/2 max-pool fused into the epilogue (npix = N * (H/2) * (W/2) * 4, quad-major)
};

// Two chained 1x1 convs (conv1x1_chain.hip): Y = W2 relu(W1 X + b1) + b2 per group (a CPM
// branch of a scale); X: cin_g * 8 channels, W1: m1 rows, Y: cout2 <= 64 channels
struct X6ChainGroup {
    const uint8_t* in;           // X6 input (plane 0)
    const uint8_t* w1;           // [cin_g/4][3][4][m1] units (x6_pack_weights)
    const float* b1;             // [m1]
    const uint8_t* w2;           // [m1/32][3][4][64] units
    const float* b2;             // [cout2]
    void* out;                   // X6 slice, or fp32 NCHW when out_f32
    uint32_t in_ps, out_ps;
    X6Layout in_l, out_l;
    int out_c, out_off, out_f32;
    int cout2, relu2;
    int N, H, W, npix, t0;       // geometry; first tile (set by the launcher)
};

struct X6ChainArgs {
    X6ChainGroup g[kX6Groups];
    int cin_g, m1, ngroups, tiles;
};

// ---------------------------------------------------------------- body records
struct RecordLayout {
    int peaks_per_part;  // capacity per part
    int max_people;      // subset rows
    size_t cand_off, subset_off, bytes;
    __host__ __device__ int cand_cap() const { return 18 * peaks_per_part; }
};

inline RecordLayout make_record_layout(int ppp, int maxp) {
    RecordLayout r;
    r.peaks_per_part = ppp;
    r.max_people = maxp;
    r.cand_off = 16;
    r.subset_off = r.cand_off + sizeof(double) * 4 * (size_t)r.cand_cap();
    r.bytes = r.subset_off + sizeof(double) * 20 * (size_t)maxp;
    return r;
}

// cubic-resize descriptor (OpenCV INTER_CUBIC, see imgproc.hip)
struct ResizeAxis {
    int src, dst;     // sizes
    double scale;     // source step per destination pixel (1/inv_scale)
};

}  // namespace opose
