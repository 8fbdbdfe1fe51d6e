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
    float* partial;     // stream-K partial slabs [2 * sk_grid][MT * PT]
    int* sk_cnt;        // per-tile arrival counters (zero between launches) -> the last
                        // workgroup of a split tile reduces it; nullptr: conv_sk_fixup launch
};

// ---------------------------------------------------------------- split-bf16 ("x6") convolution
// Activation format X6: every fp32 value x is stored as three bfloat16 pieces x0 + x1 + x2 == x
// (exact: round-to-nearest bf16 of x, of the remainder, of the remainder's remainder -> 24
// significant bits = the whole fp32 significand).  Layout per piece plane: [N][Cg][H*W][8]
// (8 channels of a pixel contiguous = one 16-byte unit); the three planes follow each other
// at `ps` bytes.  Channel offsets / strides are in groups of 8 channels.
struct X6Group {
    const uint8_t* in;     // X6 buffer (plane 0, frame 0, group 0)
    const uint8_t* wt;     // [nK][3 pieces][4 groups][Mpad] units of 8 bf16
    const float* bias;     // [cout]
    void* out;             // X6 buffer, or fp32 NCHW when out_f32
    void* out2;            // optional duplicate destination, same format (nullptr = none)
    uint32_t in_ps, out_ps, out2_ps;  // piece strides (bytes) of the X6 buffers
    int in_cg, in_goff;    // groups per frame of the input buffer / first group read
    int out_c, out_off;    // X6: groups per frame / first group; fp32: channels / first channel
    int out2_c, out2_off;
    int cout, relu, out_f32;
};

struct X6Args {
    X6Group g[2];
    int N, H, W, ks, pad;
    int cin_g;      // channel groups of the conv's input (Cin padded to 8)
    int small;      // 1: one group (Cin <= 8), chunks of 4 taps; 0: chunks of (4 groups, 1 tap)
    int nK;         // chunks of 32 k
    int Mpad, npix, ngroups, sk_grid;
    float* partial; // stream-K partial slabs [2 * sk_grid][MT * PT]
    int ablate;     // timing ablations (0 in production): 1 no im2col DMA, 2 no weight DMA, 4 no barrier, 8 no LDS reads
    int pool;       // 1: 2x2/2 max-pool fused into the epilogue (npix = N * (H/2) * (W/2) * 4, quad-major)
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
