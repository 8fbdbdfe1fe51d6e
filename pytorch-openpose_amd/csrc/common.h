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
