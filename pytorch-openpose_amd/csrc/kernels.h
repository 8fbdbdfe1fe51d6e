// kernels.h — host-side launchers for the libopose kernels.
#pragma once
#include <vector>

#include "common.h"

namespace opose {

constexpr int kMaxScales = 8;

// PAF maps of every scale for on-demand evaluation at paf_score's sample points: either the x8
// map mid[s] ([N][cm][hs][ws], channel 0 = PAF x) or, when low[s] is set, the network's low-res
// PAF channels ([N][lcm][hl][wl]), whose x8 values are evaluated where the final resize reads them
// (cv2.resize(fx=fy=8) then the resize to H x W, src/body.py:55-63: the same float32 expressions in
// the same order as the staged upsample, so the same values)
struct PafScales {
    const float* mid[kMaxScales];  // [N][cm][hs][ws] per scale
    const float* low[kMaxScales];  // [N][lcm][hl][wl] per scale, or nullptr
    int hs[kMaxScales], ws[kMaxScales];
    int hl[kMaxScales], wl[kMaxScales];
    double sy[kMaxScales], sx[kMaxScales];  // source step of the final resize to H x W
    int n, cm, lcm, H, W;
    int torch;  // 1: torch bicubic taps (Batch_body fast mode), 0: OpenCV INTER_CUBIC
};

struct Conn {
    int i, j;
    double s;
};

// conv.hip
void launch_conv(const ConvArgs& a, const int* ktab, int mt, int pt, hipStream_t st);
void launch_fill_hash(float* p, size_t n, uint32_t seed, hipStream_t st);
void launch_maxpool(const float* in, float* out, int NC, int H, int W, hipStream_t st);

// conv_x6.hip (split-bf16 fp32-accurate convolution, X6 activation format: common.h)
void x6_pack_weights(const float* w, int cout, int cin, int ks, int Mpad, int* nK_out, std::vector<uint16_t>& out);
void launch_conv_x6(const X6Args& a, int mt, int pt, hipStream_t st);
// X6Args with the groups' tiles and work units numbered for an mt x pt tile (X6Group::t0 / u0,
// X6Args::tiles / units)
X6Args x6_number_tiles(const X6Args& a, int mt, int pt);
// slab fixup of a 128 x 256 tile grid (conv_win_x6)
void launch_conv_x6_fixup(const X6Args& a, int mt, int pt, hipStream_t st);
void launch_to_x6(const float* in, int cstride, int coff, int C, int N, int HW, uint8_t* out, int cg, int goff,
                  uint32_t ps, hipStream_t st);
void launch_from_x6(const uint8_t* in, int cg, int goff, uint32_t ps, int C, int N, int HW, float* out, int cstride,
                    int coff, hipStream_t st);
// f32_out: fp32 units of 8 channels ([N][8][H*W] x 32 bytes) for launch_conv3_pool_win_x6's f32_in
// conv1_1 / conv1_2 of a pyramid's scales in one launch each: one segment per scale (input,
// output, piece strides, geometry); b0 is set by the launcher
constexpr int kConv1Segs = 8;
struct Conv1Seg {
    const void* in;
    uint8_t* out;
    uint32_t ips, ops;
    int N, H, W, b0;
};
struct Conv1Segs {
    Conv1Seg s[kConv1Segs];
    int n;
};
void launch_conv_first_x6_segs(Conv1Segs segs, const float* wt, int Mpad, const float* bias, bool f32_out,
                               hipStream_t st);
void launch_conv3_pool_win_x6_segs(Conv1Segs segs, const uint8_t* wt, const float* bias, bool f32_in, hipStream_t st);
void launch_conv_first_x6(const float* x, int N, int Cin, int H, int W, const float* wt, int Mpad, const float* bias,
                          uint8_t* out, uint32_t ops, bool f32_out, hipStream_t st);
// zero the padding units of `planes` X6P (piece, group) planes of an N x H x W buffer (common.h)
void launch_x6p_clear_pads(uint8_t* const* bufs, const int* planes, int nbufs, int N, int H, int W, hipStream_t st);
// 3 rows (padded row index row0 / row1) of groups [g0, g0 + ng) of a one-frame X6P buffer (ps
// bytes per piece, gs units per group plane, P units per row) <-> packed blocks blk0 / blk1
// ([piece][group][3 P] units); directions by mask bit 0 / 1
void launch_x6p_halo(uint8_t* x6p, uint32_t ps, uint32_t gs, int g0, int ng, int P, int row0, int row1, void* blk0,
                     void* blk1, int mask, bool unpack, hipStream_t st);
void launch_maxpool_x6(const uint8_t* in, uint32_t ips, uint8_t* out, uint32_t ops, int NG, int H, int W,
                       hipStream_t st);
// conv1_2 (64 -> 64, 3x3 pad 1) + MaxPool2d(2, 2) from an 8-group X6 tensor (f32_in: fp32 units,
// split in the kernel), input window in LDS
void launch_conv3_pool_win_x6(const uint8_t* in, uint32_t ips, int N, int H, int W, const uint8_t* wt,
                              const float* bias, uint8_t* out, uint32_t ops, bool f32_in, hipStream_t st);
// conv1x1_chain.hip: two chained 1x1 convs (CPM stage ends) in one launch, 64-pixel tiles
void launch_conv1x1_chain_x6(const X6ChainArgs& a, hipStream_t st);
// conv_win.hip: the 7x7 / 3x3 convs with the im2col operand from an LDS window of the padded X6P
// input (pair-order weights: x6_pack_weights_pairs); 128 x 256 tiles, work units (tile, k slab)
void x6_pack_weights_pairs(const float* w, int cout, int cin, int ks, int Mpad, int* nK_out,
                           std::vector<uint16_t>& out);
// the windows of an N x H x W batch's tiles fit the LDS
bool conv_win_fits(int N, int H, int W, int ks);
// the window of any 256-pixel run of one frame W columns wide fits the LDS (whatever the height)
bool conv_win_fits_rows(int W, int ks);
void launch_conv_win_x6(const X6Args& a, hipStream_t st);
// Winograd F(2,3) along x for 3x3 layers on X6P inputs (conv_wino.hip): weights U_v in pair order,
// tile slots per frame of a batch (-1: the window does not fit), whole-tile launch
void x6_pack_weights_wino(const float* w, int cout, int cin, int Mpad, int* nK_out, std::vector<uint16_t>& out);
int wino_tpf(int N, int H, int W);
void launch_conv_wino_x6(const X6Args& a, hipStream_t st);
// imgproc.hip
void launch_preprocess(const uint8_t* src, int64_t frame_stride, int64_t row_stride, int N, int H, int W, int Hs,
                       int Ws, double sy, double sx, int Hp, int Wp, float pad_val, float* out, hipStream_t st);
void launch_upsample8(const float* in, int in_cstride, int in_coff, int C, int N, int hl, int wl, int Hs, int Ws,
                      float* out, hipStream_t st);
void launch_heat_full(const float* mid, int Cm, int coff, int P, int N, int Hs, int Ws, int H, int W, double sy,
                      double sx, int nscales, int accumulate, double* avg, hipStream_t st);
// every scale of a pyramid's heat average in one launch (imgproc.hip heat_full_scales)
constexpr int kHeatScales = 8;
struct HeatScale {
    const float* mid;  // [N][Cm][Hs][Ws] x8 maps of this scale
    int Cm, coff, Hs, Ws;
    double sy, sx;
};
struct HeatScales {
    HeatScale s[kHeatScales];
    int n;
    float ns;  // len(multiplier): every scale's map is divided by it (float32) before the float64 add
};
bool heat_full_scales_fits(const HeatScales& S, int H, int W);
void launch_heat_full_scales(const HeatScales& S, int N, int P, int H, int W, double* avg, hipStream_t st);
void launch_heat_full_f32(const float* mid, int Cm, int coff, int P, int N, int Hs, int Ws, int H, int W, double sy,
                          double sx, float* avg, hipStream_t st);

// Batch_body fast mode (torch bicubic conventions)
void launch_preprocess_torch(const uint8_t* src, int64_t frame_stride, int64_t row_stride, int N, int H, int W, int nh,
                             int nw, float scale_y, float scale_x, int Hp, int Wp, float* out, hipStream_t st);
void launch_upsample8_torch(const float* in, int in_cstride, int in_coff, int C, int N, int hl, int wl, int nh, int nw,
                            float* out, hipStream_t st);
void launch_resize_torch_f32(const float* mid, int Cm, int coff, int P, int N, int nh, int nw, int H, int W,
                             float* out, hipStream_t st);

// post.hip
void launch_gauss_nms(const void* avg, bool f32, int NP, int H, int W, double thre, int cap, int* cnt, int* list,
                      double* list_score, hipStream_t st);
// single scale: heat_full's resize of mid channels [coff, coff+P) fused into the wide NMS
// (requires gauss_nms_resize_fits: a true resize with source step sy <= 0.618)
bool gauss_nms_resize_fits(int Hs, int Ws, int H, int W, double sy);
void launch_gauss_nms_resize(const float* mid, int Cm, int coff, int P, int N, int Hs, int Ws, int H, int W, double sy,
                             double sx, double thre, int cap, int* cnt, int* list, double* list_score,
                             hipStream_t st);
// Batch_body fast mode: 5x5 Gaussian (reflect pad, srcmx/utilmx.py:246-263) + findpeaks_torch
// (srcmx/utilmx.py:230-243) on heat [NP][H][W] float; scores = blurred values
void launch_blur5_nms(const float* heat, int NP, int H, int W, double thre, int cap, int* cnt, int* list,
                      double* list_score, hipStream_t st);
// Batch_hand fast mode: blurred (5x5, float64 out) + union-find seeds of blurred > thre
void launch_blur5_seed(const float* heat, int NP, int H, int W, double thre, double* blurred, int* lab, int* cnt,
                       hipStream_t st);
// sums: zeroed at every tile-local root (the component sums' only addresses; launch_hand_cc)
void launch_gauss_threshold(const double* avg, int NP, int H, int W, double thre, int* lab, int* cnt, double* sums,
                            hipStream_t st);
void gauss_threshold_tiles(int H, int W, int* ntx, int* nty);
void launch_peaks_finalize(const int* cnt, const int* list, const double* list_score, int N, int H, int W,
                           const RecordLayout& L, uint8_t* records, int* peak_pos, int* part_cnt, hipStream_t st);
void launch_paf_score(const PafScales& S, const int* peak_pos, const int* part_cnt, int N, int cap, double thre2,
                      double* score, hipStream_t st);
void launch_limb_greedy(const double* score, const int* part_cnt, int N, int cap, Conn* conn, int* conn_cnt,
                        hipStream_t st);
void launch_assemble(const Conn* conn, const int* conn_cnt, const int* part_cnt, int N, const RecordLayout& L,
                     uint8_t* records, hipStream_t st);

// hand.hip
size_t hand_cc_workspace_bytes(int NP);
// tile_seeds: lab labelled per gauss_threshold tile (only tile edges left to join); else run seeds
// (blur5_seed)
void launch_hand_cc(double* avg, int NP, int H, int W, int* lab, double* sums, const int* cnt, double* peaks,
                    int* found, void* ws, bool tile_seeds, hipStream_t st);

}  // namespace opose
