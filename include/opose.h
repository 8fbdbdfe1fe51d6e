/*
 * opose.h — C ABI of libopose.so, the MI355X-native OpenPose Body/Hand inference path.
 *
 * Drop-in boundary for hitmaxiang/pytorch-openpose `src/` (pure Python in the reference;
 * these entry points are what a ctypes/cffi binding of that path binds — see INTEGRATION.md):
 *
 *   reference interface (file:line)                         replaced by
 *   ------------------------------------------------------  -----------------------------------
 *   Body.__init__ / Hand.__init__  src/body.py:16-22,        opose_create + opose_load_weights
 *                                  src/hand.py:17-23
 *   util.transfer                  src/util.py:36-40         key mapping done by the caller; tensors
 *                                                            passed in reference state_dict order
 *   bodypose_model.forward         src/model.py:106-133      opose_body_forward
 *   handpose_model.forward         src/model.py:197-214      opose_hand_forward
 *   Body.__call__                  src/body.py:24-212        opose_body_infer
 *   Body.__call__ after the net    src/body.py:52-212        opose_body_post   (parity entry point)
 *   Hand.__call__                  src/hand.py:25-75         opose_hand_infer
 *   Hand.__call__ after the net    src/hand.py:51-75         opose_hand_post   (parity entry point)
 *   one scale of Body.__call__     src/body.py:36-50         opose_body_scale_maps; its output rows
 *                                                            opose_body_band_maps (C5 split)
 *
 * Conventions: plain pointers and sizes only; 0 = OK, negative = error (see opose_status).
 * Host pointers are caller-owned and read-only; the library copies them. A handle owns one
 * device, one HIP stream (or the caller's, see opose_set_stream), its weights and workspace.
 * Calls on one handle must be serialised by the caller; handles are independent.
 */
#ifndef OPOSE_H
#define OPOSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct opose_ctx opose_t;

typedef enum opose_status {
    OPOSE_OK = 0,
    OPOSE_E_ARG = -1,        /* bad argument / null pointer                         */
    OPOSE_E_SHAPE = -2,      /* unsupported shape                                   */
    OPOSE_E_HIP = -3,        /* HIP runtime error (message in opose_last_error)     */
    OPOSE_E_WEIGHTS = -4,    /* weights missing or of the wrong shape               */
    OPOSE_E_CAPACITY = -5,   /* a per-frame record overflowed (peaks/people)        */
    OPOSE_E_ASSEMBLY = -6,   /* reference IndexError: a 3rd subset row matched a
                                connection (src/body.py:170-173)                    */
    OPOSE_E_TIMEOUT = -7,    /* opose_rccl_wait: the halo exchange made no progress
                                before the deadline (communicator aborted)          */
} opose_status;

enum { OPOSE_NET_BODY = 0, OPOSE_NET_HAND = 1 };

/* flags for *_infer / *_post / *_forward */
enum {
    OPOSE_IN_DEVICE = 1,     /* input pointer is device memory                      */
    OPOSE_OUT_DEVICE = 2,    /* output pointer is device memory; call is async on the
                                handle's stream                                     */
    OPOSE_PIPELINE = 4,      /* opose_body_infer with IN_DEVICE | OUT_DEVICE only: the
                                input frames are complete when the call is made (not
                                produced by work still queued on the handle's stream) and
                                stay unmodified until the handle's stream passes the
                                call. The call's network part then runs on a second
                                stream and overlaps the previous call's post-network
                                part; records are still complete in the handle's stream
                                order. Video-batch throughput mode.                 */
    OPOSE_PIPELINE_DEFER = 8,/* with OPOSE_PIPELINE: the call's post-network part is
                                enqueued by the next OPOSE_PIPELINE call once that call's
                                network has reached its trunk's conv3_1 (so it overlaps
                                the middle of the next network, not its first layers),
                                or by opose_flush.  The records are complete in the
                                handle's stream order only after that; the records and
                                frames buffers must stay alive until then.  Every other
                                entry point (and opose_synchronize / opose_signal_stream
                                / opose_set_stream / opose_destroy) flushes first.  */
};

#define OPOSE_MAX_SCALES 8

/* Hard-coded locals of the reference, exposed with the reference defaults
 * (src/body.py:25-31, src/hand.py:26-31). */
typedef struct opose_params {
    int n_scales;
    double scales[OPOSE_MAX_SCALES]; /* scale_search; Body default {0.5}, Hand {0.5,1,1.5,2} */
    double boxsize;                  /* 368  */
    int stride;                      /* 8    */
    int pad_value;                   /* 128  */
    double thre1;                    /* 0.1  body peak threshold                  */
    double thre2;                    /* 0.05 PAF sample threshold                 */
    double thre_hand;                /* 0.03 hand component threshold             */
} opose_params;

void opose_default_params(int net, opose_params* p);

/* ---- lifetime ---------------------------------------------------------------------- */
/* A handle is used by one thread at a time; handles on different threads run concurrently. */
int opose_create(int device, opose_t** out);
void opose_destroy(opose_t* h);
const char* opose_last_error(const opose_t* h);
/* The new stream is ordered after all work queued on the previous one (and on the pipelined
 * network stream). */
int opose_set_stream(opose_t* h, void* hip_stream);   /* NULL = the handle's own stream */
void* opose_get_stream(const opose_t* h);
int opose_synchronize(opose_t* h);
/* Enqueue a post-network part deferred by OPOSE_PIPELINE_DEFER (no-op otherwise): afterwards the
 * last call's records are complete in the handle's stream order. */
int opose_flush(opose_t* h);
/* Ordering against a caller's stream (e.g. the framework's current stream) for OPOSE_IN_DEVICE /
 * OPOSE_OUT_DEVICE calls.  The reference computes synchronously on one device, so these replace
 * the implicit ordering of its `torch.from_numpy(...).cuda()` / `.cpu()` round trips
 * (src/body.py:44-50).
 *   opose_wait_stream:   the handle's next work (either stream) starts after everything queued on
 *                        `hip_stream` so far: device inputs produced there are complete.
 *   opose_signal_stream: work queued on `hip_stream` from now on starts after everything queued
 *                        on the handle's stream so far: device outputs are complete, and buffers
 *                        the handle read can be freed or reused by `hip_stream`. */
int opose_wait_stream(opose_t* h, void* hip_stream);
int opose_signal_stream(opose_t* h, void* hip_stream);
/*   opose_signal_input:  work queued on `hip_stream` from now on starts once the handle has read
 *                        the device inputs of every call made so far, so those buffers may be
 *                        refilled there.  After OPOSE_PIPELINE calls that is the end of the last
 *                        call's network part, before its post-network part: the next frames'
 *                        upload overlaps the post-network kernels instead of waiting for them
 *                        (the reference's per-frame `.cuda()` upload, src/body.py:44-45, in a
 *                        video loop).  Otherwise it is opose_signal_stream. */
int opose_signal_input(opose_t* h, void* hip_stream);

/* Capacity of one Body record: peaks kept per part and people kept per frame.
 * Defaults 96 / 96.  Overflow makes the frame's status OPOSE_E_CAPACITY. */
int opose_set_capacity(opose_t* h, int peaks_per_part, int max_people);

/* Per-frame Body record (fixed size, the unit of the multi-GPU gather):
 *   int32  status, n_cand, n_people, reserved
 *   double candidate[18*peaks_per_part][4]    x, y, score, id  (src/body.py:160,211)
 *   double subset[max_people][20]             ids (-1) | total score | part count */
size_t opose_body_record_bytes(const opose_t* h);

/* ---- weights ------------------------------------------------------------------------ */
/* tensors[i] = host fp32 data of the i-th state_dict tensor in reference order
 * (weight, bias per conv; OIHW); shapes = n x 4 int64 (bias: {C,1,1,1}). */
int opose_load_weights(opose_t* h, int net, const float* const* tensors,
                       const int64_t* shapes, int n);

/* ---- network only (src/model.py forward) ------------------------------------------- */
/* x [N,3,Hp,Wp] fp32 NCHW (Hp, Wp multiples of 8); paf [N,38,Hp/8,Wp/8], heat [N,19,..] */
int opose_body_forward(opose_t* h, const float* x, int N, int Hp, int Wp,
                       float* paf, float* heat, int flags);
/* heat [N,22,Hp/8,Wp/8] */
int opose_hand_forward(opose_t* h, const float* x, int N, int Hp, int Wp, float* heat, int flags);
/* The networks of a scale pyramid in one lockstep pass, as Hand() runs them (src/hand.py:33-57
 * evaluates self.model once per scale_search entry): xs[i] [N[i],3,Hp[i],Wp[i]] -> heats[i]
 * [N[i],22,Hp[i]/8,Wp[i]/8], i < n <= OPOSE_MAX_SCALES; one conv launch per layer covers
 * every scale (split-bf16 path; the fp32 path runs the scales one after another). */
int opose_hand_forward_pyramid(opose_t* h, int n, const float* const* xs, const int* N, const int* Hp,
                               const int* Wp, float* const* heats, int flags);

/* ---- end to end ---------------------------------------------------------------------- */
/* bgr: N frames uint8 [H][W][3] (row stride `row_stride` bytes, frame stride
 * `frame_stride` bytes); records: N * opose_body_record_bytes(). Returns the worst
 * per-frame status (each record carries its own). */
int opose_body_infer(opose_t* h, const uint8_t* bgr, int N, int H, int W,
                     int64_t row_stride, int64_t frame_stride, const opose_params* p,
                     void* records, int flags);

/* Post-network body path on a single scale (what follows src/body.py:50):
 * maps [N,57,h,w] fp32 (channels 0..37 PAF, 38..56 heat), padded net input (h*8, w*8),
 * pad_down / pad_right as util.padRightDownCorner, frame H x W. */
int opose_body_post(opose_t* h, const float* maps, int N, int hl, int wl, int pad_down,
                    int pad_right, int H, int W, const opose_params* p, void* records, int flags);

/* ---- scale-sharded single-frame latency (one scale of src/body.py:34-50 per rank) ------- */
/* Geometry of scale s of p->scales for an H x W frame (src/body.py:35-41): out4 = {hl, wl,
 * pad_down, pad_right} = network output size and util.padRightDownCorner's pads. */
int opose_body_scale_geom(int H, int W, const opose_params* p, int s, int* out4);

/* Network maps of scale s only (src/body.py:36-50 for one m): maps [N,57,hl,wl] fp32
 * (channels 0..37 PAF, 38..56 heat), host memory unless OPOSE_OUT_DEVICE. */
int opose_body_scale_maps(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride,
                          int64_t frame_stride, const opose_params* p, int s, float* maps, int flags);

/* Row band [r0, r1) of scale s's network maps for ONE frame, for splitting a large scale across
 * ranks (736x1312 is 53 % of the pyramid's FLOPs; src/body.py:36-50 for one
 * m, cut into output rows).  Every rank of a band group runs the VGG trunk on its band's rows
 * plus a 10-row margin past each cut (recomputed, not exchanged), then the six CPM stages
 * (src/model.py:106-133) on its own rows only.  Before each 3x3 / 7x7 stage layer that needs
 * them, the 3 rows on either side of the band are exchanged with the neighbouring bands: the
 * library packs its top and bottom 3 rows
 * into xbuf's send halves on its stream, calls fn(user, bytes, stream), and unpacks the recv
 * halves.  fn moves send_up to the band above (its recv_dn) and send_dn to the band below (its
 * recv_up), ordered on `stream` (a hipStream_t) or synchronously, and returns 0; it is called
 * 27 times per frame and never for a single band covering every row (fn == NULL: see below).
 *   xbuf: device memory, 4 x opose_body_band_halo_bytes(wl) bytes = [send_up | send_dn |
 *         recv_up | recv_dn];  r1 - r0 >= 3;  maps [57, r1-r0, wl] fp32 (host unless
 *         OPOSE_OUT_DEVICE);  bgr one H x W frame (device with OPOSE_IN_DEVICE).
 * Every conv sums each pixel in the order the whole frame's network does (k slabs fixed by the
 * layer and the frame), so concatenating every band's maps gives
 * opose_body_scale_maps(s) bit for bit. */
typedef int (*opose_halo_fn)(void* user, size_t bytes, void* stream);
/* fn == NULL: the library exchanges the halos itself, RCCL send/recv on the handle's stream with
 * the ranks set by opose_set_band_peers, over the communicator of opose_rccl_init (no host code
 * between the stage layers). */
int opose_rccl_unique_id(void* id, size_t len);  /* len >= 128; call on one rank, share the bytes */
int opose_rccl_init(opose_t* h, const void* id, int rank, int nranks);
/* A band rank failed: ncclCommAbort on the handle's communicator (this rank's own queued halo
 * send / recv exit) and drop it; opose_rccl_init builds a new one.  The abort does not reach the
 * neighbours' queued kernels: they bound their wait with opose_rccl_wait. */
int opose_rccl_abort(opose_t* h);
/* Wait for the handle's stream (where the RCCL halo send / recv of opose_body_band_maps run) with a
 * deadline.  Returns OPOSE_OK when the work completed.  If the communicator reports an
 * asynchronous error, or the stream is still busy after timeout_ms (a band neighbour failed and
 * will never post its side of an exchange), the handle's own communicator is aborted: RCCL's abort
 * flag makes this rank's queued send / recv kernels exit, so the stream drains instead of waiting
 * forever; returns OPOSE_E_HIP / OPOSE_E_TIMEOUT, and opose_rccl_init builds a new communicator.
 * A failing rank's ncclCommAbort cannot reach its neighbours' queued kernels (xGMI P2P has no
 * peer-failure signal), so each neighbour bounds its own wait with this call (src/dist.py). */
int opose_rccl_wait(opose_t* h, int timeout_ms);
int opose_set_band_peers(opose_t* h, int up, int dn);  /* communicator ranks; -1: none */
size_t opose_body_band_halo_bytes(int wl);
int opose_body_band_maps(opose_t* h, const uint8_t* bgr, int H, int W, int64_t row_stride,
                         const opose_params* p, int s, int r0, int r1, float* maps,
                         opose_halo_fn fn, void* user, void* xbuf, size_t xbuf_bytes, int flags);

/* Multi-scale post-network body path (src/body.py:51-203): maps[s] = [N,57,hl[s],wl[s]] of
 * every scale (any rank's output of opose_body_scale_maps, gathered); the per-scale x8 /
 * crop / resize, the float64 scale average and everything after it, as opose_body_infer. */
int opose_body_post_scales(opose_t* h, const float* const* maps, const int* hl, const int* wl,
                           const int* pad_down, const int* pad_right, int n_scales, int N, int H,
                           int W, const opose_params* p, void* records, int flags);

/* Batched "fast mode" of the reference (srcmx/Batch_model.py:137-204 Batch_body.__call__):
 * torch-bicubic pre/post-processing (inputs as transforms.ToTensor would give: uint8 / 255),
 * single scale p->scales[0] (Batch_body: 0.5), 5x5 Gaussian + peak scores from the blurred
 * heat map, then the same limb scoring / matching / assembly as Body.  Records as
 * opose_body_infer. */
int opose_batch_body_infer(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride,
                           int64_t frame_stride, const opose_params* p, void* records, int flags);

/* Post-network part of the fast mode (srcmx/Batch_model.py:159-204): maps = [N,57,hl,wl]
 * (PAF 38 | heat 19), nh x nw = int(H*s) x int(W*s) = the crop of the x8 maps, frame H x W. */
int opose_batch_body_post(opose_t* h, const float* maps, int N, int hl, int wl, int nh, int nw,
                          int H, int W, const opose_params* p, void* records, int flags);

/* Fast-mode hand (srcmx/Batch_model.py:310-354 Batch_hand.__call__): N crops already resized
 * to H x W (the data loader's boxsize, a multiple of 8) as uint8 BGR; network at scale 1,
 * torch bicubic x8, 5x5 Gaussian, components of blurred > p->thre_hand (Batch_hand: 0.035)
 * selected on the blurred map.  peaks [N][21][3] in the H x W frame, found [N][21]. */
int opose_batch_hand_infer(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride,
                           int64_t frame_stride, const opose_params* p, double* peaks, int32_t* found,
                           int flags);

/* Post-network part of the fast-mode hand (srcmx/Batch_model.py:334-354): maps = [N,22,hl,wl]
 * network outputs; peaks in the (8 hl) x (8 wl) frame. */
int opose_batch_hand_post(opose_t* h, const float* maps, int N, int hl, int wl, const opose_params* p,
                          double* peaks, int32_t* found, int flags);

/* Hand on N crops uint8 [H][W][3] (util.handDetect gives squares): peaks [N][21][3]
 * (x, y, score), found [N][21] (0 = part missing, the reference's [0,0,0] row). */
int opose_hand_infer(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride,
                     int64_t frame_stride, const opose_params* p, double* peaks,
                     int32_t* found, int flags);

/* Hand on n square crops of different sizes (the hands util.handDetect finds in a batch of
 * frames): crops[i] = uint8 [sizes[i]][sizes[i]][3] with row stride row_strides[i].  Every
 * crop maps to the same network input per scale (scale * boxsize), so the network runs once
 * per scale for all crops; resize-back and component selection run per crop.  peaks [n][21][3],
 * found [n][21]; same per-crop results as opose_hand_infer up to fp32 network noise.
 * Replaces a loop of Hand.__call__ over crops (srcmx/MotionEstimation.py:186-201). */
int opose_hand_infer_crops(opose_t* h, const uint8_t* const* crops, const int* sizes,
                           const int64_t* row_strides, int n, const opose_params* p,
                           double* peaks, int32_t* found, int flags);

/* Post-network hand path: maps[s] = [N,22,hl[s],wl[s]] per scale s (pads per scale),
 * crop H x W. */
int opose_hand_post(opose_t* h, const float* const* maps, const int* hl, const int* wl,
                    const int* pad_down, const int* pad_right, int n_scales, int N, int H, int W,
                    const opose_params* p, double* peaks, int32_t* found, int flags);

/* ---- measurement ---------------------------------------------------------------------- */
/* When enabled, every kernel launch is bracketed by HIP events on the stream it runs on and
 * accumulated per kernel class.  enable: 0 off, 1 per class, 2 per class and per layer,
 * 3 the 7x7 conv class only (the dominant kernel: bench.py's live roofline at ~1/4 of the
 * event overhead).  opose_profile_read writes one JSON object. */
int opose_profile_enable(opose_t* h, int enable);
int opose_profile_reset(opose_t* h);
int opose_profile_read(opose_t* h, char* buf, size_t len);

/* ---- test hooks (parity tests call single stages; host pointers, synchronous) ----- */
/* one stride-1 conv: x [N,Cin,H,W], w [Cout,Cin,ks,ks], b [Cout] -> out [N,Cout,H,W];
 * mt/pt <= 0 select the production tile heuristic; splits > 0 forces that many stream-K
 * workgroups (== number of tiles: plain data-parallel grid) */
int opose_debug_conv(opose_t* h, const float* x, const float* w, const float* b, int N, int Cin, int H, int W,
                     int Cout, int ks, int pad, int relu, int mt, int pt, int splits, float* out);
/* mean time (ms) of one conv launch (ngroups GEMM groups) on hashed data over `reps`
 * launches; ablate bit 1 skips the im2col gather, bit 2 the weight load (timing only) */
int opose_debug_conv_time(opose_t* h, int N, int Cin, int H, int W, int Cout, int ks, int ngroups,
                          int mt, int pt, int splits, int ablate, int reps, float* ms);
/* The split-bf16 ("x6") conv kernel on one layer: x fp32 NCHW is split into three bf16 pieces,
 * convolved with six bf16 MFMA piece products per fp32 product, written fp32 (out_x6 = 0) or
 * split and rebuilt (out_x6 = 1). */
int opose_debug_conv_x6(opose_t* h, const float* x, const float* w, const float* b, int N, int Cin, int H,
                        int W, int Cout, int ks, int pad, int relu, int mt, int pt, int splits, int out_x6,
                        float* out);
int opose_debug_conv_x6_time(opose_t* h, int N, int Cin, int H, int W, int Cout, int ks, int ngroups,
                             int mt, int pt, int splits, int reps, float* ms);
/* src/body.py:38-41 for one frame and one scale: out [3,Hp,Wp]; HpWp receives (Hp, Wp)
 * (out may be NULL to query the size) */
int opose_debug_preprocess(opose_t* h, const uint8_t* bgr, int H, int W, double scale, int pad_value,
                           float* out, int* HpWp);
/* src/body.py:54-57,67 for one frame: maps [57,hl,wl] -> heat_avg [18,H,W] float64 and
 * (optional) the x8-upsampled, cropped PAF maps [38,Hs,Ws] float32 */
int opose_debug_heat(opose_t* h, const float* maps, int hl, int wl, int pad_down, int pad_right, int H, int W,
                     double* heat_avg, float* paf_mid);
/* src/hand.py:62-64 on NP float64 maps [NP,H,W]: binary = gaussian_filter(map, 3) > thre, then
 * label(binary, connectivity 2) -> labels [NP,H,W] int32: -1 off the binary map, else the
 * linear index (y * W + x) of the component's first pixel in raster order -- scipy.ndimage.label's
 * numbering order -- and sums [NP,H,W] float64: at a component's first pixel, the sum of the
 * map over the component (elsewhere undefined) */
int opose_debug_hand_label(opose_t* h, const double* maps, int NP, int H, int W, double thre, int32_t* labels,
                           double* sums);

#ifdef __cplusplus
}
#endif
#endif /* OPOSE_H */
