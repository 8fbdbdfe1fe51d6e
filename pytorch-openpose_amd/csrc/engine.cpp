// engine.cpp — libopose host runtime: weights, network plans, workspace, C ABI.
//
// Mirrors hitmaxiang/pytorch-openpose:
//  * topology + state_dict order      src/model.py:25-104 (body), :136-195 (hand)
//  * Body.__call__ orchestration      src/body.py:24-212
//  * Hand.__call__ orchestration      src/hand.py:25-75
// The network runs as one launch per layer of the split-bf16 implicit-GEMM kernels (conv_win.hip,
// conv_x6.hip, conv1x1_chain.hip; conv.hip is the fp32 alternative): the two CPM branches of a
// stage and the scales of a pyramid share a launch as groups, each conv sums a pixel in an order
// fixed by its layer (k slabs, slab_count); stage concatenation is implicit (channel-slice writes).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <map>
#include <mutex>
#include <memory>
#include <string>
#include <thread>
#include <queue>
#include <vector>

#include "../../include/opose.h"
#include "common.h"
#include "kernels.h"

using namespace opose;

namespace {

struct Spec {
    std::string name;
    int cin, cout, ks, pad;
};

// ---------------------------------------------------------------- topology (src/model.py)
std::vector<Spec> vgg_body() {
    return {{"conv1_1", 3, 64, 3, 1},     {"conv1_2", 64, 64, 3, 1},     {"conv2_1", 64, 128, 3, 1},
            {"conv2_2", 128, 128, 3, 1},  {"conv3_1", 128, 256, 3, 1},   {"conv3_2", 256, 256, 3, 1},
            {"conv3_3", 256, 256, 3, 1},  {"conv3_4", 256, 256, 3, 1},   {"conv4_1", 256, 512, 3, 1},
            {"conv4_2", 512, 512, 3, 1},  {"conv4_3_CPM", 512, 256, 3, 1}, {"conv4_4_CPM", 256, 128, 3, 1}};
}
std::vector<Spec> vgg_hand() {
    return {{"conv1_1", 3, 64, 3, 1},    {"conv1_2", 64, 64, 3, 1},    {"conv2_1", 64, 128, 3, 1},
            {"conv2_2", 128, 128, 3, 1}, {"conv3_1", 128, 256, 3, 1},  {"conv3_2", 256, 256, 3, 1},
            {"conv3_3", 256, 256, 3, 1}, {"conv3_4", 256, 256, 3, 1},  {"conv4_1", 256, 512, 3, 1},
            {"conv4_2", 512, 512, 3, 1}, {"conv4_3", 512, 512, 3, 1},  {"conv4_4", 512, 512, 3, 1},
            {"conv5_1", 512, 512, 3, 1}, {"conv5_2", 512, 512, 3, 1},  {"conv5_3_CPM", 512, 128, 3, 1}};
}
std::vector<Spec> body_branch(int stage, int br) {
    const int out = br == 1 ? 38 : 19;
    const std::string L = "_L" + std::to_string(br);
    if (stage == 1)
        return {{"conv5_1_CPM" + L, 128, 128, 3, 1}, {"conv5_2_CPM" + L, 128, 128, 3, 1},
                {"conv5_3_CPM" + L, 128, 128, 3, 1}, {"conv5_4_CPM" + L, 128, 512, 1, 0},
                {"conv5_5_CPM" + L, 512, out, 1, 0}};
    const std::string sfx = "_stage" + std::to_string(stage) + L;
    std::vector<Spec> v = {{"Mconv1" + sfx, 185, 128, 7, 3}};
    for (int i = 2; i <= 5; ++i) v.push_back({"Mconv" + std::to_string(i) + sfx, 128, 128, 7, 3});
    v.push_back({"Mconv6" + sfx, 128, 128, 1, 0});
    v.push_back({"Mconv7" + sfx, 128, out, 1, 0});
    return v;
}
std::vector<Spec> hand_stage(int stage) {
    if (stage == 1) return {{"conv6_1_CPM", 128, 512, 1, 0}, {"conv6_2_CPM", 512, 22, 1, 0}};
    const std::string sfx = "_stage" + std::to_string(stage);
    std::vector<Spec> v = {{"Mconv1" + sfx, 150, 128, 7, 3}};
    for (int i = 2; i <= 5; ++i) v.push_back({"Mconv" + std::to_string(i) + sfx, 128, 128, 7, 3});
    v.push_back({"Mconv6" + sfx, 128, 128, 1, 0});
    v.push_back({"Mconv7" + sfx, 128, 22, 1, 0});
    return v;
}
std::vector<Spec> state_dict_order(int net) {
    std::vector<Spec> all;
    if (net == OPOSE_NET_BODY) {
        all = vgg_body();
        for (int br = 1; br <= 2; ++br)
            for (int s = 1; s <= 6; ++s) {
                auto b = body_branch(s, br);
                all.insert(all.end(), b.begin(), b.end());
            }
    } else {
        all = vgg_hand();
        for (int s = 1; s <= 6; ++s) {
            auto b = hand_stage(s);
            all.insert(all.end(), b.begin(), b.end());
        }
    }
    return all;
}

int round_up(int v, int m) { return (v + m - 1) / m * m; }

// OPOSE_PIPELINE_DEFER gate: the layer before which the next network records it ("stageN": before
// CPM stage N).  Swept on the bench, same box: conv4_1 2,101, stage2 2,100, stage3 2,105, stage4
// 2,107 frames/s against 2,110 with no gate (a round-4 A/B, kept in git history)
static const std::string& gate_layer() {
    static const std::string g = "conv3_1";
    return g;
}

// ---------------------------------------------------------------- streams
// Streams come from a process-wide pool and go back to it when a handle is destroyed (drained
// first), so test suites and services that create and destroy handles do not churn HIP streams.
struct StreamPool {
    std::mutex mu;
    std::map<std::pair<int, int>, std::vector<hipStream_t>> free;  // (device, priority) -> streams
};
StreamPool& stream_pool() {
    static StreamPool* p = new StreamPool();  // never destroyed: handles may outlive static teardown
    return *p;
}
hipError_t pooled_stream(hipStream_t* s, int priority) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    {
        std::lock_guard<std::mutex> g(stream_pool().mu);
        auto& v = stream_pool().free[{dev, priority}];
        if (!v.empty()) {
            *s = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, priority);
}
void return_stream(hipStream_t s, int device, int priority) {
    if (!s) return;
    (void)hipStreamSynchronize(s);
    std::lock_guard<std::mutex> g(stream_pool().mu);
    stream_pool().free[{device, priority}].push_back(s);
}

// ---------------------------------------------------------------- device memory helpers
// Bumped whenever device memory that a captured hipGraph may reference is (re)allocated:
// graphs captured under an older epoch are dropped instead of replayed.
std::atomic<uint64_t> g_alloc_epoch{1};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    uint64_t pad_key = 0;  // X6P geometry whose padding units are known zero (0: none)
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T* ensure(size_t n, hipStream_t st) {
        size_t b = n * sizeof(T);
        if (b > bytes) {
            if (p) {
                (void)st;
                OPOSE_HIP_CHECK(hipDeviceSynchronize());  // the handle may have work on two streams
                OPOSE_HIP_CHECK(hipFree(p));
                p = nullptr;
            }
            size_t nb = std::max(b, bytes + bytes / 4);
            OPOSE_HIP_CHECK(hipMalloc(&p, nb));
            bytes = nb;
            pad_key = 0;
            g_alloc_epoch.fetch_add(1);
        }
        return static_cast<T*>(p);
    }
};

// Pinned host staging (small results copied back each call: a device-to-host copy into pageable
// memory goes through the runtime's staging buffer, ~35 us per copy on the box)
struct PinnedBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    template <class T>
    T* ensure(size_t n) {
        const size_t b = n * sizeof(T);
        if (b > bytes) {
            if (p) {
                OPOSE_HIP_CHECK(hipDeviceSynchronize());  // a copy into it may still be in flight
                OPOSE_HIP_CHECK(hipHostFree(p));
                p = nullptr;
            }
            OPOSE_HIP_CHECK(hipHostMalloc(&p, b, hipHostMallocDefault));
            bytes = b;
        }
        return static_cast<T*>(p);
    }
};

// A GEMM-ready conv: one or two (combined) reference layers.
struct DevConv {
    std::string name;
    int cin = 0, cout = 0, ks = 0, pad = 0, K = 0, Kpad = 0, Mpad = 0;
    bool tap_major = false;  // K = (channel block of 32, tap, channel); see conv.hip
    float* wt = nullptr;
    float* bias = nullptr;
    int* ktab = nullptr;
    // split-bf16 (X6) form: [nK6][3][4][Mpad] units of 8 bf16, input channels in the physical
    // (group-aligned) order of the X6 activation buffers; see conv_x6.hip
    uint8_t* wx6 = nullptr;
    int nK6 = 0, cin_g = 0;
    bool small6 = false;
    // 3x3 / 7x7 layers: the same weights in pair order for conv_win_x6 (conv_win.hip)
    uint8_t* wx6p = nullptr;
    int nK6p = 0;
    // 3x3 layers: the Winograd F(2,3) weights U_v (x6_pack_weights_wino) for conv_wino_x6
    uint8_t* wwino = nullptr;
    int nKw = 0;
    // k-slab policy inputs (engine slab_count): the network, the layer's resolution level
    // (0: H .. 3: H/8) and whether it is one branch of a CPM pair (two GEMMs per launch)
    int net = 0, lvl = 0;
    bool pair = false;
    ~DevConv() {
        if (wx6) (void)hipFree(wx6);
        if (wx6p) (void)hipFree(wx6p);
        if (wwino) (void)hipFree(wwino);
        if (wt) (void)hipFree(wt);
        if (bias) (void)hipFree(bias);
        if (ktab) (void)hipFree(ktab);
    }
};

struct ProfEntry {
    std::string cls;
    std::string detail;  // optional second aggregation key (per layer / tile choice)
    double flops = 0;
    double bytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;  // null: not recorded (profiling off / filtered)
};

struct ProfAgg {
    long count = 0;
    double ms = 0, flops = 0, bytes = 0;
};

// geometry of one pyramid scale (engine.cpp geom)
struct ScaleGeom {
    double mult;      // scale * boxsize / H
    int Hs, Ws;       // cv2.resize output (cvRound(H * mult))
    int Hp, Wp;       // padded to stride
    int hl, wl;       // network output
    double up_sy, up_sx;  // final resize (Hs,Ws) -> (H,W) source steps
};

}  // namespace

struct GraphEntry {
    hipGraphExec_t exec = nullptr;
    uint64_t epoch = 0;
    bool eager = false;  // its capture was not one chain of nodes: run eagerly from then on
};

struct opose_ctx {
    // launch-sequence cache: per call signature, the device work of the first call runs
    // eagerly (allocating every buffer), the second is captured into a hipGraph, later calls
    // replay it (one launch instead of ~150: single-frame latency is launch bound)
    std::map<std::string, GraphEntry> graphs;
    bool use_graphs = getenv("OPOSE_NO_GRAPH") == nullptr;
    // set while run_graphed captures: run_scales_concurrently then keeps the capture on one
    // stream (no forked branches in any captured graph, see run_graphed)
    bool capturing = false;
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    int ppp = 128, maxp = 96;
    // weights
    std::map<std::string, std::unique_ptr<DevConv>> convs[2];
    bool loaded[2] = {false, false};
    // workspace
    // network convolutions: fp32-accurate split-bf16 kernel (default) or the fp32 MFMA kernel
    // (OPOSE_CONV=f32)
    bool x6 = [] {
        const char* e = getenv("OPOSE_CONV");
        return !(e && std::string(e) == "f32");
    }();
    // MaxPool2d fused into the preceding conv's epilogue (default); OPOSE_FUSED_POOL=0 at handle
    // creation: separate maxpool_x6 launches (A/B; bit-identical results)
    bool fused_pool = [] {
        const char* e = getenv("OPOSE_FUSED_POOL");
        return !(e && e[0] == '0');
    }();
    // conv1_1 by the direct first-layer kernel (default); OPOSE_FIRST_DIRECT=0: implicit GEMM
    bool first_direct = [] {
        const char* e = getenv("OPOSE_FIRST_DIRECT");
        return !(e && e[0] == '0');
    }();
    // the batched 3x3 / 7x7 convs on padded inputs by conv_win_x6 (input window in LDS;
    // OPOSE_CONV7_WIN=0: conv_x6 over the im2col stream, the cross-check of tests/test_gpu_x6.py)
    bool win7 = [] {
        const char* e = getenv("OPOSE_CONV7_WIN");
        return !(e && e[0] == '0');
    }();
    // OPOSE_WINO=1: 3x3 layers that would run whole tiles on the window kernel run as Winograd
    // F(2,3) along x instead (conv_wino_x6, 2/3 of the MFMAs).  Opt-in: fp32-accurate and correct
    // (tests/test_gpu_x6.py), but slower than the window kernel on this hardware
    bool wino = [] {
        const char* e = getenv("OPOSE_WINO");
        return e && e[0] == '1';
    }();
    int force_kernel = -1;  // opose_debug_conv_x6's X6P path: the family under test
    // a pyramid's heat-map average in one launch (heat_full_scales); OPOSE_HEAT_SCALES=0: one
    // launch per scale into the float64 accumulator (the bit-identity cross-check of
    // tests/test_gpu_scale_shard.py)
    bool heat_scales = [] {
        const char* e = getenv("OPOSE_HEAT_SCALES");
        return !(e && e[0] == '0');
    }();
    // a CPM stage's closing 1x1 pair in one launch (conv1x1_chain_x6); OPOSE_FUSE_1X1=0: two
    // launches through an HBM intermediate (the cross-check of tests/test_gpu_x6.py)
    bool fuse1x1 = [] {
        const char* e = getenv("OPOSE_FUSE_1X1");
        return !(e && e[0] == '0');
    }();
    // conv1_1 -> conv1_2 (window kernel) hand-off as fp32 units, split by conv1_2 (default);
    // OPOSE_C11_F32=0: as X6 (A/B, bit-identical)
    bool c11_f32 = [] {
        const char* e = getenv("OPOSE_C11_F32");
        return !(e && e[0] == '0');
    }();
    // multi-frame segments whose windows overflow the LDS run as one segment per frame on the
    // window kernel (run_conv_x6_segs); OPOSE_SPLIT_FRAMES=0: conv_x6 for such launches (A/B)
    bool split_frames = [] {
        const char* e = getenv("OPOSE_SPLIT_FRAMES");
        return !(e && e[0] == '0');
    }();
    // conv1_2 + pool by conv3_pool_win_x6 (input window in LDS; OPOSE_CONV12_WIN=0: conv_x6's
    // pooled 64 x 128 tile over the im2col stream)
    bool win12 = [] {
        const char* e = getenv("OPOSE_CONV12_WIN");
        return !(e && e[0] == '0');
    }();
    // conv launch plans per launch signature (tile, grid) and the device copies of their unit
    // schedules (X6Args::sched; never freed while the handle lives: captured graphs hold them)
    struct ConvPlan {
        int mt = 0, pt = 0, grid = 0;
        int* sched = nullptr;
    };
    std::map<std::string, ConvPlan> plans;
    std::map<std::string, int> slab_cache;  // engine slab_count
    std::vector<int*> sched_mem;
    std::vector<std::vector<int>> sched_host;  // sources of the asynchronous uploads
    DevBuf frames, mids[2][kMaxScales], avg, cnt, list, peak_pos, part_cnt, score, conn, conn_cnt, records, maps_in,
        hlab, hsums, hpeaks, hfound, list_score, hsel;
    PinnedBuf hand_out;  // Hand() peaks + found, staged for the host
    // network workspace, one set per concurrently running scale (slot s runs on scale_stream(s);
    // slot 0 is the handle's stream): input, activations, k-slab partials
    struct NetWS {
        DevBuf x, xband, x6in, x6A, x6B, x6P0, x6P1, x6Q0, x6Q1, x6S0, x6S1, x6T0, x6T1, x6U, bufA, bufB, S0, S1, T0, T1, U, partial;
    };
    NetWS ws[kMaxScales];
    int slot = 0;
    NetWS& w() { return ws[slot]; }
    // the scales of one Hand() call run concurrently on their own streams (OPOSE_SCALE_STREAMS=0:
    // one after another on the handle's stream, captured into a hipGraph)
    bool scale_streams = [] {
        const char* e = getenv("OPOSE_SCALE_STREAMS");
        return !(e && e[0] == '0');
    }();
    // split-bf16 path: a pyramid's networks (Hand()'s four scales, a multi-scale Body's) in
    // lockstep, one conv launch per layer for all of them (default); OPOSE_LOCKSTEP=0: one network
    // per scale, concurrent streams when scale_streams (the reference of the lockstep tests; the
    // same outputs bit for bit: a pixel's summation order does not depend on the launch).
    int lockstep = [] {
        const char* e = getenv("OPOSE_LOCKSTEP");
        return e ? std::atoi(e) : 1;
    }();
    hipStream_t sstream[kMaxScales] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kMaxScales] = {};
    // Cross-call pipelining of opose_body_infer calls flagged OPOSE_PIPELINE (device input and
    // output).  Call k's network part (preprocess, conv stack,
    // x8 upsample) runs on `nstream`, its post-network part on `stream` after an event; call
    // k+1's network then overlaps call k's post-network kernels (latency-bound launches of a few
    // dozen workgroups, and the CUs a 236-tile conv grid leaves idle).  The x8 maps (the only
    // buffers both parts touch) alternate between two sets; `nstream` waits for the post part
    // of the call two back before overwriting a set, and for `stream` whenever another entry
    // point used the shared network workspace there since (main_dirty).  Every call ends with
    // `stream` ordered after its own network part.
    hipStream_t nstream = nullptr;
    int nstream_prio = 0;
    // OPOSE_PIPELINE_DEFER: the last call's post-network part, enqueued by the next pipelined
    // call after that call's network recorded ev_gate (before its trunk's conv3_1), or by
    // flush_post.  gate_ev: set while a network part should record the gate.
    struct DeferredPost {
        bool pending = false;
        int N = 0, H = 0, W = 0, set = 0;
        std::vector<ScaleGeom> gs;
        opose_params p{};
        uint8_t* rec = nullptr;
    } dpost;
    hipEvent_t ev_gate = nullptr, gate_ev = nullptr;
    bool gate_done = false;
    hipEvent_t ev_net = nullptr, ev_main = nullptr, ev_post[2] = {nullptr, nullptr};
    // opose_wait_stream / opose_signal_stream / opose_set_stream: ordering against streams the
    // caller owns (a framework's current stream)
    hipEvent_t ev_ext = nullptr, ev_sig = nullptr;
    hipEvent_t ev_in = nullptr;  // opose_signal_input
    bool post_pending[2] = {false, false};
    bool main_dirty = false;
    int mid_set = 0, next_set = 0;
    DevBuf& mid(int s) { return mids[mid_set][s]; }
    // profiling
    bool prof = false;
    bool detail = false;  // per-layer aggregation (opose_profile_enable(h, 2))
    bool prof_conv7_only = false;  // opose_profile_enable(h, 3)
    std::vector<ProfEntry> pending;
    std::map<std::string, ProfAgg> agg;
    std::vector<hipEvent_t> event_pool;

    hipEvent_t get_event() {
        if (!event_pool.empty()) {
            hipEvent_t e = event_pool.back();
            event_pool.pop_back();
            return e;
        }
        // timing-only events: no system-scope fence on record (no L2 writeback / invalidate
        // between the bracketed launches; only hipEventElapsedTime reads them)
        hipEvent_t e;
        OPOSE_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        return e;
    }
    void prof_begin(ProfEntry& pe, const char* cls, double flops, double bytes) {
        if (!prof || (prof_conv7_only && std::strcmp(cls, "conv7x7") != 0)) return;
        pe.cls = cls;
        pe.flops = flops;
        pe.bytes = bytes;
        pe.e0 = get_event();
        pe.e1 = get_event();
        OPOSE_HIP_CHECK(hipEventRecord(pe.e0, stream));
    }
    void prof_end(ProfEntry& pe) {
        if (!prof || !pe.e0) return;
        OPOSE_HIP_CHECK(hipEventRecord(pe.e1, stream));
        pending.push_back(pe);
    }
    // fold finished event pairs into agg; non-blocking (stops at the first unfinished pair, so a
    // call does not wait for its own kernels) unless `all`
    void prof_drain(bool all = false) {
        size_t done = 0;
        for (auto& pe : pending) {
            if (!all && hipEventQuery(pe.e1) != hipSuccess) break;
            ++done;
            OPOSE_HIP_CHECK(hipEventSynchronize(pe.e1));
            float ms = 0;
            OPOSE_HIP_CHECK(hipEventElapsedTime(&ms, pe.e0, pe.e1));
            for (const std::string* key : {&pe.cls, &pe.detail}) {
                if (key->empty() || (key == &pe.detail && !detail)) continue;
                auto& a = agg[*key];
                a.count++;
                a.ms += ms;
                a.flops += pe.flops;
                a.bytes += pe.bytes;
            }
            event_pool.push_back(pe.e0);
            event_pool.push_back(pe.e1);
        }
        pending.erase(pending.begin(), pending.begin() + done);
    }
    // RCCL communicator for row-band halo exchanges (opose_rccl_init) and this handle's band
    // neighbours (opose_set_band_peers; -1: none)
    ncclComm_t comm = nullptr;
    int band_up = -1, band_dn = -1;
    ~opose_ctx();
    void release() {
        // drain every stream first, then the graph executables (they may reference the scale
        // streams' captured work), then streams, events and memory
        if (stream) (void)hipStreamSynchronize(stream);
        if (nstream) (void)hipStreamSynchronize(nstream);
        for (int i = 0; i < kMaxScales; ++i)
            if (sstream[i]) (void)hipStreamSynchronize(sstream[i]);
        for (auto& kv : graphs)
            if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
        graphs.clear();
        return_stream(nstream, device, nstream_prio);
        for (hipEvent_t e : {ev_net, ev_main, ev_post[0], ev_post[1], ev_ext, ev_sig, ev_in, ev_fork})
            if (e) (void)hipEventDestroy(e);
        for (int i = 0; i < kMaxScales; ++i) {
            return_stream(sstream[i], device, 0);
            if (ev_join[i]) (void)hipEventDestroy(ev_join[i]);
        }
        for (int* p : sched_mem) (void)hipFree(p);
        for (auto e : event_pool) (void)hipEventDestroy(e);
        return_stream(own_stream, device, 0);
    }
};

namespace {

struct Act {  // a channel slice of an NCHW activation buffer
    float* p;
    int cstride, coff;
};

// --------------------------------------------------------------- conv launch planning
// choose_tile: the fp32 MFMA path (OPOSE_CONV=f32, conv.hip stream-K) and the whole-tile choice of
// the split-bf16 debug entry points; the split-bf16 network plans with slab_count / pick_tile
struct TileChoice {
    int mt, pt, grid;  // tile shape, workgroups (grid == tiles: data parallel; else stream-K)
};

// Cost model in units of one 32-deep k-chunk of a 64x64 output tile on one CU.  A CU that
// holds k >= 2 co-resident workgroups finishes them in k * work; a lone workgroup (one wave per
// SIMD) runs at ~60 %.  Stream-K (grid = all resident slots) balances the chip exactly and
// pays for the partial slabs of tiles it splits plus one fixup launch.
TileChoice choose_tile(int Mpad, const std::vector<int>& gpix, int nK, bool x6 = false, bool dp_only = false,
                       double* cost_out = nullptr) {
    long npix_all = 0;
    for (int n : gpix) npix_all += n;
    static const int cfg[6][3] = {{128, 128, 2}, {128, 256, 1}, {256, 128, 1},
                                  {128, 64, 3},  {64, 128, 3},  {64, 64, 4}};  // mt, pt, WG/CU
    // split-bf16 kernel: 2.5x the MFMA rate per chunk, more LDS per workgroup
    static const int occ6[6] = {1, 1, 1, 2, 2, 3};
    // (256x128 measured 0-2.5 % faster than 128x256 where both fit: half the im2col DMA per MFMA;
    // a 64x256 tile (four 64x64 waves) for the M = 64 layers measured 91 vs 109 TF/s with 64x128
    // on conv1_2 -- an M = 64 tile loads the same im2col bytes per MFMA whatever its width -- and
    // was deleted)
    static const double ovh6_big[6] = {1.5, 1.0, 0.96, 1.1, 1.1, 1.2};
    // layers of one or two small frames (C2 / C3 / single-frame C5, stream-K over the whole chip):
    // 128x128 priced like the 8-wave tiles and 64x64 higher -- measured, C2 1.91 -> 1.72 ms and
    // Hand() 10.0 -> 9.9 ms, C5 and the bench unchanged; the same weights on the bench's
    // 32-frame layers cost 6 % (a round-4 A/B, kept in git history)
    static const double ovh6_small[6] = {1.0, 1.0, 0.96, 1.1, 1.1, 1.6};
    const double* ovh6 = npix_all <= 16384 ? ovh6_small : ovh6_big;
    const double rate = x6 ? 0.4 : 1.0;
    // relative cost per MFMA of the smaller tiles of the fp32 kernel (more load/issue work per
    // MFMA), measured with scripts/conv_timing.py
    static const double ovh[6] = {1.0, 0.95, 0.93, 1.02, 1.02, 1.06};
    TileChoice best{64, 64, 1};
    double best_cost = 1e300;
    for (int c = 0; c < 6; ++c) {
        const int mt = cfg[c][0], pt = cfg[c][1], occ = x6 ? occ6[c] : cfg[c][2];
        if (Mpad % mt) continue;
        long tiles = 0;
        for (int n : gpix) tiles += (long)(Mpad / mt) * ((n + pt - 1) / pt);
        const double unit = (mt / 64.0) * (pt / 64.0) * (x6 ? ovh6[c] : ovh[c]) * rate;
        // data parallel
        const long per_cu = (tiles + 255) / 256;
        // one resident workgroup of a 2-per-CU config runs at ~60 % (floor 1.6); the 8-wave
        // 128x256 config fills the CU on its own
        const double floor1 = occ >= 2 ? 1.6 : 1.0;
        const double dp = std::max<double>(per_cu, floor1) * nK * unit;
        if (dp < best_cost * 0.97) {
            best_cost = dp;
            best = {mt, pt, (int)tiles};
        }
        // stream-K over every resident slot (each workgroup >= 4 chunks)
        const long iters = tiles * nK;
        long grid = std::min<long>(256L * occ, iters / 4);
        if (!dp_only && grid >= 1 && grid != tiles) {
            const double per_wg = (double)iters / grid;
            const double cu_load = std::max(floor1, std::ceil(grid / 256.0)) * per_wg * unit;
            // partial slabs: every workgroup segment that is not a whole tile writes one, the
            // fixup re-reads them all (grid > tiles: ~grid + tiles segments, each tile cut in
            // grid / tiles parts -- the dominant cost of tiny single-frame layers)
            // (measured: with grid <= 2 x tiles the slabs stay cache resident and the old
            // tiles-with-partials estimate ranks configurations better)
            const long segs = grid > 2 * tiles ? grid + tiles : std::min<long>(tiles, 2 * grid);
            const double slab_bytes = grid > 2 * tiles
                                          ? (double)segs * mt * pt * 4.0 * 2.0 + (double)tiles * mt * pt * 4.0
                                          : (double)segs * mt * pt * 4.0 * 3.0;
            const double sk = cu_load + slab_bytes / 5e12 / 0.42e-6 + 8.0;      // + fixup launch
            if (sk < best_cost * 0.97) {
                best_cost = sk;
                best = {mt, pt, (int)grid};
            }
        }
    }
    if (cost_out) *cost_out = best_cost;
    return best;
}

// ---------------------------------------------------------------- fixed k slabs (split-bf16 path)
// A tile of a group with S slabs sums chunks [s nK / S, (s + 1) nK / S) from zero for each s and
// the slabs are folded in slab order (common.h X6Group::slabs).  S is a function of the layer and
// the segment (slab_count), so the work units (tile, slab) of a launch are fixed before its grid
// is chosen; the grid only decides which workgroup runs which unit.

struct SlabGroup {
    long tiles;
    int S;
};

// per-unit fixed cost in chunks (prologue: weight stages / window DMA; epilogue stores)
constexpr double kUnitOvh = 1.5;

// Longest-first assignment of the units of `gs` (numbered group, tile, slab) to G workgroups:
// each unit costs its chunks + kUnitOvh and goes to the least loaded workgroup (ties: the lowest
// index).  Returns the largest load in chunks; `lists`: per workgroup its units, ascending.
double lpt_units(const std::vector<SlabGroup>& gs, int nK, int G, std::vector<std::vector<int>>* lists) {
    struct Un {
        double c;
        int id;
    };
    std::vector<Un> us;
    int u = 0;
    double total = 0, big = 0;
    for (const SlabGroup& g : gs)
        for (long t = 0; t < g.tiles; ++t)
            for (int s = 0; s < g.S; ++s, ++u) {
                const double c = (double)((s + 1) * nK / g.S - s * nK / g.S) + kUnitOvh;
                us.push_back({c, u});
                total += c;
                big = std::max(big, c);
            }
    if (!lists && us.size() > 8192) return std::max(total / G, big);  // planning estimate of a large launch
    std::stable_sort(us.begin(), us.end(), [](const Un& a, const Un& b) { return a.c > b.c; });
    std::priority_queue<std::pair<double, int>, std::vector<std::pair<double, int>>, std::greater<>> pq;
    for (int w = 0; w < G; ++w) pq.push({0.0, w});
    if (lists) lists->assign(G, {});
    double mk = 0;
    for (const Un& x : us) {
        auto top = pq.top();
        pq.pop();
        top.first += x.c;
        mk = std::max(mk, top.first);
        if (lists) (*lists)[top.second].push_back(x.id);
        pq.push(top);
    }
    if (lists)
        for (auto& L : *lists) std::sort(L.begin(), L.end());
    return mk;
}

}  // namespace

// ======================================================================== engine
namespace opose {

// RCCL entry points, resolved on first use: the library shares the RCCL a host framework already
// loaded (torch's), and callers that never split a frame never load it.
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
};
static const Rccl& rccl() {
    static const Rccl r = [] {
        void* lib = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
        if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!lib) lib = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!lib) throw std::runtime_error("RCCL (librccl.so) not found");
        auto sym = [&](const char* n) {
            void* f = dlsym(lib, n);
            if (!f) throw std::runtime_error(std::string("RCCL without ") + n);
            return f;
        };
        Rccl x;
        x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(sym("ncclGetUniqueId"));
        x.comm_init_rank = reinterpret_cast<decltype(x.comm_init_rank)>(sym("ncclCommInitRank"));
        x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(sym("ncclCommDestroy"));
        x.comm_abort = reinterpret_cast<decltype(x.comm_abort)>(sym("ncclCommAbort"));
        x.send = reinterpret_cast<decltype(x.send)>(sym("ncclSend"));
        x.recv = reinterpret_cast<decltype(x.recv)>(sym("ncclRecv"));
        x.group_start = reinterpret_cast<decltype(x.group_start)>(sym("ncclGroupStart"));
        x.group_end = reinterpret_cast<decltype(x.group_end)>(sym("ncclGroupEnd"));
        x.error_string = reinterpret_cast<decltype(x.error_string)>(sym("ncclGetErrorString"));
        x.async_error = reinterpret_cast<decltype(x.async_error)>(sym("ncclCommGetAsyncError"));
        return x;
    }();
    return r;
}
static void rccl_check(ncclResult_t r) {
    if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL: ") + rccl().error_string(r));
}

}  // namespace opose

opose_ctx::~opose_ctx() {
    if (comm) (void)opose::rccl().comm_destroy(comm);
    release();
}

namespace opose {

static DevConv* find_conv(opose_ctx* h, int net, const std::string& name) {
    auto it = h->convs[net].find(name);
    if (it == h->convs[net].end()) throw std::runtime_error("missing layer " + name);
    return it->second.get();
}

static void upload_conv(opose_ctx* h, int net, const std::string& key, const std::vector<const Spec*>& parts,
                        const std::vector<const float*>& w, const std::vector<const float*>& b,
                        const std::vector<int>& cmap = {}) {
    auto dc = std::make_unique<DevConv>();
    const Spec& s0 = *parts[0];
    dc->name = key;
    dc->net = net;
    dc->lvl = key.rfind("conv1_", 0) == 0 ? 0 : key.rfind("conv2_", 0) == 0 ? 1 : key.rfind("conv3_", 0) == 0 ? 2 : 3;
    dc->pair = key.size() > 3 && (key.compare(key.size() - 3, 3, "_L1") == 0 || key.compare(key.size() - 3, 3, "_L2") == 0);
    dc->cin = s0.cin;
    dc->ks = s0.ks;
    dc->pad = s0.pad;
    dc->K = s0.cin * s0.ks * s0.ks;
    dc->tap_major = s0.cin >= 32;
    const int cin_pad = round_up(s0.cin, 32);
    dc->Kpad = dc->tap_major ? s0.ks * s0.ks * cin_pad : round_up(dc->K, 32);
    int cout = 0;
    for (auto* p : parts) cout += p->cout;
    dc->cout = cout;
    dc->Mpad = cout <= 64 ? 64 : round_up(cout, 128);
    std::vector<float> wt((size_t)dc->Kpad * dc->Mpad, 0.f), bias(cout, 0.f);
    int m0 = 0;
    for (size_t i = 0; i < parts.size(); ++i) {
        for (int m = 0; m < parts[i]->cout; ++m) {
            for (int k = 0; k < dc->K; ++k) {
                // reference layout OIHW: k = c * ks*ks + tap
                const int c = k / (s0.ks * s0.ks), tap = k % (s0.ks * s0.ks);
                // blocked layout: K = (32-channel block, tap, channel in block) -- a workgroup
                // walks all taps of one channel block before the next, so the im2col rows it
                // gathers are re-read from L2 while still resident (see conv.hip)
                const int kk = dc->tap_major ? ((c / 32) * (s0.ks * s0.ks) + tap) * 32 + (c % 32) : k;
                wt[(size_t)kk * dc->Mpad + m0 + m] = w[i][(size_t)m * dc->K + k];
            }
            bias[m0 + m] = b[i][m];
        }
        m0 += parts[i]->cout;
    }
    std::vector<int> ktab(dc->Kpad, 0);  // padding rows: any in-range tap (weights are 0)
    for (int k = 0; k < dc->K; ++k) {
        int c = k / (dc->ks * dc->ks), r = k % (dc->ks * dc->ks);
        ktab[k] = (c << 8) | ((r / dc->ks) << 4) | (r % dc->ks);
    }
    // X6 weights: input channel c of the reference layer sits at physical channel cmap[c]
    {
        const int cin_phys = cmap.empty() ? s0.cin : cmap.back() + 1;
        const int taps = s0.ks * s0.ks;
        std::vector<float> wp((size_t)cout * cin_phys * taps, 0.f);
        int mm = 0;
        for (size_t i = 0; i < parts.size(); ++i)
            for (int m = 0; m < parts[i]->cout; ++m, ++mm)
                for (int c = 0; c < s0.cin; ++c) {
                    const int pc = cmap.empty() ? c : cmap[c];
                    for (int t = 0; t < taps; ++t)
                        wp[((size_t)mm * cin_phys + pc) * taps + t] = w[i][((size_t)m * s0.cin + c) * taps + t];
                }
        std::vector<uint16_t> wx;
        x6_pack_weights(wp.data(), cout, cin_phys, s0.ks, dc->Mpad, &dc->nK6, wx);
        dc->cin_g = (cin_phys + 7) / 8;
        dc->small6 = dc->cin_g == 1;
        OPOSE_HIP_CHECK(hipMalloc(&dc->wx6, wx.size() * 2));
        OPOSE_HIP_CHECK(hipMemcpy(dc->wx6, wx.data(), wx.size() * 2, hipMemcpyHostToDevice));
        if ((s0.ks == 7 || s0.ks == 3) && dc->Mpad % 128 == 0 && cin_phys > 8) {
            x6_pack_weights_pairs(wp.data(), cout, cin_phys, s0.ks, dc->Mpad, &dc->nK6p, wx);
            OPOSE_HIP_CHECK(hipMalloc(&dc->wx6p, wx.size() * 2));
            OPOSE_HIP_CHECK(hipMemcpy(dc->wx6p, wx.data(), wx.size() * 2, hipMemcpyHostToDevice));
        }
        if (s0.ks == 3 && dc->Mpad % 128 == 0 && cin_phys > 8) {
            x6_pack_weights_wino(wp.data(), cout, cin_phys, dc->Mpad, &dc->nKw, wx);
            OPOSE_HIP_CHECK(hipMalloc(&dc->wwino, wx.size() * 2));
            OPOSE_HIP_CHECK(hipMemcpy(dc->wwino, wx.data(), wx.size() * 2, hipMemcpyHostToDevice));
        }
    }
    OPOSE_HIP_CHECK(hipMalloc(&dc->wt, wt.size() * 4));
    OPOSE_HIP_CHECK(hipMalloc(&dc->bias, bias.size() * 4));
    OPOSE_HIP_CHECK(hipMalloc(&dc->ktab, ktab.size() * 4));
    g_alloc_epoch.fetch_add(1);  // captured graphs may hold the replaced layer's pointers
    OPOSE_HIP_CHECK(hipMemcpy(dc->wt, wt.data(), wt.size() * 4, hipMemcpyHostToDevice));
    OPOSE_HIP_CHECK(hipMemcpy(dc->bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
    OPOSE_HIP_CHECK(hipMemcpy(dc->ktab, ktab.data(), ktab.size() * 4, hipMemcpyHostToDevice));
    h->convs[net][key] = std::move(dc);
}

static const char* conv_class(int ks) { return ks == 7 ? "conv7x7" : (ks == 3 ? "conv3x3" : "conv1x1"); }

// run one (possibly 2-group) conv: out = act(conv(in))
static void run_conv(opose_ctx* h, DevConv* c0, DevConv* c1, int N, int H, int W, Act in0, Act out0, Act in1,
                     Act out1, bool relu0, bool relu1, Act dup = {nullptr, 0, 0}) {
    ConvArgs a{};
    const int ng = c1 ? 2 : 1;
    a.N = N;
    a.H = H;
    a.W = W;
    a.Cin = c0->cin;
    a.ks = c0->ks;
    a.pad = c0->pad;
    a.K = c0->K;
    a.Kpad = c0->Kpad;
    a.Mpad = c0->Mpad;
    a.npix = N * H * W;
    a.tap_major = c0->tap_major ? 1 : 0;
    DevConv* cs[2] = {c0, c1};
    Act ins[2] = {in0, in1}, outs[2] = {out0, out1};
    bool relus[2] = {relu0, relu1};
    for (int g = 0; g < ng; ++g) {
        ConvGroup& G = a.g[g];
        G.in = ins[g].p;
        G.in_cstride = ins[g].cstride;
        G.in_coff = ins[g].coff;
        G.wt = cs[g]->wt;
        G.bias = cs[g]->bias;
        G.out = outs[g].p;
        G.out_cstride = outs[g].cstride;
        G.out_coff = outs[g].coff;
        G.out2 = nullptr;
        G.cout = cs[g]->cout;
        G.relu = relus[g] ? 1 : 0;
    }
    if (dup.p) {
        a.g[0].out2 = dup.p;
        a.g[0].out2_cstride = dup.cstride;
        a.g[0].out2_coff = dup.coff;
    }
    if (ng == 1) a.g[1] = a.g[0];
    for (int g = 0; g < ng; ++g)  // the im2col gather addresses the input with 32-bit byte offsets
        if ((double)N * ins[g].cstride * H * W * 4.0 >= 2147483648.0)
            throw std::invalid_argument("activation slab >= 2 GiB: split the batch");
    const TileChoice t = choose_tile(a.Mpad, std::vector<int>(ng, a.npix), a.Kpad / 32);
    a.ngroups = ng;
    a.sk_grid = t.grid;
    a.partial = h->w().partial.ensure<float>((size_t)2 * t.grid * t.mt * t.pt, h->stream);
    double flops = 0;
    for (int g = 0; g < ng; ++g) flops += 2.0 * cs[g]->cout * (double)a.K * a.npix;
    ProfEntry pe;
    h->prof_begin(pe, conv_class(c0->ks), flops, 0);
    if (h->detail)
        pe.detail = "layer/" + c0->name + "/" + std::to_string(t.mt) + "x" + std::to_string(t.pt) + "s" +
                    std::to_string(t.grid) + "/n" + std::to_string(a.npix);
    launch_conv(a, c0->ktab, t.mt, t.pt, h->stream);
    h->prof_end(pe);
}

static void run_pool(opose_ctx* h, const float* in, float* out, int NC, int H, int W) {
    ProfEntry pe;
    h->prof_begin(pe, "maxpool", 0, (double)NC * H * W * 4 * 1.25);
    launch_maxpool(in, out, NC, H, W, h->stream);
    h->prof_end(pe);
}

// VGG trunk: x [N,3,H,W] -> final trunk conv written via `last` (+ optional duplicate)
static void run_trunk(opose_ctx* h, int net, const float* x, int N, int H, int W, Act last, Act dup) {
    const std::vector<Spec> vgg = net == OPOSE_NET_BODY ? vgg_body() : vgg_hand();
    size_t act = (size_t)N * 64 * H * W;
    float* A = h->w().bufA.ensure<float>(act, h->stream);
    float* B = h->w().bufB.ensure<float>(act, h->stream);
    const float* cur = x;
    int cc = 3, hh = H, ww = W;
    for (size_t i = 0; i < vgg.size(); ++i) {
        const Spec& s = vgg[i];
        DevConv* c = find_conv(h, net, s.name);
        const bool final_layer = i + 1 == vgg.size();
        float* dst = (cur == A) ? B : A;
        Act out = final_layer ? last : Act{dst, s.cout, 0};
        run_conv(h, c, nullptr, N, hh, ww, Act{const_cast<float*>(cur), cc, 0}, out, Act{}, Act{}, true, false,
                 final_layer ? dup : Act{nullptr, 0, 0});
        cur = dst;
        cc = s.cout;
        // pools follow conv1_2, conv2_2, conv3_4 (src/model.py:37,40,45 / :147,150,155)
        if (s.name == "conv1_2" || s.name == "conv2_2" || s.name == "conv3_4") {
            float* pd = (cur == A) ? B : A;
            run_pool(h, cur, pd, N * cc, hh, ww);
            hh /= 2;
            ww /= 2;
            cur = pd;
        }
    }
}

// ---------------------------------------------------------------- split-bf16 network path
struct XAct {  // a group slice of an X6 buffer (or, f32: a channel slice of an fp32 NCHW buffer)
    void* p = nullptr;
    int c = 0, off = 0;  // f32: channels per frame / first channel
    uint32_t ps = 0;     // X6 piece stride (bytes)
    X6Layout l{};        // X6 unit addressing (common.h)
    bool f32 = false;
    bool padded = false;
    int ylo = 0, yhi = 0;  // X6P row-band view: rows conv taps may read (yhi == 0: the frame's)
};

static XAct f32act(float* p, int c, int off) {
    XAct a;
    a.p = p;
    a.c = c;
    a.off = off;
    a.f32 = true;
    return a;
}

static uint32_t checked_ps(size_t ps) {
    if (ps * 3 >= 2147483648.0) throw std::invalid_argument("X6 activation >= 2 GiB: split the batch");
    return (uint32_t)ps;
}

// dense X6 [N][cg][H*W], groups [goff, ...)
static XAct x6act(uint8_t* p, int cg, int goff, int N, int H, int W) {
    const size_t hw = (size_t)H * W;
    XAct a;
    a.p = p;
    a.ps = checked_ps((size_t)N * cg * hw * 16);
    a.l = X6Layout{(uint32_t)(cg * hw), (uint32_t)hw, (uint32_t)W, (uint32_t)(goff * hw)};
    return a;
}

// padded X6P (common.h): units per (piece, group) plane
static size_t x6p_plane(int N, int H, int W) { return (size_t)(N * (H + 3) + 4) * x6p_pitch(W); }

static XAct x6pact(uint8_t* p, int cg, int goff, int N, int H, int W) {
    const size_t P = (size_t)x6p_pitch(W), plane = x6p_plane(N, H, W);
    XAct a;
    a.p = p;
    a.ps = checked_ps((size_t)cg * plane * 16);
    a.l = X6Layout{(uint32_t)((H + 3) * P), (uint32_t)plane, (uint32_t)P, (uint32_t)(goff * plane + 3 * P + 3)};
    a.padded = true;
    return a;
}

// One GEMM of a conv launch (an X6Group): a scale's frames through one branch's weights.
// Hl: the frame height the k-slab policy sees (a row band's view passes its whole frame's rows;
// 0: H); slabs: set by the planner (a frame view inherits its segment's).
struct ConvSeg {
    DevConv* c;
    int N, H, W;
    XAct in, out, dup;  // dup: optional duplicate X6 destination
    bool relu;
    int Hl = 0;
    int slabs = 0;
};

// Run convs of one shape (ks, Cin, Mpad) over up to kX6Groups segments per launch: the CPM
// branch pair of a stage and the scales of a pyramid share one grid (X6Args groups).
// pool: MaxPool2d(2, 2) (src/model.py:10-13, floor mode) fused into the epilogue; out is then the
// pooled [N][(H/2)(W/2)] X6 tensor (conv outputs the floor mode drops are never computed)
static void run_conv_x6_segs(opose_ctx* h, const std::vector<ConvSeg>& segs, bool pool = false);

// frame n of an activation (N frames of H x W) as a one-frame activation of the same buffer
static XAct frame_view(const XAct& a, int n, int H, int W) {
    XAct v = a;
    if (!a.p) return v;
    if (a.f32) v.p = static_cast<float*>(a.p) + (size_t)n * a.c * H * W;
    else v.l.o0 = a.l.o0 + (uint32_t)n * a.l.fs;
    return v;
}

// The kernel family of a segment -- conv_x6's (4 groups, 1 tap) chunks or conv_win_x6's pair
// order -- is part of each pixel's summation order, so like the slab count it is a function of
// the layer and the segment only:
//  * the window kernel for 3x3 / 7x7 layers on padded inputs whose window fits the LDS: one frame
//    of any height (conv_win_fits_rows: a 256-pixel run at W columns, so a row band and its whole
//    frame agree), or a batch whose tiles straddle frames;
//  * a 7x7 batch whose straddling windows do not fit but one frame's do: the window kernel on
//    one segment per frame (frame views of the same buffers; a crop batch's 92 x 92 scale);
//  * body layers of fewer than 4096 pixels (C2's single frame, a pyramid's 0.5 scale): conv_x6,
//    whose 128 x 64 tiles spread a small layer over the chip;
//  * the hand's 512-channel 3x3 layers at H/8 (conv4_x, conv5_1/5_2; not conv5_3_CPM's 128 outputs,
//    which take the 7x7 layers' slab layout on the window kernel): conv_x6, whose 256 x 128 tiles
//    cover a 368 crop's 4-scale pyramid in one data-parallel round (254 tiles; the window
//    kernel's 128 x 256 tiles make 260: 225 vs 270 TF/s);
//  * everything else (dense inputs, pooled convs, 1x1): conv_x6.
enum { kKernelX6 = 0, kKernelWin = 1, kKernelWinFrames = 2, kKernelWino = 3 };
static int slab_count(opose_ctx* h, const DevConv* c, bool win, int N, int H, int W, bool pool);
static int seg_kernel_direct(const opose_ctx* h, const ConvSeg& sg, bool pool);
//  * Winograd (conv_wino_x6): a 3x3 segment the window kernel would run as whole tiles (one k
//    slab) whose Winograd window fits (wino_tpf, a function of N, H, W; one frame: of W only);
//    the output pairs sit at even x of the frame, so a row band and its frame still agree.
static int seg_kernel(opose_ctx* h, const ConvSeg& sg, bool pool) {
    if (h->force_kernel >= 0) return h->force_kernel;
    const int k = seg_kernel_direct(h, sg, pool);
    const DevConv* c = sg.c;
    if (k == kKernelWin && h->wino && c->ks == 3 && c->wwino &&
        slab_count(h, c, true, sg.N, sg.Hl ? sg.Hl : sg.H, sg.W, pool) == 1 &&
        wino_tpf(sg.N, sg.Hl ? sg.Hl : sg.H, sg.W) >= 0)
        return kKernelWino;
    return k;
}
static int seg_kernel_direct(const opose_ctx* h, const ConvSeg& sg, bool pool) {
    const DevConv* c = sg.c;
    if (!h->win7 || pool || !c->wx6p || !sg.in.padded || (c->ks != 3 && c->ks != 7)) return kKernelX6;
    const long lpix = (long)sg.N * (sg.Hl ? sg.Hl : sg.H) * sg.W;
    if (c->net == OPOSE_NET_BODY && lpix < 4096) return kKernelX6;
    if (c->net == OPOSE_NET_HAND && c->ks == 3 && c->lvl == 3 && c->Mpad > 128) return kKernelX6;
    if (sg.N == 1) return conv_win_fits_rows(sg.W, c->ks) ? kKernelWin : kKernelX6;
    if (conv_win_fits(sg.N, sg.H, sg.W, c->ks)) return kKernelWin;
    if (c->ks == 7 && h->split_frames && conv_win_fits_rows(sg.W, c->ks)) return kKernelWinFrames;
    return kKernelX6;
}

// conv_x6 tile configurations: mt, pt, co-resident workgroups per CU, cost per chunk relative to
// a 64 x 64 tile's (measured, scripts/conv_timing.py; rounds 1-2)
static const int kX6Cfg[6][3] = {{128, 128, 1}, {128, 256, 1}, {256, 128, 1}, {128, 64, 2}, {64, 128, 2}, {64, 64, 3}};
static const double kX6Ovh[6] = {1.5, 1.0, 0.96, 1.1, 1.1, 1.2};
// launches of at most 16,384 columns (one small frame, C2's layers): 128x128 priced like the
// 8-wave tiles and 64x64 higher (round 3, choose_tile: C2 1.91 -> 1.72 ms)
static const double kX6OvhSmall[6] = {1.0, 1.0, 0.96, 1.1, 1.1, 1.6};

// GEMM columns and slab count of one group of a launch
struct ColGroup {
    long cols;
    int S;
};

static std::vector<SlabGroup> slab_groups(const std::vector<ColGroup>& cg, int Mpad, int mt, int pt) {
    std::vector<SlabGroup> gs;
    for (const ColGroup& c : cg) gs.push_back({(long)(Mpad / mt) * ((c.cols + pt - 1) / pt), c.S});
    return gs;
}

// Tile shape and grid of one launch (window kernel: 128 x 256 only) priced in choose_tile's units
// (a 32-deep chunk of a 64 x 64 tile = 0.4): the largest workgroup load (one-slab launches: rounds
// of whole tiles over the hardware dispatcher; else the longest-first unit schedule) times the
// tile's chunk cost, plus the slab partials' HBM round trip and the fixup launch.
struct TilePick {
    int mt = 0, pt = 0, grid = 0;
    double cost = 1e300;
};
static TilePick pick_tile(const std::vector<ColGroup>& cg, bool win, int nK, int Mpad, bool pool = false,
                          bool small_tiles = true) {
    bool multi = false;
    long cols_all = 0;
    for (const ColGroup& c : cg) {
        multi = multi || c.S > 1;
        cols_all += c.cols;
    }
    const double* ovh = cols_all <= 16384 ? kX6OvhSmall : kX6Ovh;
    // multi-slab launches of one small frame's layers (C2; slab_count's small-frame rule): 128 x 64 tiles,
    // one work unit per workgroup slot (slab_count) -- the measured best of 128 x 64 / 128 x 128 /
    // 64 x 128 / 64 x 64 / 128 x 256 at 6-32 slabs on C2's 7x7 layers (round 4 sweep)
    const bool small1 =
        small_tiles && !win && cols_all <= (pool ? 16384L : 4096L) * (long)cg.size() && Mpad % 128 == 0 && multi;
    TilePick best;
    for (int ci = 0; ci < 6; ++ci) {
        const int mt = win ? 128 : kX6Cfg[ci][0], pt = win ? 256 : kX6Cfg[ci][1], occ = win ? 1 : kX6Cfg[ci][2];
        if (win && ci > 0) break;
        if (Mpad % mt) continue;
        if (small1 && (mt != 128 || pt != 64)) continue;
        const std::vector<SlabGroup> gs = slab_groups(cg, Mpad, mt, pt);
        long units = 0, tiles = 0;
        for (const SlabGroup& g : gs) {
            units += g.tiles * g.S;
            tiles += g.tiles;
        }
        // one-slab launches: one workgroup per tile, the hardware dispatcher balancing them
        const long G = multi ? std::min<long>(units, 256L * occ) : tiles;
        const double mk = multi ? lpt_units(gs, nK, (int)G, nullptr) : (double)((tiles + 256L * occ - 1) / (256L * occ)) * nK;
        const double unit = (mt / 64.0) * (pt / 64.0) * (win ? 0.8 : ovh[ci]) * 0.4;
        // co-resident workgroups share a CU; a lone one of a 2-3 per CU tile runs at ~60 %
        const double share = G <= 256 ? (occ >= 2 ? 1.6 : 1.0) : (multi ? std::min<double>(occ, (double)G / 256.0) : occ);
        double cost = mk * unit * share;
        if (multi) cost += (double)units * mt * pt * 4.0 * 2.0 / 5e12 / 0.42e-6 + 8.0;  // slab partials + fixup
        if (cost < best.cost * 0.97) {
            best.cost = cost;
            best.mt = mt;
            best.pt = pt;
            best.grid = (int)G;
        }
    }
    return best;
}

// k slabs of a segment (common.h X6Group::slabs): a function of the layer, its kernel family and
// the segment's logical geometry (N frames of H x W) -- never of the launch that runs it, its
// grid, its other groups or a row band's rows.  Large layers keep one slab (one run over all
// chunks, the data-parallel grids of the bench's 32-frame batch); smaller ones are cut so that
// their work units fill the chip, counting tiles of the kernel's smallest tile (window: 128 x 256,
// conv_x6: 128 x 64) and both branches of a CPM pair.  The hand's layers run as one launch per
// layer for a 4-scale pyramid (lockstep): its 3x3 layers fill the chip with whole tiles (254 /
// 502 tiles over the pyramid), and the 7x7 counts are set per scale size so that the pyramid's
// units pack evenly over 256 workgroups (longest-first, lpt_units).
static int slab_count(opose_ctx* h, const DevConv* c, bool win, int N, int H, int W, bool pool) {
    const int nK = win ? c->nK6p : c->nK6;
    if (c->ks == 1 || nK < 8) return 1;  // 1x1: the closing pairs' unfused form sums like the fused chain
    const int smax = nK / 4;
    const long npix = (long)N * H * W;
    const double mr = c->Mpad / 128.0;
    auto clampS = [&](long s) { return (int)std::max<long>(1, std::min<long>(s, smax)); };
    if (c->net == OPOSE_NET_HAND) {
        if (pool) return 1;
        // the 7x7 stages, and conv5_3_CPM (3x3 at H/8, 128 outputs: 65 whole tiles for a 368 crop);
        // conv2_1 (128 outputs at H/2: 994 tiles) runs whole tiles
        if (!(c->ks == 7 && win) && !(c->ks == 3 && c->Mpad <= 128 && c->lvl == 3)) return 1;
        // A 368 crop's scales have 3 / 9 / 19 / 34 tiles: 4 / 7 / 8 / 4 slabs make 363 units whose
        // longest-first packing over 256 workgroups is within a chunk of the best of every table of
        // 1-16 slabs per scale (a makespan model with a per-unit overhead of 4 chunks), with the
        // fewest units of those (fewer partials, a shorter fixup).  Measured, same box: one crop
        // 7.39-7.53 -> 7.09 ms, a 368 + 256 crop batch 13.85-13.97 -> 13.50 ms (round 4's
        // 16 / 12 / 8 / 7; profiles/r5_hand_slabs.log).
        const double T = std::ceil(npix / 256.0) * mr;
        return clampS(T < 6 ? 4 : T < 12 ? 7 : T < 30 ? 8 : T < 60 ? 4 : T < 120 ? 4 : T < 240 ? 2 : 1);
    }
    const int mult = c->pair ? 2 : 1;
    if (std::ceil(npix / 256.0) * mr * mult >= 160) return 1;  // the bench's batches: whole tiles fill the chip
    if (!win && npix <= (pool ? 16384 : 4096) && c->Mpad % 128 == 0) {
        // one small frame (C2 and the pyramid's small scales on conv_x6): 128 x 64 tiles (pick_tile),
        // as many slabs as keep (tiles x slabs) within the 512 workgroup slots (two per CU) -- one
        // unit per workgroup.  C2's 7x7 layers: 10 slabs (300 units) 35.4 us, 16 (480) 33.6 us,
        // 20-32 (several units per workgroup) 40-43 us
        // (pooled convs: conv_x6_fixup pools the folded quads)
        const long tiles = (long)(c->Mpad / 128) * ((npix + 63) / 64) * mult;
        return clampS(std::max<long>(1, 512 / tiles));
    }
    if (pool) return 1;
    // otherwise the count that prices lowest for the segment run alone (with its CPM sibling), as
    // Body(frame) runs a scale -- plus, for one frame whose H/8 map has >= 40 rows (a scale the
    // balanced C5 split may cut into row bands, src/dist.py split_plan), the same layer on a fifth
    // of the rows (+ the band trunk's margin), as a band rank runs it.  A band's smaller launch
    // may take smaller tiles: the tile does not change a pixel's sum, the slab count does.
    const int h8 = H >> (3 - std::min(3, c->lvl));
    const long bpix = N == 1 && h8 >= 40
                          ? (long)std::min(H, H / 5 + (c->lvl < 3 ? 20 << (3 - c->lvl) : 0)) * W
                          : 0;
    const std::string key = std::to_string(win) + "/" + std::to_string(nK) + "/" + std::to_string(c->Mpad) + "/" +
                            std::to_string(npix) + "/" + std::to_string(mult) + "/" + std::to_string(bpix);
    auto it = h->slab_cache.find(key);
    if (it != h->slab_cache.end()) return it->second;
    static const int cand[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32, 40, 48, 64};
    int best = 1;
    double best_cost = 1e300;
    for (int S : cand) {
        if (S > std::max(1, smax)) break;
        double cost = pick_tile(std::vector<ColGroup>(mult, ColGroup{npix, S}), win, nK, c->Mpad).cost;
        // (the band proxy is a slice of a large scale: any tile, not the small-frame rule's)
        if (bpix) cost += pick_tile(std::vector<ColGroup>(mult, ColGroup{bpix, S}), win, nK, c->Mpad, false, false).cost;
        if (cost < best_cost * 0.97) {
            best_cost = cost;
            best = S;
        }
    }
    h->slab_cache[key] = best;
    return best;
}

// Launch plan of one kernel family over segments whose slab counts are set: tile shape, grid,
// and (multi-slab launches) the longest-first unit schedule.  Cached per signature.
static opose_ctx::ConvPlan plan_launch(opose_ctx* h, const std::vector<ConvSeg>& segs, bool win, bool pool, int nK,
                                       int Mpad) {
    std::string key = (win ? "w" : "x") + std::to_string(pool) + "/" + std::to_string(nK) + "/" + std::to_string(Mpad);
    for (const ConvSeg& s : segs)
        key += "/" + std::to_string((long)s.N * s.H * s.W) + ":" + std::to_string(s.slabs) + ":" +
               std::to_string(pool ? s.W : 0);
    auto it = h->plans.find(key);
    if (it != h->plans.end()) return it->second;
    std::vector<ColGroup> cg;
    bool multi = false;
    for (const ConvSeg& s : segs) {
        cg.push_back({pool ? (long)s.N * (s.H / 2) * (s.W / 2) * 4 : (long)s.N * s.H * s.W, s.slabs});
        multi = multi || s.slabs > 1;
    }
    const TilePick tp = pick_tile(cg, win, nK, Mpad, pool);
    opose_ctx::ConvPlan best;
    best.mt = tp.mt;
    best.pt = tp.pt;
    best.grid = tp.grid;
    best.sched = nullptr;
    if (multi) {
        std::vector<std::vector<int>> lists;
        lpt_units(slab_groups(cg, Mpad, best.mt, best.pt), nK, best.grid, &lists);
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        OPOSE_HIP_CHECK(hipStreamIsCapturing(h->stream, &cs));
        if (cs != hipStreamCaptureStatusNone) return best;  // (captured: contiguous unit ranges, same sums)
        std::vector<int> flat(best.grid + 1, 0);
        for (int w = 0; w < best.grid; ++w) flat[w + 1] = flat[w] + (int)lists[w].size();
        for (const auto& L : lists) flat.insert(flat.end(), L.begin(), L.end());
        int* d = nullptr;
        OPOSE_HIP_CHECK(hipMalloc(&d, flat.size() * sizeof(int)));
        h->sched_host.push_back(std::move(flat));
        const std::vector<int>& src = h->sched_host.back();
        OPOSE_HIP_CHECK(hipMemcpyAsync(d, src.data(), src.size() * sizeof(int), hipMemcpyHostToDevice, h->stream));
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));  // (once per launch signature)
        h->sched_mem.push_back(d);
        best.sched = d;
    }
    h->plans[key] = best;
    return best;
}

// One launch: segments of one kernel family, at most kX6Groups of them, slab counts set.
static void launch_segs(opose_ctx* h, const std::vector<ConvSeg>& segs, int family, bool pool) {
    const bool win = family == kKernelWin, wino = family == kKernelWino;
    DevConv* c0 = segs[0].c;
    X6Args a{};
    const int ng = (int)segs.size();
    a.ks = c0->ks;
    a.pad = c0->pad;
    a.cin_g = c0->cin_g;
    a.small = c0->small6 ? 1 : 0;
    a.nK = wino ? c0->nKw : win ? c0->nK6p : c0->nK6;
    a.Mpad = c0->Mpad;
    a.pool = pool ? 1 : 0;
    a.ngroups = ng;
    double flops = 0;
    long npix_all = 0;
    for (int g = 0; g < ng; ++g) {
        const ConvSeg& sg = segs[g];
        DevConv* c = sg.c;
        if (c->ks != c0->ks || c->cin_g != c0->cin_g || c->Mpad != c0->Mpad || c->nK6 != c0->nK6 || c->nK6p != c0->nK6p)
            throw std::invalid_argument("conv segments of different shapes");
        if (pool && (sg.dup.p || sg.out.f32)) throw std::invalid_argument("pooled conv: single X6 output only");
        X6Group& G = a.g[g];
        G.in = static_cast<const uint8_t*>(sg.in.p);
        G.in_ps = sg.in.ps;
        G.in_l = sg.in.l;
        G.wt = wino ? c->wwino : win ? c->wx6p : c->wx6;
        G.bias = c->bias;
        G.out = sg.out.p;
        G.out_ps = sg.out.ps;
        G.out_l = sg.out.l;
        G.out_c = sg.out.c;
        G.out_off = sg.out.off;
        G.out_f32 = sg.out.f32 ? 1 : 0;
        G.out2 = sg.dup.p;
        G.out2_ps = sg.dup.ps;
        G.out2_l = sg.dup.l;
        G.cout = c->cout;
        G.relu = sg.relu ? 1 : 0;
        G.N = sg.N;
        G.H = sg.H;
        G.W = sg.W;
        G.npix = pool ? sg.N * (sg.H / 2) * (sg.W / 2) * 4 : sg.N * sg.H * sg.W;
        G.ylo = sg.in.ylo;
        G.yhi = sg.in.yhi;
        G.slabs = sg.slabs;
        G.tpf = wino ? wino_tpf(sg.N, sg.Hl ? sg.Hl : sg.H, sg.W) : 0;
        if (G.yhi && (sg.N != 1 || pool)) throw std::invalid_argument("row band views: one frame, no pooling");
        npix_all += G.npix;
        flops += 2.0 * c->cout * (double)c->K * (pool ? 4.0 * sg.N * (sg.H / 2) * (sg.W / 2) : (double)G.npix);
    }
    if (wino) {
        ProfEntry pe;
        h->prof_begin(pe, conv_class(c0->ks), flops, 0);
        if (h->detail) {
            std::string nm = c0->name;
            for (int g = 1; g < ng; ++g)
                if (segs[g].c != c0 && nm.find(segs[g].c->name) == std::string::npos) nm += "|" + segs[g].c->name;
            pe.detail = "layer/" + nm + "/wino/g" + std::to_string(ng) + "/n" + std::to_string(npix_all);
        }
        launch_conv_wino_x6(a, h->stream);
        h->prof_end(pe);
        return;
    }
    const opose_ctx::ConvPlan p = plan_launch(h, segs, win, pool, a.nK, a.Mpad);
    a.sk_grid = p.grid;
    a.sched = p.sched;
    const X6Args num = x6_number_tiles(a, p.mt, p.pt);
    a.partial = num.units != num.tiles ? h->w().partial.ensure<float>((size_t)num.units * p.mt * p.pt, h->stream) : nullptr;
    ProfEntry pe;
    h->prof_begin(pe, conv_class(c0->ks), flops, 0);
    if (h->detail) {
        std::string nm = c0->name;
        for (int g = 1; g < ng; ++g)
            if (segs[g].c != c0 && nm.find(segs[g].c->name) == std::string::npos) nm += "|" + segs[g].c->name;
        pe.detail = "layer/" + nm + "/" + (win ? "win" : "x6") + "/" + std::to_string(p.mt) + "x" + std::to_string(p.pt) +
                    "g" + std::to_string(p.grid) + "u" + std::to_string(num.units) + "/g" + std::to_string(ng) + "/n" +
                    std::to_string(npix_all);
    }
    if (win) launch_conv_win_x6(a, h->stream);
    else launch_conv_x6(a, p.mt, p.pt, h->stream);
    h->prof_end(pe);
}

static void run_conv_x6_segs(opose_ctx* h, const std::vector<ConvSeg>& segs, bool pool) {
    if (segs.empty()) return;
    // kernel family and slab count per segment, frames of kKernelWinFrames segments as segments
    std::vector<ConvSeg> parts[3];  // conv_x6, conv_win_x6, conv_wino_x6
    for (const ConvSeg& s0 : segs) {
        ConvSeg sg = s0;
        const int kind = seg_kernel(h, sg, pool);
        const bool win = kind != kKernelX6;
        if (kind == kKernelWino) {
            sg.slabs = 1;
            parts[2].push_back(sg);
            continue;
        }
        if (!sg.slabs) sg.slabs = slab_count(h, sg.c, win, sg.N, sg.Hl ? sg.Hl : sg.H, sg.W, pool);
        if (kind == kKernelWinFrames) {
            for (int n = 0; n < sg.N; ++n) {
                ConvSeg f = sg;
                f.N = 1;
                f.in = frame_view(sg.in, n, sg.H, sg.W);
                f.out = frame_view(sg.out, n, sg.H, sg.W);
                f.dup = frame_view(sg.dup, n, sg.H, sg.W);
                parts[1].push_back(f);
            }
        } else {
            parts[win ? 1 : 0].push_back(sg);
        }
    }
    for (int k = 0; k < 3; ++k)
        for (size_t i = 0; i < parts[k].size(); i += kX6Groups)
            launch_segs(h,
                        std::vector<ConvSeg>(parts[k].begin() + i,
                                             parts[k].begin() + std::min(parts[k].size(), i + (size_t)kX6Groups)),
                        k == 0 ? kKernelX6 : k == 1 ? kKernelWin : kKernelWino, pool);
}

// A CPM stage's closing 1x1 pair (conv5_4 -> conv5_5, conv6_1 -> conv6_2, Mconv6 -> Mconv7) on one
// segment: out = c2(relu(c1(in))) (+ ReLU when relu2); `mid` holds c1's output when the pair runs
// as two launches.
struct ChainSeg {
    DevConv *c1, *c2;
    int N, H, W;
    XAct in, mid, out;
    bool relu2;
    int Hl = 0;  // ConvSeg::Hl of the two-launch form
};

// One launch of conv1x1_chain_x6 for every segment (the intermediate never leaves the CU), or,
// with OPOSE_FUSE_1X1=0 or a shape the kernel does not take, the two convs as separate launches
// through `mid`.
static void run_chain_x6(opose_ctx* h, const std::vector<ChainSeg>& segs) {
    // a small frame's 512-wide stage-1 pair (C2: 943 pixels, 15 workgroups of 64 pixels per
    // branch in the fused kernel, 42 us) runs as two launches over 128 x 64 tiles: the same sums
    // (1x1 convs never split k, the fused kernel rounds the intermediate like conv_x6's epilogue).
    // Not a hand pyramid's small scales: they share the fused launch of the large ones.
    auto small_pair = [&](const ChainSeg& sg) {
        return (long)sg.N * (sg.Hl ? sg.Hl : sg.H) * sg.W <= 4096 && sg.c1->cout >= 256 && sg.c1->net == OPOSE_NET_BODY;
    };
    {
        std::vector<ChainSeg> small, rest;
        for (const ChainSeg& sg : segs) (small_pair(sg) ? small : rest).push_back(sg);
        if (!small.empty() && !rest.empty()) {
            run_chain_x6(h, small);
            run_chain_x6(h, rest);
            return;
        }
    }
    bool fuse = h->fuse1x1 && !segs.empty() && segs.size() <= (size_t)kX6Groups && !small_pair(segs[0]);
    for (const ChainSeg& sg : segs) {
        const DevConv *c1 = sg.c1, *c2 = sg.c2;
        fuse = fuse && c1->ks == 1 && c2->ks == 1 && c1->cin_g == 16 && c1->cout == c1->Mpad && c1->Mpad % 128 == 0 &&
               c2->cin == c1->cout && c2->Mpad == 64 && c2->nK6 == c1->cout / 32 && !c1->small6 &&
               c1->cin_g == segs[0].c1->cin_g && c1->cout == segs[0].c1->cout;
    }
    if (!fuse) {
        std::vector<ConvSeg> first, second;
        for (const ChainSeg& sg : segs) {
            first.push_back(ConvSeg{sg.c1, sg.N, sg.H, sg.W, sg.in, sg.mid, XAct{}, true, sg.Hl});
            second.push_back(ConvSeg{sg.c2, sg.N, sg.H, sg.W, sg.mid, sg.out, XAct{}, sg.relu2, sg.Hl});
        }
        run_conv_x6_segs(h, first);
        run_conv_x6_segs(h, second);
        return;
    }
    X6ChainArgs a{};
    a.cin_g = segs[0].c1->cin_g;
    a.m1 = segs[0].c1->cout;
    a.ngroups = (int)segs.size();
    double flops = 0;
    long npix_all = 0;
    for (size_t g = 0; g < segs.size(); ++g) {
        const ChainSeg& sg = segs[g];
        X6ChainGroup& G = a.g[g];
        G.in = static_cast<const uint8_t*>(sg.in.p);
        G.in_ps = sg.in.ps;
        G.in_l = sg.in.l;
        G.w1 = sg.c1->wx6;
        G.b1 = sg.c1->bias;
        G.w2 = sg.c2->wx6;
        G.b2 = sg.c2->bias;
        G.out = sg.out.p;
        G.out_ps = sg.out.ps;
        G.out_l = sg.out.l;
        G.out_c = sg.out.c;
        G.out_off = sg.out.off;
        G.out_f32 = sg.out.f32 ? 1 : 0;
        G.cout2 = sg.c2->cout;
        G.relu2 = sg.relu2 ? 1 : 0;
        G.N = sg.N;
        G.H = sg.H;
        G.W = sg.W;
        G.npix = sg.N * sg.H * sg.W;
        npix_all += G.npix;
        flops += 2.0 * G.npix * ((double)sg.c1->cout * sg.c1->K + (double)sg.c2->cout * sg.c2->K);
    }
    ProfEntry pe;
    h->prof_begin(pe, "conv1x1", flops, 0);
    if (h->detail)
        pe.detail = "layer/" + segs[0].c1->name + ">" + segs[0].c2->name + "/chain/g" + std::to_string(a.ngroups) + "/n" +
                    std::to_string(npix_all);
    launch_conv1x1_chain_x6(a, h->stream);
    h->prof_end(pe);
}

// Zero the padding units of X6P buffers (cg groups each) for an N x H x W geometry.  The convs
// never write them, so a buffer stays valid for its geometry until a forward of another geometry
// writes pixels where this one has pads: clear only on a geometry change (or a reallocation),
// and then invalidate the captured graphs, whose replays assume their own geometry's pads are
// zero.  Inside a stream capture the clear becomes part of the graph (replayed every time) and
// the keys stay unset.
static void clear_x6p_pads(opose_ctx* h, std::initializer_list<std::pair<DevBuf*, int>> bufs, int N, int H, int W) {
    uint8_t* p[8];
    int planes[8];
    DevBuf* owner[8];
    int n = 0;
    for (const auto& b : bufs) {
        const uint64_t key = ((uint64_t)N << 40) ^ ((uint64_t)H << 20) ^ (uint64_t)W ^ ((uint64_t)b.second << 58) ^ 1u;
        if (b.first->pad_key == key) continue;
        p[n] = static_cast<uint8_t*>(b.first->p);
        planes[n] = 3 * b.second;
        owner[n] = b.first;
        ++n;
    }
    if (!n) return;
    ProfEntry pe;
    h->prof_begin(pe, "x6p_pads", 0, 0);
    launch_x6p_clear_pads(p, planes, n, N, H, W, h->stream);
    h->prof_end(pe);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    OPOSE_HIP_CHECK(hipStreamIsCapturing(h->stream, &cs));
    if (cs != hipStreamCaptureStatusNone) return;
    int i = 0;
    for (const auto& b : bufs) {
        const uint64_t key = ((uint64_t)N << 40) ^ ((uint64_t)H << 20) ^ (uint64_t)W ^ ((uint64_t)b.second << 58) ^ 1u;
        if (i < n && owner[i] == b.first) {
            b.first->pad_key = key;
            ++i;
        }
    }
    g_alloc_epoch.fetch_add(1);
}

// One scale of a network forward.  The scales of a pyramid (Hand()'s four, C5's) run in lockstep:
// layer by layer, one conv launch covers every scale (X6 groups with their own geometry), so a
// single crop's small layers share one grid instead of each filling a fraction of the chip.
struct NetSeg {
    const float* x;  // [N][3][Hp][Wp] fp32 network input
    int N, Hp, Wp;
    int slot;  // workspace set (opose_ctx::ws)
    int Hl = 0;  // the whole frame's input rows when x is a row band's rows (ConvSeg::Hl); 0: Hp
};

static void run_scales_concurrently(opose_ctx* h, int ns, const std::function<void(int)>& fn);

// VGG trunk on X6 activations: every segment's x -> its final trunk conv written via last[i]
// (+ dup[i]).  Full and half resolution run on dense X6 buffers (A / B); from the second pool on
// (H/4: conv3_x, H/8: conv4_x, conv5_x of the hand) the activations are padded X6P (P0 / P1,
// Q0 / Q1), which the windowed conv_win_x6 reads (conv_x6 reads either layout).
static void run_trunk_x6(opose_ctx* h, int net, const std::vector<NetSeg>& segs, const std::vector<XAct>& last,
                         const std::vector<XAct>& dup) {
    const std::vector<Spec> vgg = net == OPOSE_NET_BODY ? vgg_body() : vgg_hand();
    const size_t ns = segs.size();
    // padded levels (fused pooling only: the separate maxpool_x6 reads and writes dense X6)
    const bool padded = h->fused_pool;
    int maxg4 = 0, maxg8 = 0;  // widest activation (groups) at H/4 and H/8
    {
        int lvl = 0;
        for (const Spec& s : vgg) {
            const int og = (s.cout + 7) / 8;
            const bool pooled = s.name == "conv1_2" || s.name == "conv2_2" || s.name == "conv3_4";
            const int out_lvl = lvl + (pooled ? 1 : 0);
            if (out_lvl == 2) maxg4 = std::max(maxg4, og);
            if (out_lvl == 3) maxg8 = std::max(maxg8, og);
            lvl = out_lvl;
        }
    }
    struct Bufs {
        uint8_t *A, *B, *P0, *P1, *Q0, *Q1;
        XAct cur;
    };
    std::vector<Bufs> bs(ns);
    for (size_t i = 0; i < ns; ++i) {
        const NetSeg& sg = segs[i];
        auto& w = h->ws[sg.slot];
        const int N = sg.N, H = sg.Hp, W = sg.Wp;
        const size_t act = (size_t)N * H * W * 8 * 16 * 3;  // 64 channels at full resolution: the largest dense tensor
        Bufs& b = bs[i];
        b.A = w.x6A.ensure<uint8_t>(act, h->stream);
        b.B = w.x6B.ensure<uint8_t>(act, h->stream);
        b.P0 = b.P1 = b.Q0 = b.Q1 = nullptr;
        if (padded) {
            const int H4 = H / 4, W4 = W / 4, H8 = H / 8, W8 = W / 8;
            b.P0 = w.x6P0.ensure<uint8_t>(x6p_plane(N, H4, W4) * maxg4 * 48, h->stream);
            b.P1 = w.x6P1.ensure<uint8_t>(x6p_plane(N, H4, W4) * maxg4 * 48, h->stream);
            b.Q0 = w.x6Q0.ensure<uint8_t>(x6p_plane(N, H8, W8) * maxg8 * 48, h->stream);
            b.Q1 = w.x6Q1.ensure<uint8_t>(x6p_plane(N, H8, W8) * maxg8 * 48, h->stream);
            clear_x6p_pads(h, {{&w.x6P0, maxg4}, {&w.x6P1, maxg4}}, N, H4, W4);
            clear_x6p_pads(h, {{&w.x6Q0, maxg8}, {&w.x6Q1, maxg8}}, N, H8, W8);
        }
    }
    // output buffer of segment i for a layer at resolution level `lvl` (0: H, 1: H/2, 2: H/4,
    // 3: H/8), not the one its input is in
    auto out_buf = [&](size_t i, int lvl, int og) -> XAct {
        const Bufs& b = bs[i];
        const void* avoid = b.cur.p;
        const int N = segs[i].N, hh = segs[i].Hp >> lvl, ww = segs[i].Wp >> lvl;
        if (!padded || lvl < 2) return x6act(avoid == b.A ? b.B : b.A, og, 0, N, hh, ww);
        uint8_t* p = lvl == 2 ? (avoid == b.P0 ? b.P1 : b.P0) : (avoid == b.Q0 ? b.Q1 : b.Q0);
        return x6pact(p, og, 0, N, hh, ww);
    };
    // conv1_1 straight from the fp32 input (conv_first_x6, no input split) of segment i; f32: its
    // output as fp32 units for the windowed conv1_2, which splits them itself
    auto conv11_direct = [&](size_t i, const Spec& s, DevConv* c, bool f32) {
        const NetSeg& sg = segs[i];
        const size_t npix = (size_t)sg.N * sg.Hp * sg.Wp;
        ProfEntry pe;
        h->prof_begin(pe, "conv3x3", 2.0 * 64 * 27 * (double)npix, 0);
        if (h->detail) pe.detail = "layer/" + s.name + "/first_direct/n" + std::to_string(npix);
        launch_conv_first_x6(sg.x, sg.N, 3, sg.Hp, sg.Wp, c->wt, c->Mpad, c->bias, bs[i].A, (uint32_t)(npix * 8 * 16),
                             f32, h->stream);
        h->prof_end(pe);
        bs[i].cur = x6act(bs[i].A, 8, 0, sg.N, sg.Hp, sg.Wp);
        bs[i].cur.f32 = f32;  // (fp32 units at the X6 unit addresses x 2)
    };
    // conv1_2 + pool with the input window in LDS instead of the 9-tap im2col stream (segment i,
    // input at resolution level lvl)
    auto conv12_win_ok = [&](const Spec& s, const DevConv* c) {
        return h->fused_pool && h->win12 && s.name == "conv1_2" && c->cin == 64 && c->cout == 64 && c->ks == 3 &&
               c->pad == 1 && c->Mpad == 64 && c->nK6 == 18 && !c->small6;
    };
    auto conv12_win = [&](size_t i, const Spec& s, DevConv* c, int lvl) {
        const NetSeg& sg = segs[i];
        const int og = (s.cout + 7) / 8;
        const int hh = sg.Hp >> lvl, ww = sg.Wp >> lvl;
        if (bs[i].cur.padded || bs[i].cur.l.fs != 8u * hh * ww) throw std::logic_error("conv1_2 input layout");
        const size_t np = (size_t)sg.N * hh * ww, npo = (size_t)sg.N * (hh / 2) * (ww / 2);
        const XAct out = out_buf(i, lvl + 1, og);
        ProfEntry pe;
        h->prof_begin(pe, "conv3x3", 2.0 * 64 * 576 * (double)(npo * 4), 0);
        if (h->detail) pe.detail = "layer/" + s.name + "/x6win/n" + std::to_string(npo * 4);
        launch_conv3_pool_win_x6(static_cast<const uint8_t*>(bs[i].cur.p), (uint32_t)(np * 8 * 16), sg.N, hh, ww,
                                 c->wx6, c->bias, static_cast<uint8_t*>(out.p), (uint32_t)(npo * 8 * 16),
                                 bs[i].cur.f32, h->stream);
        h->prof_end(pe);
        bs[i].cur = out;
    };
    int lvl = 0;
    for (size_t li = 0; li < vgg.size(); ++li) {
        const Spec& s = vgg[li];
        DevConv* c = find_conv(h, net, s.name);
        if (h->gate_ev && s.name == gate_layer()) {  // OPOSE_PIPELINE_DEFER: the previous post may start
            OPOSE_HIP_CHECK(hipEventRecord(h->gate_ev, h->stream));
            h->gate_done = true;
        }
        if (li == 0 && s.cin == 3 && s.cout == 64 && s.ks == 3 && s.pad == 1 && vgg.size() > 1 && h->first_direct) {
            DevConv* c2 = find_conv(h, net, vgg[1].name);
            const bool pair12 = conv12_win_ok(vgg[1], c2);
            const bool f32 = pair12 && h->c11_f32;
            if (ns > 1 && ns <= (size_t)kConv1Segs && pair12) {
                // a pyramid's conv1_1 and conv1_2 as one launch each over every segment: the
                // small scales' tiles fill the large scale's tail (round 3 ran the per-scale
                // chains on concurrent streams, which a captured graph may not fork any more)
                Conv1Segs S1{}, S2{};
                S1.n = S2.n = (int)ns;
                double f1 = 0, f2 = 0;
                long px1 = 0, px2 = 0;
                for (size_t i = 0; i < ns; ++i) {
                    const NetSeg& sg = segs[i];
                    const size_t npix = (size_t)sg.N * sg.Hp * sg.Wp;
                    const size_t npo = (size_t)sg.N * (sg.Hp / 2) * (sg.Wp / 2);
                    bs[i].cur = x6act(bs[i].A, 8, 0, sg.N, sg.Hp, sg.Wp);  // conv1_1's output
                    const XAct o2 = out_buf(i, 1, 8);                        // (not A)
                    if (o2.p == bs[i].A) throw std::logic_error("conv1_2 output aliases its input");
                    S1.s[i] = Conv1Seg{sg.x, bs[i].A, 0u, (uint32_t)(npix * 8 * 16), sg.N, sg.Hp, sg.Wp, 0};
                    S2.s[i] = Conv1Seg{bs[i].A, static_cast<uint8_t*>(o2.p), (uint32_t)(npix * 8 * 16),
                                       (uint32_t)(npo * 8 * 16), sg.N, sg.Hp, sg.Wp, 0};
                    f1 += 2.0 * 64 * 27 * (double)npix;
                    f2 += 2.0 * 64 * 576 * (double)(npo * 4);
                    px1 += (long)npix;
                    px2 += (long)npo * 4;
                    bs[i].cur = o2;
                }
                ProfEntry pe;
                h->prof_begin(pe, "conv3x3", f1, 0);
                if (h->detail) pe.detail = "layer/" + s.name + "/first_direct/g" + std::to_string(ns) + "/n" + std::to_string(px1);
                launch_conv_first_x6_segs(S1, c->wt, c->Mpad, c->bias, f32, h->stream);
                h->prof_end(pe);
                h->prof_begin(pe, "conv3x3", f2, 0);
                if (h->detail) pe.detail = "layer/" + vgg[1].name + "/x6win/g" + std::to_string(ns) + "/n" + std::to_string(px2);
                launch_conv3_pool_win_x6_segs(S2, c2->wx6, c2->bias, f32, h->stream);
                h->prof_end(pe);
                ++li;
                ++lvl;
                continue;
            }
            for (size_t i = 0; i < ns; ++i) conv11_direct(i, s, c, f32);
            continue;
        }
        if (li == 0) {
            for (size_t i = 0; i < ns; ++i) {
                const NetSeg& sg = segs[i];
                const size_t npix = (size_t)sg.N * sg.Hp * sg.Wp;
                uint8_t* X = h->ws[sg.slot].x6in.ensure<uint8_t>(npix * 16 * 3, h->stream);
                ProfEntry pe;
                h->prof_begin(pe, "to_x6", 0, (double)npix * (12 + 48));
                launch_to_x6(sg.x, 3, 0, 3, sg.N, sg.Hp * sg.Wp, X, 1, 0, (uint32_t)(npix * 16), h->stream);
                h->prof_end(pe);
                bs[i].cur = x6act(X, 1, 0, sg.N, sg.Hp, sg.Wp);
            }
        }
        const bool final_layer = li + 1 == vgg.size();
        const int og = (s.cout + 7) / 8;
        const bool pooled = s.name == "conv1_2" || s.name == "conv2_2" || s.name == "conv3_4";
        if (pooled && conv12_win_ok(s, c)) {
            for (size_t i = 0; i < ns; ++i) conv12_win(i, s, c, lvl);
            ++lvl;
            continue;
        }
        std::vector<ConvSeg> cs;
        std::vector<XAct> outs;
        const bool fuse = pooled && h->fused_pool;  // conv + MaxPool2d(2, 2) in one launch
        for (size_t i = 0; i < ns; ++i) {
            const NetSeg& sg = segs[i];
            const XAct out = fuse ? out_buf(i, lvl + 1, og) : final_layer ? last[i] : out_buf(i, lvl, og);
            outs.push_back(out);
            cs.push_back(ConvSeg{c, sg.N, sg.Hp >> lvl, sg.Wp >> lvl, bs[i].cur, out,
                                 final_layer && !fuse ? dup[i] : XAct{}, true, sg.Hl >> lvl});
        }
        run_conv_x6_segs(h, cs, fuse);
        for (size_t i = 0; i < ns; ++i) bs[i].cur = outs[i];
        if (fuse) {
            ++lvl;
            continue;
        }
        if (pooled) {  // separate MaxPool2d(2, 2) (fused_pool off: dense buffers throughout)
            for (size_t i = 0; i < ns; ++i) {
                const NetSeg& sg = segs[i];
                const int hh = sg.Hp >> lvl, ww = sg.Wp >> lvl;
                const size_t np = (size_t)sg.N * hh * ww;
                Bufs& b = bs[i];
                const XAct pd = x6act(b.cur.p == b.A ? b.B : b.A, og, 0, sg.N, hh / 2, ww / 2);
                ProfEntry pe;
                h->prof_begin(pe, "maxpool", 0, (double)np * og * 48 * 1.25);
                launch_maxpool_x6(static_cast<const uint8_t*>(b.cur.p), (uint32_t)(np * og * 16),
                                  static_cast<uint8_t*>(pd.p), (uint32_t)((size_t)sg.N * (hh / 2) * (ww / 2) * og * 16),
                                  sg.N * og, hh, ww, h->stream);
                h->prof_end(pe);
                b.cur = pd;
            }
            ++lvl;
        }
    }
}

// Output rows [r0, r1) of one frame's CPM stages (opose_body_band_maps).  The stage buffers keep
// the whole frame's geometry; every stage layer runs on a view of the band's rows (X6P origin
// moved down r0 rows), whose padding rows are the neighbouring bands' rows: band_halo refreshes
// them before each 3x3 / 7x7 layer that reads them.  The trunk before the stages runs on the
// band's rows plus kBandTrunkMargin rows past each cut (recomputed, not exchanged).  Every conv of
// the band sums each pixel in the order of the whole frame's (ConvSeg::Hl = the frame's rows), so
// the band's maps are the whole frame's rows bit for bit.
struct Band {
    int r0, r1;
    float* maps;  // [57][r1 - r0][wl] fp32 device
    opose_halo_fn fn;  // nullptr: the library's RCCL send / recv (opose_rccl_init)
    void* user;
    uint8_t* xbuf;  // [send_up | send_dn | recv_up | recv_dn], cap bytes each
    size_t cap;
};

// output rows of a band's trunk past each cut edge (engine body_net_x6; src/dist.py BAND_MARGIN)
constexpr int kBandTrunkMargin = 10;

// bytes of one direction of a band's halo exchange at wl columns: 3 pieces x 32 groups (the
// widest stage tensor, 256 channels) x 3 rows x P units x 16 B
static size_t band_halo_bytes(int wl) { return (size_t)3 * 32 * 3 * x6p_pitch(wl) * 16; }

// bodypose_model.forward on X6 activations, every segment in lockstep; per segment the fp32
// output in its slot's S0 with the fp32 path's layout (channel stride 185: paf [0,38), heat [38,57)).
// band: one segment of one frame, stages on rows [band->r0, band->r1) only, output in band->maps.
static std::vector<float*> body_net_x6(opose_ctx* h, const std::vector<NetSeg>& segs, const Band* band = nullptr) {
    const int SG = 24, TG = 32, UG = 128;  // [L1 | L2 | trunk] = 5 + 3 + 16 groups; 256 / 1024 channels
    const int net = OPOSE_NET_BODY;
    const size_t ns = segs.size();
    // per segment: S (stage inputs) and T (branch activations): padded X6P, read by the 7x7 / 3x3
    // convs; U (conv5_4 output, read by the 1x1 conv5_5): dense
    struct Bufs {
        uint8_t *S[2], *T[2], *U;
        float* O;
        int N, hl, wl;
    };
    std::vector<Bufs> bs(ns);
    std::vector<XAct> last, dup;
    for (size_t i = 0; i < ns; ++i) {
        auto& w = h->ws[segs[i].slot];
        Bufs& b = bs[i];
        b.N = segs[i].N;
        b.hl = segs[i].Hp / 8;
        b.wl = segs[i].Wp / 8;
        const size_t px = (size_t)b.N * b.hl * b.wl, plane = x6p_plane(b.N, b.hl, b.wl);
        b.S[0] = w.x6S0.ensure<uint8_t>(plane * SG * 48, h->stream);
        b.S[1] = w.x6S1.ensure<uint8_t>(plane * SG * 48, h->stream);
        b.T[0] = w.x6T0.ensure<uint8_t>(plane * TG * 48, h->stream);
        b.T[1] = w.x6T1.ensure<uint8_t>(plane * TG * 48, h->stream);
        b.U = w.x6U.ensure<uint8_t>(px * UG * 48, h->stream);
        b.O = w.S0.ensure<float>(px * 185, h->stream);
        clear_x6p_pads(h, {{&w.x6S0, SG}, {&w.x6S1, SG}, {&w.x6T0, TG}, {&w.x6T1, TG}}, b.N, b.hl, b.wl);
        last.push_back(x6pact(b.S[0], SG, 8, b.N, b.hl, b.wl));
        dup.push_back(x6pact(b.S[1], SG, 8, b.N, b.hl, b.wl));
    }
    if (band && (ns != 1 || bs[0].N != 1 || band->r0 < 0 || band->r1 > bs[0].hl || band->r1 - band->r0 < 3))
        throw std::invalid_argument("row band: one frame, 3 <= r1 - r0 rows inside the map");
    // rows a stage layer computes, and the band view of a full-height X6P activation
    const int hb = band ? band->r1 - band->r0 : 0;
    auto rows = [&](size_t i) { return band ? hb : bs[i].hl; };
    auto bview = [&](XAct a) {
        if (band) {
            a.l.o0 += (uint32_t)band->r0 * a.l.rs;
            a.l.fs = (uint32_t)(hb + 3) * a.l.rs;
            a.ylo = band->r0 > 0 ? -3 : 0;
            a.yhi = band->r1 < bs[0].hl ? hb + 3 : hb;
        }
        return a;
    };
    auto s_ = [&](size_t i, int k, int goff) { return bview(x6pact(bs[i].S[k], SG, goff, bs[i].N, bs[i].hl, bs[i].wl)); };
    auto t_ = [&](size_t i, int k, int goff) { return bview(x6pact(bs[i].T[k], TG, goff, bs[i].N, bs[i].hl, bs[i].wl)); };
    auto u_ = [&](size_t i, int goff) { return x6act(bs[i].U, UG, goff, bs[i].N, rows(i), bs[i].wl); };
    // band edges: send the band's first / last 3 rows of groups [g0, g0 + ng) of X6P buffer buf
    // (cg groups) up / down, receive the neighbours' rows into the rows above / below the band
    auto band_halo = [&](uint8_t* buf, int cg, int g0, int ng) {
        if (!band) return;
        const int hl = bs[0].hl, P = x6p_pitch(bs[0].wl);
        const size_t plane = x6p_plane(1, hl, bs[0].wl), bytes = (size_t)9 * ng * P * 16;
        const int mask = (band->r0 > 0 ? 1 : 0) | (band->r1 < hl ? 2 : 0);
        if (!mask) return;
        if (bytes > band->cap) throw std::invalid_argument("row band: halo buffer too small");
        const uint32_t ps = checked_ps((size_t)cg * plane * 16);
        uint8_t* x = band->xbuf;
        const size_t c = band->cap;
        ProfEntry pe;
        h->prof_begin(pe, "band_halo", 0, 4.0 * (double)bytes);
        launch_x6p_halo(buf, ps, (uint32_t)plane, g0, ng, P, 3 + band->r0, band->r1, x, x + c, mask, false, h->stream);
        if (!band->fn) {  // the library's own exchange: RCCL P2P on the handle's stream
            const Rccl& R = rccl();
            rccl_check(R.group_start());
            if (mask & 1) {
                rccl_check(R.send(x, bytes, ncclUint8, h->band_up, h->comm, h->stream));
                rccl_check(R.recv(x + 2 * c, bytes, ncclUint8, h->band_up, h->comm, h->stream));
            }
            if (mask & 2) {
                rccl_check(R.send(x + c, bytes, ncclUint8, h->band_dn, h->comm, h->stream));
                rccl_check(R.recv(x + 3 * c, bytes, ncclUint8, h->band_dn, h->comm, h->stream));
            }
            rccl_check(R.group_end());
        } else if (band->fn(band->user, bytes, h->stream) != 0) {
            throw std::runtime_error("row band: halo exchange failed");
        }
        launch_x6p_halo(buf, ps, (uint32_t)plane, g0, ng, P, band->r0, 3 + band->r1, x + 2 * c, x + 3 * c, mask, true,
                        h->stream);
        h->prof_end(pe);
    };
    // one layer over every segment: branch L1 (conv c1) and, when c2, branch L2
    auto layer = [&](const std::string& n1, const std::string& n2, const std::function<XAct(size_t)>& in1,
                     const std::function<XAct(size_t)>& out1, const std::function<XAct(size_t)>& in2,
                     const std::function<XAct(size_t)>& out2, bool relu1, bool relu2) {
        DevConv* c1 = find_conv(h, net, n1);
        DevConv* c2 = n2.empty() ? nullptr : find_conv(h, net, n2);
        std::vector<ConvSeg> cs;
        for (size_t i = 0; i < ns; ++i) {
            cs.push_back(ConvSeg{c1, bs[i].N, rows(i), bs[i].wl, in1(i), out1(i), XAct{}, relu1, bs[i].hl});
            if (c2) cs.push_back(ConvSeg{c2, bs[i].N, rows(i), bs[i].wl, in2(i), out2(i), XAct{}, relu2, bs[i].hl});
        }
        run_conv_x6_segs(h, cs);
    };
    auto none = [](size_t) { return XAct{}; };
    if (band) {
        // the band's trunk on the input rows its stages need: out1 rows [r0 - 3, r1 + 3) (the 7x7
        // Mconv1 halo) plus kBandTrunkMargin - 3 rows that a cut edge's zero padding corrupts
        // (1 + 1 rows at H, 2 at H/2, 4 at H/4, 4 at H/8: 6.75 rows at H/8); rows a multiple of 8
        // so the three pools see the whole frame's 2x2 windows
        const int hl = bs[0].hl, Wp = segs[0].Wp, Hp = segs[0].Hp;
        const int a = std::max(0, band->r0 - kBandTrunkMargin), b = std::min(hl, band->r1 + kBandTrunkMargin);
        const int Hs = 8 * (b - a);
        float* xs = h->ws[segs[0].slot].xband.ensure<float>((size_t)3 * Hs * Wp, h->stream);
        OPOSE_HIP_CHECK(hipMemcpy2DAsync(xs, (size_t)Hs * Wp * 4, segs[0].x + (size_t)8 * a * Wp, (size_t)Hp * Wp * 4,
                                         (size_t)Hs * Wp * 4, 3, hipMemcpyDeviceToDevice, h->stream));
        auto sub = [&](XAct v) {
            v.l.o0 += (uint32_t)a * v.l.rs;
            v.l.fs = (uint32_t)(b - a + 3) * v.l.rs;
            return v;
        };
        run_trunk_x6(h, net, {NetSeg{xs, 1, Hs, Wp, segs[0].slot, Hp}}, {sub(last[0])}, {sub(dup[0])});
    } else {
        run_trunk_x6(h, net, segs, last, dup);
    }
    layer("conv5_1_CPM_L1+L2", "", [&](size_t i) { return s_(i, 0, 8); }, [&](size_t i) { return t_(i, 0, 0); }, none,
          none, true, false);
    band_halo(bs[0].T[0], TG, 0, TG);
    layer("conv5_2_CPM_L1", "conv5_2_CPM_L2", [&](size_t i) { return t_(i, 0, 0); },
          [&](size_t i) { return t_(i, 1, 0); }, [&](size_t i) { return t_(i, 0, 16); },
          [&](size_t i) { return t_(i, 1, 16); }, true, true);
    band_halo(bs[0].T[1], TG, 0, TG);
    layer("conv5_3_CPM_L1", "conv5_3_CPM_L2", [&](size_t i) { return t_(i, 1, 0); },
          [&](size_t i) { return t_(i, 0, 0); }, [&](size_t i) { return t_(i, 1, 16); },
          [&](size_t i) { return t_(i, 0, 16); }, true, true);
    // 1x1 pairs of both branches and every segment: L1 then L2 of each segment
    auto chain = [&](const std::string& a1, const std::string& a2, const std::string& b1, const std::string& b2,
                     const std::function<ChainSeg(size_t, int, DevConv*, DevConv*)>& mk) {
        DevConv *ca1 = find_conv(h, net, a1), *ca2 = find_conv(h, net, a2);
        DevConv *cb1 = find_conv(h, net, b1), *cb2 = find_conv(h, net, b2);
        std::vector<ChainSeg> cs;
        for (size_t i = 0; i < ns; ++i) {
            cs.push_back(mk(i, 0, ca1, ca2));
            cs.push_back(mk(i, 1, cb1, cb2));
        }
        run_chain_x6(h, cs);
    };
    chain("conv5_4_CPM_L1", "conv5_5_CPM_L1", "conv5_4_CPM_L2", "conv5_5_CPM_L2",
          [&](size_t i, int br, DevConv* c1, DevConv* c2) {
              return ChainSeg{c1, c2, bs[i].N, rows(i), bs[i].wl, t_(i, 0, br ? 16 : 0), u_(i, br ? 64 : 0),
                              s_(i, 1, br ? 5 : 0), false, bs[i].hl};
          });
    band_halo(bs[0].S[1], SG, 0, 8);
    int cur = 1;
    for (int st = 2; st <= 6; ++st) {
        const std::string sf = "_stage" + std::to_string(st);
        if (h->gate_ev && gate_layer() == "stage" + std::to_string(st)) {
            OPOSE_HIP_CHECK(hipEventRecord(h->gate_ev, h->stream));
            h->gate_done = true;
        }
        layer("Mconv1" + sf + "_L1+L2", "", [&](size_t i) { return s_(i, cur, 0); },
              [&](size_t i) { return t_(i, 0, 0); }, none, none, true, false);
        int t = 0;
        for (int k = 2; k <= 5; ++k) {
            band_halo(bs[0].T[t], TG, 0, TG);  // Mconv2..5 read 3 rows past the band
            const std::string nm = "Mconv" + std::to_string(k) + sf;
            layer(nm + "_L1", nm + "_L2", [&](size_t i) { return t_(i, t, 0); },
                  [&](size_t i) { return t_(i, t ^ 1, 0); }, [&](size_t i) { return t_(i, t, 16); },
                  [&](size_t i) { return t_(i, t ^ 1, 16); }, true, true);
            t ^= 1;
        }
        // Mconv6 -> Mconv7; Mconv7: no ReLU, except Mconv7_stage6_L2 (no_relu list quirk,
        // src/model.py:30-33)
        chain("Mconv6" + sf + "_L1", "Mconv7" + sf + "_L1", "Mconv6" + sf + "_L2", "Mconv7" + sf + "_L2",
              [&](size_t i, int br, DevConv* c1, DevConv* c2) {
                  const XAct o = st < 6 ? s_(i, cur ^ 1, br ? 5 : 0)
                                 : band ? f32act(band->maps, 57, br ? 38 : 0) : f32act(bs[i].O, 185, br ? 38 : 0);
                  return ChainSeg{c1, c2, bs[i].N, rows(i), bs[i].wl, t_(i, t, br ? 16 : 0), t_(i, t ^ 1, br ? 16 : 0), o,
                                  br == 1 && st == 6, bs[i].hl};
              });
        if (st < 6) band_halo(bs[0].S[cur ^ 1], SG, 0, 8);  // the next Mconv1 (7x7) reads them
        cur ^= 1;
    }
    std::vector<float*> outs;
    for (const Bufs& b : bs) outs.push_back(b.O);
    return outs;
}

// handpose_model.forward on X6 activations, every segment in lockstep; per segment the fp32
// output in its slot's S0, channel stride 150 (heat [0,22))
static std::vector<float*> hand_net_x6(opose_ctx* h, const std::vector<NetSeg>& segs) {
    const int SG = 19, TG = 16, UG = 64;  // [L 22 + 2 | trunk 128] = 3 + 16 groups; 128 / 512 channels
    const int net = OPOSE_NET_HAND;
    const size_t ns = segs.size();
    struct Bufs {
        uint8_t *S[2], *T[2], *U;
        float* O;
        int N, hl, wl;
    };
    std::vector<Bufs> bs(ns);
    std::vector<XAct> last, dup;
    for (size_t i = 0; i < ns; ++i) {
        auto& w = h->ws[segs[i].slot];
        Bufs& b = bs[i];
        b.N = segs[i].N;
        b.hl = segs[i].Hp / 8;
        b.wl = segs[i].Wp / 8;
        const size_t px = (size_t)b.N * b.hl * b.wl, plane = x6p_plane(b.N, b.hl, b.wl);
        b.S[0] = w.x6S0.ensure<uint8_t>(plane * SG * 48, h->stream);
        b.S[1] = w.x6S1.ensure<uint8_t>(plane * SG * 48, h->stream);
        b.T[0] = w.x6T0.ensure<uint8_t>(plane * TG * 48, h->stream);
        b.T[1] = w.x6T1.ensure<uint8_t>(plane * TG * 48, h->stream);
        b.U = w.x6U.ensure<uint8_t>(px * UG * 48, h->stream);
        b.O = w.S0.ensure<float>(px * 150, h->stream);
        clear_x6p_pads(h, {{&w.x6S0, SG}, {&w.x6S1, SG}, {&w.x6T0, TG}, {&w.x6T1, TG}}, b.N, b.hl, b.wl);
        last.push_back(x6pact(b.S[0], SG, 3, b.N, b.hl, b.wl));
        dup.push_back(x6pact(b.S[1], SG, 3, b.N, b.hl, b.wl));
    }
    auto s_ = [&](size_t i, int k, int goff) { return x6pact(bs[i].S[k], SG, goff, bs[i].N, bs[i].hl, bs[i].wl); };
    auto t_ = [&](size_t i, int k) { return x6pact(bs[i].T[k], TG, 0, bs[i].N, bs[i].hl, bs[i].wl); };
    auto u_ = [&](size_t i) { return x6act(bs[i].U, UG, 0, bs[i].N, bs[i].hl, bs[i].wl); };
    auto layer = [&](const std::string& name, const std::function<XAct(size_t)>& in,
                     const std::function<XAct(size_t)>& out, bool relu) {
        DevConv* c = find_conv(h, net, name);
        std::vector<ConvSeg> cs;
        for (size_t i = 0; i < ns; ++i) cs.push_back(ConvSeg{c, bs[i].N, bs[i].hl, bs[i].wl, in(i), out(i), XAct{}, relu});
        run_conv_x6_segs(h, cs);
    };
    auto chain = [&](const std::string& n1, const std::string& n2, const std::function<ChainSeg(size_t, DevConv*, DevConv*)>& mk) {
        DevConv *c1 = find_conv(h, net, n1), *c2 = find_conv(h, net, n2);
        std::vector<ChainSeg> cs;
        for (size_t i = 0; i < ns; ++i) cs.push_back(mk(i, c1, c2));
        run_chain_x6(h, cs);
    };
    run_trunk_x6(h, net, segs, last, dup);
    chain("conv6_1_CPM", "conv6_2_CPM", [&](size_t i, DevConv* c1, DevConv* c2) {
        return ChainSeg{c1, c2, bs[i].N, bs[i].hl, bs[i].wl, s_(i, 0, 3), u_(i), s_(i, 1, 0), false};
    });
    int cur = 1;
    for (int st = 2; st <= 6; ++st) {
        const std::string sf = "_stage" + std::to_string(st);
        layer("Mconv1" + sf, [&](size_t i) { return s_(i, cur, 0); }, [&](size_t i) { return t_(i, 0); }, true);
        int t = 0;
        for (int k = 2; k <= 5; ++k) {
            layer("Mconv" + std::to_string(k) + sf, [&](size_t i) { return t_(i, t); },
                  [&](size_t i) { return t_(i, t ^ 1); }, true);
            t ^= 1;
        }
        chain("Mconv6" + sf, "Mconv7" + sf, [&](size_t i, DevConv* c1, DevConv* c2) {
            const XAct o = st == 6 ? f32act(bs[i].O, 150, 0) : s_(i, cur ^ 1, 0);
            return ChainSeg{c1, c2, bs[i].N, bs[i].hl, bs[i].wl, t_(i, t), t_(i, t ^ 1), o, false};
        });
        cur ^= 1;
    }
    std::vector<float*> outs;
    for (const Bufs& b : bs) outs.push_back(b.O);
    return outs;
}

// bodypose_model.forward (src/model.py:106-133). Output: S-buffer with paf [0,38), heat [38,57)
static float* body_net(opose_ctx* h, const float* x, int N, int Hp, int Wp) {
    if (!h->loaded[OPOSE_NET_BODY]) throw std::runtime_error("body weights not loaded");
    if (h->x6) return body_net_x6(h, {NetSeg{x, N, Hp, Wp, h->slot}})[0];
    const int hl = Hp / 8, wl = Wp / 8;
    const size_t px = (size_t)N * hl * wl;
    float* S[2] = {h->w().S0.ensure<float>(px * 185, h->stream), h->w().S1.ensure<float>(px * 185, h->stream)};
    float* T[2] = {h->w().T0.ensure<float>(px * 256, h->stream), h->w().T1.ensure<float>(px * 256, h->stream)};
    float* U = h->w().U.ensure<float>(px * 1024, h->stream);
    const int net = OPOSE_NET_BODY;
    run_trunk(h, net, x, N, Hp, Wp, Act{S[0], 185, 57}, Act{S[1], 185, 57});
    // stage 1 (src/model.py:52-62): input = trunk slice of S0
    run_conv(h, find_conv(h, net, "conv5_1_CPM_L1+L2"), nullptr, N, hl, wl, Act{S[0], 185, 57}, Act{T[0], 256, 0},
             Act{}, Act{}, true, false);
    run_conv(h, find_conv(h, net, "conv5_2_CPM_L1"), find_conv(h, net, "conv5_2_CPM_L2"), N, hl, wl,
             Act{T[0], 256, 0}, Act{T[1], 256, 0}, Act{T[0], 256, 128}, Act{T[1], 256, 128}, true, true);
    run_conv(h, find_conv(h, net, "conv5_3_CPM_L1"), find_conv(h, net, "conv5_3_CPM_L2"), N, hl, wl,
             Act{T[1], 256, 0}, Act{T[0], 256, 0}, Act{T[1], 256, 128}, Act{T[0], 256, 128}, true, true);
    run_conv(h, find_conv(h, net, "conv5_4_CPM_L1"), find_conv(h, net, "conv5_4_CPM_L2"), N, hl, wl,
             Act{T[0], 256, 0}, Act{U, 1024, 0}, Act{T[0], 256, 128}, Act{U, 1024, 512}, true, true);
    run_conv(h, find_conv(h, net, "conv5_5_CPM_L1"), find_conv(h, net, "conv5_5_CPM_L2"), N, hl, wl,
             Act{U, 1024, 0}, Act{S[1], 185, 0}, Act{U, 1024, 512}, Act{S[1], 185, 38}, false, false);
    int cur = 1;
    for (int st = 2; st <= 6; ++st) {
        const std::string s = "_stage" + std::to_string(st);
        float* in = S[cur];
        float* out = S[cur ^ 1];
        run_conv(h, find_conv(h, net, "Mconv1" + s + "_L1+L2"), nullptr, N, hl, wl, Act{in, 185, 0},
                 Act{T[0], 256, 0}, Act{}, Act{}, true, false);
        int t = 0;
        for (int i = 2; i <= 6; ++i) {
            const std::string nm = "Mconv" + std::to_string(i) + s;
            run_conv(h, find_conv(h, net, nm + "_L1"), find_conv(h, net, nm + "_L2"), N, hl, wl, Act{T[t], 256, 0},
                     Act{T[t ^ 1], 256, 0}, Act{T[t], 256, 128}, Act{T[t ^ 1], 256, 128}, true, true);
            t ^= 1;
        }
        // Mconv7: no ReLU, except Mconv7_stage6_L2 (no_relu list quirk, src/model.py:30-33)
        run_conv(h, find_conv(h, net, "Mconv7" + s + "_L1"), find_conv(h, net, "Mconv7" + s + "_L2"), N, hl, wl,
                 Act{T[t], 256, 0}, Act{out, 185, 0}, Act{T[t], 256, 128}, Act{out, 185, 38}, false, st == 6);
        cur ^= 1;
    }
    return S[cur];
}

// handpose_model.forward (src/model.py:197-214). Output: S-buffer with heat [0,22)
static float* hand_net(opose_ctx* h, const float* x, int N, int Hp, int Wp) {
    if (!h->loaded[OPOSE_NET_HAND]) throw std::runtime_error("hand weights not loaded");
    if (h->x6) return hand_net_x6(h, {NetSeg{x, N, Hp, Wp, h->slot}})[0];
    const int hl = Hp / 8, wl = Wp / 8;
    const size_t px = (size_t)N * hl * wl;
    float* S[2] = {h->w().S0.ensure<float>(px * 150, h->stream), h->w().S1.ensure<float>(px * 150, h->stream)};
    float* T[2] = {h->w().T0.ensure<float>(px * 128, h->stream), h->w().T1.ensure<float>(px * 128, h->stream)};
    float* U = h->w().U.ensure<float>(px * 512, h->stream);
    const int net = OPOSE_NET_HAND;
    run_trunk(h, net, x, N, Hp, Wp, Act{S[0], 150, 22}, Act{S[1], 150, 22});
    run_conv(h, find_conv(h, net, "conv6_1_CPM"), nullptr, N, hl, wl, Act{S[0], 150, 22}, Act{U, 512, 0}, Act{},
             Act{}, true, false);
    run_conv(h, find_conv(h, net, "conv6_2_CPM"), nullptr, N, hl, wl, Act{U, 512, 0}, Act{S[1], 150, 0}, Act{},
             Act{}, false, false);
    int cur = 1;
    for (int st = 2; st <= 6; ++st) {
        const std::string s = "_stage" + std::to_string(st);
        float* in = S[cur];
        float* out = S[cur ^ 1];
        run_conv(h, find_conv(h, net, "Mconv1" + s), nullptr, N, hl, wl, Act{in, 150, 0}, Act{T[0], 128, 0}, Act{},
                 Act{}, true, false);
        int t = 0;
        for (int i = 2; i <= 6; ++i) {
            run_conv(h, find_conv(h, net, "Mconv" + std::to_string(i) + s), nullptr, N, hl, wl, Act{T[t], 128, 0},
                     Act{T[t ^ 1], 128, 0}, Act{}, Act{}, true, false);
            t ^= 1;
        }
        run_conv(h, find_conv(h, net, "Mconv7" + s), nullptr, N, hl, wl, Act{T[t], 128, 0}, Act{out, 150, 0}, Act{},
                 Act{}, false, false);
        cur ^= 1;
    }
    return S[cur];
}

// ---------------------------------------------------------------- geometry (src/body.py:32-41)
static int cv_round(double v) { return (int)std::nearbyint(v); }

static ScaleGeom geom(double s, const opose_params& p, int H, int W) {
    ScaleGeom g;
    g.mult = s * p.boxsize / H;
    g.Hs = cv_round(H * g.mult);
    g.Ws = cv_round(W * g.mult);
    if (g.Hs <= 0 || g.Ws <= 0) throw std::invalid_argument("scale produces an empty image");
    g.Hp = round_up(g.Hs, p.stride);
    g.Wp = round_up(g.Ws, p.stride);
    g.hl = g.Hp / 8;
    g.wl = g.Wp / 8;
    g.up_sy = 1.0 / ((double)H / g.Hs);
    g.up_sx = 1.0 / ((double)W / g.Ws);
    return g;
}

// Body mid set of one scale: the x8 heat channels [N][18][Hs][Ws] (read whole by the heat resize),
// then the network's low-res PAF channels [N][38][hl][wl], whose x8 values paf_score evaluates at
// its sample points only (the x8 PAF maps are never written: PafScales::low)
static size_t body_mid_heat(int N, const ScaleGeom& g) { return (size_t)N * 18 * g.Hs * g.Ws; }

// post-network body path from per-scale mid sets (body_to_mid) to records
static void body_post_common(opose_ctx* h, int N, int H, int W, const std::vector<ScaleGeom>& gs,
                             const opose_params& p, uint8_t* rec_dev) {
    const RecordLayout L = make_record_layout(h->ppp, h->maxp);
    const int cap = h->ppp;
    const int ns = (int)gs.size();
    PafScales S{};
    for (int s = 0; s < ns; ++s) {
        S.mid[s] = h->mid(s).ensure<float>(0, h->stream);
        S.low[s] = S.mid[s] + body_mid_heat(N, gs[s]);
        S.hs[s] = gs[s].Hs;
        S.ws[s] = gs[s].Ws;
        S.hl[s] = gs[s].hl;
        S.wl[s] = gs[s].wl;
        S.sy[s] = gs[s].up_sy;
        S.sx[s] = gs[s].up_sx;
    }
    S.n = ns;
    S.cm = 18;
    S.lcm = 38;
    S.H = H;
    S.W = W;
    int* cnt = h->cnt.ensure<int>((size_t)N * 18, h->stream);
    int* list = h->list.ensure<int>((size_t)N * 18 * cap, h->stream);
    double* lscore = h->list_score.ensure<double>((size_t)N * 18 * cap, h->stream);
    int* pos = h->peak_pos.ensure<int>((size_t)N * 18 * cap, h->stream);
    int* pcnt = h->part_cnt.ensure<int>((size_t)N * 18, h->stream);
    double* score = h->score.ensure<double>((size_t)N * 19 * cap * cap, h->stream);
    Conn* conn = h->conn.ensure<Conn>((size_t)N * 19 * cap, h->stream);
    int* ccnt = h->conn_cnt.ensure<int>((size_t)N * 19, h->stream);
    OPOSE_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * N * 18, h->stream));
    ProfEntry pe;
    // single scale: the float64 average equals the float32 resize output exactly -> f32 map
    const bool f32 = ns == 1;
    if (f32 && gauss_nms_resize_fits(gs[0].Hs, gs[0].Ws, H, W, gs[0].up_sy)) {
        // one scale, a true upsampling resize (the reference's 368-row frames at scale 0.5): the
        // resize runs inside the NMS tiles (post.hip gauss_nms_resize) and tiles whose sources
        // cannot produce a peak are dropped, so no full-resolution map is written or read.
        // float64-VALU bound: flops = the reference filter's 2 x 37 float64 operations per
        // full-resolution part-map pixel (bench.py GAUSS_OPS_PER_PIXEL); bytes: the x8 heat
        // channels the tiles read
        h->prof_begin(pe, "gauss_nms_resize", 74.0 * N * 18 * (double)H * W, (double)N * 18 * 4.0 * gs[0].Hs * gs[0].Ws);
        launch_gauss_nms_resize(S.mid[0], 18, 0, 18, N, gs[0].Hs, gs[0].Ws, H, W, gs[0].up_sy, gs[0].up_sx, p.thre1,
                                cap, cnt, list, lscore, h->stream);
        h->prof_end(pe);
    } else {
    double* avg = h->avg.ensure<double>((size_t)N * 18 * H * W, h->stream);
    HeatScales hsc{};
    hsc.n = ns;
    hsc.ns = (float)ns;
    double mid_bytes = 0;
    for (int s = 0; s < ns && s < kHeatScales; ++s) {
        hsc.s[s] = HeatScale{S.mid[s], 18, 0, gs[s].Hs, gs[s].Ws, gs[s].up_sy, gs[s].up_sx};
        mid_bytes += (double)N * 18 * 4.0 * gs[s].Hs * gs[s].Ws;
    }
    const bool fused_avg = !f32 && h->heat_scales && heat_full_scales_fits(hsc, H, W);  // several scales: one launch
    if (fused_avg) {
        h->prof_begin(pe, "heat_full", 0, (double)N * 18 * H * W * 8.0 + mid_bytes);
        launch_heat_full_scales(hsc, N, 18, H, W, avg, h->stream);
        h->prof_end(pe);
    }
    for (int s = 0; s < ns && !fused_avg; ++s) {
        h->prof_begin(pe, "heat_full", 0,
                      (double)N * 18 * (H * W * (f32 ? 4.0 : 8.0) * (s ? 2 : 1) + 4.0 * gs[s].Hs * gs[s].Ws));
        if (f32)
            launch_heat_full_f32(S.mid[s], 18, 0, 18, N, gs[s].Hs, gs[s].Ws, H, W, gs[s].up_sy, gs[s].up_sx,
                                 reinterpret_cast<float*>(avg), h->stream);
        else
            launch_heat_full(S.mid[s], 18, 0, 18, N, gs[s].Hs, gs[s].Ws, H, W, gs[s].up_sy, gs[s].up_sx, ns, s > 0,
                             avg, h->stream);
        h->prof_end(pe);
    }
    h->prof_begin(pe, "gauss_nms", 0, (double)N * 18 * H * W * (f32 ? 4 : 8));
    launch_gauss_nms(avg, f32, N * 18, H, W, p.thre1, cap, cnt, list, lscore, h->stream);
    h->prof_end(pe);
    }
    h->prof_begin(pe, "peaks_finalize", 0, 0);
    launch_peaks_finalize(cnt, list, lscore, N, H, W, L, rec_dev, pos, pcnt, h->stream);
    h->prof_end(pe);
    // bytes: the low-res PAF channels, read once from HBM (every sample after the first hits L2)
    double paf_bytes = 0;
    for (int s = 0; s < ns; ++s) paf_bytes += (double)N * 38 * 4 * gs[s].hl * gs[s].wl;
    h->prof_begin(pe, "paf_score", 0, paf_bytes);
    launch_paf_score(S, pos, pcnt, N, cap, p.thre2, score, h->stream);
    h->prof_end(pe);
    h->prof_begin(pe, "limb_greedy", 0, 0);
    launch_limb_greedy(score, pcnt, N, cap, conn, ccnt, h->stream);
    h->prof_end(pe);
    h->prof_begin(pe, "assemble", 0, 0);
    launch_assemble(conn, ccnt, pcnt, N, L, rec_dev, h->stream);
    h->prof_end(pe);
}

static void upsample_to_mid(opose_ctx* h, int s, const float* maps, int cstride, int N, const ScaleGeom& g, int C) {
    float* mid = h->mid(s).ensure<float>((size_t)N * C * g.Hs * g.Ws, h->stream);
    ProfEntry pe;
    h->prof_begin(pe, "upsample8", 0, (double)N * C * g.Hs * g.Ws * 4);
    launch_upsample8(maps, cstride, 0, C, N, g.hl, g.wl, g.Hs, g.Ws, mid, h->stream);
    h->prof_end(pe);
}

// body maps (PAF channels 0..37, heat 38..55 of [N][cstride][hl][wl]) -> mid set s (body_mid_heat)
static void body_to_mid(opose_ctx* h, int s, const float* maps, int cstride, int N, const ScaleGeom& g) {
    const size_t heat = body_mid_heat(N, g), lp = (size_t)g.hl * g.wl;
    float* mid = h->mid(s).ensure<float>(heat + (size_t)N * 38 * lp, h->stream);
    ProfEntry pe;
    h->prof_begin(pe, "upsample8", 0, (double)heat * 4 + (double)N * 56 * lp * 4 + (double)N * 38 * lp * 4);
    launch_upsample8(maps, cstride, 38, 18, N, g.hl, g.wl, g.Hs, g.Ws, mid, h->stream);
    OPOSE_HIP_CHECK(hipMemcpy2DAsync(mid + heat, 38 * lp * 4, maps, (size_t)cstride * lp * 4, 38 * lp * 4, N,
                                     hipMemcpyDeviceToDevice, h->stream));
    h->prof_end(pe);
}

// Every scale's network in lockstep on the handle's stream (split-bf16 path): per scale the
// preprocess into its slot's input, one conv launch per layer for all scales (hand_net_x6 /
// body_net_x6 segments), per scale the x8 upsample of its C heat / PAF channels into mid(s).
static void run_scales_lockstep(opose_ctx* h, int net, const uint8_t* fd, int64_t frame_stride, int64_t row_stride,
                                int N, int H, int W, const std::vector<ScaleGeom>& gs, const opose_params& p) {
    if (!h->loaded[net]) throw std::runtime_error(net == OPOSE_NET_BODY ? "body weights not loaded" : "hand weights not loaded");
    std::vector<NetSeg> segs;
    for (size_t s = 0; s < gs.size(); ++s) {
        const ScaleGeom& g = gs[s];
        float* x = h->ws[s].x.ensure<float>((size_t)N * 3 * g.Hp * g.Wp, h->stream);
        ProfEntry pe;
        h->prof_begin(pe, "preprocess", 0, (double)N * (3.0 * H * W + 12.0 * g.Hp * g.Wp));
        launch_preprocess(fd, frame_stride, row_stride, N, H, W, g.Hs, g.Ws, 1.0 / g.mult, 1.0 / g.mult, g.Hp, g.Wp,
                          (float)p.pad_value / 256.f - 0.5f, x, h->stream);
        h->prof_end(pe);
        segs.push_back(NetSeg{x, N, g.Hp, g.Wp, (int)s});
    }
    const std::vector<float*> outs = net == OPOSE_NET_BODY ? body_net_x6(h, segs) : hand_net_x6(h, segs);
    for (size_t s = 0; s < gs.size(); ++s)
        if (net == OPOSE_NET_BODY)
            body_to_mid(h, (int)s, outs[s], 185, N, gs[s]);
        else
            upsample_to_mid(h, (int)s, outs[s], 150, N, gs[s], 21);
}

// bytes a strided uint8 [N][H][W][3] host view spans: the last row ends 3*W bytes after its start,
// so a view cut from the bottom-right of a larger buffer is never read past its end
static size_t host_span(int N, int H, int W, int64_t row_stride, int64_t frame_stride) {
    return (size_t)(N - 1) * (size_t)frame_stride + (size_t)(H - 1) * (size_t)row_stride + (size_t)W * 3;
}

static int worst_status(const uint8_t* rec, int N, size_t bytes) {
    int w = 0;
    for (int n = 0; n < N; ++n) {
        int s = reinterpret_cast<const int32_t*>(rec + (size_t)n * bytes)[0];
        if (s < w) w = s;
    }
    return w;
}

}  // namespace opose

// ======================================================================== C ABI
namespace opose {
// every entry point that enqueues work on the handle's stream (other than the pipelined body
// path): select the device, and make the next pipelined network wait for that stream
static void flush_post(opose_ctx* h);
static void enter_main(opose_ctx* h) {
    OPOSE_HIP_CHECK(hipSetDevice(h->device));
    flush_post(h);
    h->main_dirty = true;
}
}  // namespace opose

#define OPOSE_TRY(h, ...)                      \
    try {                                      \
        __VA_ARGS__;                           \
    } catch (const std::invalid_argument& e) { \
        if (h) (h)->err = e.what();            \
        return OPOSE_E_SHAPE;                  \
    } catch (const opose::HipError& e) {       \
        if (h) (h)->err = e.what();            \
        return OPOSE_E_HIP;                    \
    } catch (const std::exception& e) {        \
        if (h) (h)->err = e.what();            \
        return OPOSE_E_WEIGHTS;                \
    }

// Batch_body fast mode after the network (srcmx/Batch_model.py:159-204): torch bicubic x8
// cropped to nh x nw, torch bicubic to H x W, 5x5 blur + peaks on the blurred map, then the
// shared limb scoring / greedy matching / assembly.  maps: [N][cstride][hl][wl] with PAF
// channels 0..37 and heat 38..56.
static void batch_post_common(opose_ctx* h, int N, int H, int W, const float* maps, int cstride, int hl, int wl,
                              int nh, int nw, const opose_params& p, uint8_t* rec_dev) {
    const RecordLayout L = make_record_layout(h->ppp, h->maxp);
    const int cap = h->ppp;
    ProfEntry pe;
    float* mid = h->mid(0).ensure<float>((size_t)N * 56 * nh * nw, h->stream);
    h->prof_begin(pe, "upsample8", 0, (double)N * 56 * nh * nw * 4);
    launch_upsample8_torch(maps, cstride, 0, 56, N, hl, wl, nh, nw, mid, h->stream);
    h->prof_end(pe);
    float* heat = reinterpret_cast<float*>(h->avg.ensure<double>((size_t)N * 18 * H * W, h->stream));
    h->prof_begin(pe, "heat_full", 0, (double)N * 18 * (4.0 * H * W + 4.0 * nh * nw));
    launch_resize_torch_f32(mid, 56, 38, 18, N, nh, nw, H, W, heat, h->stream);
    h->prof_end(pe);
    PafScales S{};
    S.mid[0] = mid;
    S.hs[0] = nh;
    S.ws[0] = nw;
    S.sy[0] = (double)((float)nh / (float)H);
    S.sx[0] = (double)((float)nw / (float)W);
    S.n = 1;
    S.cm = 56;
    S.H = H;
    S.W = W;
    S.torch = 1;
    int* cnt = h->cnt.ensure<int>((size_t)N * 18, h->stream);
    int* list = h->list.ensure<int>((size_t)N * 18 * cap, h->stream);
    double* lscore = h->list_score.ensure<double>((size_t)N * 18 * cap, h->stream);
    int* pos = h->peak_pos.ensure<int>((size_t)N * 18 * cap, h->stream);
    int* pcnt = h->part_cnt.ensure<int>((size_t)N * 18, h->stream);
    double* score = h->score.ensure<double>((size_t)N * 19 * cap * cap, h->stream);
    Conn* conn = h->conn.ensure<Conn>((size_t)N * 19 * cap, h->stream);
    int* ccnt = h->conn_cnt.ensure<int>((size_t)N * 19, h->stream);
    OPOSE_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * N * 18, h->stream));
    h->prof_begin(pe, "gauss_nms", 0, (double)N * 18 * H * W * 4);
    launch_blur5_nms(heat, N * 18, H, W, p.thre1, cap, cnt, list, lscore, h->stream);
    h->prof_end(pe);
    h->prof_begin(pe, "peaks_finalize", 0, 0);
    launch_peaks_finalize(cnt, list, lscore, N, H, W, L, rec_dev, pos, pcnt, h->stream);
    h->prof_end(pe);
    h->prof_begin(pe, "paf_score", 0, 0);
    launch_paf_score(S, pos, pcnt, N, cap, p.thre2, score, h->stream);
    h->prof_end(pe);
    h->prof_begin(pe, "limb_greedy", 0, 0);
    launch_limb_greedy(score, pcnt, N, cap, conn, ccnt, h->stream);
    h->prof_end(pe);
    h->prof_begin(pe, "assemble", 0, 0);
    launch_assemble(conn, ccnt, pcnt, N, L, rec_dev, h->stream);
    h->prof_end(pe);
}

// Run `work` (device work only: kernels, device memsets/copies on h->stream, no host sync,
// no allocation once warm) through the launch-sequence cache keyed by `key`.  Captures stay on
// the one stream (h->capturing: run_scales_concurrently runs its scales one after another), and
// a captured graph that is not a single chain of nodes is refused (linear_graph).  Cause: in a
// torch process the library runs on torch's bundled HIP runtime (libamdhip64 7.0.2, SONAME
// libamdhip64.so.7, loaded before ours), whose hipGraphLaunch segfaults on a freshly instantiated
// forked graph after other forked executables were destroyed.  scripts/graph_fork_repro.hip
// reproduces it without libopose: the same program crashes under 7.0.2 and runs clean
// under /opt/rocm's 7.2, with no fork in captures, or with no executable destroyed.
// a chain: one root, nodes - 1 edges, and no node with more than one successor (a tree with
// nodes - 1 edges and one root may still branch)
static bool linear_graph(hipGraph_t g) {
    size_t nodes = 0, edges = 0, roots = 0;
    OPOSE_HIP_CHECK(hipGraphGetNodes(g, nullptr, &nodes));
    OPOSE_HIP_CHECK(hipGraphGetEdges(g, nullptr, nullptr, &edges));
    OPOSE_HIP_CHECK(hipGraphGetRootNodes(g, nullptr, &roots));
    if (nodes == 0) return true;
    if (roots != 1 || edges != nodes - 1) return false;
    std::vector<hipGraphNode_t> all(nodes);
    OPOSE_HIP_CHECK(hipGraphGetNodes(g, all.data(), &nodes));
    for (hipGraphNode_t n : all) {
        size_t succ = 0;
        OPOSE_HIP_CHECK(hipGraphNodeGetDependentNodes(n, nullptr, &succ));
        if (succ > 1) return false;
    }
    return true;
}

template <class F>
static void run_graphed(opose_ctx* h, const std::string& key, F&& work) {
    if (!h->use_graphs || h->prof || !h->stream) {
        work();
        return;
    }
    const uint64_t epoch = g_alloc_epoch.load();
    auto it = h->graphs.find(key);
    if (it != h->graphs.end() && it->second.eager) {  // refused once: never captured again
        work();
        return;
    }
    if (it != h->graphs.end() && it->second.exec && it->second.epoch == epoch) {
        OPOSE_HIP_CHECK(hipGraphLaunch(it->second.exec, h->stream));
        return;
    }
    if (it == h->graphs.end() || it->second.epoch != epoch) {  // first sighting: eager, allocates
        if (it != h->graphs.end() && it->second.exec) OPOSE_HIP_CHECK(hipGraphExecDestroy(it->second.exec));
        work();
        h->graphs[key] = GraphEntry{nullptr, g_alloc_epoch.load()};
        return;
    }
    // second sighting with nothing reallocated since: capture, instantiate, launch
    OPOSE_HIP_CHECK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    h->capturing = true;
    try {
        work();
        h->capturing = false;
    } catch (...) {
        h->capturing = false;
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(h->stream, &g);
        if (g) (void)hipGraphDestroy(g);
        throw;
    }
    hipGraph_t g = nullptr;
    OPOSE_HIP_CHECK(hipStreamEndCapture(h->stream, &g));
    if (!linear_graph(g)) {
        // a fork inside a capture (see above): never instantiated.  The captured work did not run,
        // so run it eagerly now, and keep this signature eager (no capture on every later call)
        (void)hipGraphDestroy(g);
        it->second.eager = true;
        work();
        return;
    }
    if (g_alloc_epoch.load() != epoch) {  // something allocated inside the capture: not replayable
        (void)hipGraphDestroy(g);
        h->graphs.erase(key);
        work();
        return;
    }
    hipGraphExec_t ex = nullptr;
    const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    OPOSE_HIP_CHECK(e);
    it->second.exec = ex;
    OPOSE_HIP_CHECK(hipGraphLaunch(ex, h->stream));
}

static std::string call_key(const char* what, int N, int H, int W, int64_t rs, int64_t fs, const opose_params& p,
                            const void* in_dev, const void* out_dev, int ppp, int maxp) {
    std::string k(what);
    char tmp[256];
    std::snprintf(tmp, sizeof tmp, "|%d|%d|%d|%lld|%lld|%p|%p|%d|%d|", N, H, W, (long long)rs, (long long)fs, in_dev,
                  out_dev, ppp, maxp);
    k += tmp;
    k.append(reinterpret_cast<const char*>(&p), sizeof p);
    return k;
}

extern "C" {

void opose_default_params(int net, opose_params* p) {
    std::memset(p, 0, sizeof(*p));
    if (net == OPOSE_NET_HAND) {
        p->n_scales = 4;
        p->scales[0] = 0.5;
        p->scales[1] = 1.0;
        p->scales[2] = 1.5;
        p->scales[3] = 2.0;
    } else {
        p->n_scales = 1;
        p->scales[0] = 0.5;
    }
    p->boxsize = 368;
    p->stride = 8;
    p->pad_value = 128;
    p->thre1 = 0.1;
    p->thre2 = 0.05;
    p->thre_hand = 0.03;
}

int opose_create(int device, opose_t** out) {
    if (!out) return OPOSE_E_ARG;
    *out = nullptr;
    auto* h = new opose_ctx();
    h->device = device;
    if (hipSetDevice(device) != hipSuccess || pooled_stream(&h->own_stream, 0) != hipSuccess) {
        delete h;
        return OPOSE_E_HIP;
    }
    h->stream = h->own_stream;
    *out = h;
    return OPOSE_OK;
}

void opose_destroy(opose_t* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)opose_flush(h);
    (void)hipStreamSynchronize(h->stream);
    delete h;
}

const char* opose_last_error(const opose_t* h) { return h ? h->err.c_str() : "null handle"; }

namespace opose {
static hipEvent_t lazy_event(hipEvent_t& e) {
    if (!e) OPOSE_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
}
}  // namespace opose

int opose_set_stream(opose_t* h, void* s) {
    if (!h) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipSetDevice(h->device));
        flush_post(h);
        const hipStream_t ns = s ? static_cast<hipStream_t>(s) : h->own_stream;
        if (ns != h->stream) {
            // work still queued on the old stream (and on the pipelined network stream) uses the
            // workspace the new stream's calls reuse: order the new stream after both
            hipEvent_t e = lazy_event(h->ev_sig);
            OPOSE_HIP_CHECK(hipEventRecord(e, h->stream));
            OPOSE_HIP_CHECK(hipStreamWaitEvent(ns, e, 0));
            if (h->nstream) {
                OPOSE_HIP_CHECK(hipEventRecord(e, h->nstream));
                OPOSE_HIP_CHECK(hipStreamWaitEvent(ns, e, 0));
            }
            h->stream = ns;
            h->main_dirty = true;  // the next pipelined network waits for the new stream
        }
    });
    return OPOSE_OK;
}

int opose_wait_stream(opose_t* h, void* s) {
    if (!h) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipSetDevice(h->device));
        const hipStream_t xs = static_cast<hipStream_t>(s);
        // Both library streams must come after `xs`: the handle's stream directly (nothing to do
        // when `xs` is that stream), the pipelined network stream through the event even then --
        // back-to-back pipelined calls do not otherwise order it after the handle's stream.
        // Before the network stream exists, the first pipelined call orders it after the
        // handle's stream (main_dirty), which by then has waited on every such `xs`.
        hipEvent_t e = lazy_event(h->ev_ext);
        OPOSE_HIP_CHECK(hipEventRecord(e, xs));
        if (xs != h->stream) OPOSE_HIP_CHECK(hipStreamWaitEvent(h->stream, e, 0));
        if (h->nstream) {
            if (xs != h->nstream) OPOSE_HIP_CHECK(hipStreamWaitEvent(h->nstream, e, 0));
        } else {
            h->main_dirty = true;
        }
    });
    return OPOSE_OK;
}

int opose_signal_stream(opose_t* h, void* s) {
    if (!h) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipSetDevice(h->device));
        flush_post(h);
        const hipStream_t xs = static_cast<hipStream_t>(s);
        if (xs == h->stream) return OPOSE_OK;
        hipEvent_t e = lazy_event(h->ev_sig);
        OPOSE_HIP_CHECK(hipEventRecord(e, h->stream));
        OPOSE_HIP_CHECK(hipStreamWaitEvent(xs, e, 0));
    });
    return OPOSE_OK;
}

int opose_signal_input(opose_t* h, void* s) {
    if (!h) return OPOSE_E_ARG;
    // Since the last entry point that queued work on the handle's stream (main_dirty), only
    // OPOSE_PIPELINE calls ran, and each read its device inputs on the network stream only (its
    // post-network part reads the mid buffers).  That stream waited for the handle's stream when
    // main_dirty was last cleared, so an event on it after the last network covers every input
    // read so far.  Otherwise the handle's stream holds input reads: opose_signal_stream.
    if (!h->nstream || h->main_dirty) return opose_signal_stream(h, s);
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipSetDevice(h->device));
        const hipStream_t xs = static_cast<hipStream_t>(s);
        if (xs == h->nstream) return OPOSE_OK;
        hipEvent_t e = lazy_event(h->ev_in);
        OPOSE_HIP_CHECK(hipEventRecord(e, h->nstream));
        OPOSE_HIP_CHECK(hipStreamWaitEvent(xs, e, 0));
    });
    return OPOSE_OK;
}

void* opose_get_stream(const opose_t* h) { return h ? h->stream : nullptr; }

int opose_flush(opose_t* h) {
    if (!h) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipSetDevice(h->device));
        flush_post(h);
    });
    return OPOSE_OK;
}

int opose_synchronize(opose_t* h) {
    if (!h) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        flush_post(h);
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        if (h->nstream) OPOSE_HIP_CHECK(hipStreamSynchronize(h->nstream));
    });
    return OPOSE_OK;
}

int opose_set_capacity(opose_t* h, int ppp, int maxp) {
    if (!h || ppp < 1 || maxp < 1 || ppp > 1024 || maxp > 256) return OPOSE_E_ARG;
    if (opose_flush(h) != OPOSE_OK) return OPOSE_E_HIP;
    h->ppp = ppp;
    h->maxp = maxp;
    return OPOSE_OK;
}

size_t opose_body_record_bytes(const opose_t* h) { return h ? make_record_layout(h->ppp, h->maxp).bytes : 0; }

int opose_load_weights(opose_t* h, int net, const float* const* tensors, const int64_t* shapes, int n) {
    if (!h || !tensors || !shapes || (net != OPOSE_NET_BODY && net != OPOSE_NET_HAND)) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const std::vector<Spec> order = state_dict_order(net);
        if ((size_t)n != 2 * order.size()) {
            h->err = "expected " + std::to_string(2 * order.size()) + " tensors, got " + std::to_string(n);
            return OPOSE_E_WEIGHTS;
        }
        std::map<std::string, std::pair<const float*, const float*>> byname;
        for (size_t i = 0; i < order.size(); ++i) {
            const Spec& s = order[i];
            const int64_t* ws = shapes + 8 * i;
            const int64_t* bs = shapes + 8 * i + 4;
            if (ws[0] != s.cout || ws[1] != s.cin || ws[2] != s.ks || ws[3] != s.ks || bs[0] != s.cout) {
                h->err = "shape mismatch for " + s.name;
                return OPOSE_E_WEIGHTS;
            }
            byname[s.name] = {tensors[2 * i], tensors[2 * i + 1]};
        }
        h->convs[net].clear();
        // physical channel order of the X6 stage-input concat (8-channel groups): body
        // [L1 38 | pad 2 | L2 19 | pad 5 | trunk 128], hand [L 22 | pad 2 | trunk 128]
        std::vector<int> cmap;
        if (net == OPOSE_NET_BODY)
            for (int c = 0; c < 185; ++c) cmap.push_back(c < 38 ? c : (c < 57 ? c + 2 : c + 7));
        else
            for (int c = 0; c < 150; ++c) cmap.push_back(c < 22 ? c : c + 2);
        for (const Spec& s : order)
            upload_conv(h, net, s.name, {&s}, {byname[s.name].first}, {byname[s.name].second},
                        s.name.rfind("Mconv1_", 0) == 0 ? cmap : std::vector<int>{});
        if (net == OPOSE_NET_BODY) {
            // branch-pair layers sharing an input become one GEMM with M = 256
            std::vector<std::string> shared = {"conv5_1_CPM"};
            for (int st = 2; st <= 6; ++st) shared.push_back("Mconv1_stage" + std::to_string(st));
            for (const auto& base : shared) {
                const std::string l1 = base + "_L1", l2 = base + "_L2";
                const Spec *s1 = nullptr, *s2 = nullptr;
                for (const Spec& s : order) {
                    if (s.name == l1) s1 = &s;
                    if (s.name == l2) s2 = &s;
                }
                upload_conv(h, net, base + "_L1+L2", {s1, s2}, {byname[l1].first, byname[l2].first},
                            {byname[l1].second, byname[l2].second},
                            base.rfind("Mconv1_", 0) == 0 ? cmap : std::vector<int>{});
            }
        }
        h->loaded[net] = true;
    });
    return OPOSE_OK;
}

static int net_forward(opose_t* h, int net, const float* x, int N, int Hp, int Wp, float* o1, float* o2, int flags) {
    if (!h || !x || N <= 0 || Hp < 8 || Wp < 8 || Hp % 8 || Wp % 8) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const size_t in_n = (size_t)N * 3 * Hp * Wp;
        const float* xd = x;
        if (!(flags & OPOSE_IN_DEVICE)) {
            float* buf = h->w().x.ensure<float>(in_n, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, x, in_n * 4, hipMemcpyHostToDevice, h->stream));
            xd = buf;
        }
        const int hl = Hp / 8, wl = Wp / 8;
        const size_t plane = (size_t)hl * wl;
        const hipMemcpyKind kind = (flags & OPOSE_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        if (net == OPOSE_NET_BODY) {
            float* S = body_net(h, xd, N, Hp, Wp);
            // S: [N][185][hl][wl]; paf = ch 0..37, heat = 38..56
            OPOSE_HIP_CHECK(hipMemcpy2DAsync(o1, 38 * plane * 4, S, 185 * plane * 4, 38 * plane * 4, N, kind, h->stream));
            OPOSE_HIP_CHECK(hipMemcpy2DAsync(o2, 19 * plane * 4, S + 38 * plane, 185 * plane * 4, 19 * plane * 4, N,
                                             kind, h->stream));
        } else {
            float* S = hand_net(h, xd, N, Hp, Wp);
            OPOSE_HIP_CHECK(hipMemcpy2DAsync(o1, 22 * plane * 4, S, 150 * plane * 4, 22 * plane * 4, N, kind, h->stream));
        }
        if (!(flags & OPOSE_OUT_DEVICE)) OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        h->prof_drain();
    });
    return OPOSE_OK;
}

int opose_hand_forward_pyramid(opose_t* h, int n, const float* const* xs, const int* N, const int* Hp, const int* Wp,
                               float* const* heats, int flags) {
    if (!h || !xs || !N || !Hp || !Wp || !heats || n < 1 || n > OPOSE_MAX_SCALES) return OPOSE_E_ARG;
    for (int i = 0; i < n; ++i)
        if (!xs[i] || !heats[i] || N[i] <= 0 || Hp[i] < 8 || Wp[i] < 8 || Hp[i] % 8 || Wp[i] % 8) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        if (!h->loaded[OPOSE_NET_HAND]) throw std::runtime_error("hand weights not loaded");
        const hipMemcpyKind kind = (flags & OPOSE_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        std::vector<NetSeg> segs;
        for (int i = 0; i < n; ++i) {
            const size_t in_n = (size_t)N[i] * 3 * Hp[i] * Wp[i];
            const float* xd = xs[i];
            if (!(flags & OPOSE_IN_DEVICE)) {
                float* buf = h->ws[i].x.ensure<float>(in_n, h->stream);
                OPOSE_HIP_CHECK(hipMemcpyAsync(buf, xs[i], in_n * 4, hipMemcpyHostToDevice, h->stream));
                xd = buf;
            }
            segs.push_back(NetSeg{xd, N[i], Hp[i], Wp[i], i});
        }
        std::vector<float*> outs;
        if (h->x6) {
            outs = hand_net_x6(h, segs);
        } else {
            for (int i = 0; i < n; ++i) {
                h->slot = i;
                outs.push_back(hand_net(h, segs[i].x, N[i], Hp[i], Wp[i]));
            }
            h->slot = 0;
        }
        for (int i = 0; i < n; ++i) {
            const size_t plane = (size_t)(Hp[i] / 8) * (Wp[i] / 8);
            OPOSE_HIP_CHECK(hipMemcpy2DAsync(heats[i], 22 * plane * 4, outs[i], 150 * plane * 4, 22 * plane * 4, N[i],
                                             kind, h->stream));
        }
        if (!(flags & OPOSE_OUT_DEVICE)) OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        h->prof_drain();
    });
    return OPOSE_OK;
}

int opose_body_forward(opose_t* h, const float* x, int N, int Hp, int Wp, float* paf, float* heat, int flags) {
    if (!paf || !heat) return OPOSE_E_ARG;
    return net_forward(h, OPOSE_NET_BODY, x, N, Hp, Wp, paf, heat, flags);
}

int opose_hand_forward(opose_t* h, const float* x, int N, int Hp, int Wp, float* heat, int flags) {
    if (!heat) return OPOSE_E_ARG;
    return net_forward(h, OPOSE_NET_HAND, x, N, Hp, Wp, heat, nullptr, flags);
}

static int finish_records(opose_t* h, int N, void* records, uint8_t* rec_dev, int flags) {
    const RecordLayout L = make_record_layout(h->ppp, h->maxp);
    if (flags & OPOSE_OUT_DEVICE) {
        if (rec_dev != records)
            OPOSE_HIP_CHECK(hipMemcpyAsync(records, rec_dev, L.bytes * N, hipMemcpyDeviceToDevice, h->stream));
        h->prof_drain();
        return OPOSE_OK;
    }
    OPOSE_HIP_CHECK(hipMemcpyAsync(records, rec_dev, L.bytes * N, hipMemcpyDeviceToHost, h->stream));
    OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
    h->prof_drain();
    return worst_status(static_cast<const uint8_t*>(records), N, L.bytes);
}

static opose_params fill_params(const opose_params* p, int net) {
    opose_params q;
    if (p) q = *p;
    else opose_default_params(net, &q);
    if (q.n_scales < 1 || q.n_scales > OPOSE_MAX_SCALES || q.stride != 8 || q.boxsize <= 0)
        throw std::invalid_argument("bad opose_params");
    return q;
}

namespace opose {
// fn(s) for every scale s, scale s on stream s (0: the handle's stream, others its scale
// streams), each with workspace slot s; the handle's stream continues after all of them
static void run_scales_concurrently(opose_ctx* h, int ns, const std::function<void(int)>& fn) {
    if (h->capturing) {  // one stream while capturing (run_graphed): same work, same slots
        try {
            for (int s = ns - 1; s >= 0; --s) {
                h->slot = s;
                fn(s);
            }
        } catch (...) {
            h->slot = 0;
            throw;
        }
        h->slot = 0;
        return;
    }
    const hipStream_t main = h->stream;
    if (!h->ev_fork) OPOSE_HIP_CHECK(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
    OPOSE_HIP_CHECK(hipEventRecord(h->ev_fork, main));
    for (int s = 1; s < ns; ++s) {
        if (!h->sstream[s]) {
            OPOSE_HIP_CHECK(pooled_stream(&h->sstream[s], 0));
            OPOSE_HIP_CHECK(hipEventCreateWithFlags(&h->ev_join[s], hipEventDisableTiming));
        }
        OPOSE_HIP_CHECK(hipStreamWaitEvent(h->sstream[s], h->ev_fork, 0));
    }
    // largest scale first: it is the critical path
    try {
        for (int s = ns - 1; s >= 0; --s) {
            h->stream = s ? h->sstream[s] : main;
            h->slot = s;
            fn(s);
            if (s) OPOSE_HIP_CHECK(hipEventRecord(h->ev_join[s], h->sstream[s]));
        }
    } catch (...) {
        h->stream = main;
        h->slot = 0;
        throw;
    }
    h->stream = main;
    h->slot = 0;
    for (int s = 1; s < ns; ++s) OPOSE_HIP_CHECK(hipStreamWaitEvent(main, h->ev_join[s], 0));
}

// the deferred post-network part (OPOSE_PIPELINE_DEFER) on the handle's stream, after `after`
static void enqueue_deferred_post(opose_ctx* h, hipEvent_t after) {
    opose_ctx::DeferredPost& d = h->dpost;
    if (!d.pending) return;
    d.pending = false;
    OPOSE_HIP_CHECK(hipStreamWaitEvent(h->stream, after, 0));
    h->mid_set = d.set;
    try {
        body_post_common(h, d.N, d.H, d.W, d.gs, d.p, d.rec);
    } catch (...) {
        h->mid_set = 0;
        throw;
    }
    h->mid_set = 0;
    OPOSE_HIP_CHECK(hipEventRecord(h->ev_post[d.set], h->stream));
    h->post_pending[d.set] = true;
}

// enqueue a deferred post-network part now (after its whole network)
static void flush_post(opose_ctx* h) {
    if (h->dpost.pending) enqueue_deferred_post(h, h->ev_net);
}

static void pipelined_body(opose_ctx* h, int N, int H, int W, const std::vector<ScaleGeom>& gs,
                           const opose_params& p, uint8_t* rec, const std::function<void()>& net_part,
                           bool defer) {
    if (h->dpost.pending && !(h->dpost.N == N && h->dpost.H == H && h->dpost.W == W)) flush_post(h);
    if (!h->nstream) {
        int lo = 0, hi = 0;
        OPOSE_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        // the network stream gets the higher priority: its conv grids should not wait for
        // post-network workgroups that can run on whatever CUs are left (network high / post
        // high / both default measured the same)
        OPOSE_HIP_CHECK(pooled_stream(&h->nstream, hi));
        h->nstream_prio = hi;
        for (hipEvent_t* e : {&h->ev_net, &h->ev_main, &h->ev_post[0], &h->ev_post[1], &h->ev_gate})
            OPOSE_HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    const int set = h->next_set;
    h->next_set ^= 1;
    if (h->post_pending[set]) OPOSE_HIP_CHECK(hipStreamWaitEvent(h->nstream, h->ev_post[set], 0));
    if (h->main_dirty) {
        OPOSE_HIP_CHECK(hipEventRecord(h->ev_main, h->stream));
        OPOSE_HIP_CHECK(hipStreamWaitEvent(h->nstream, h->ev_main, 0));
        h->main_dirty = false;
    }
    hipStream_t main = h->stream;
    const bool gate = h->dpost.pending;  // the previous call's post waits for this network's gate
    h->mid_set = set;
    h->stream = h->nstream;
    h->gate_ev = gate ? h->ev_gate : nullptr;
    h->gate_done = false;
    try {
        net_part();
        if (gate && !h->gate_done) OPOSE_HIP_CHECK(hipEventRecord(h->ev_gate, h->nstream));
    } catch (...) {
        h->stream = main;
        h->mid_set = 0;
        h->gate_ev = nullptr;
        throw;
    }
    h->gate_ev = nullptr;
    h->stream = main;
    h->mid_set = 0;
    // ev_net is re-recorded every call: take the gate first (the deferred post's network ran
    // before this one on nstream, so the gate implies it)
    if (gate) enqueue_deferred_post(h, h->ev_gate);
    OPOSE_HIP_CHECK(hipEventRecord(h->ev_net, h->nstream));
    if (defer) {
        opose_ctx::DeferredPost& d = h->dpost;
        d.pending = true;
        d.N = N;
        d.H = H;
        d.W = W;
        d.set = set;
        d.gs = gs;
        d.p = p;
        d.rec = rec;
        return;
    }
    OPOSE_HIP_CHECK(hipStreamWaitEvent(main, h->ev_net, 0));
    h->mid_set = set;
    body_post_common(h, N, H, W, gs, p, rec);
    OPOSE_HIP_CHECK(hipEventRecord(h->ev_post[set], main));
    h->post_pending[set] = true;
    h->mid_set = 0;
}
}  // namespace opose

int opose_body_infer(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride, int64_t frame_stride,
                     const opose_params* pp, void* records, int flags) {
    if (!h || !bgr || !records || N <= 0 || H <= 0 || W <= 0) return OPOSE_E_ARG;
    if (row_stride < (int64_t)W * 3 || frame_stride < row_stride * H) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipSetDevice(h->device));  // pipelined or not: decided below
        const opose_params p = fill_params(pp, OPOSE_NET_BODY);
        const RecordLayout L = make_record_layout(h->ppp, h->maxp);
        const uint8_t* fd = bgr;
        if (!(flags & OPOSE_IN_DEVICE)) {
            uint8_t* buf = h->frames.ensure<uint8_t>((size_t)frame_stride * N, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, bgr, host_span(N, H, W, row_stride, frame_stride),
                                           hipMemcpyHostToDevice, h->stream));
            fd = buf;
        }
        std::vector<ScaleGeom> gs;
        for (int s = 0; s < p.n_scales; ++s) gs.push_back(geom(p.scales[s], p, H, W));
        uint8_t* rec = (flags & OPOSE_OUT_DEVICE) ? static_cast<uint8_t*>(records)
                                                  : h->records.ensure<uint8_t>(L.bytes * N, h->stream);
        auto scale_net = [&](int s) {
            const ScaleGeom& g = gs[s];
            float* x = h->w().x.ensure<float>((size_t)N * 3 * g.Hp * g.Wp, h->stream);
            ProfEntry pe;
            h->prof_begin(pe, "preprocess", 0, (double)N * (3.0 * H * W + 12.0 * g.Hp * g.Wp));
            launch_preprocess(fd, frame_stride, row_stride, N, H, W, g.Hs, g.Ws, 1.0 / g.mult, 1.0 / g.mult, g.Hp,
                              g.Wp, (float)p.pad_value / 256.f - 0.5f, x, h->stream);
            h->prof_end(pe);
            float* S = body_net(h, x, N, g.Hp, g.Wp);
            body_to_mid(h, s, S, 185, N, g);
        };
        const bool lockstep = h->x6 && h->lockstep && p.n_scales > 1;
        auto net_part = [&] {
            if (lockstep)
                run_scales_lockstep(h, OPOSE_NET_BODY, fd, frame_stride, row_stride, N, H, W, gs, p);
            else if (h->scale_streams && p.n_scales > 1)  // (pipelined: forked from and joined into nstream)
                run_scales_concurrently(h, p.n_scales, scale_net);
            else
                for (int s = 0; s < p.n_scales; ++s) scale_net(s);
        };
        if ((flags & OPOSE_PIPELINE) && (flags & OPOSE_IN_DEVICE) && (flags & OPOSE_OUT_DEVICE)) {
            pipelined_body(h, N, H, W, gs, p, rec, net_part, (flags & OPOSE_PIPELINE_DEFER) != 0);
        } else if (!lockstep && h->scale_streams && p.n_scales > 1) {  // multi-scale pyramid (C5): scales concurrently
            enter_main(h);
            h->mid_set = 0;
            run_scales_concurrently(h, p.n_scales, scale_net);
            body_post_common(h, N, H, W, gs, p, rec);
        } else {
            enter_main(h);
            h->mid_set = 0;
            const std::string key = call_key("body", N, H, W, row_stride, frame_stride, p, fd, rec, h->ppp, h->maxp);
            run_graphed(h, key, [&] {
                net_part();
                body_post_common(h, N, H, W, gs, p, rec);
            });
        }
        return finish_records(h, N, records, rec, flags);
    });
}

int opose_body_post(opose_t* h, const float* maps, int N, int hl, int wl, int pad_down, int pad_right, int H, int W,
                    const opose_params* pp, void* records, int flags) {
    if (!h || !maps || !records || N <= 0 || hl <= 0 || wl <= 0 || H <= 0 || W <= 0) return OPOSE_E_ARG;
    if (pad_down < 0 || pad_right < 0 || pad_down >= 8 * hl || pad_right >= 8 * wl) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        opose_params p = fill_params(pp, OPOSE_NET_BODY);
        p.n_scales = 1;
        const RecordLayout L = make_record_layout(h->ppp, h->maxp);
        const size_t n_in = (size_t)N * 57 * hl * wl;
        const float* md = maps;
        if (!(flags & OPOSE_IN_DEVICE)) {
            float* buf = h->maps_in.ensure<float>(n_in, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, maps, n_in * 4, hipMemcpyHostToDevice, h->stream));
            md = buf;
        }
        ScaleGeom g;
        g.mult = 0;
        g.hl = hl;
        g.wl = wl;
        g.Hp = 8 * hl;
        g.Wp = 8 * wl;
        g.Hs = g.Hp - pad_down;
        g.Ws = g.Wp - pad_right;
        g.up_sy = 1.0 / ((double)H / g.Hs);
        g.up_sx = 1.0 / ((double)W / g.Ws);
        body_to_mid(h, 0, md, 57, N, g);
        uint8_t* rec = (flags & OPOSE_OUT_DEVICE) ? static_cast<uint8_t*>(records)
                                                  : h->records.ensure<uint8_t>(L.bytes * N, h->stream);
        body_post_common(h, N, H, W, {g}, p, rec);
        return finish_records(h, N, records, rec, flags);
    });
}

// ---- scale-sharded single-frame latency ---------------------------------
int opose_body_scale_geom(int H, int W, const opose_params* pp, int s, int* out4) {
    if (!out4 || H <= 0 || W <= 0) return OPOSE_E_ARG;
    try {
        const opose_params p = fill_params(pp, OPOSE_NET_BODY);
        if (s < 0 || s >= p.n_scales) return OPOSE_E_ARG;
        const ScaleGeom g = geom(p.scales[s], p, H, W);
        out4[0] = g.hl;
        out4[1] = g.wl;
        out4[2] = g.Hp - g.Hs;
        out4[3] = g.Wp - g.Ws;
        return OPOSE_OK;
    } catch (const std::exception&) {
        return OPOSE_E_SHAPE;
    }
}

int opose_body_scale_maps(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride,
                          int64_t frame_stride, const opose_params* pp, int s, float* maps, int flags) {
    if (!h || !bgr || !maps || N <= 0 || H <= 0 || W <= 0) return OPOSE_E_ARG;
    if (row_stride < (int64_t)W * 3 || frame_stride < row_stride * H) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const opose_params p = fill_params(pp, OPOSE_NET_BODY);
        if (s < 0 || s >= p.n_scales) return OPOSE_E_ARG;
        const uint8_t* fd = bgr;
        if (!(flags & OPOSE_IN_DEVICE)) {
            uint8_t* buf = h->frames.ensure<uint8_t>((size_t)frame_stride * N, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, bgr, host_span(N, H, W, row_stride, frame_stride),
                                           hipMemcpyHostToDevice, h->stream));
            fd = buf;
        }
        const ScaleGeom g = geom(p.scales[s], p, H, W);
        float* x = h->w().x.ensure<float>((size_t)N * 3 * g.Hp * g.Wp, h->stream);
        launch_preprocess(fd, frame_stride, row_stride, N, H, W, g.Hs, g.Ws, 1.0 / g.mult, 1.0 / g.mult, g.Hp, g.Wp,
                          (float)p.pad_value / 256.f - 0.5f, x, h->stream);
        const float* S = body_net(h, x, N, g.Hp, g.Wp);
        // channels 0..56 of the stage-6 concat buffer [N][185][hl*wl] -> [N][57][hl*wl]
        const size_t plane = (size_t)g.hl * g.wl * 4;
        OPOSE_HIP_CHECK(hipMemcpy2DAsync(maps, 57 * plane, S, 185 * plane, 57 * plane, N,
                                         (flags & OPOSE_OUT_DEVICE) ? hipMemcpyDeviceToDevice
                                                                    : hipMemcpyDeviceToHost,
                                         h->stream));
        if (!(flags & OPOSE_OUT_DEVICE)) OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        return OPOSE_OK;
    });
}

int opose_rccl_unique_id(void* id, size_t len) {
    if (!id || len < sizeof(ncclUniqueId)) return OPOSE_E_ARG;
    try {
        ncclUniqueId u;
        rccl_check(rccl().get_unique_id(&u));
        std::memcpy(id, &u, sizeof(u));
        return OPOSE_OK;
    } catch (const std::exception&) {
        return OPOSE_E_HIP;
    }
}

int opose_rccl_init(opose_t* h, const void* id, int rank, int nranks) {
    if (!h || !id || nranks < 1 || rank < 0 || rank >= nranks) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipSetDevice(h->device));
        if (h->comm) {
            rccl_check(rccl().comm_destroy(h->comm));
            h->comm = nullptr;
        }
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        rccl_check(rccl().comm_init_rank(&h->comm, nranks, u, rank));
        return OPOSE_OK;
    });
}

int opose_rccl_abort(opose_t* h) {
    if (!h) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        if (h->comm) {
            ncclComm_t c = h->comm;
            h->comm = nullptr;
            h->band_up = h->band_dn = -1;
            rccl_check(rccl().comm_abort(c));
        }
        return OPOSE_OK;
    });
}

int opose_rccl_wait(opose_t* h, int timeout_ms) {
    if (!h || timeout_ms < 0) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipSetDevice(h->device));
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t q = hipStreamQuery(h->stream);
            if (q == hipSuccess) return OPOSE_OK;
            if (q != hipErrorNotReady) OPOSE_HIP_CHECK(q);
            ncclResult_t ae = ncclSuccess;
            if (h->comm) rccl_check(rccl().async_error(h->comm, &ae));
            const bool late = std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms);
            if ((ae != ncclSuccess && ae != ncclInProgress) || late) {
                // a band neighbour failed or never arrived: abort this rank's communicator, which
                // raises RCCL's abort flag that the queued send / recv kernels poll, so this rank's
                // stream drains instead of waiting on a peer that will not come
                if (h->comm) {
                    ncclComm_t c = h->comm;
                    h->comm = nullptr;
                    h->band_up = h->band_dn = -1;
                    (void)rccl().comm_abort(c);
                }
                h->err = late ? "RCCL halo exchange: no progress within the deadline (communicator aborted)"
                              : std::string("RCCL halo exchange: ") + rccl().error_string(ae) + " (communicator aborted)";
                return late ? OPOSE_E_TIMEOUT : OPOSE_E_HIP;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    });
}

int opose_set_band_peers(opose_t* h, int up, int dn) {
    if (!h) return OPOSE_E_ARG;
    h->band_up = up;
    h->band_dn = dn;
    return OPOSE_OK;
}

size_t opose_body_band_halo_bytes(int wl) { return wl > 0 ? band_halo_bytes(wl) : 0; }

int opose_body_band_maps(opose_t* h, const uint8_t* bgr, int H, int W, int64_t row_stride, const opose_params* pp,
                         int s, int r0, int r1, float* maps, opose_halo_fn fn, void* user, void* xbuf,
                         size_t xbuf_bytes, int flags) {
    if (!h || !bgr || !maps || !xbuf || H <= 0 || W <= 0 || row_stride < (int64_t)W * 3) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const opose_params p = fill_params(pp, OPOSE_NET_BODY);
        if (s < 0 || s >= p.n_scales) return OPOSE_E_ARG;
        const ScaleGeom g = geom(p.scales[s], p, H, W);
        if (r0 < 0 || r1 > g.hl || r1 - r0 < 3) return OPOSE_E_ARG;
        if (!fn && ((r0 > 0 && (!h->comm || h->band_up < 0)) || (r1 < g.hl && (!h->comm || h->band_dn < 0))))
            return OPOSE_E_ARG;  // the library's exchange needs opose_rccl_init + opose_set_band_peers
        if (xbuf_bytes < 4 * band_halo_bytes(g.wl)) return OPOSE_E_ARG;
        if (!h->x6) throw std::invalid_argument("row bands need the split-bf16 path (OPOSE_CONV=f32 is set)");
        if (!h->loaded[OPOSE_NET_BODY]) throw std::runtime_error("body weights not loaded");
        const uint8_t* fd = bgr;
        if (!(flags & OPOSE_IN_DEVICE)) {
            uint8_t* buf = h->frames.ensure<uint8_t>((size_t)row_stride * H, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, bgr, host_span(1, H, W, row_stride, row_stride * H),
                                           hipMemcpyHostToDevice, h->stream));
            fd = buf;
        }
        const int hb = r1 - r0;
        float* out = (flags & OPOSE_OUT_DEVICE) ? maps : h->maps_in.ensure<float>((size_t)57 * hb * g.wl, h->stream);
        float* x = h->w().x.ensure<float>((size_t)3 * g.Hp * g.Wp, h->stream);
        launch_preprocess(fd, row_stride * H, row_stride, 1, H, W, g.Hs, g.Ws, 1.0 / g.mult, 1.0 / g.mult, g.Hp, g.Wp,
                          (float)p.pad_value / 256.f - 0.5f, x, h->stream);
        const size_t cap = xbuf_bytes / 4;
        const Band band{r0, r1, out, fn, user, static_cast<uint8_t*>(xbuf), cap};
        body_net_x6(h, {NetSeg{x, 1, g.Hp, g.Wp, h->slot}}, &band);
        if (!(flags & OPOSE_OUT_DEVICE)) {
            OPOSE_HIP_CHECK(hipMemcpyAsync(maps, out, (size_t)57 * hb * g.wl * 4, hipMemcpyDeviceToHost, h->stream));
            OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        }
        return OPOSE_OK;
    });
}

int opose_body_post_scales(opose_t* h, const float* const* maps, const int* hl, const int* wl, const int* pad_down,
                           const int* pad_right, int n_scales, int N, int H, int W, const opose_params* pp,
                           void* records, int flags) {
    if (!h || !maps || !hl || !wl || !pad_down || !pad_right || !records || N <= 0 || H <= 0 || W <= 0 ||
        n_scales < 1 || n_scales > OPOSE_MAX_SCALES)
        return OPOSE_E_ARG;
    for (int s = 0; s < n_scales; ++s)
        if (!maps[s] || hl[s] <= 0 || wl[s] <= 0 || pad_down[s] < 0 || pad_right[s] < 0 ||
            pad_down[s] >= 8 * hl[s] || pad_right[s] >= 8 * wl[s])
            return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        opose_params p = fill_params(pp, OPOSE_NET_BODY);
        const RecordLayout L = make_record_layout(h->ppp, h->maxp);
        std::vector<ScaleGeom> gs;
        for (int s = 0; s < n_scales; ++s) {
            ScaleGeom g;
            g.mult = 0;
            g.hl = hl[s];
            g.wl = wl[s];
            g.Hp = 8 * hl[s];
            g.Wp = 8 * wl[s];
            g.Hs = g.Hp - pad_down[s];
            g.Ws = g.Wp - pad_right[s];
            g.up_sy = 1.0 / ((double)H / g.Hs);
            g.up_sx = 1.0 / ((double)W / g.Ws);
            const float* md = maps[s];
            if (!(flags & OPOSE_IN_DEVICE)) {
                const size_t n_in = (size_t)N * 57 * g.hl * g.wl;
                float* buf = h->maps_in.ensure<float>(n_in, h->stream);
                OPOSE_HIP_CHECK(hipMemcpyAsync(buf, maps[s], n_in * 4, hipMemcpyHostToDevice, h->stream));
                md = buf;
            }
            body_to_mid(h, s, md, 57, N, g);
            gs.push_back(g);
        }
        uint8_t* rec = (flags & OPOSE_OUT_DEVICE) ? static_cast<uint8_t*>(records)
                                                  : h->records.ensure<uint8_t>(L.bytes * N, h->stream);
        body_post_common(h, N, H, W, gs, p, rec);
        return finish_records(h, N, records, rec, flags);
    });
}

int opose_batch_body_infer(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride,
                           int64_t frame_stride, const opose_params* pp, void* records, int flags) {
    if (!h || !bgr || !records || N <= 0 || H <= 0 || W <= 0) return OPOSE_E_ARG;
    if (row_stride < (int64_t)W * 3 || frame_stride < row_stride * H) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const opose_params p = fill_params(pp, OPOSE_NET_BODY);
        const RecordLayout L = make_record_layout(h->ppp, h->maxp);
        // Batch_body.calculate_size_pad (srcmx/Batch_model.py:302-307): int() truncation
        const double scale = p.boxsize * p.scales[0] / H;
        const int nh = (int)(H * scale), nw = (int)(W * scale);
        if (nh <= 0 || nw <= 0) throw std::invalid_argument("scale produces an empty image");
        const int Hp = round_up(nh, p.stride), Wp = round_up(nw, p.stride);
        const uint8_t* fd = bgr;
        if (!(flags & OPOSE_IN_DEVICE)) {
            uint8_t* buf = h->frames.ensure<uint8_t>((size_t)frame_stride * N, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, bgr, host_span(N, H, W, row_stride, frame_stride),
                                           hipMemcpyHostToDevice, h->stream));
            fd = buf;
        }
        uint8_t* rec = (flags & OPOSE_OUT_DEVICE) ? static_cast<uint8_t*>(records)
                                                  : h->records.ensure<uint8_t>(L.bytes * N, h->stream);
        const std::string key = call_key("batch_body", N, H, W, row_stride, frame_stride, p, fd, rec, h->ppp, h->maxp);
        run_graphed(h, key, [&] {
            float* x = h->w().x.ensure<float>((size_t)N * 3 * Hp * Wp, h->stream);
            ProfEntry pe;
            h->prof_begin(pe, "preprocess", 0, (double)N * (3.0 * H * W + 12.0 * Hp * Wp));
            const float sc = (float)(1.0 / scale);  // torch: float(1 / scale_factor)
            launch_preprocess_torch(fd, frame_stride, row_stride, N, H, W, nh, nw, sc, sc, Hp, Wp, x, h->stream);
            h->prof_end(pe);
            float* S = body_net(h, x, N, Hp, Wp);
            batch_post_common(h, N, H, W, S, 185, Hp / 8, Wp / 8, nh, nw, p, rec);
        });
        return finish_records(h, N, records, rec, flags);
    });
}

int opose_batch_body_post(opose_t* h, const float* maps, int N, int hl, int wl, int nh, int nw, int H, int W,
                          const opose_params* pp, void* records, int flags) {
    if (!h || !maps || !records || N <= 0 || hl <= 0 || wl <= 0 || H <= 0 || W <= 0) return OPOSE_E_ARG;
    if (nh <= 0 || nw <= 0 || nh > 8 * hl || nw > 8 * wl) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const opose_params p = fill_params(pp, OPOSE_NET_BODY);
        const RecordLayout L = make_record_layout(h->ppp, h->maxp);
        const size_t n_in = (size_t)N * 57 * hl * wl;
        const float* md = maps;
        if (!(flags & OPOSE_IN_DEVICE)) {
            float* buf = h->maps_in.ensure<float>(n_in, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, maps, n_in * 4, hipMemcpyHostToDevice, h->stream));
            md = buf;
        }
        uint8_t* rec = (flags & OPOSE_OUT_DEVICE) ? static_cast<uint8_t*>(records)
                                                  : h->records.ensure<uint8_t>(L.bytes * N, h->stream);
        batch_post_common(h, N, H, W, md, 57, hl, wl, nh, nw, p, rec);
        return finish_records(h, N, records, rec, flags);
    });
}

// Hand post path from per-scale x8 maps (mids[s] = [N][21][Hs][Ws]) to peaks / found.
// mid_crop: first crop of this call inside mids[s] (crop-batched hand path); out_crop: first
// crop's slot in the peaks / found outputs
static void hand_post_common(opose_ctx* h, int N, int H, int W, const std::vector<ScaleGeom>& gs,
                             const opose_params& p, double* peaks_out, int32_t* found_out, int flags,
                             int mid_crop = 0, int out_crop = 0) {
    const int ns = (int)gs.size();
    const int NP = N * 21;
    double* avg = h->avg.ensure<double>((size_t)NP * H * W, h->stream);
    ProfEntry pe;
    HeatScales hsc{};
    hsc.n = ns;
    hsc.ns = (float)ns;
    double mid_bytes = 0;
    for (int s = 0; s < ns && s < kHeatScales; ++s) {
        hsc.s[s] = HeatScale{h->mid(s).ensure<float>(0, h->stream) + (size_t)mid_crop * 21 * gs[s].Hs * gs[s].Ws, 21, 0,
                             gs[s].Hs, gs[s].Ws, gs[s].up_sy, gs[s].up_sx};
        mid_bytes += (double)NP * 4.0 * gs[s].Hs * gs[s].Ws;
    }
    if (h->heat_scales && heat_full_scales_fits(hsc, H, W)) {  // every scale in one launch, the average written once
        h->prof_begin(pe, "heat_full", 0, (double)NP * H * W * 8 + mid_bytes);
        launch_heat_full_scales(hsc, N, 21, H, W, avg, h->stream);
        h->prof_end(pe);
    } else {
        for (int s = 0; s < ns; ++s) {
            h->prof_begin(pe, "heat_full", 0, (double)NP * H * W * 8 * (s ? 2 : 1));
            const float* mid = h->mid(s).ensure<float>(0, h->stream) + (size_t)mid_crop * 21 * gs[s].Hs * gs[s].Ws;
            launch_heat_full(mid, 21, 0, 21, N, gs[s].Hs, gs[s].Ws, H, W, gs[s].up_sy, gs[s].up_sx, ns, s > 0, avg,
                             h->stream);
            h->prof_end(pe);
        }
    }
    int* lab = h->hlab.ensure<int>((size_t)NP * H * W, h->stream);
    double* sums = h->hsums.ensure<double>((size_t)NP * H * W, h->stream);
    int* cnt = h->cnt.ensure<int>((size_t)NP, h->stream);
    double* pk = ((flags & OPOSE_OUT_DEVICE) ? peaks_out
                                             : h->hpeaks.ensure<double>((size_t)(out_crop * 21 + NP) * 3, h->stream)) +
                 (size_t)out_crop * 21 * 3;
    int* fd = ((flags & OPOSE_OUT_DEVICE) ? found_out : h->hfound.ensure<int>((size_t)(out_crop * 21 + NP), h->stream)) +
              (size_t)out_crop * 21;
    OPOSE_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * NP, h->stream));
    h->prof_begin(pe, "gauss_threshold", 0, (double)NP * H * W * 12);
    launch_gauss_threshold(avg, NP, H, W, p.thre_hand, lab, cnt, sums, h->stream);
    h->prof_end(pe);
    h->prof_begin(pe, "hand_cc", 0, 0);
    void* ws = h->hsel.ensure<uint8_t>(hand_cc_workspace_bytes(NP), h->stream);
    launch_hand_cc(avg, NP, H, W, lab, sums, cnt, pk, fd, ws, true, h->stream);
    h->prof_end(pe);
}

// copy the hand results to the host (unless they were written to device buffers)
static void hand_finish(opose_ctx* h, int N, double* peaks_out, int32_t* found_out, int flags) {
    const int NP = N * 21;
    if (!(flags & OPOSE_OUT_DEVICE)) {
        double* st = h->hand_out.ensure<double>((size_t)NP * 4);  // NP * 3 peaks, then NP found
        int32_t* sf = reinterpret_cast<int32_t*>(st + (size_t)NP * 3);
        OPOSE_HIP_CHECK(hipMemcpyAsync(st, h->hpeaks.ensure<double>((size_t)NP * 3, h->stream), sizeof(double) * NP * 3,
                                       hipMemcpyDeviceToHost, h->stream));
        OPOSE_HIP_CHECK(hipMemcpyAsync(sf, h->hfound.ensure<int>((size_t)NP, h->stream), sizeof(int) * NP,
                                       hipMemcpyDeviceToHost, h->stream));
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        std::memcpy(peaks_out, st, sizeof(double) * NP * 3);
        std::memcpy(found_out, sf, sizeof(int32_t) * NP);
    }
    h->prof_drain();
}

int opose_hand_infer(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride, int64_t frame_stride,
                     const opose_params* pp, double* peaks, int32_t* found, int flags) {
    if (!h || !bgr || !peaks || !found || N <= 0 || H <= 0 || W <= 0) return OPOSE_E_ARG;
    if (row_stride < (int64_t)W * 3 || frame_stride < row_stride * H) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const opose_params p = fill_params(pp, OPOSE_NET_HAND);
        const uint8_t* fd = bgr;
        if (!(flags & OPOSE_IN_DEVICE)) {
            uint8_t* buf = h->frames.ensure<uint8_t>((size_t)frame_stride * N, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, bgr, host_span(N, H, W, row_stride, frame_stride),
                                           hipMemcpyHostToDevice, h->stream));
            fd = buf;
        }
        std::vector<ScaleGeom> gs;
        for (int s = 0; s < p.n_scales; ++s) gs.push_back(geom(p.scales[s], p, H, W));
        const bool od = flags & OPOSE_OUT_DEVICE;
        char fk[32];
        std::snprintf(fk, sizeof fk, "%p", od ? (const void*)found : nullptr);
        const std::string key =
            call_key("hand", N, H, W, row_stride, frame_stride, p, fd, od ? (const void*)peaks : nullptr, 0, 0) + fk;
        auto scale_net = [&](int s) {
            const ScaleGeom& g = gs[s];
            float* x = h->w().x.ensure<float>((size_t)N * 3 * g.Hp * g.Wp, h->stream);
            ProfEntry pe;
            h->prof_begin(pe, "preprocess", 0, (double)N * (3.0 * H * W + 12.0 * g.Hp * g.Wp));
            launch_preprocess(fd, frame_stride, row_stride, N, H, W, g.Hs, g.Ws, 1.0 / g.mult, 1.0 / g.mult, g.Hp,
                              g.Wp, (float)p.pad_value / 256.f - 0.5f, x, h->stream);
            h->prof_end(pe);
            float* Sb = hand_net(h, x, N, g.Hp, g.Wp);
            upsample_to_mid(h, s, Sb, 150, N, g, 21);
        };
        if (h->x6 && h->lockstep && p.n_scales > 1) {
            run_graphed(h, key, [&] {
                run_scales_lockstep(h, OPOSE_NET_HAND, fd, frame_stride, row_stride, N, H, W, gs, p);
                hand_post_common(h, N, H, W, gs, p, peaks, found, flags & OPOSE_OUT_DEVICE);
            });
        } else if (h->scale_streams && p.n_scales > 1) {
            // the scales' networks are independent until the heat average: each on its own stream
            // with its own workspace (a single crop's layers fill a fraction of the chip each)
            run_scales_concurrently(h, p.n_scales, scale_net);
            hand_post_common(h, N, H, W, gs, p, peaks, found, flags & OPOSE_OUT_DEVICE);
        } else {
            run_graphed(h, key, [&] {
                for (int s = 0; s < p.n_scales; ++s) scale_net(s);
                hand_post_common(h, N, H, W, gs, p, peaks, found, flags & OPOSE_OUT_DEVICE);
            });
        }
        hand_finish(h, N, peaks, found, flags & OPOSE_OUT_DEVICE);
    });
    return OPOSE_OK;
}

// Batch_hand after the network (srcmx/Batch_model.py:334-354): maps [N][cstride][H/8][W/8]
// with the 22 heat channels first
static void batch_hand_post_common(opose_ctx* h, int N, int H, int W, const float* maps, int cstride,
                                   const opose_params& p, double* peaks, int32_t* found, int flags) {
    const int NP = N * 21;
    ProfEntry pe;
    float* mid = h->mid(0).ensure<float>((size_t)NP * H * W, h->stream);
    h->prof_begin(pe, "upsample8", 0, (double)NP * H * W * 4);
    launch_upsample8_torch(maps, cstride, 0, 21, N, H / 8, W / 8, H, W, mid, h->stream);
    h->prof_end(pe);
    double* avg = h->avg.ensure<double>((size_t)NP * H * W, h->stream);
    int* lab = h->hlab.ensure<int>((size_t)NP * H * W, h->stream);
    double* sums = h->hsums.ensure<double>((size_t)NP * H * W, h->stream);
    int* cnt = h->cnt.ensure<int>((size_t)NP, h->stream);
    const bool od = flags & OPOSE_OUT_DEVICE;
    double* pk = od ? peaks : h->hpeaks.ensure<double>((size_t)NP * 3, h->stream);
    int* fo = od ? found : h->hfound.ensure<int>((size_t)NP, h->stream);
    OPOSE_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * NP, h->stream));
    h->prof_begin(pe, "gauss_threshold", 0, (double)NP * H * W * 16);
    launch_blur5_seed(mid, NP, H, W, p.thre_hand, avg, lab, cnt, h->stream);
    h->prof_end(pe);
    h->prof_begin(pe, "hand_cc", 0, 0);
    void* ws = h->hsel.ensure<uint8_t>(hand_cc_workspace_bytes(NP), h->stream);
    launch_hand_cc(avg, NP, H, W, lab, sums, cnt, pk, fo, ws, false, h->stream);
    h->prof_end(pe);
    hand_finish(h, N, peaks, found, flags & OPOSE_OUT_DEVICE);
}

int opose_batch_hand_post(opose_t* h, const float* maps, int N, int hl, int wl, const opose_params* pp, double* peaks,
                          int32_t* found, int flags) {
    if (!h || !maps || !peaks || !found || N <= 0 || hl <= 0 || wl <= 0) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const opose_params p = fill_params(pp, OPOSE_NET_HAND);
        const size_t n_in = (size_t)N * 22 * hl * wl;
        const float* md = maps;
        if (!(flags & OPOSE_IN_DEVICE)) {
            float* buf = h->maps_in.ensure<float>(n_in, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, maps, n_in * 4, hipMemcpyHostToDevice, h->stream));
            md = buf;
        }
        batch_hand_post_common(h, N, 8 * hl, 8 * wl, md, 22, p, peaks, found, flags);
    });
    return OPOSE_OK;
}

int opose_batch_hand_infer(opose_t* h, const uint8_t* bgr, int N, int H, int W, int64_t row_stride,
                           int64_t frame_stride, const opose_params* pp, double* peaks, int32_t* found, int flags) {
    if (!h || !bgr || !peaks || !found || N <= 0 || H <= 0 || W <= 0 || H % 8 || W % 8) return OPOSE_E_ARG;
    if (row_stride < (int64_t)W * 3 || frame_stride < row_stride * H) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const opose_params p = fill_params(pp, OPOSE_NET_HAND);
        const uint8_t* fd = bgr;
        if (!(flags & OPOSE_IN_DEVICE)) {
            uint8_t* buf = h->frames.ensure<uint8_t>((size_t)frame_stride * N, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(buf, bgr, host_span(N, H, W, row_stride, frame_stride),
                                           hipMemcpyHostToDevice, h->stream));
            fd = buf;
        }
        // ToTensor - 0.5 at scale 1 (torch bicubic at scale 1 is the identity)
        float* x = h->w().x.ensure<float>((size_t)N * 3 * H * W, h->stream);
        ProfEntry pe;
        h->prof_begin(pe, "preprocess", 0, (double)N * 15.0 * H * W);
        launch_preprocess_torch(fd, frame_stride, row_stride, N, H, W, H, W, 1.f, 1.f, H, W, x, h->stream);
        h->prof_end(pe);
        float* Sb = hand_net(h, x, N, H, W);
        batch_hand_post_common(h, N, H, W, Sb, 150, p, peaks, found, flags);
        hand_finish(h, N, peaks, found, flags & OPOSE_OUT_DEVICE);
    });
    return OPOSE_OK;
}

int opose_hand_infer_crops(opose_t* h, const uint8_t* const* crops, const int* sizes, const int64_t* row_strides,
                           int n, const opose_params* pp, double* peaks, int32_t* found, int flags) {
    if (!h || !crops || !sizes || !row_strides || !peaks || !found || n <= 0) return OPOSE_E_ARG;
    for (int i = 0; i < n; ++i)
        if (!crops[i] || sizes[i] <= 0 || row_strides[i] < (int64_t)sizes[i] * 3) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const opose_params p = fill_params(pp, OPOSE_NET_HAND);
        const int ns = p.n_scales;
        // per-crop geometry; the network side (Hs, Ws, Hp, Wp per scale) must agree across crops
        std::vector<std::vector<ScaleGeom>> gs(n);
        for (int i = 0; i < n; ++i)
            for (int s = 0; s < ns; ++s) gs[i].push_back(geom(p.scales[s], p, sizes[i], sizes[i]));
        for (int i = 1; i < n; ++i)
            for (int s = 0; s < ns; ++s)
                if (gs[i][s].Hs != gs[0][s].Hs || gs[i][s].Ws != gs[0][s].Ws)
                    throw std::invalid_argument("crops do not share the network input size of a scale");
        // stage the crops (host -> one device buffer)
        std::vector<size_t> off(n + 1, 0);
        for (int i = 0; i < n; ++i) off[i + 1] = off[i] + (size_t)row_strides[i] * sizes[i];
        const uint8_t* base = nullptr;
        uint8_t* buf = nullptr;
        if (!(flags & OPOSE_IN_DEVICE)) {
            buf = h->frames.ensure<uint8_t>(off[n], h->stream);
            for (int i = 0; i < n; ++i)
                OPOSE_HIP_CHECK(hipMemcpyAsync(buf + off[i], crops[i], host_span(1, sizes[i], sizes[i], row_strides[i], 0),
                                               hipMemcpyHostToDevice, h->stream));
        }
        // all crops of a scale form one batch; with the split-bf16 path all scales run in lockstep
        // (one conv launch per layer for every crop and scale).  Batches are cut so that the
        // largest activation (64 channels at the largest scale's full resolution, X6: 3 x 128 B
        // per pixel) stays below the 2 GiB the conv kernels address with 32-bit offsets.
        const bool lockstep = h->x6 && h->lockstep && ns > 1;
        if (lockstep && !h->loaded[OPOSE_NET_HAND]) throw std::runtime_error("hand weights not loaded");
        size_t maxpix = 0;
        for (int s = 0; s < ns; ++s) maxpix = std::max(maxpix, (size_t)gs[0][s].Hp * gs[0][s].Wp);
        const int chunk = (int)std::max<size_t>(1, (((size_t)1 << 31) - 1) / (3 * 128 * maxpix));
        // size every per-crop buffer for the largest crop / all crops up front: a reallocation
        // after the first batch would drop the results of the crops already done
        const int wmax = *std::max_element(sizes, sizes + n);
        h->avg.ensure<double>((size_t)21 * wmax * wmax, h->stream);
        h->hlab.ensure<int>((size_t)21 * wmax * wmax, h->stream);
        h->hsums.ensure<double>((size_t)21 * wmax * wmax, h->stream);
        if (!(flags & OPOSE_OUT_DEVICE)) {
            h->hpeaks.ensure<double>((size_t)n * 21 * 3, h->stream);
            h->hfound.ensure<int>((size_t)n * 21, h->stream);
        }
        for (int c0 = 0; c0 < n; c0 += chunk) {
            const int nc = std::min(chunk, n - c0);
            std::vector<NetSeg> segs;
            for (int s = 0; s < ns; ++s) {
                const ScaleGeom& g0 = gs[0][s];
                float* x = h->ws[lockstep ? s : h->slot].x.ensure<float>((size_t)nc * 3 * g0.Hp * g0.Wp, h->stream);
                ProfEntry pe;
                h->prof_begin(pe, "preprocess", 0, 0);
                for (int i = c0; i < c0 + nc; ++i) {
                    const ScaleGeom& g = gs[i][s];
                    const uint8_t* src = buf ? buf + off[i] : crops[i];
                    launch_preprocess(src, (int64_t)(off[i + 1] - off[i]), row_strides[i], 1, sizes[i], sizes[i], g.Hs,
                                      g.Ws, 1.0 / g.mult, 1.0 / g.mult, g.Hp, g.Wp, (float)p.pad_value / 256.f - 0.5f,
                                      x + (size_t)(i - c0) * 3 * g.Hp * g.Wp, h->stream);
                }
                h->prof_end(pe);
                if (lockstep) {
                    segs.push_back(NetSeg{x, nc, g0.Hp, g0.Wp, s});
                    continue;
                }
                float* Sb = hand_net(h, x, nc, g0.Hp, g0.Wp);
                upsample_to_mid(h, s, Sb, 150, nc, g0, 21);
            }
            if (lockstep) {
                const std::vector<float*> outs = hand_net_x6(h, segs);
                for (int s = 0; s < ns; ++s) upsample_to_mid(h, s, outs[s], 150, nc, gs[0][s], 21);
            }
            for (int i = c0; i < c0 + nc; ++i)
                hand_post_common(h, 1, sizes[i], sizes[i], gs[i], p, peaks, found, flags & OPOSE_OUT_DEVICE, i - c0, i);
        }
        (void)base;
        hand_finish(h, n, peaks, found, flags & OPOSE_OUT_DEVICE);
    });
    return OPOSE_OK;
}

int opose_hand_post(opose_t* h, const float* const* maps, const int* hl, const int* wl, const int* pad_down,
                    const int* pad_right, int n_scales, int N, int H, int W, const opose_params* pp,
                    double* peaks, int32_t* found, int flags) {
    if (!h || !maps || !hl || !wl || !pad_down || !pad_right || !peaks || !found || N <= 0 || H <= 0 || W <= 0 ||
        n_scales < 1 || n_scales > OPOSE_MAX_SCALES)
        return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        opose_params p = fill_params(pp, OPOSE_NET_HAND);
        std::vector<ScaleGeom> gs;
        for (int s = 0; s < n_scales; ++s) {
            ScaleGeom g;
            g.mult = 0;
            g.hl = hl[s];
            g.wl = wl[s];
            g.Hp = 8 * hl[s];
            g.Wp = 8 * wl[s];
            g.Hs = g.Hp - pad_down[s];
            g.Ws = g.Wp - pad_right[s];
            if (g.Hs <= 0 || g.Ws <= 0) throw std::invalid_argument("bad pad");
            g.up_sy = 1.0 / ((double)H / g.Hs);
            g.up_sx = 1.0 / ((double)W / g.Ws);
            const size_t n_in = (size_t)N * 22 * g.hl * g.wl;
            const float* md = maps[s];
            if (!(flags & OPOSE_IN_DEVICE)) {
                float* buf = h->maps_in.ensure<float>(n_in, h->stream);
                OPOSE_HIP_CHECK(hipMemcpyAsync(buf, maps[s], n_in * 4, hipMemcpyHostToDevice, h->stream));
                md = buf;
            }
            upsample_to_mid(h, s, md, 22, N, g, 21);
            gs.push_back(g);
        }
        hand_post_common(h, N, H, W, gs, p, peaks, found, flags & OPOSE_OUT_DEVICE);
        hand_finish(h, N, peaks, found, flags & OPOSE_OUT_DEVICE);
    });
    return OPOSE_OK;
}

// ------------------------------------------------------------------ test hooks
int opose_debug_conv(opose_t* h, const float* x, const float* w, const float* b, int N, int Cin, int H, int W,
                     int Cout, int ks, int pad, int relu, int mt, int pt, int splits, float* out) {
    if (!h || !x || !w || !b || !out || ks > 15 || pad > 7) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        Spec s{"debug", Cin, Cout, ks, pad};
        upload_conv(h, 0, "__debug__", {&s}, {w}, {b});
        DevConv* c = h->convs[0]["__debug__"].get();
        DevBuf xin, yout;
        const size_t nx = (size_t)N * Cin * H * W, ny = (size_t)N * Cout * H * W;
        float* xd = xin.ensure<float>(nx, h->stream);
        float* yd = yout.ensure<float>(ny, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(xd, x, nx * 4, hipMemcpyHostToDevice, h->stream));
        ConvArgs a{};
        a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.ks = ks; a.pad = pad;
        a.K = c->K; a.Kpad = c->Kpad; a.Mpad = c->Mpad; a.npix = N * H * W;
        a.tap_major = c->tap_major ? 1 : 0;
        ConvGroup& G = a.g[0];
        G.in = xd; G.in_cstride = Cin; G.in_coff = 0; G.wt = c->wt; G.bias = c->bias;
        G.out = yd; G.out_cstride = Cout; G.out_coff = 0; G.out2 = nullptr; G.cout = Cout; G.relu = relu;
        a.g[1] = a.g[0];
        TileChoice t = choose_tile(a.Mpad, {a.npix}, a.Kpad / 32);
        if (mt > 0) { t.mt = mt; t.pt = pt; t.grid = (a.Mpad / mt) * ((a.npix + pt - 1) / pt); }
        if (splits > 0) t.grid = splits;
        if (a.Mpad % t.mt) throw std::invalid_argument("tile M does not divide Mpad");
        a.ngroups = 1;
        a.sk_grid = t.grid;
        a.partial = h->w().partial.ensure<float>((size_t)2 * t.grid * t.mt * t.pt, h->stream);
        launch_conv(a, c->ktab, t.mt, t.pt, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(out, yd, ny * 4, hipMemcpyDeviceToHost, h->stream));
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        h->convs[0].erase("__debug__");
    });
    return OPOSE_OK;
}

// Test-hook plan of a conv_x6 launch (groups filled): tile mt x pt (0: choose_tile's data-parallel
// pick), `slabs` k slabs per tile (<= 1: one; clamped to nK), one workgroup per whole tile or,
// with slabs, min(units, 256) workgroups over contiguous unit ranges; sets grid, units, partials.
static TileChoice debug_x6_plan(opose_ctx* h, X6Args& a, int mt, int pt, int slabs) {
    std::vector<int> gpix;
    for (int g = 0; g < a.ngroups; ++g) gpix.push_back(a.g[g].npix);
    TileChoice t = choose_tile(a.Mpad, gpix, a.nK, true, true);
    if (mt > 0) {
        t.mt = mt;
        t.pt = pt;
    }
    if (a.Mpad % t.mt) throw std::invalid_argument("tile M does not divide Mpad");
    for (int g = 0; g < a.ngroups; ++g) a.g[g].slabs = std::max(1, std::min(slabs, a.nK));
    const X6Args num = x6_number_tiles(a, t.mt, t.pt);
    t.grid = num.units == num.tiles ? num.tiles : std::min(num.units, 256);
    a.sk_grid = t.grid;
    a.sched = nullptr;
    a.partial = h->w().partial.ensure<float>((size_t)num.units * t.mt * t.pt, h->stream);
    return t;
}

// split-bf16 conv of one layer: x fp32 NCHW -> X6 -> conv_x6 -> fp32 (out_x6: through an X6
// output buffer and back, exercising the split epilogue)
int opose_debug_conv_x6(opose_t* h, const float* x, const float* w, const float* b, int N, int Cin, int H, int W,
                        int Cout, int ks, int pad, int relu, int mt, int pt, int splits, int out_x6, float* out) {
    if (!h || !x || !w || !b || !out || ks > 15 || pad > 7) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        Spec s{"debug", Cin, Cout, ks, pad};
        upload_conv(h, 0, "__debug__", {&s}, {w}, {b});
        DevConv* c = h->convs[0]["__debug__"].get();
        const int HW = H * W;
        const int cg = c->cin_g, og = (Cout + 7) / 8;
        if (mt <= -2) {
            // padded (X6P) input and output through run_conv_x6_segs with the family under test
            // forced: -2 the window kernel, -3 Winograd (conv_wino_x6); the host splits and joins
            const size_t plane = x6p_plane(N, H, W), P = (size_t)x6p_pitch(W);
            auto rne = [](float v) -> uint16_t {
                uint32_t u;
                std::memcpy(&u, &v, 4);
                u += 0x7fffu + ((u >> 16) & 1u);
                return (uint16_t)(u >> 16);
            };
            auto f16 = [](uint16_t hb) {
                const uint32_t u = (uint32_t)hb << 16;
                float v;
                std::memcpy(&v, &u, 4);
                return v;
            };
            std::vector<uint16_t> hx((size_t)3 * cg * plane * 8, 0);
            const size_t ipl = (size_t)cg * plane * 8;  // bf16 per piece
            for (int n = 0; n < N; ++n)
                for (int ch = 0; ch < Cin; ++ch)
                    for (int y = 0; y < H; ++y)
                        for (int xx0 = 0; xx0 < W; ++xx0) {
                            const float v = x[(((size_t)n * Cin + ch) * H + y) * W + xx0];
                            const size_t u = (size_t)(ch / 8) * plane + (3 + (size_t)n * (H + 3) + y) * P + 3 + xx0;
                            const uint16_t h0 = rne(v);
                            const float r = v - f16(h0);
                            const uint16_t h1 = rne(r);
                            const uint16_t h2 = rne(r - f16(h1));
                            hx[u * 8 + ch % 8] = h0;
                            hx[ipl + u * 8 + ch % 8] = h1;
                            hx[2 * ipl + u * 8 + ch % 8] = h2;
                        }
            DevBuf bi, bo;
            uint8_t* xi = bi.ensure<uint8_t>(hx.size() * 2, h->stream);
            const size_t opl = (size_t)og * plane * 8;
            uint8_t* yo = bo.ensure<uint8_t>(3 * opl * 2, h->stream);
            OPOSE_HIP_CHECK(hipMemcpyAsync(xi, hx.data(), hx.size() * 2, hipMemcpyHostToDevice, h->stream));
            OPOSE_HIP_CHECK(hipMemsetAsync(yo, 0, 3 * opl * 2, h->stream));
            ConvSeg sg{c, N, H, W, x6pact(xi, cg, 0, N, H, W), x6pact(yo, og, 0, N, H, W), XAct{}, relu != 0};
            if (mt == -3) sg.slabs = 1;
            h->force_kernel = mt == -3 ? kKernelWino : kKernelWin;
            try {
                run_conv_x6_segs(h, {sg});
            } catch (...) {
                h->force_kernel = -1;
                throw;
            }
            h->force_kernel = -1;
            std::vector<uint16_t> hy(3 * opl);
            OPOSE_HIP_CHECK(hipMemcpyAsync(hy.data(), yo, hy.size() * 2, hipMemcpyDeviceToHost, h->stream));
            OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
            for (int n = 0; n < N; ++n)
                for (int ch = 0; ch < Cout; ++ch)
                    for (int y = 0; y < H; ++y)
                        for (int xx0 = 0; xx0 < W; ++xx0) {
                            const size_t u = (size_t)(ch / 8) * plane + (3 + (size_t)n * (H + 3) + y) * P + 3 + xx0;
                            out[(((size_t)n * Cout + ch) * H + y) * W + xx0] =
                                (f16(hy[u * 8 + ch % 8]) + f16(hy[opl + u * 8 + ch % 8])) + f16(hy[2 * opl + u * 8 + ch % 8]);
                        }
            h->convs[0].erase("__debug__");
            return OPOSE_OK;
        }
        DevBuf xin, xx, yx, yout;
        const size_t nx = (size_t)N * Cin * HW, ny = (size_t)N * Cout * HW;
        const uint32_t ips = (uint32_t)((size_t)N * cg * HW * 16), ops = (uint32_t)((size_t)N * og * HW * 16);
        float* xd = xin.ensure<float>(nx, h->stream);
        uint8_t* x6 = xx.ensure<uint8_t>((size_t)ips * 3, h->stream);
        uint8_t* y6 = yx.ensure<uint8_t>((size_t)ops * 3, h->stream);
        float* yd = yout.ensure<float>(ny, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(xd, x, nx * 4, hipMemcpyHostToDevice, h->stream));
        launch_to_x6(xd, Cin, 0, Cin, N, HW, x6, cg, 0, ips, h->stream);
        X6Args a{};
        a.ks = ks; a.pad = pad;
        a.cin_g = cg; a.small = c->small6 ? 1 : 0; a.nK = c->nK6; a.Mpad = c->Mpad;
        X6Group& G = a.g[0];
        G.N = N; G.H = H; G.W = W; G.npix = N * HW;
        G.in = x6; G.in_ps = ips; G.in_l = x6act(x6, cg, 0, N, H, W).l;
        G.wt = c->wx6; G.bias = c->bias; G.cout = Cout; G.relu = relu; G.out2 = nullptr;
        if (out_x6) { G.out = y6; G.out_ps = ops; G.out_l = x6act(y6, og, 0, N, H, W).l; G.out_f32 = 0; }
        else { G.out = yd; G.out_c = Cout; G.out_off = 0; G.out_f32 = 1; }
        a.ngroups = 1;
        const TileChoice t = debug_x6_plan(h, a, mt, pt, splits);
        launch_conv_x6(a, t.mt, t.pt, h->stream);
        if (out_x6) launch_from_x6(y6, og, 0, ops, Cout, N, HW, yd, Cout, 0, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(out, yd, ny * 4, hipMemcpyDeviceToHost, h->stream));
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        h->convs[0].erase("__debug__");
    });
    return OPOSE_OK;
}

// timing of one split-bf16 conv launch configuration on hashed data
int opose_debug_conv_x6_time(opose_t* h, int N, int Cin, int H, int W, int Cout, int ks, int ngroups, int mt, int pt,
                             int splits, int reps, float* ms) {
    if (!h || !ms || reps < 1 || ngroups < 1 || ngroups > 2) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        Spec s{"timing", Cin, Cout, ks, ks / 2};
        std::vector<float> w((size_t)Cout * Cin * ks * ks), b(Cout, 0.f);
        for (size_t i = 0; i < w.size(); ++i) w[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
        upload_conv(h, 0, "__timing__", {&s}, {w.data()}, {b.data()});
        DevConv* c = h->convs[0]["__timing__"].get();
        const int HW = H * W;
        const int cg = c->cin_g, og = (Cout + 7) / 8;
        const uint32_t ips = (uint32_t)((size_t)ngroups * N * cg * HW * 16);
        const uint32_t ops = (uint32_t)((size_t)ngroups * N * og * HW * 16);
        DevBuf xin, xx, yx;
        float* xd = xin.ensure<float>((size_t)ngroups * N * cg * 8 * HW, h->stream);
        launch_fill_hash(xd, (size_t)ngroups * N * cg * 8 * HW, 0x80000003u, h->stream);
        uint8_t* x6 = xx.ensure<uint8_t>((size_t)ips * 3, h->stream);
        uint8_t* y6 = yx.ensure<uint8_t>((size_t)ops * 3, h->stream);
        launch_to_x6(xd, cg * 8, 0, cg * 8, ngroups * N, HW, x6, cg, 0, ips, h->stream);
        X6Args a{};
        a.ks = ks; a.pad = ks / 2;
        a.cin_g = cg; a.small = c->small6 ? 1 : 0; a.nK = c->nK6; a.Mpad = c->Mpad;
        for (int g = 0; g < ngroups; ++g) {
            X6Group& G = a.g[g];
            const int gg = g;
            G.N = N; G.H = H; G.W = W; G.npix = N * HW;
            G.in = x6 + (size_t)gg * N * cg * HW * 16; G.in_ps = ips; G.in_l = x6act(x6, cg, 0, N, H, W).l;
            G.wt = c->wx6; G.bias = c->bias; G.cout = Cout; G.relu = 1; G.out2 = nullptr;
            G.out = y6 + (size_t)gg * N * og * HW * 16; G.out_ps = ops; G.out_l = x6act(y6, og, 0, N, H, W).l;
            G.out_f32 = 0;
        }
        a.ngroups = ngroups;
        const TileChoice t = debug_x6_plan(h, a, mt, pt, splits);
        launch_conv_x6(a, t.mt, t.pt, h->stream);  // warm-up
        hipEvent_t e0, e1;
        OPOSE_HIP_CHECK(hipEventCreate(&e0));
        OPOSE_HIP_CHECK(hipEventCreate(&e1));
        OPOSE_HIP_CHECK(hipEventRecord(e0, h->stream));
        for (int r = 0; r < reps; ++r) launch_conv_x6(a, t.mt, t.pt, h->stream);
        OPOSE_HIP_CHECK(hipEventRecord(e1, h->stream));
        OPOSE_HIP_CHECK(hipEventSynchronize(e1));
        OPOSE_HIP_CHECK(hipEventElapsedTime(ms, e0, e1));
        *ms /= reps;
        OPOSE_HIP_CHECK(hipEventDestroy(e0));
        OPOSE_HIP_CHECK(hipEventDestroy(e1));
        h->convs[0].erase("__timing__");
    });
    return OPOSE_OK;
}

// timing of one conv launch configuration on hashed data (ablate: see ConvArgs::ablate)
int opose_debug_conv_time(opose_t* h, int N, int Cin, int H, int W, int Cout, int ks, int ngroups, int mt, int pt,
                          int splits, int ablate, int reps, float* ms) {
    if (!h || !ms || reps < 1 || ngroups < 1 || ngroups > 2) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        Spec s{"timing", Cin, Cout, ks, ks / 2};
        std::vector<float> w((size_t)Cout * Cin * ks * ks, 0.01f), b(Cout, 0.f);
        upload_conv(h, 0, "__timing__", {&s}, {w.data()}, {b.data()});
        DevConv* c = h->convs[0]["__timing__"].get();
        launch_fill_hash(c->wt, (size_t)c->Kpad * c->Mpad, 7, h->stream);
        DevBuf xin, yout;
        const size_t nx = (size_t)ngroups * N * Cin * H * W, ny = (size_t)ngroups * N * Cout * H * W;
        float* xd = xin.ensure<float>(nx, h->stream);
        float* yd = yout.ensure<float>(ny, h->stream);
        launch_fill_hash(xd, nx, 3u, h->stream);
        ConvArgs a{};
        a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.ks = ks; a.pad = ks / 2;
        a.K = c->K; a.Kpad = c->Kpad; a.Mpad = c->Mpad; a.npix = N * H * W;
        a.tap_major = c->tap_major ? 1 : 0;
        for (int g = 0; g < 2; ++g) {
            ConvGroup& G = a.g[g];
            const int gg = g < ngroups ? g : 0;
            G.in = xd + (size_t)gg * N * Cin * H * W; G.in_cstride = Cin; G.in_coff = 0; G.wt = c->wt; G.bias = c->bias;
            G.out = yd + (size_t)gg * N * Cout * H * W; G.out_cstride = Cout; G.out_coff = 0; G.out2 = nullptr;
            G.cout = Cout; G.relu = 1;
        }
        TileChoice t = choose_tile(a.Mpad, std::vector<int>(ngroups, a.npix), a.Kpad / 32);
        if (mt > 0) { t.mt = mt; t.pt = pt; t.grid = (a.Mpad / mt) * ((a.npix + pt - 1) / pt) * ngroups; }
        if (splits > 0) t.grid = splits;
        if (a.Mpad % t.mt) throw std::invalid_argument("tile M does not divide Mpad");
        a.ngroups = ngroups;
        a.sk_grid = t.grid;
        a.partial = h->w().partial.ensure<float>((size_t)2 * t.grid * t.mt * t.pt, h->stream);
        if (ablate) throw std::invalid_argument("timing ablations were removed");
        auto go = [&]() { launch_conv(a, c->ktab, t.mt, t.pt, h->stream); };
        go();  // warm-up
        hipEvent_t e0, e1;
        OPOSE_HIP_CHECK(hipEventCreate(&e0));
        OPOSE_HIP_CHECK(hipEventCreate(&e1));
        OPOSE_HIP_CHECK(hipEventRecord(e0, h->stream));
        for (int r = 0; r < reps; ++r) go();
        OPOSE_HIP_CHECK(hipEventRecord(e1, h->stream));
        OPOSE_HIP_CHECK(hipEventSynchronize(e1));
        OPOSE_HIP_CHECK(hipEventElapsedTime(ms, e0, e1));
        *ms /= reps;
        OPOSE_HIP_CHECK(hipEventDestroy(e0));
        OPOSE_HIP_CHECK(hipEventDestroy(e1));
        h->convs[0].erase("__timing__");
    });
    return OPOSE_OK;
}

int opose_debug_preprocess(opose_t* h, const uint8_t* bgr, int H, int W, double scale, int pad_value, float* out,
                           int* HpWp) {
    if (!h || !bgr || !HpWp) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        opose_params p;
        opose_default_params(OPOSE_NET_BODY, &p);
        const ScaleGeom g = geom(scale, p, H, W);
        HpWp[0] = g.Hp;
        HpWp[1] = g.Wp;
        if (!out) return OPOSE_OK;
        DevBuf fin, xo;
        uint8_t* fd = fin.ensure<uint8_t>((size_t)H * W * 3, h->stream);
        float* xd = xo.ensure<float>((size_t)3 * g.Hp * g.Wp, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(fd, bgr, (size_t)H * W * 3, hipMemcpyHostToDevice, h->stream));
        launch_preprocess(fd, (int64_t)H * W * 3, (int64_t)W * 3, 1, H, W, g.Hs, g.Ws, 1.0 / g.mult, 1.0 / g.mult, g.Hp,
                          g.Wp, (float)pad_value / 256.f - 0.5f, xd, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(out, xd, (size_t)3 * g.Hp * g.Wp * 4, hipMemcpyDeviceToHost, h->stream));
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
    });
    return OPOSE_OK;
}

// maps [57][hl][wl] -> heat_avg [18][H][W] (float64) and PAF x8 map [38][Hs][Ws] (float32)
int opose_debug_heat(opose_t* h, const float* maps, int hl, int wl, int pad_down, int pad_right, int H, int W,
                     double* heat_avg, float* paf_mid) {
    if (!h || !maps || !heat_avg) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        DevBuf min_;
        float* md = min_.ensure<float>((size_t)57 * hl * wl, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(md, maps, (size_t)57 * hl * wl * 4, hipMemcpyHostToDevice, h->stream));
        ScaleGeom g;
        g.hl = hl; g.wl = wl; g.Hp = 8 * hl; g.Wp = 8 * wl; g.Hs = g.Hp - pad_down; g.Ws = g.Wp - pad_right;
        g.up_sy = 1.0 / ((double)H / g.Hs);
        g.up_sx = 1.0 / ((double)W / g.Ws);
        upsample_to_mid(h, 0, md, 57, 1, g, 56);
        double* avg = h->avg.ensure<double>((size_t)18 * H * W, h->stream);
        launch_heat_full(h->mid(0).ensure<float>(0, h->stream), 56, 38, 18, 1, g.Hs, g.Ws, H, W, g.up_sy, g.up_sx, 1, 0,
                         avg, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(heat_avg, avg, (size_t)18 * H * W * 8, hipMemcpyDeviceToHost, h->stream));
        if (paf_mid)
            OPOSE_HIP_CHECK(hipMemcpyAsync(paf_mid, h->mid(0).ensure<float>(0, h->stream),
                                           (size_t)38 * g.Hs * g.Ws * 4, hipMemcpyDeviceToHost, h->stream));
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
    });
    return OPOSE_OK;
}

int opose_debug_hand_label(opose_t* h, const double* maps, int NP, int H, int W, double thre, int32_t* labels,
                           double* sums) {
    if (!h || !maps || !labels || !sums || NP <= 0 || H <= 0 || W <= 0) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        enter_main(h);
        const size_t n = (size_t)NP * H * W;
        DevBuf mb, lb, sb, cb, pk, fd, ws;
        double* md = mb.ensure<double>(n, h->stream);
        int* lab = lb.ensure<int>(n, h->stream);
        double* sd = sb.ensure<double>(n, h->stream);
        int* cnt = cb.ensure<int>((size_t)NP, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(md, maps, n * 8, hipMemcpyHostToDevice, h->stream));
        OPOSE_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * NP, h->stream));
        launch_gauss_threshold(md, NP, H, W, thre, lab, cnt, sd, h->stream);
        launch_hand_cc(md, NP, H, W, lab, sd, cnt, pk.ensure<double>((size_t)NP * 3, h->stream),
                       fd.ensure<int>((size_t)NP, h->stream), ws.ensure<uint8_t>(hand_cc_workspace_bytes(NP), h->stream),
                       true, h->stream);
        OPOSE_HIP_CHECK(hipMemcpyAsync(labels, lab, n * 4, hipMemcpyDeviceToHost, h->stream));
        OPOSE_HIP_CHECK(hipMemcpyAsync(sums, sd, n * 8, hipMemcpyDeviceToHost, h->stream));
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
    });
    return OPOSE_OK;
}

int opose_profile_enable(opose_t* h, int enable) {
    if (!h) return OPOSE_E_ARG;
    h->prof = enable != 0;
    h->detail = enable == 2;
    h->prof_conv7_only = enable == 3;
    return OPOSE_OK;
}

int opose_profile_reset(opose_t* h) {
    if (!h) return OPOSE_E_ARG;
    OPOSE_TRY(h, h->prof_drain(true));
    h->agg.clear();
    return OPOSE_OK;
}

int opose_profile_read(opose_t* h, char* buf, size_t len) {
    if (!h || !buf || !len) return OPOSE_E_ARG;
    OPOSE_TRY(h, {
        OPOSE_HIP_CHECK(hipStreamSynchronize(h->stream));
        if (h->nstream) OPOSE_HIP_CHECK(hipStreamSynchronize(h->nstream));
        h->prof_drain(true);
    });
    std::string s = "{";
    bool first = true;
    for (auto& kv : h->agg) {
        char tmp[512];
        std::snprintf(tmp, sizeof tmp, "%s\"%s\":{\"count\":%ld,\"ms\":%.6f,\"flops\":%.6e,\"bytes\":%.6e}",
                      first ? "" : ",", kv.first.c_str(), kv.second.count, kv.second.ms, kv.second.flops,
                      kv.second.bytes);
        s += tmp;
        first = false;
    }
    s += "}";
    if (s.size() + 1 > len) return OPOSE_E_ARG;
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return OPOSE_OK;
}

}  // extern "C"
