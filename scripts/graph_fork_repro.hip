// Standalone HIP repro of the round-4 hipGraphLaunch segfault: no libopose.
// It follows engine.cpp's order: run_graphed (eager first sighting, capture on the second,
// replay after) over run_scales_concurrently's fork (event record on the main stream, the side
// stream waits, work on both, join back), and release() (drain, destroy the graph executables,
// destroy the events, return the side and main streams to a process-wide pool).
//
// Scenario of gpurun_out/c3d.log / c3f.log: handle B exists first; handle A (OPOSE_LOCKSTEP=0)
// forks inside its captures, then is destroyed; B's next forked call takes A's pooled side
// stream, captures on it and replays.
//
//   hipcc --offload-arch=gfx950 -O2 -o scripts/graph_fork_repro scripts/graph_fork_repro.hip
//   ./scripts/graph_fork_repro <variant> [replays]
//
// variants (one per process; the crash, if any, ends that process):
//   fresh        B's side stream is newly created (no reuse of A's)
//   reuse        B's side stream is A's, returned to the pool after A's release
//   reuse_keep   as reuse, but A's graph executable is never destroyed
//   reuse_nofork as reuse, but A's captures stay on one stream (the round-4 workaround)
//   reuse_nocap  as reuse, but A never captures (eager forks only)
//   reuse_newev  as reuse, and B's side-stream work is issued on a stream that has never been
//                part of any capture, with A's side stream only waited on
//   stress N     N random operations over several live handles (see stress() below);
//                STRESS_NOFORK=1 keeps every capture on one stream, STRESS_LEAK=1 never destroys
//                an executable graph
//
// libopose runs under the HIP runtime the process loaded first: torch's bundled libamdhip64
// (SONAME libamdhip64.so.7, ROCm 7.0.2) whenever torch is imported before the library, as in the
// test suite.  Run this binary under both: as built (/opt/rocm, 7.2) and with
// LD_LIBRARY_PATH=<torch>/lib.
#include <hip/hip_runtime.h>

#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(3);                                                                      \
        }                                                                                      \
    } while (0)

__global__ void bump(float* p, int n, float v) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.5f + v;
}

static std::vector<hipStream_t> g_pool;  // engine.cpp stream_pool()

static hipStream_t pooled() {
    if (!g_pool.empty()) {
        hipStream_t s = g_pool.back();
        g_pool.pop_back();
        return s;
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
}
static void give_back(hipStream_t s) {
    CK(hipStreamSynchronize(s));
    g_pool.push_back(s);
}

struct Handle {
    const char* name;
    hipStream_t main = nullptr, side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipGraphExec_t exec = nullptr;
    int sightings = 0;
    bool fork_in_capture = true;
    bool capture = true;
    float *a = nullptr, *b = nullptr;
    int n = 1 << 16;

    void init(const char* nm) {
        name = nm;
        sightings = 0;
        main = pooled();
        CK(hipMalloc(&a, n * sizeof(float)));
        CK(hipMalloc(&b, n * sizeof(float)));
        CK(hipMemsetAsync(a, 0, n * sizeof(float), main));
        CK(hipMemsetAsync(b, 0, n * sizeof(float), main));
    }
    // run_scales_concurrently: scale 1 on the side stream, scale 0 on main, join
    void work(bool capturing, bool fork) {
        const int bs = 256, gs = (n + bs - 1) / bs;
        if (!fork) {
            for (int k = 0; k < 4; ++k) bump<<<gs, bs, 0, main>>>(b, n, 1.f);
            for (int k = 0; k < 4; ++k) bump<<<gs, bs, 0, main>>>(a, n, 2.f);
            return;
        }
        if (!side) side = pooled();
        if (!ev_fork) CK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
        if (!ev_join) CK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
        CK(hipEventRecord(ev_fork, main));
        CK(hipStreamWaitEvent(side, ev_fork, 0));
        for (int k = 0; k < 4; ++k) bump<<<gs, bs, 0, side>>>(b, n, 1.f);
        CK(hipEventRecord(ev_join, side));
        for (int k = 0; k < 4; ++k) bump<<<gs, bs, 0, main>>>(a, n, 2.f);
        CK(hipStreamWaitEvent(main, ev_join, 0));
        (void)capturing;
    }
    // run_graphed
    void call(bool fork) {
        ++sightings;
        if (!capture || sightings == 1) {
            work(false, fork);
            return;
        }
        if (exec) {
            CK(hipGraphLaunch(exec, main));
            return;
        }
        CK(hipStreamBeginCapture(main, hipStreamCaptureModeThreadLocal));
        work(true, fork && fork_in_capture);
        hipGraph_t g = nullptr;
        CK(hipStreamEndCapture(main, &g));
        CK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
        CK(hipGraphLaunch(exec, main));
    }
    // release()
    void release(bool destroy_exec) {
        CK(hipStreamSynchronize(main));
        if (side) CK(hipStreamSynchronize(side));
        if (exec && destroy_exec) CK(hipGraphExecDestroy(exec));
        exec = nullptr;
        if (ev_fork) CK(hipEventDestroy(ev_fork));
        if (ev_join) CK(hipEventDestroy(ev_join));
        ev_fork = ev_join = nullptr;
        if (side) give_back(side);
        give_back(main);
        side = main = nullptr;
        CK(hipFree(a));
        CK(hipFree(b));
    }
};

// ---------------------------------------------------------------------------------------------
// "stress": the GPU test list's pattern, closer to the library's graphs.  Several handles live at
// once; each call signature is eager on its first sighting, captured on its second, replayed
// after; an allocation bumps a process-wide epoch that makes every handle recapture (destroying
// the old executable).  A forked call is the round-4 lockstep pyramid's conv1_x: one event
// recorded on the main stream, three pooled scale streams wait on it, run kernels, and the main
// stream waits on each scale's join event; around it a memset, kernels, a device copy and a copy
// into pinned host memory.  Handles are destroyed in release()'s order and their streams pooled.
static unsigned g_rng = 12345;
static unsigned rnd(unsigned n) {
    g_rng = g_rng * 1103515245u + 12345u;
    return (g_rng >> 8) % n;
}
static int g_epoch = 1;
// STRESS_NOFORK=1: calls never fork (captures stay on one stream); STRESS_LEAK=1: executable graphs
// are never destroyed (neither on recapture nor at release)
static const bool g_nofork = std::getenv("STRESS_NOFORK") && std::getenv("STRESS_NOFORK")[0] == '1';
static const bool g_leak = std::getenv("STRESS_LEAK") && std::getenv("STRESS_LEAK")[0] == '1';
// the last runtime call in flight, printed by the SIGSEGV handler
static char g_last[256] = "start";
static int g_op = -1;
static void on_segv(int sig) {
    char msg[320];
    int n = std::snprintf(msg, sizeof msg, "SIGNAL %d at stress op %d during: %s\n", sig, g_op, g_last);
    (void)!write(2, msg, n > 0 ? (size_t)n : 0);
    _exit(139);
}

struct Handle3 {
    hipStream_t main = nullptr, side[4] = {};
    hipEvent_t ev_fork = nullptr, ev_join[4] = {};
    struct Entry {
        hipGraphExec_t exec = nullptr;
        int epoch = 0;
        bool seen = false;
    };
    Entry entries[4];
    float* buf[4] = {};
    float* host = nullptr;
    int n = 1 << 15;
    bool capturing = false;
    long launches = 0;

    void init() {
        main = pooled();
        for (auto& b : buf) CK(hipMalloc(&b, n * sizeof(float)));
        CK(hipHostMalloc(&host, n * sizeof(float), hipHostMallocDefault));
        ++g_epoch;
    }
    void work(int sig) {
        const int bs = 256, gs = (n + bs - 1) / bs;
        CK(hipMemsetAsync(buf[0], 0, n * sizeof(float), main));
        bump<<<gs, bs, 0, main>>>(buf[0], n, 1.f);
        if ((sig & 1) && !g_nofork) {  // forked: the pyramid's per-scale chains
            if (!ev_fork) CK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
            CK(hipEventRecord(ev_fork, main));
            for (int s = 1; s < 4; ++s) {
                if (!side[s]) {
                    side[s] = pooled();
                    CK(hipEventCreateWithFlags(&ev_join[s], hipEventDisableTiming));
                }
                CK(hipStreamWaitEvent(side[s], ev_fork, 0));
                for (int k = 0; k <= s; ++k) bump<<<gs, bs, 0, side[s]>>>(buf[s], n, (float)s);
                CK(hipEventRecord(ev_join[s], side[s]));
            }
            for (int k = 0; k < 3; ++k) bump<<<gs, bs, 0, main>>>(buf[0], n, 2.f);
            for (int s = 1; s < 4; ++s) CK(hipStreamWaitEvent(main, ev_join[s], 0));
        }
        for (int k = 0; k < 2 + sig; ++k) bump<<<gs, bs, 0, main>>>(buf[0], n, 3.f);
        CK(hipMemcpyAsync(buf[1], buf[0], n * sizeof(float), hipMemcpyDeviceToDevice, main));
        CK(hipMemcpyAsync(host, buf[1], 256 * sizeof(float), hipMemcpyDeviceToHost, main));
    }
    void call(int sig) {
        Entry& e = entries[sig];
        if (e.exec && e.epoch == g_epoch) {
            std::snprintf(g_last, sizeof g_last, "hipGraphLaunch (replay) sig %d exec %p", sig, (void*)e.exec);
            CK(hipGraphLaunch(e.exec, main));
            ++launches;
            return;
        }
        if (!e.seen || e.epoch != g_epoch) {
            std::snprintf(g_last, sizeof g_last, "hipGraphExecDestroy (recapture) sig %d exec %p", sig, (void*)e.exec);
            if (e.exec && !g_leak) CK(hipGraphExecDestroy(e.exec));
            e.exec = nullptr;
            std::snprintf(g_last, sizeof g_last, "eager call sig %d", sig);
            work(sig);
            e.seen = true;
            e.epoch = g_epoch;
            return;
        }
        std::snprintf(g_last, sizeof g_last, "capture sig %d", sig);
        CK(hipStreamBeginCapture(main, hipStreamCaptureModeThreadLocal));
        work(sig);
        hipGraph_t g = nullptr;
        CK(hipStreamEndCapture(main, &g));
        std::snprintf(g_last, sizeof g_last, "hipGraphInstantiate sig %d", sig);
        CK(hipGraphInstantiate(&e.exec, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
        std::snprintf(g_last, sizeof g_last, "hipGraphLaunch (first) sig %d exec %p", sig, (void*)e.exec);
        CK(hipGraphLaunch(e.exec, main));
        ++launches;
    }
    void release() {
        CK(hipStreamSynchronize(main));
        for (int s = 1; s < 4; ++s)
            if (side[s]) CK(hipStreamSynchronize(side[s]));
        std::snprintf(g_last, sizeof g_last, "release: hipGraphExecDestroy");
        for (auto& e : entries)
            if (e.exec && !g_leak) CK(hipGraphExecDestroy(e.exec));
        std::snprintf(g_last, sizeof g_last, "release: events, streams, memory");
        if (ev_fork) CK(hipEventDestroy(ev_fork));
        for (int s = 1; s < 4; ++s) {
            if (side[s]) give_back(side[s]);
            if (ev_join[s]) CK(hipEventDestroy(ev_join[s]));
        }
        for (auto& b : buf) CK(hipFree(b));
        CK(hipHostFree(host));
        give_back(main);
    }
};

static int stress(int ops) {
    std::signal(SIGSEGV, on_segv);
    std::printf("stress: fork %s, executables %s\n", g_nofork ? "off" : "on", g_leak ? "leaked" : "destroyed");
    std::vector<Handle3*> hs;
    long launches = 0;
    for (int i = 0; i < ops; ++i) {
        g_op = i;
        const unsigned r = rnd(100);
        if (hs.empty() || (r < 6 && hs.size() < 6)) {
            hs.push_back(new Handle3());
            hs.back()->init();
        } else if (r < 10 && hs.size() > 1) {
            const unsigned k = rnd((unsigned)hs.size());
            hs[k]->release();
            launches += hs[k]->launches;
            delete hs[k];
            hs.erase(hs.begin() + k);
        } else if (r < 12) {
            ++g_epoch;  // another allocation somewhere: every handle recaptures
        } else {
            Handle3* h = hs[rnd((unsigned)hs.size())];
            const int sig = (int)rnd(4);
            for (int k = 0; k < 3; ++k) h->call(sig);
            if (rnd(4) == 0) CK(hipStreamSynchronize(h->main));
        }
        if (i % 500 == 0) {
            std::printf("stress op %d: %zu handles, %ld graph launches so far\n", i, hs.size(), launches);
            std::fflush(stdout);
        }
    }
    for (Handle3* h : hs) {
        h->release();
        launches += h->launches;
        delete h;
    }
    std::printf("variant stress: ok (%d ops, %ld graph launches; fork %s, executables %s)\n", ops, launches,
                g_nofork ? "off" : "on", g_leak ? "leaked" : "destroyed");
    return 0;
}

int main(int argc, char** argv) {
    const char* v = argc > 1 ? argv[1] : "reuse";
    const int replays = argc > 2 ? std::atoi(argv[2]) : 200;
    {
        int rv = 0;
        CK(hipRuntimeGetVersion(&rv));
        char line[512], lib[512] = "?";
        if (FILE* f = std::fopen("/proc/self/maps", "r")) {
            while (std::fgets(line, sizeof line, f))
                if (const char* q = std::strstr(line, "/")) {
                    if (std::strstr(q, "libamdhip64")) {
                        std::snprintf(lib, sizeof lib, "%s", q);
                        break;
                    }
                }
            std::fclose(f);
        }
        lib[std::strcspn(lib, "\n")] = 0;
        std::printf("runtime %d from %s\n", rv, lib);
    }
    if (std::strcmp(v, "stress") == 0) return stress(replays);
    const bool reuse = std::strncmp(v, "reuse", 5) == 0;
    std::printf("variant %s, %d replays\n", v, replays);
    std::fflush(stdout);

    Handle B;  // the lockstep C5 handle: exists first, its first graphs never fork
    B.init("B");
    for (int i = 0; i < 3; ++i) B.call(false);
    B.release(true);  // new signature below: start B's graph cache over, keep its streams
    B.init("B");

    Handle A;  // the OPOSE_LOCKSTEP=0 handle: forks inside its captures
    A.init("A");
    A.fork_in_capture = std::strcmp(v, "reuse_nofork") != 0;
    A.capture = std::strcmp(v, "reuse_nocap") != 0;
    for (int i = 0; i < 8; ++i) A.call(true);
    CK(hipStreamSynchronize(A.main));
    hipStream_t a_side = A.side;
    A.release(std::strcmp(v, "reuse_keep") != 0);
    std::printf("A released (side stream %p back in the pool)\n", (void*)a_side);
    std::fflush(stdout);

    if (!reuse) {  // keep A's streams out of B's reach
        g_pool.clear();
    }
    if (std::strcmp(v, "reuse_newev") == 0) {
        hipStream_t fresh;
        CK(hipStreamCreateWithFlags(&fresh, hipStreamNonBlocking));
        B.side = fresh;
    }
    for (int i = 0; i < replays; ++i) {
        B.call(true);
        if (i < 4 || i % 50 == 0) {
            CK(hipStreamSynchronize(B.main));
            std::printf("B call %d ok (side %p%s)\n", i, (void*)B.side, B.side == a_side ? " = A's" : "");
            std::fflush(stdout);
        }
    }
    CK(hipStreamSynchronize(B.main));
    std::vector<float> h(B.n);
    CK(hipMemcpy(h.data(), B.a, B.n * sizeof(float), hipMemcpyDeviceToHost));
    std::printf("variant %s: ok (a[0] = %g)\n", v, h[0]);
    return 0;
}
