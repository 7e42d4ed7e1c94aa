// common.cpp -- what every libpt unit uses: the error channel, the PT_TUNE switch,
// the RCCL loader, per-device stream pools and properties, the scene's device copy,
// and pt_device_init (the HIP runtime's start, beside the scene's parse).
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "api_internal.h"

namespace pti {

namespace {
thread_local std::string g_err;
}

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
const std::string& last_error() { return g_err; }

// RCCL is loaded on first use (the multi-GPU gather only): librccl is a ~570 MB
// library, and mapping it at process start costs the one-GPU CLI its start-up.
const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return x;
        x.CommInitAll = reinterpret_cast<decltype(&ncclCommInitAll)>(dlsym(h, "ncclCommInitAll"));
        x.Gather = reinterpret_cast<decltype(&ncclGather)>(dlsym(h, "ncclGather"));
        x.GroupStart = reinterpret_cast<decltype(&ncclGroupStart)>(dlsym(h, "ncclGroupStart"));
        x.GroupEnd = reinterpret_cast<decltype(&ncclGroupEnd)>(dlsym(h, "ncclGroupEnd"));
        x.GetErrorString = reinterpret_cast<decltype(&ncclGetErrorString)>(dlsym(h, "ncclGetErrorString"));
        x.ok = x.CommInitAll && x.Gather && x.GroupStart && x.GroupEnd && x.GetErrorString;
        return x;
    }();
    return r;
}

// Tuning and diagnostics switch: ONE environment variable, read where a
// session or pass starts, PT_TUNE="key=value,key=value".  None of it is needed
// for a correct or a fast render; the keys exist for A/B runs and diagnostics
// (INTEGRATION.md "Tuning and diagnostics"):
//   engine=mega       megakernel instead of the wavefront path engine (replay traversal)
//   budget_us=N       path engine: a round ends N us after its work ran out, for every wave at once
//                     (default 2500; 0: each wave after `budget` trips of its own)
//   lowq_budget_us=N  ... the same for the low-chain rounds (default 5000; 0: trip budgets, as
//                     budget_us=0)
//   budget=N          ... trips a query wave keeps its chains after the round's work ran out, when
//                     budget_us is 0 or budget alone is given (default 1024)
//   wg_per_cu=N       path engine: workgroups per CU (grid)
//   runend=N          a round with at most N chains runs them to the end of the pass
//   sparse=N          rounds with fewer than N chains run the end-of-pass kernel
//   sparse_steps=N    steps per loop trip of the end-of-pass kernel
//   coop=N            a round with at most N chains runs the cooperative engine (one team of
//                     lanes per chain) to the end of the pass (0: never)
//   round_batch=N     path rounds launched per chain count while the chains are far above
//                     the hand-over (default 1)
//   probe_every=N, probe_min=N, aux_extra=N, end_min=N
//                     path engine step mix: candidate probes every N-th trip or with N lanes
//                     waiting, extra aux-node steps per trip, ended paths per fold batch
//                     (defaults 3, 32, 1, 64)
//   lowq=N, lowq_probe_every=N, lowq_probe_min=N, lowq_aux_extra=N, lowq_end_min=N
//                     the step mix of rounds that start with fewer than N chains (default
//                     768 per CU; the mix of the other rounds, except lowq_end_min: 48)
//   lowq_wg=N         ... and their path workgroups per CU (PT_CMAX chains each; default 2)
//   coop_team=T       lanes per chain in the cooperative engine (4 default, 8, 16, 32, 64)
//   coop_grow=N       the final cooperative launch (teams of 4) hands its last N chains to a launch
//                     of whole-wave teams (default: 16 per CU; 0 = never; at most the carry queue)
//   coop_grow_mid=N   ... and, before that, its last N chains to teams of 32 (default 0: no such stage)
//   coop_order=0      the pass's final cooperative launch takes its chains in queue order (default:
//                     the pixels with the most samples left first)
//   early=K, early_at=N, early_wg=W
//                     once a pass's chains fall below N (default 768 per CU), each path round runs
//                     its K heaviest chains (1: what W cooperative workgroups per CU hold) in a
//                     cooperative launch on a second stream beside it; the launch hands its chains
//                     back when the round's path workgroups finish (default: 1; 0 = off)
//   side_team=T       that launch's teams of T lanes: 4 (default), 8, 16, 32 or 64
//   side_prio=0|1|2   that launch's stream: 0 normal priority (may share a main stream's
//                     hardware queue), 1 the greatest priority (a queue pool of its own; default),
//                     2 a CU-masked stream over every CU (always a queue of its own); take_stream
//   inject_fail=G     pt_render: rank G fails after its set-up (tests of the error paths)
//   inject_rccl=1     pt_render: the RCCL gather fails before any RCCL call (tests of the
//                     host fail-over)
//   prespin_us=N      diagnostics, same_device=2: N us of FMA work on the device before each
//                     rank's render (outside its time)
//   staging=0         pt_render: no pinned staging buffer for the framebuffer's copy out
//   shortlog=1        diagnostics: on a lost-chain error, the short pixels' sample counts on stderr
//   dupcheck=1        diagnostics: after every round, a slot that appears twice in the next round's work
//   Hand-off test hooks (DESIGN.md §4 "Hand-off sites": one per place where work changes hands):
//   side_late=1       the early launch's workgroups all act as late ones (take no chain, hand every
//                     work item on to the next round)
//   handon=0          ... and drop those items instead (lost chains: the resolve fails)
//   grow_late=1       the final launch's grow stop (coop_grow) with its odd workgroups acting as
//                     late ones (they hand their untaken items on through the intake order)
//   side_stop_now=1   the early launch stops at its first chain cycle's end (every team yields
//                     its chain to the next round's carry queue)
//   shade_hold=1      path rounds with a budget: the shade wave shades nothing until every query
//                     wave has left, so everything it shades is flushed to the next round
//   drop=<site>       the items of one hand-off site (PT_HO_*: suspend, flush, ringout, exact,
//                     side_take, side_yield, side_handon, grow_yield, grow_handon) are dropped
//                     instead of handed on (lost chains: the resolve fails); pt_stats.handoff
//                     counts every site's items
//   cap=N             chains a workgroup may hold
//   batch=N           round-queue entries a query wave takes per pull (1..64, default 32)
//   lstack=N          aux stack words a path-engine query may use (default and maximum PT_LSTACK;
//                     a query needing more takes the exact DFS)
//   roundlog=1|2|3    per-round kernel times / each round's chains, wall time and rays / and the
//                     pixels' remaining samples, on stderr
//   wgprof=FILE       per-workgroup timelines (-DPT_WPROF builds)
//   cprof=1           per-phase cycles of the cooperative engine on stderr (-DPT_CPROF builds)
//   qstats=FILE       per-query work counters of the host self-test render
//   qengine=coop      host self-tests: the cooperative engine's query algorithm (pt_coop.h)
//   prepstats=1       pt_scene_prepare's per-stage times on stderr
std::string tune_str(const char* key) {
    // the single-variable switches of earlier builds are ignored now: say so once
    static const bool warned = [] {
        for (const char* old : {"PT_ENGINE", "PT_PATH_BUDGET", "PT_STRAGGLER", "PT_QSTATS", "PT_WGPROF", "PT_COOP"})
            if (getenv(old)) fprintf(stderr, "libpt: %s is ignored; use PT_TUNE=\"key=value,...\" (INTEGRATION.md)\n", old);
        // keys of earlier builds, measured without a gain and removed
        if (const char* e = getenv("PT_TUNE"))
            for (const char* old : {"coop_stop", "near_budget", "near_k", "lowq2", "lowq2_wg", "variant", "rowmajor"}) {
                const std::string k = std::string(old) + "=";
                for (const char* p = e; (p = strstr(p, k.c_str())) != nullptr; p += k.size())
                    if (p == e || p[-1] == ',') {
                        fprintf(stderr, "libpt: PT_TUNE key %s was removed and is ignored (INTEGRATION.md)\n", old);
                        break;
                    }
            }
        return true;
    }();
    (void)warned;
    const char* e = getenv("PT_TUNE");
    if (!e) return {};
    const std::string k = std::string(key) + "=";
    for (const char* p = e; *p;) {
        const char* q = strchr(p, ',');
        const std::string item(p, q ? (size_t)(q - p) : strlen(p));
        if (item.compare(0, k.size(), k) == 0) return item.substr(k.size());
        if (!q) break;
        p = q + 1;
    }
    return {};
}
bool tune_has(const char* key) { return !tune_str(key).empty(); }
int tune_int(const char* key, int def) {
    const std::string v = tune_str(key);
    return v.empty() ? def : atoi(v.c_str());
}
int stats_level() {
    const char* e = getenv("PT_STATS");
    return e ? atoi(e) : 0;
}

int handoff_site(const char* name) {
    static const char* names[PT_HO_N] = {"suspend", "flush", "ringout", "exact", "side_take",
                                         "side_yield", "side_handon", "grow_yield", "grow_handon"};
    for (int k = 0; k < PT_HO_N; ++k)
        if (strcmp(name, names[k]) == 0) return k;
    return -1;
}

unsigned prep_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }

// streams made ahead of time by pt_device_init (stream creation costs ~8 ms of
// the runtime's first use), adopted by the next session on that device
namespace {
std::mutex g_spare_mu;
std::map<int, std::vector<hipStream_t>> g_spare_streams, g_spare_side;
}
// side: the early cooperative launch's stream.  It must run BESIDE the session's path
// round, so it must never share a hardware queue with a main stream: the runtime maps
// streams onto at most GPU_MAX_HW_QUEUES (4) queues per priority level and, past that,
// hands a new stream an existing queue of the same priority, where its kernels run in
// submission order after the other stream's.  A side launch queued behind (or ahead of)
// its own path round then runs alone: it holds the pass's heaviest chains to the end of
// the pass at the cooperative engine's rate (round 4: with 4 and 8 sessions on one
// device, the ranks past the third rendered 1.3-1.7x slower).  Side streams are made at
// the greatest priority, a queue pool of their own.
hipError_t take_stream(int dev, hipStream_t* s, bool side) {
    {
        std::lock_guard<std::mutex> lk(g_spare_mu);
        auto& v = side ? g_spare_side[dev] : g_spare_streams[dev];
        if (!v.empty()) {
            *s = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    const int mode = side ? tune_int("side_prio", 1) : 0;
    if (mode == 2) {
        // a CU-masked stream (every CU) always gets a hardware queue of its own
        std::vector<uint32_t> m(64, 0xffffffffu);
        return hipExtStreamCreateWithCUMask(s, (uint32_t)m.size(), m.data());
    }
    if (mode == 0) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    int least = 0, greatest = 0;
    if (const hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest)) return e;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}
void give_stream(int dev, hipStream_t s, bool side) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_spare_mu);
    (side ? g_spare_side : g_spare_streams)[dev].push_back(s);
}

// ------------------------------------------------------------- devices ---
// Device properties, queried once per device.  The runtime's start is split for
// PT_STATS=3: hipInit, device enumeration, and the two attributes check_device needs
// (the CU count, and the architecture name from the property query); each is timed.
namespace {
struct StartTimes { double init = -1, count = -1; };
StartTimes g_start;
}
int device_props(int dev, DevProps* out) {
    static std::mutex mu;
    static std::map<int, DevProps> cache;
    static int count = -1;
    std::lock_guard<std::mutex> lk(mu);
    if (count < 0) {
        auto t0 = std::chrono::steady_clock::now();
        auto lap = [&t0] {
            const auto n = std::chrono::steady_clock::now();
            const double ms = std::chrono::duration<double, std::milli>(n - t0).count();
            t0 = n;
            return ms;
        };
        if (hipInit(0) != hipSuccess) return fail(PT_E_NO_GPU, "hipInit failed (no HIP device visible)");
        g_start.init = lap();
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(PT_E_NO_GPU, "no HIP device visible");
        g_start.count = lap();
        count = n;
    }
    if (dev < 0 || dev >= count) return fail(PT_E_NO_GPU, "device index out of range");
    DevProps& p = cache[dev];
    if (!p.ok) {
        const auto t0 = std::chrono::steady_clock::now();
        int cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        hipDeviceProp_t pr;
        HIP_TRY(hipGetDeviceProperties(&pr, dev));
        p.cus = std::max(1, cus);
        strncpy(p.arch, pr.gcnArchName, sizeof(p.arch) - 1);
        p.props_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        p.ok = true;
    }
    *out = p;
    return PT_OK;
}

int check_device(int dev) {
    DevProps p;
    if (const int rc = device_props(dev, &p)) return rc;
    if (strncmp(p.arch, "gfx950", 6) != 0)
        return fail(PT_E_NO_GPU, std::string("device is ") + p.arch + ", this build targets gfx950");
    return PT_OK;
}

// The scene on device `dev`, uploaded on first use: one allocation and one copy
// of the upload image.  Devices upload in parallel (a lock per device).  mega:
// also the BVH2 aux of the megakernel traversal.
int ensure_device_scene(pt_scene* s, int dev, bool mega, DevScene** out, double* upload_ms) {
    DevEntry* e;
    {
        std::lock_guard<std::mutex> lk(s->mu);
        auto& slot = s->dev[dev];
        if (!slot) slot.reset(new DevEntry());
        e = slot.get();
    }
    std::lock_guard<std::mutex> lk(e->mu);
    DevScene& d = e->d;
    *upload_ms = 0.0;
    HIP_TRY(hipSetDevice(dev));
    if (!e->ready) {
        const auto t0 = std::chrono::steady_clock::now();
        void* p = nullptr;
        const size_t bytes = s->blob.size() * sizeof(pt::F4);
        HIP_TRY(hipMalloc(&p, bytes));
        if (hipMemcpy(p, s->blob.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(p);
            return fail(PT_E_HIP, "scene upload failed");
        }
        unsigned char* b = static_cast<unsigned char*>(p);
        d.base = b;
        d.blob = reinterpret_cast<const pt::F4*>(b);
        d.nodes = reinterpret_cast<const pt::Node*>(b + s->o_nodes);
        d.prims = reinterpret_cast<const pt::Prim*>(b + s->o_prim);
        d.anc_info = reinterpret_cast<const uint32_t*>(b + s->o_ainfo);
        d.anc = reinterpret_cast<const uint32_t*>(b + s->o_anc);
        d.shade = reinterpret_cast<const pt::Shade*>(b + s->i_shade);
        d.planes = reinterpret_cast<const uint32_t*>(b + s->i_planes);
        d.emitters = reinterpret_cast<const uint32_t*>(b + s->i_emit);
        d.thr = reinterpret_cast<const float*>(b + s->i_thr);
        d.top = reinterpret_cast<const pt::AuxSL*>(b + s->i_top);
        d.n_top = s->n_top;
        *upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        e->ready = true;
    }
    if (mega && !d.aux) {
        const size_t bytes = std::max<size_t>(sizeof(pt::AuxNode), s->aux.size() * sizeof(pt::AuxNode));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d.aux), bytes));
        if (!s->aux.empty())
            HIP_TRY(hipMemcpy(d.aux, s->aux.data(), s->aux.size() * sizeof(pt::AuxNode), hipMemcpyHostToDevice));
    }
    *out = &d;
    return PT_OK;
}

void free_device_scene(DevScene& d) {
    (void)hipFree(d.base);
    (void)hipFree(d.aux);
}

}  // namespace pti

using namespace pti;

extern "C" {

const char* pt_last_error(void) { return last_error().c_str(); }

int pt_abi_version(void) { return PT_ABI_VERSION; }

int pt_device_init(int device) {
    // (PT_STATS=3: the phases on stderr)
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&t0] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    const bool st = stats_level() >= 3;
    int rc = check_device(device);
    if (rc) return rc;
    DevProps pp;
    (void)device_props(device, &pp);
    const double t_props = ms();
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipFree(nullptr));                // creates the device context
    const double t_ctx = ms();
    HIP_TRY(pt_preload_kernels_base());       // loads both code objects (no launch)
    const double t_base = ms();
    HIP_TRY(pt_preload_kernels_wave());
    const double t_wave = ms();
    double t_copy = 0.0, t_s1 = 0.0;
    {
        // the runtime's copy path starts on its first transfer (tens of ms): do one
        // now, and make the first session's stream (a lock per device: the CLI's
        // per-device threads warm their devices at the same time)
        struct Warm { std::mutex mu; bool done = false; };
        static std::mutex mu;
        static std::map<int, std::unique_ptr<Warm>> warmed;
        Warm* w;
        {
            std::lock_guard<std::mutex> lk(mu);
            auto& e = warmed[device];
            if (!e) e.reset(new Warm());
            w = e.get();
        }
        std::lock_guard<std::mutex> lk(w->mu);
        if (!w->done) {
            void* d = nullptr;
            uint32_t h = 0;
            hipStream_t s = nullptr;
            // (the stream on a second thread, beside the copy path's start; on this thread
            // after it if no thread can be started)
            hipError_t se = hipSuccess;
            auto make = [&s, &se, device] {
                se = hipSetDevice(device);
                if (se == hipSuccess) se = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
            };
            std::thread sth;
            try {
                sth = std::thread(make);
            } catch (const std::system_error&) {
            }
            hipError_t ce = hipMalloc(&d, 64);
            if (ce == hipSuccess) ce = hipMemcpy(d, &h, 4, hipMemcpyHostToDevice);
            if (ce == hipSuccess) ce = hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
            if (d) (void)hipFree(d);
            t_copy = ms();
            if (sth.joinable()) sth.join();
            else make();
            t_s1 = ms();
            HIP_TRY(ce);
            HIP_TRY(se);
            give_stream(device, s, false);
            w->done = true;
        }
    }
    if (st)
        fprintf(stderr, "pt_device_init(%d) ms: hip_init %.1f device_count %.1f props %.1f context %.1f code_base %.1f "
                "code_wave %.1f copy %.1f stream (beside it) +%.1f\n", device,
                g_start.init >= 0 ? g_start.init : 0.0, g_start.count >= 0 ? g_start.count : 0.0, pp.props_ms,
                t_ctx - t_props,
                t_base - t_ctx, t_wave - t_base, t_copy ? t_copy - t_wave : 0.0, t_s1 ? t_s1 - t_copy : 0.0);
    return PT_OK;
}

}  // extern "C"
