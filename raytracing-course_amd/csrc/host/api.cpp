// api.cpp -- C ABI of libpt (include/pt.h): scene lifecycle (Scene::Load /
// InitScene equivalents), device residency, tile sessions and the render
// driver (Scene::Render equivalent).  Host C++; kernels live in
// ../device/pt_kernels.hip.
#include "pt.h"

#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <math.h>
#include <cmath>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <functional>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../device/pt_coop.h"
#include "../device/pt_kernels.h"
#include "pt_scene.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// RCCL is loaded on first use (the multi-GPU gather only): librccl is a ~570 MB
// library, and mapping it at process start costs the one-GPU CLI its start-up.
struct Rccl {
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclGather) Gather = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    bool ok = false;
};
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
//   lowq_budget_us=N  ... the same for the low-chain rounds (default 5000)
//   budget=N          ... trips a query wave keeps its chains after the round's work ran out, when
//                     budget_us is 0 or budget alone is given (default 1024)
//   wg_per_cu=N       path engine: workgroups per CU (grid)
//   runend=N          a round with at most N chains runs them to the end of the pass
//   sparse=N          rounds with fewer than N chains run the end-of-pass kernel
//   sparse_steps=N    steps per loop trip of the end-of-pass kernel
//   coop=N            a round with at most N chains runs the cooperative engine (one wave
//                     per chain) to the end of the pass (0: never)
//   round_batch=N     path rounds launched per chain count while the chains are far above
//                     the hand-over (default 1)
//   probe_every=N, probe_min=N, aux_extra=N, end_min=N
//                     path engine step mix: candidate probes every N-th trip or with N lanes
//                     waiting, extra aux-node steps per trip (defaults 3, 16, 1)
//   lowq=N, lowq_probe_every=N, lowq_probe_min=N, lowq_aux_extra=N, lowq_end_min=N
//                     the step mix of rounds that start with fewer than N chains (default
//                     768 per CU; the mix of the other rounds)
//   lowq_wg=N         ... and their path workgroups per CU (PT_CMAX chains each; default 2)
//   coop_team=T       lanes per chain in the cooperative engine (8, 16, 32, 64)
//   coop_grow=N       the final cooperative launch (teams of 8) hands its last N chains to a launch
//                     of whole-wave teams (default: 16 per CU; 0 = never)
//   coop_grow_mid=N   ... and, before that, its last N chains to teams of 32 (default 0: no such stage)
//   coop_order=0      the pass's final cooperative launch takes its chains in queue order (default:
//                     the pixels with the most samples left first)
//   early=K, early_at=N, early_wg=W
//                     once a pass's chains fall below N (default 768 per CU), each path round runs
//                     its K heaviest chains (1: what W cooperative workgroups per CU hold) in a
//                     cooperative launch on a second stream beside it; the launch hands its chains
//                     back when the round's path workgroups finish (default: 1; 0 = off)
//   side_team=T       that launch's teams of T lanes: 8 (default), 16, 32 or 64
//   side_prio=0|1|2   that launch's stream: 0 normal priority (may share a main stream's
//                     hardware queue), 1 the greatest priority (a queue pool of its own; default),
//                     2 a CU-masked stream over every CU (always a queue of its own); take_stream
//   inject_fail=G     pt_render: rank G fails after its set-up (tests of the error paths)
//   prespin_us=N      diagnostics, same_device=2: N us of FMA work on the device before each
//                     rank's render (outside its time)
//   staging=0         pt_render: no pinned staging buffer for the framebuffer's copy out
//   shortlog=1        diagnostics: on a lost-chain error, the short pixels' sample counts on stderr
//   dupcheck=1        diagnostics: after every round, a slot that appears twice in the next round's work
//   side_late=1       test hook: the early launch's workgroups all act as late ones (take no
//                     chain, hand every work item on to the next round)
//   handon=0          test hook: ... and drop those items instead (lost chains: the resolve fails)
//   grow_late=1       test hook: the final launch's grow stop (coop_grow) with its odd workgroups
//                     acting as late ones (they hand their untaken items on through the intake order)
//   cap=N            chains a workgroup may hold
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

// streams made ahead of time by pt_device_init (stream creation costs ~8 ms of
// the runtime's first use), adopted by the next session on that device
std::mutex g_spare_mu;
std::map<int, std::vector<hipStream_t>> g_spare_streams, g_spare_side;
// side: the early cooperative launch's stream.  It must run BESIDE the session's path
// round, so it must never share a hardware queue with a main stream: the runtime maps
// streams onto at most GPU_MAX_HW_QUEUES (4) queues per priority level and, past that,
// hands a new stream an existing queue of the same priority, where its kernels run in
// submission order after the other stream's.  A side launch queued behind (or ahead of)
// its own path round then runs alone: it holds the pass's heaviest chains to the end of
// the pass at the cooperative engine's rate (round 4: with 4 and 8 sessions on one
// device, the ranks past the third rendered 1.3-1.7x slower).  Side streams are made at
// the greatest priority, a queue pool of their own.
hipError_t take_stream(int dev, hipStream_t* s, bool side = false) {
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

#define HIP_TRY(expr)                                                                                 \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail(PT_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_));            \
    } while (0)

// A scene's device copy: ONE allocation holding the query blob (which also holds
// the reference nodes, primitives and ancestor lists the other kernels read:
// the views below point into it), the shading records, the plane and emitter
// lists, the gamma thresholds and k_wcamera's copy of the aux BVH's top two
// levels -- uploaded with one copy from one host image.  The BVH2 aux (the
// megakernel's traversal) is uploaded on first use only.
struct DevScene {
    unsigned char* base = nullptr;
    const pt::F4* blob = nullptr;
    const pt::Node* nodes = nullptr;
    const pt::Prim* prims = nullptr;
    const uint32_t* anc_info = nullptr;
    const uint32_t* anc = nullptr;
    const pt::Shade* shade = nullptr;
    const uint32_t* planes = nullptr;
    const uint32_t* emitters = nullptr;
    const float* thr = nullptr;
    const pt::AuxSL* top = nullptr;   // aux root entries + their child nodes' entries (k_wcamera)
    uint32_t n_top = 0;
    pt::AuxNode* aux = nullptr;       // BVH2 aux (megakernel only)
};
struct DevEntry {
    std::mutex mu;                    // this device's upload (devices upload in parallel)
    bool ready = false;
    DevScene d;
};

constexpr uint32_t kCandCap = 24;   // candidate-list words per lane (per replay pass)

}  // namespace

struct pt_scene {
    pth::HScene hs;
    bool prepared = false;
    std::vector<pth::HNode> nodes;
    uint32_t n_bvh = 0;
    std::vector<uint32_t> planes, emitters;
    std::vector<pt::Node> dnodes;
    std::vector<pt::Prim> dprims;
    std::vector<pt::Shade> dshade;
    std::vector<pt::AuxNode> aux;
    std::vector<pt::AuxSL> auxsl;
    uint32_t tree_depth = 0, max_stack = 0, aux_depth = 0, auxsl_depth = 0;
    float box_extent = 0.f;     // max |coordinate| of the reference node boxes
    std::vector<uint32_t> anc_info, anc;   // per-leaf ancestor lists (replay walk)
    std::vector<pt::F4> blob;   // the wavefront query's fetch space (pt_core.h SceneView::blob)
    uint32_t o_nodes = 0, o_aux = 0, o_ainfo = 0, o_anc = 0, o_qprim = 0, o_prim = 0, o_bundle = 0;
    uint32_t auxw_stack = 0;    // per-lane stack words of the wide aux traversal
    uint32_t aux_rshift = 0;    // leaf-range packing of the wide aux entries (annotate_aux_ranges)
    std::vector<float> regions;   // per reference node: its leaf's hit region {lo, hi} (lo > hi: unbounded)
    uint32_t aux_coarse_leaves = 0;   // leaf entries whose binary16 own box is > 4x wider than the f32 one
    float thr[256];
    // the device-only sections of the blob (byte offsets; the device copy is the blob)
    size_t i_shade = 0, i_planes = 0, i_emit = 0, i_thr = 0, i_top = 0;
    uint32_t n_top = 0;
    std::map<int, std::unique_ptr<DevEntry>> dev;
    std::mutex mu;                    // the image and the device map (not the uploads)
};

struct pt_session {
    pt_scene* sc = nullptr;
    int dev = 0;
    const DevScene* ds = nullptr;   // the scene's copy on this device
    double upload_ms = 0.0;         // time this session spent uploading it (0: already there)
    pt::TileMap tm{};
    uint32_t n_tiles_local = 0, n_slots = 0, depth = 0;
    pt::PixelState st{};          // per-slot records + fold records (device)
    unsigned long long* counters = nullptr;
    uint8_t* out = nullptr;
    uint8_t* fb = nullptr;            // rank 0: the window's row-major framebuffer (device)
    float* rad = nullptr;
    unsigned long long* wg_prof = nullptr;
    // wavefront engine buffers (replay traversal)
    bool wave = false;
    uint32_t path_grid = 0, path_budget = 1024, path_ticks = 0, low_ticks = 0, path_runend = 0, path_sparse = 0, sparse_steps = 8;
    uint32_t coop_max = 0, coop_grid = 0, coop_reserve = 0;   // cooperative engine (k_wcoop) at the end of a pass
    uint32_t round_batch = 1;     // rounds launched per count while the chains are far above the hand-over
    // k_wpath's per-trip step mix: {probe_every, probe_min, aux_extra, end_min}, and the one of
    // rounds that start with fewer than lowq chains (latency-bound: few chains per lane)
    uint32_t mix[4] = {PT_PROBE_EVERY, PT_PROBE_MIN, PT_AUX2, PT_END_MIN},
             mix_low[4] = {PT_PROBE_EVERY, PT_PROBE_MIN, PT_AUX2, PT_END_MIN_LOW};
    uint32_t lowq = 0;
    uint32_t low_grid = 0;        // path workgroups of those rounds
    bool coop_order = true;       // the cooperative engine takes the pixels furthest from the target first
    uint32_t* order = nullptr;    // 2 x 256 bucket counters + the intake order (a round's work: <= pixels)
    // early cooperative launch: once a pass's chains fall below early_at, the early_k chains
    // with the most samples left run in a cooperative launch on a second stream (early_wg
    // workgroups per CU, beside the path engine's low-chain rounds) to the end of the pass
    uint32_t early_k = 0, early_at = 0, early_wg = 1, side_team = 8;
    pt::RayQ side = {};           // its queue (early_k entries) ...
    uint32_t* side_carry = nullptr;   // ... its suspended queries' restart records (early_k x carry_words)
    uint32_t* side_ctl = nullptr;     // ... and its two round-counter sets
    hipStream_t side_stream = nullptr;
    hipEvent_t side_taken = nullptr, side_end = nullptr;   // its queue is taken / it has stopped
    std::thread side_th;          // makes the three above (joined before their first use)
    hipError_t side_rc = hipSuccess;
    uint32_t coop_grow = 0;       // the final launch's last chains handed to whole-wave teams (0: never)
    uint32_t coop_grow_mid = 0;   // ... and an earlier stage of teams of 32 (0: none)
    uint32_t coop_team = 8;       // lanes per chain in the cooperative engine (pure-coop rate, teams of
                                  // 64 / 32 / 16 / 8: 283 / 392 / 572 / 815 Mray/s)
    // every device buffer below lives in one allocation (pt_session_create)
    unsigned char* arena = nullptr;
    size_t arena_bytes = 0;
    pt::RayQ fq[2] = {};          // fresh rays (n_slots each)
    pt::DoneQ done = {};          // exact-DFS results (n_slots)
    pt::RayQ ex = {};             // rays handed to the exact DFS (n_slots)
    uint32_t* carry = nullptr;    // 2 * carry_cap * carry_words
    uint2* endq = nullptr;        // path_grid * PT_CMAX: the shade waves' ended paths
    unsigned long long short_seen = 0;   // CTR_SHORT at the last resolve
    uint32_t lane_cap = 0;        // min(pixels, query lanes): what one round can suspend
    uint32_t carry_cap = 0, carry_words = 0;
    uint32_t* ctl = nullptr;      // 2 x PT_CTL_SET round counters
    uint32_t* ctl_host = nullptr; // pinned copy of one counter set
    double roundlog_t = 0.0;      // (roundlog>=2: the last round's end, host clock, and the rays by then)
    unsigned long long roundlog_rays = 0;
    uint32_t shade_grid = 0, rounds = 0;
    hipStream_t stream = nullptr;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, pending_isect;
    std::vector<bool> pending_isect_coop;   // which of pending_isect are cooperative-engine launches
    double kernel_ms = 0.0, resolve_ms = 0.0, isect_ms = 0.0, coop_ms = 0.0;
    uint64_t isect_launches = 0, coop_launches = 0;
    uint64_t samples_done = 0;
    uint32_t deferred_spp = 0;    // wavefront engine: trace() calls not yet run (one pass at the next sync point)
    uint32_t* tile_order = nullptr;   // local tiles in Z-order of their image position (k_wcamera)
    std::vector<uint32_t> gtiles;     // this rank's window tiles (local -> window tile), tm.gtile on the device
    // optional progress report during a pass (pt_render's bar): finished samples,
    // counted by the kernels into host-mapped memory and polled at the round syncs
    std::function<void(uint64_t)> on_progress;
    unsigned long long* prog_host = nullptr;
    unsigned long long* prog_dev = nullptr;
    pt::CamView cam{};
    int traversal = PT_TRAVERSAL_REPLAY;
};

namespace {

// ------------------------------------------------------------- prepare ---
void build_device_layout(pt_scene* s) {
    const auto& P = s->hs.prims;
    // end[i] = one past node i's subtree in preorder
    std::vector<uint32_t> end(s->nodes.size());
    for (size_t k = s->nodes.size(); k-- > 0;)
        end[k] = s->nodes[k].left == 0xFFFFFFFFu ? (uint32_t)k + 1u : end[s->nodes[k].right];
    s->dnodes.resize(s->nodes.size());
    for (size_t i = 0; i < s->nodes.size(); ++i) {
        const pth::HNode& n = s->nodes[i];
        // AABB_t::Intersect (src/bvh.cpp:90-91): s = 0.5f*(max-min), center = 0.5f*(max+min)
        float c[3], h[3];
        for (int a = 0; a < 3; ++a) {
            h[a] = 0.5f * (n.mx[a] - n.mn[a]);
            c[a] = 0.5f * (n.mx[a] + n.mn[a]);
        }
        const bool leaf = n.left == 0xFFFFFFFFu;
        if (!leaf && n.left != (uint32_t)i + 1u) throw std::runtime_error("BVH not in preorder");
        const uint32_t ref = leaf ? n.first : n.right;
        const uint32_t cnt = leaf ? n.count : (PT_NODE_INTERIOR | end[i]);
        if (leaf && (cnt == 0u || (cnt & PT_NODE_INTERIOR))) throw std::runtime_error("bad BVH leaf size");
        pt::Node d;
        d.a = pt::F4{c[0], c[1], c[2], h[0]};
        d.b = pt::F4{h[1], h[2], pt::u2f(ref), pt::u2f(cnt)};
        s->dnodes[i] = d;
    }
    s->dprims.resize(P.size());
    s->dshade.resize(P.size());
    for (size_t i = 0; i < P.size(); ++i) {
        const pth::HPrim& p = P[i];
        pt::Prim d;
        d.p0 = pt::F4{p.pos[0], p.pos[1], p.pos[2], pt::u2f(p.type)};
        d.p1 = pt::F4{p.rot[0], p.rot[1], p.rot[2], p.rot[3]};
        d.p2 = pt::F4{p.a[0], p.a[1], p.a[2], 0.f};
        d.p3 = pt::F4{p.b[0], p.b[1], p.b[2], p.c[0]};
        d.p4 = pt::F4{p.c[1], p.c[2], 0.f, 0.f};
        s->dprims[i] = d;
        pt::Shade sh;
        sh.s0 = pt::F4{p.col[0], p.col[1], p.col[2], p.ior};
        sh.s1 = pt::F4{p.emis[0], p.emis[1], p.emis[2], pt::u2f(p.mat)};
        s->dshade[i] = sh;
    }
    // tree depth and the stack the exact DFS needs: need(v) = max(1 + need(left), need(right))
    std::vector<uint32_t> need(s->nodes.size(), 0), dep(s->nodes.size(), 0);
    uint32_t maxdep = 0;
    for (size_t i = 0; i < s->nodes.size(); ++i) {
        const pth::HNode& n = s->nodes[i];
        if (n.left != 0xFFFFFFFFu) { dep[n.left] = dep[i] + 1; dep[n.right] = dep[i] + 1; }
        maxdep = std::max(maxdep, dep[i]);
    }
    for (size_t k = s->nodes.size(); k-- > 0;) {
        const pth::HNode& n = s->nodes[k];
        if (n.left != 0xFFFFFFFFu) need[k] = std::max(1u + need[n.left], need[n.right]);
    }
    s->tree_depth = maxdep + 1;
    s->max_stack = need.empty() ? 0 : need[0];
    // ancestor lists of the leaves (root .. parent), for the replay walk (pt_query.h)
    std::vector<uint32_t> parent(s->nodes.size(), 0xFFFFFFFFu);
    for (size_t i = 0; i < s->nodes.size(); ++i)
        if (s->nodes[i].left != 0xFFFFFFFFu) { parent[s->nodes[i].left] = (uint32_t)i; parent[s->nodes[i].right] = (uint32_t)i; }
    s->anc_info.assign(s->nodes.size(), 0u);
    s->anc.clear();
    std::vector<uint32_t> path;
    for (size_t i = 0; i < s->nodes.size(); ++i) {
        if (s->nodes[i].left != 0xFFFFFFFFu) continue;
        // root .. parent, then the leaf itself, padded to 4 entries (16-B pieces)
        path.clear();
        for (uint32_t a = parent[i]; a != 0xFFFFFFFFu; a = parent[a]) path.push_back(a);
        if (path.size() + 1 > 63 || s->anc.size() + path.size() + 4 >= (1u << 26))
            throw std::runtime_error("BVH too deep for the ancestor lists");
        s->anc_info[i] = (uint32_t)s->anc.size() | ((uint32_t)(path.size() + 1) << 26);
        s->anc.insert(s->anc.end(), path.rbegin(), path.rend());
        s->anc.push_back((uint32_t)i);
        while (s->anc.size() & 3u) s->anc.push_back(0xFFFFFFFFu);
    }
    if (s->anc.empty()) s->anc.assign(4, 0xFFFFFFFFu);
    if (s->nodes.size() >= (1u << 24)) throw std::runtime_error("BVH larger than 2^24 nodes");
}

// The region where a reference leaf's primitives can report a hit, as a box for
// its wide aux leaf entry (pt_query.h PT_LEAF_MARGIN).  IntersectTriangle hits
// the plane through the local origin (src/primitives.cpp:156-157) and accepts a
// point whose projection along n lies in the triangle, so a plain triangle (pos
// = +0, identity rotation) can only be hit on T' = T - (a.n) n, the triangle
// moved onto that plane, with n the float normal the test itself computes.
// Rounding (u = 2^-24, X = scene box extent; derivation in DESIGN.md §2):
//  * each edge test dot(cross(e, p - a), n) > 0 is decided within 36u |e| |p - a|,
//    i.e. a point up to 36u |p - a| <= 144u X outside an edge may pass; at a corner
//    of angle phi that widens the accepted region by 1/sin(phi/2): the box here is
//    widened by 4 x 144u X / sin(phi_min/2);
//  * the computed point p = o + t d lies within ~22u (2|o| + 3X) of the ray and of
//    the plane: the per-ray margin the query adds (64 dl = 4096u (X + |o|) / |d|min).
// Degenerate triangles (an angle under ~0.1 degree) and non-plain primitives keep
// the leaf's own box, which is the candidate test of the first replay: correct,
// just unfiltered.
bool leaf_hit_region(const pt_scene* s, uint32_t leaf, float lo[3], float hi[3]) {
    if (!(s->box_extent < INFINITY)) return false;
    const pt::Node& n = s->dnodes[leaf];
    const uint32_t first = pt::f2u(n.b.z), cnt = pt::f2u(n.b.w);
    double l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = first; i < first + cnt; ++i) {
        const pt::Prim& P = s->dprims.at(i);
        const bool plain = pt::f2u(P.p0.w) == pt::T_TRIANGLE && pt::f2u(P.p0.x) == 0u && pt::f2u(P.p0.y) == 0u &&
                           pt::f2u(P.p0.z) == 0u && pt::f2u(P.p1.x) == 0u && pt::f2u(P.p1.y) == 0u &&
                           pt::f2u(P.p1.z) == 0u && pt::f2u(P.p1.w) == 0x3f800000u;
        if (!plain) return false;
        const pt::f3 a = pt::mk3(P.p2.x, P.p2.y, P.p2.z), b = pt::mk3(P.p3.x, P.p3.y, P.p3.z),
                     c = pt::mk3(P.p3.w, P.p4.x, P.p4.y);
        const pt::f3 nf = pt::normalize(pt::cross(b - a, c - a));   // the test's own float normal
        if (!(std::isfinite(nf.x) && std::isfinite(nf.y) && std::isfinite(nf.z))) return false;
        const double V[3][3] = {{a.x, a.y, a.z}, {b.x, b.y, b.z}, {c.x, c.y, c.z}};
        double smin = 1.0;   // sin(phi/2) of the sharpest corner
        for (int k = 0; k < 3; ++k) {
            const double* o = V[k];
            const double* p1 = V[(k + 1) % 3];
            const double* p2 = V[(k + 2) % 3];
            double uu = 0, vv = 0, uv = 0;
            for (int j = 0; j < 3; ++j) {
                const double u = p1[j] - o[j], v = p2[j] - o[j];
                uu += u * u; vv += v * v; uv += u * v;
            }
            if (!(uu > 0 && vv > 0)) return false;
            smin = std::min(smin, sqrt(std::max(0.0, (1.0 - uv / sqrt(uu * vv)) * 0.5)));
        }
        if (!(smin > 1e-3)) return false;
        const double wid = 4.0 * 144.0 * 0x1p-24 * (double)s->box_extent / smin;
        const double nd[3] = {nf.x, nf.y, nf.z};
        const double d = V[0][0] * nd[0] + V[0][1] * nd[1] + V[0][2] * nd[2];
        for (int k = 0; k < 3; ++k)
            for (int j = 0; j < 3; ++j) {
                const double x = V[k][j] - d * nd[j];
                l[j] = std::min(l[j], x - wid);
                h[j] = std::max(h[j], x + wid);
            }
    }
    if (!(l[0] <= h[0])) return false;
    for (int j = 0; j < 3; ++j) {
        // outward to float, with the aux build's static widening
        lo[j] = (float)(l[j] - fabs(l[j]) * 1.52587890625e-05 - 7.62939453125e-06);
        hi[j] = (float)(h[j] + fabs(h[j]) * 1.52587890625e-05 + 7.62939453125e-06);
    }
    return true;
}

// fn(begin, end, part) over [0, n) in at most `parts` contiguous chunks, one thread each
// (host preparation loops whose items are independent)
template <class F>
void parallel_chunks(size_t n, unsigned parts, F fn) {
    parts = std::max(1u, std::min<unsigned>(parts, (unsigned)((n + 8191) / 8192)));
    if (parts == 1) { fn((size_t)0, n, 0u); return; }
    std::vector<std::thread> th;
    for (unsigned k = 0; k < parts; ++k)
        th.emplace_back(fn, n * k / parts, n * (k + 1) / parts, k);
    for (auto& t : th) t.join();
}
unsigned prep_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }

// binary16 bits of x rounded toward -inf (down) or +inf (up)
uint32_t f16_out(float x, bool up) {
    const _Float16 h = (_Float16)x;
    uint16_t b = __builtin_bit_cast(uint16_t, h);
    const float back = (float)h;
    if (up ? back < x : back > x) {
        // one step outward
        const bool neg = (b & 0x8000u) != 0u;
        if ((b & 0x7fffu) == 0u) b = up ? 0x0001u : 0x8001u;
        else if (neg == up) b = (uint16_t)(b - 1u);
        else b = (uint16_t)(b + 1u);
    }
    return b;
}

// The query blob's form of the wide aux entries (pt_query.h PT_LEAF_MARGIN):
// own box and hit region, both binary16 rounded outward, then {range, code}.
// A leaf's hit region is leaf_hit_region's box, or unbounded; an internal
// entry's is the union over its child node's entries (children follow their
// parent in the wide tree's numbering).
void encode_aux_entries(pt_scene* s, std::vector<pt::AuxSL>& aux) {
    const uint32_t W = PT_AUXW, nn = (uint32_t)(aux.size() / W);
    std::vector<std::array<float, 6>> nodeB(nn), entB(aux.size());
    const std::array<float, 6> unb = {-INFINITY, -INFINITY, -INFINITY, INFINITY, INFINITY, INFINITY};
    for (uint32_t n = nn; n-- > 0;) {
        std::array<float, 6> u = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
        for (uint32_t k = 0; k < W; ++k) {
            const pt::AuxSL& e = aux[(size_t)n * W + k];
            const uint32_t code = pt::f2u(e.b.w);
            if (code == 0xFFFFFFFFu) continue;
            std::array<float, 6> b;
            if (code & 0x80000000u) {
                const float* r = &s->regions.at(6ull * (code & 0x7FFFFFFFu));
                if (r[0] <= r[3]) b = {r[0], r[1], r[2], r[3], r[4], r[5]};
                else b = unb;
            } else {
                if (code <= n || code >= nn) throw std::runtime_error("aux wide tree: child before its parent");
                b = nodeB[code];
            }
            entB[(size_t)n * W + k] = b;
            for (int j = 0; j < 3; ++j) { u[j] = std::min(u[j], b[j]); u[3 + j] = std::max(u[3 + j], b[3 + j]); }
        }
        nodeB[n] = u;
    }
    // binary16 keeps parity (outward rounding) but not culling: past |x| = 65504 a bound
    // becomes infinite, and its step is 2 or more above 2048 -- leaf boxes much smaller
    // than that step are then visited by far more rays (counted, warned about once)
    const unsigned parts = prep_threads();
    std::vector<size_t> coarse_k(parts, 0), leaves_k(parts, 0);
    parallel_chunks(aux.size(), parts, [&](size_t i0, size_t i1, unsigned part) {
    size_t coarse = 0, leaves = 0;
    for (size_t i = i0; i < i1; ++i) {
        pt::AuxSL& e = aux[i];
        if (pt::f2u(e.b.w) == 0xFFFFFFFFu) continue;
        const float A[6] = {e.a.x, e.a.y, e.a.z, e.a.w, e.b.x, e.b.y};
        const std::array<float, 6>& B = entB[i];
        uint32_t h[12];
        for (int j = 0; j < 6; ++j) {
            h[j] = f16_out(A[j], j >= 3);
            h[6 + j] = f16_out(B[j], j >= 3);
        }
        if (pt::f2u(e.b.w) & 0x80000000u) {
            ++leaves;
            bool c = false;
            for (int j = 0; j < 3; ++j) {
                const float w32 = A[3 + j] - A[j];
                const float w16 = (float)__builtin_bit_cast(_Float16, (uint16_t)h[3 + j]) -
                                  (float)__builtin_bit_cast(_Float16, (uint16_t)h[j]);
                c = c || !(w16 <= 4.f * w32 + 1e-3f);
            }
            coarse += c ? 1u : 0u;
        }
        const uint32_t range = pt::f2u(e.b.z), code = pt::f2u(e.b.w);
        // {lo.x, lo.y}, {lo.z, hi.x}, {hi.y, hi.z} per box
        e.a = pt::F4{pt::u2f(h[0] | h[1] << 16), pt::u2f(h[2] | h[3] << 16), pt::u2f(h[4] | h[5] << 16),
                     pt::u2f(h[6] | h[7] << 16)};
        e.b = pt::F4{pt::u2f(h[8] | h[9] << 16), pt::u2f(h[10] | h[11] << 16), pt::u2f(range), pt::u2f(code)};
    }
    coarse_k[part] = coarse;
    leaves_k[part] = leaves;
    });
    size_t coarse = 0, leaves = 0;
    for (unsigned k = 0; k < parts; ++k) { coarse += coarse_k[k]; leaves += leaves_k[k]; }
    s->aux_coarse_leaves = (uint32_t)coarse;
    if (leaves && coarse * 100 > leaves)
        fprintf(stderr, "pt: %zu of %zu leaf boxes are more than 4x wider in the binary16 aux BVH (coordinates "
                        "beyond ~2048 or +-65504): results stay exact, traversal visits more nodes\n", coarse, leaves);
}

// k_wcamera's costly-class test reads the wide aux root's entries and, for each
// inner one, its child node's entries (f32 host form): entries 0..W-1 = the root,
// entries W (1 + k) .. = the child of root entry k, whose code is rewritten to 1 + k
std::vector<pt::AuxSL> aux_top(const pt_scene* s) {
    const uint32_t W = PT_AUXW;
    std::vector<pt::AuxSL> t;
    if (s->auxsl.size() < W) return t;
    t.assign(s->auxsl.begin(), s->auxsl.begin() + W);
    for (uint32_t k = 0; k < W; ++k) {
        const uint32_t code = pt::f2u(t[k].b.w);
        if (code == 0xFFFFFFFFu || (code & 0x80000000u)) continue;
        if ((size_t)(code + 1) * W > s->auxsl.size()) throw std::runtime_error("aux root child out of range");
        const uint32_t at = (uint32_t)(t.size() / W);
        t.insert(t.end(), s->auxsl.begin() + (size_t)code * W, s->auxsl.begin() + (size_t)(code + 1) * W);
        t[k].b.w = pt::u2f(at);
    }
    return t;
}

// one 16-B-aligned blob holding every array the wavefront query reads
// (SceneView::blob; 32-bit byte offsets).  The compact primitive records
// (pt_query.h qprim_expand) are built here.
void build_query_blob(pt_scene* s, const std::function<void(const char*)>& tick) {
    std::vector<pt::F4>& b = s->blob;
    b.clear();
    // every section's 16-B pieces, reserved at once (the blob is tens of MB; a
    // reallocation would copy it): nodes, aux, ancestor lists, compact primitives (4),
    // full primitives (5), shading records (2), leaf bundles (6 per leaf), the small
    // device-only tables and the 256-B section padding
    b.reserve(s->dnodes.size() * 2 + s->auxsl.size() * 2 + (s->anc_info.size() + s->anc.size()) / 4 + 4 +
              s->dprims.size() * (4 + 5 + 2) + (s->dnodes.size() / 2 + 1) * 6 +
              (s->planes.size() + s->emitters.size()) / 4 + 64 + 2 * 5 * PT_AUXW + 16 * 12);
    auto append = [&b](const void* p, size_t bytes) {
        // sections are addressed by 32-bit byte offsets (and the device forms record
        // offsets from them in 32 bits): the whole blob must stay below 4 GiB
        if (b.size() * 16 + bytes >= 0xFFFFFFF0ull) throw std::runtime_error("scene too large for 32-bit query offsets");
        const uint32_t o = (uint32_t)(b.size() * 16);
        const size_t n = (bytes + 15) / 16;
        b.resize(b.size() + n, pt::F4{0.f, 0.f, 0.f, 0.f});
        if (bytes) memcpy(&b[o / 16], p, bytes);
        return o;
    };
    // leaf ordinals: each wide aux leaf entry carries in b.z the index of its leaf's
    // bundle; bundles are numbered in the order the wide aux nodes hold the leaves,
    // so the leaves of one aux node (spatial neighbours, often probed by the same
    // ray) share cache lines
    std::vector<uint32_t> leaves;
    std::vector<uint8_t> seen(s->dnodes.size(), 0);
    std::vector<pt::AuxSL> aux = s->auxsl;
    for (pt::AuxSL& e : aux) {
        const uint32_t code = pt::f2u(e.b.w);
        if (code == 0xFFFFFFFFu || !(code & 0x80000000u)) continue;
        const uint32_t leaf = code & 0x7FFFFFFFu;
        if (leaf >= s->dnodes.size() || (pt::f2u(s->dnodes[leaf].b.w) & 0x80000000u) || seen[leaf]++)
            throw std::runtime_error("aux leaf entry names an internal node or a leaf twice");
        e.b.z = pt::u2f((uint32_t)leaves.size());
        leaves.push_back(leaf);
    }
    tick("blob: leaf ordinals");
    encode_aux_entries(s, aux);
    tick("blob: aux encode");
    s->o_nodes = append(s->dnodes.data(), s->dnodes.size() * sizeof(pt::Node));
    s->o_aux = append(aux.data(), aux.size() * sizeof(pt::AuxSL));
    s->o_ainfo = append(s->anc_info.data(), s->anc_info.size() * 4);
    s->o_anc = append(s->anc.data(), s->anc.size() * 4);
    std::vector<pt::F4> qp(4 * s->dprims.size());
    parallel_chunks(s->dprims.size(), prep_threads(), [&](size_t i0, size_t i1, unsigned) {
    for (size_t i = i0; i < i1; ++i) {
        const pt::Prim& P = s->dprims[i];
        const uint32_t type = pt::f2u(P.p0.w);
        const bool pos0 = pt::f2u(P.p0.x) == 0u && pt::f2u(P.p0.y) == 0u && pt::f2u(P.p0.z) == 0u;
        const bool rot1 = pt::f2u(P.p1.x) == 0u && pt::f2u(P.p1.y) == 0u && pt::f2u(P.p1.z) == 0u &&
                          pt::f2u(P.p1.w) == 0x3f800000u;
        pt::F4* r = &qp[4 * i];
        if (type == pt::T_TRIANGLE && pos0 && rot1) {
            // with the triangle's normal exactly as IntersectTriangle computes it
            const pt::f3 a = pt::mk3(P.p2.x, P.p2.y, P.p2.z), b = pt::mk3(P.p3.x, P.p3.y, P.p3.z),
                         c = pt::mk3(P.p3.w, P.p4.x, P.p4.y);
            const pt::f3 n = pt::normalize(pt::cross(b - a, c - a));
            r[0] = pt::F4{a.x, a.y, a.z, P.p0.w};
            r[1] = pt::F4{b.x, b.y, b.z, n.x};
            r[2] = pt::F4{c.x, c.y, c.z, n.y};
            r[3] = pt::F4{n.z, 0.f, 0.f, 0.f};
        } else if (type == pt::T_BOX || type == pt::T_ELLIPSOID) {
            r[0] = pt::F4{P.p2.x, P.p2.y, P.p2.z, P.p0.w};
            r[1] = pt::F4{P.p0.x, P.p0.y, P.p0.z, P.p1.x};
            r[2] = pt::F4{P.p1.y, P.p1.z, P.p1.w, 0.f};
        } else {
            r[0] = pt::F4{0.f, 0.f, 0.f, pt::u2f(type | PT_QP_FULL)};
            r[1] = r[2] = r[3] = pt::F4{0.f, 0.f, 0.f, 0.f};
        }
    }
    });
    tick("blob: sections + qprims");
    s->o_qprim = append(qp.data(), qp.size() * sizeof(pt::F4));
    // leaf bundles (pt_query.h): the compact record of the leaf's first primitive
    // (pieces 0-2), then {leaf node index, first primitive, primitive count, its n.z}
    std::vector<pt::F4> bu(6 * leaves.size());
    for (size_t k = 0; k < leaves.size(); ++k) {
        const pt::Node& n = s->dnodes[leaves[k]];
        pt::F4* r = &bu[6 * k];
        const uint32_t first = pt::f2u(n.b.z), cnt = pt::f2u(n.b.w);
        if (cnt) {
            if (first >= s->dprims.size()) throw std::runtime_error("leaf primitive out of range");
            r[0] = qp[4 * first]; r[1] = qp[4 * first + 1]; r[2] = qp[4 * first + 2];
        }
        r[3] = pt::F4{pt::u2f(leaves[k]), pt::u2f(first), pt::u2f(cnt), cnt ? qp[4 * first + 3].x : 0.f};
        // the leaf's box exactly as its node record holds it (c, s)
        r[4] = n.a;
        r[5] = pt::F4{n.b.x, n.b.y, 0.f, 0.f};
    }
    s->o_bundle = append(bu.data(), bu.size() * sizeof(pt::F4));
    s->o_prim = append(s->dprims.data(), s->dprims.size() * sizeof(pt::Prim));
    tick("blob: bundles + prims");
    // The device copy is the blob itself plus the tables only the kernels read (shading
    // records, plane and emitter lists, gamma thresholds, k_wcamera's top aux levels),
    // each at a 256-B offset: one host image, uploaded with one copy (ensure_device_scene)
    auto align256 = [&b] { b.resize((b.size() + 15) & ~(size_t)15, pt::F4{0.f, 0.f, 0.f, 0.f}); };
    const std::vector<pt::AuxSL> top = aux_top(s);
    align256(); s->i_shade = append(s->dshade.data(), s->dshade.size() * sizeof(pt::Shade));
    align256(); s->i_planes = append(s->planes.data(), s->planes.size() * 4);
    align256(); s->i_emit = append(s->emitters.data(), s->emitters.size() * 4);
    align256(); s->i_thr = append(s->thr, sizeof(s->thr));
    align256(); s->i_top = append(top.data(), top.size() * sizeof(pt::AuxSL));
    s->n_top = (uint32_t)top.size();
    align256();
    if (b.size() * 16 >= 0xFFFFFFF0ull) throw std::runtime_error("scene too large for 32-bit query offsets");
}

// ------------------------------------------------------------- devices ---
// device properties, queried once per device (hipGetDeviceProperties costs
// milliseconds, and every session creation needs the CU count)
struct DevProps { bool ok = false; int cus = 0; char arch[64] = {0}; };
int device_props(int dev, DevProps* out) {
    static std::mutex mu;
    static std::map<int, DevProps> cache;
    static int count = -1;
    std::lock_guard<std::mutex> lk(mu);
    if (count < 0) {
        const auto t0 = std::chrono::steady_clock::now();
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(PT_E_NO_GPU, "no HIP device visible");
        count = n;
        if (getenv("PT_STATS") && atoi(getenv("PT_STATS")) >= 3)
            fprintf(stderr, "hip runtime start (hipGetDeviceCount): %.1f ms, %d device(s)\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), n);
    }
    if (dev < 0 || dev >= count) return fail(PT_E_NO_GPU, "device index out of range");
    DevProps& p = cache[dev];
    if (!p.ok) {
        hipDeviceProp_t pr;
        HIP_TRY(hipGetDeviceProperties(&pr, dev));
        p.cus = std::max(1, pr.multiProcessorCount);
        strncpy(p.arch, pr.gcnArchName, sizeof(p.arch) - 1);
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

// per-lane LDS words: replay needs [aux stack | candidates], the exact DFS its stack
pt::ReplayCfg replay_cfg(const pt_scene* s) {
    pt::ReplayCfg c;
    c.as = std::max<uint32_t>(s->aux_depth, 1u);
    c.cap = kCandCap;
    return c;
}
uint32_t lane_words(const pt_scene* s, int traversal) {
    const pt::ReplayCfg c = replay_cfg(s);
    const uint32_t dfs = std::max<uint32_t>(s->max_stack, 1u);
    return traversal == PT_TRAVERSAL_EXACT ? dfs : std::max(dfs, c.as + c.cap);
}

void set_blob(pt::SceneView& v, const pt_scene* s, const pt::F4* blob) {
    v.blob = blob;
    v.o_nodes = s->o_nodes; v.o_aux = s->o_aux; v.o_ainfo = s->o_ainfo;
    v.o_anc = s->o_anc; v.o_qprim = s->o_qprim; v.o_prim = s->o_prim; v.o_bundle = s->o_bundle;
    v.aux_rshift = s->aux_rshift;
}

pt::SceneView host_view(const pt_scene* s, int traversal) {
    pt::SceneView v;
    v.aux = traversal == PT_TRAVERSAL_EXACT ? nullptr : s->aux.data();
    v.nodes = s->dnodes.data();
    v.prims = s->dprims.data();
    v.shade = s->dshade.data();
    v.planes = s->planes.data();
    v.emitters = s->emitters.data();
    v.n_planes = (uint32_t)s->planes.size();
    v.n_emitters = (uint32_t)s->emitters.size();
    v.inv_emitters = s->emitters.empty() ? 0.f : 1.f / (float)s->emitters.size();
    v.bg = pt::mk3(s->hs.bg[0], s->hs.bg[1], s->hs.bg[2]);
    v.box_extent = s->box_extent;
    v.anc_info = s->anc_info.data();
    v.anc = s->anc.data();
    set_blob(v, s, s->blob.data());
    return v;
}

pt::CamView make_cam(const pt_scene* s) {
    const pth::HScene& h = s->hs;
    pt::CamView c;
    c.pos = pt::mk3(h.cam_pos[0], h.cam_pos[1], h.cam_pos[2]);
    c.right = pt::mk3(h.cam_right[0], h.cam_right[1], h.cam_right[2]);
    c.up = pt::mk3(h.cam_up[0], h.cam_up[1], h.cam_up[2]);
    c.fwd = pt::mk3(h.cam_fwd[0], h.cam_fwd[1], h.cam_fwd[2]);
    // src/scene.cpp:181-182: float tan_fov_x = tan(fov_x / 2) -> ::tan(double); tan_y = tan_x*H/W
    c.tx = (float)tan((double)(h.fov_x / 2));
    c.ty = c.tx * (float)h.H / (float)h.W;
    c.W = (float)h.W;
    c.H = (float)h.H;
    return c;
}

int finish_pending(pt_session* ss) {
    for (auto& e : ss->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) ss->kernel_ms += ms;
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    ss->pending.clear();
    // diagnostics (PT_TUNE roundlog=1): per-launch ms of the rounds, one line per sync
    const bool log = tune_int("roundlog", 0) == 1 && !ss->pending_isect.empty();
    if (log) fprintf(stderr, "rounds_ms");
    for (size_t i = 0; i < ss->pending_isect.size(); ++i) {
        const auto& e = ss->pending_isect[i];
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) {
            ss->isect_ms += ms;
            if (i < ss->pending_isect_coop.size() && ss->pending_isect_coop[i]) ss->coop_ms += ms;
        }
        if (log) fprintf(stderr, " %.3f", ms);
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    if (log) fprintf(stderr, "\n");
    ss->pending_isect.clear();
    ss->pending_isect_coop.clear();
    return PT_OK;
}

// the window tiles dealt to `rank` (pt_kernels.h tile_owner), ascending
std::vector<uint32_t> rank_tiles(uint32_t n_tiles, uint32_t tiles_x, uint32_t rank, uint32_t world) {
    std::vector<uint32_t> v;
    v.reserve(n_tiles / world + 1);
    for (uint32_t t = 0; t < n_tiles; ++t)
        if (pt::tile_owner(t, tiles_x, world) == rank) v.push_back(t);
    return v;
}

uint64_t owned_pixels(const pt_session* ss) {
    uint64_t px = 0;
    for (uint32_t t = 0; t < ss->n_tiles_local; ++t) {
        const uint32_t gt = ss->gtiles[t];
        const uint32_t tx = gt % ss->tm.tiles_x, ty = gt / ss->tm.tiles_x;
        const uint32_t w = std::min(16u, ss->tm.ww - tx * 16u), h = std::min(16u, ss->tm.wh - ty * 16u);
        px += (uint64_t)w * h;
    }
    return px;
}

void progress_bar(uint64_t done, uint64_t total, int& last) {
    // the reference prints "Loading: [ ##...   x% ]" every 10 % (src/scene.cpp:232-240)
    const int ct = total ? (int)((done * 10) / total) : 10;
    while (last < ct && last < 10) {
        ++last;
        std::string bar = "Loading: [ ";
        bar += std::string((size_t)last, '#');
        bar += std::string((size_t)(11 - last), ' ');
        bar += std::to_string(last * 10);
        bar += "% ]\n";
        fputs(bar.c_str(), stdout);
        fflush(stdout);
    }
}

}  // namespace

extern "C" {

const char* pt_last_error(void) { return g_err.c_str(); }

int pt_device_init(int device) {
    // (PT_STATS=3: the phases on stderr)
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&t0] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    const bool st = getenv("PT_STATS") && atoi(getenv("PT_STATS")) >= 3;
    int rc = check_device(device);
    if (rc) return rc;
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
            // (the stream on a second thread, beside the copy path's start)
            hipError_t se = hipSuccess;
            std::thread sth([&s, &se, device] {
                se = hipSetDevice(device);
                if (se == hipSuccess) se = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
            });
            hipError_t ce = hipMalloc(&d, 64);
            if (ce == hipSuccess) ce = hipMemcpy(d, &h, 4, hipMemcpyHostToDevice);
            if (ce == hipSuccess) ce = hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
            if (d) (void)hipFree(d);
            t_copy = ms();
            sth.join();
            t_s1 = ms();
            HIP_TRY(ce);
            HIP_TRY(se);
            std::lock_guard<std::mutex> lk2(g_spare_mu);
            g_spare_streams[device].push_back(s);
            w->done = true;
        }
    }
    if (st)
        fprintf(stderr, "pt_device_init(%d) ms: runtime+props %.1f context %.1f code_base %.1f code_wave %.1f copy %.1f "
                "stream (beside it) +%.1f\n", device, t_props, t_ctx - t_props, t_base - t_ctx, t_wave - t_base,
                t_copy ? t_copy - t_wave : 0.0, t_s1 ? t_s1 - t_copy : 0.0);
    return PT_OK;
}
int pt_abi_version(void) { return PT_ABI_VERSION; }

int pt_scene_load_mem(const char* text, size_t len, pt_scene** out) {
    if (!out || (!text && len)) return fail(PT_E_INVALID, "null argument");
    auto* s = new pt_scene();
    try {
        pth::parse_scene(text, len, s->hs);
    } catch (const std::exception& e) {
        delete s;
        return fail(PT_E_SCENE, e.what());
    }
    *out = s;
    return PT_OK;
}

int pt_scene_load(const char* path, pt_scene** out) {
    if (!path || !out) return fail(PT_E_INVALID, "null argument");
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail(PT_E_IO, std::string("cannot open ") + path);
    std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return pt_scene_load_mem(text.data(), text.size(), out);
}

int pt_scene_override(pt_scene* s, uint32_t w, uint32_t h, uint32_t samples, uint32_t depth) {
    if (!s) return fail(PT_E_INVALID, "null scene");
    if (w) s->hs.W = w;
    if (h) s->hs.H = h;
    if (samples) s->hs.samples = samples;
    if (depth) s->hs.depth = depth;
    return PT_OK;
}

// Scene::InitScene (src/scene.cpp:7-40)
int pt_scene_prepare(pt_scene* s) {
    if (!s) return fail(PT_E_INVALID, "null scene");
    if (s->prepared) return PT_OK;
    try {
        // PT_TUNE prepstats=1: per-stage times on stderr
        const bool stats = tune_int("prepstats", 0) != 0;
        auto tick = [stats, t = std::chrono::steady_clock::now()](const char* what) mutable {
            if (!stats) return;
            const auto n = std::chrono::steady_clock::now();
            fprintf(stderr, "prepare %-22s %7.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
            t = n;
        };
        auto& P = s->hs.prims;
        for (const auto& p : P)
            if (p.type != pt::T_PLANE && p.type != pt::T_BOX && p.type != pt::T_ELLIPSOID && p.type != pt::T_TRIANGLE)
                return fail(PT_E_SCENE, "primitive without a type (the reference exits in Primitive::Intersect)");
        // InitBVH: std::partition(non-planes first) on the same sequence -> same permutation
        std::vector<uint32_t> idx(P.size());
        for (uint32_t i = 0; i < (uint32_t)P.size(); ++i) idx[i] = i;
        auto mid = std::partition(idx.begin(), idx.end(), [&P](uint32_t i) { return P[i].type != pt::T_PLANE; });
        s->n_bvh = (uint32_t)(mid - idx.begin());
        std::vector<pth::HPrim> part(P.size());
        for (size_t i = 0; i < idx.size(); ++i) part[i] = P[idx[i]];
        P.swap(part);
        pth::build_reference_bvh(P, s->n_bvh, s->nodes);
        tick("reference BVH");
        s->planes.clear();
        for (uint32_t i = s->n_bvh; i < (uint32_t)P.size(); ++i) s->planes.push_back(i);
        // InitDistribution: BOX/ELLIPSOID with emission > 0, in post-BVH order
        s->emitters.clear();
        for (uint32_t i = 0; i < (uint32_t)P.size(); ++i) {
            const auto& p = P[i];
            if (!(p.emis[0] > 0 || p.emis[1] > 0 || p.emis[2] > 0)) continue;
            if (p.type == pt::T_BOX || p.type == pt::T_ELLIPSOID) s->emitters.push_back(i);
        }
        build_device_layout(s);
        tick("device layout");
        s->box_extent = 0.f;
        for (const auto& n : s->nodes)
            for (int a = 0; a < 3; ++a) s->box_extent = std::max({s->box_extent, fabsf(n.mn[a]), fabsf(n.mx[a])});
        if (!std::isfinite(s->box_extent)) s->box_extent = INFINITY;   // certification then never succeeds
        {
            // the leaves' hit regions, for the aux build's split choice
            std::vector<float>& reg = s->regions;
            reg.assign(6 * s->dnodes.size(), 1.f);
            for (uint32_t i = 0; i < (uint32_t)s->dnodes.size(); ++i) {
                float lo[3], hi[3];
                if ((pt::f2u(s->dnodes[i].b.w) & 0x80000000u) || !leaf_hit_region(s, i, lo, hi)) {
                    reg[6 * i] = 1.f; reg[6 * i + 3] = -1.f;   // none
                    continue;
                }
                for (int a = 0; a < 3; ++a) { reg[6 * i + a] = lo[a]; reg[6 * i + 3 + a] = hi[a]; }
            }
            tick("hit regions");
            pth::build_aux_bvh(s->nodes, reg, s->aux, s->aux_depth);
            tick("aux BVH2");
        }
        pth::build_aux_wide(s->aux, s->dnodes, PT_AUXW, s->auxsl, s->auxsl_depth, s->auxw_stack, s->regions);
        pth::annotate_aux_ranges(s->auxsl, PT_AUXW, (uint32_t)s->dnodes.size(), s->aux_rshift);
        // Query::sp (pt_query.h) counts pending aux nodes in a 7-bit field
        if (s->auxw_stack > PT_QUERY_SP_MAX)
            throw std::runtime_error("auxiliary BVH too deep for the query's stack counter");
        tick("aux wide + ranges");
        pth::build_gamma_thresholds(s->thr);
        build_query_blob(s, tick);
        tick("query blob");
    } catch (const std::exception& e) {
        return fail(PT_E_SCENE, e.what());
    }
    s->prepared = true;
    return PT_OK;
}

int pt_scene_get_info(const pt_scene* s, pt_scene_info* info) {
    if (!s || !info) return fail(PT_E_INVALID, "null argument");
    memset(info, 0, sizeof(*info));
    info->width = s->hs.W;
    info->height = s->hs.H;
    info->samples = s->hs.samples;
    info->ray_depth = s->hs.depth;
    info->n_prims = (uint32_t)s->hs.prims.size();
    info->n_bvh_prims = s->n_bvh;
    info->n_planes = (uint32_t)s->planes.size();
    info->n_emitters = (uint32_t)s->emitters.size();
    info->n_nodes = (uint32_t)s->nodes.size();
    info->tree_depth = s->tree_depth;
    info->max_stack = s->max_stack;
    info->n_aux_nodes = (uint32_t)(s->auxsl.size() / PT_AUXW);   // wide auxiliary BVH (wavefront query)
    info->aux_depth = s->auxsl_depth;
    info->n_warnings = (uint32_t)s->hs.warnings.size();
    return PT_OK;
}

int pt_scene_dump_bvh(const pt_scene* s, void* nodes_out, size_t nodes_bytes, void* prims_out, size_t prims_bytes) {
    if (!s || !s->prepared) return fail(PT_E_INVALID, "scene not prepared");
    if (nodes_out) {
        if (nodes_bytes < s->nodes.size() * 40) return fail(PT_E_INVALID, "nodes buffer too small");
        auto* b = static_cast<unsigned char*>(nodes_out);
        for (const auto& n : s->nodes) {
            memcpy(b, n.mn, 12); memcpy(b + 12, n.mx, 12);
            const uint32_t u[4] = {n.left, n.right, n.first, n.count};
            memcpy(b + 24, u, 16);
            b += 40;
        }
    }
    if (prims_out) {
        if (prims_bytes < s->hs.prims.size() * 52) return fail(PT_E_INVALID, "prims buffer too small");
        auto* b = static_cast<unsigned char*>(prims_out);
        for (const auto& p : s->hs.prims) {
            const bool tri = p.type == pt::T_TRIANGLE;
            const float f[12] = {p.a[0], p.a[1], p.a[2], tri ? p.b[0] : 0.f, tri ? p.b[1] : 0.f, tri ? p.b[2] : 0.f,
                                 tri ? p.c[0] : 0.f, tri ? p.c[1] : 0.f, tri ? p.c[2] : 0.f, p.pos[0], p.pos[1], p.pos[2]};
            memcpy(b, &p.type, 4);
            memcpy(b + 4, f, 48);
            b += 52;
        }
    }
    return PT_OK;
}

void pt_scene_free(pt_scene* s) {
    if (!s) return;
    for (auto& kv : s->dev) {
        (void)hipSetDevice(kv.first);
        free_device_scene(kv.second->d);
    }
    delete s;
}

// ------------------------------------------------------------- sessions ---
int pt_session_create(pt_scene* s, const pt_session_opts* o, pt_session** out) {
    if (!s || !o || !out) return fail(PT_E_INVALID, "null argument");
    if (!s->prepared) return fail(PT_E_INVALID, "scene not prepared (call pt_scene_prepare)");
    if (o->world == 0 || o->rank >= o->world) return fail(PT_E_INVALID, "bad rank/world");
    if (s->hs.W == 0 || s->hs.H == 0) return fail(PT_E_SCENE, "zero image size");
    if ((uint64_t)s->hs.W * s->hs.H >= 2147483647ull) return fail(PT_E_SCENE, "image too large for per-pixel seeds");
    // the slot record keeps the current path's vertex count in 24 bits (pt_devutil.h PixelHot)
    if (s->hs.depth >= (1u << 24)) return fail(PT_E_SCENE, "RAY_DEPTH too large (at most 16777215)");
    int rc = check_device(o->device);
    if (rc) return rc;
    // the megakernel (exact / division-form traversal, PT_TUNE engine=mega) also reads the BVH2 aux
    const bool mega = o->traversal != PT_TRAVERSAL_REPLAY || tune_str("engine") == "mega";
    DevScene* ds = nullptr;
    double up_ms = 0.0;
    if ((rc = ensure_device_scene(s, o->device, mega, &ds, &up_ms))) return rc;
    auto* ss = new pt_session();
    ss->sc = s;
    ss->dev = o->device;
    ss->ds = ds;
    ss->upload_ms = up_ms;
    ss->traversal = o->traversal;
    ss->depth = s->hs.depth;
    ss->tm.W = s->hs.W;
    ss->tm.H = s->hs.H;
    ss->tm.x0 = o->win_w ? o->win_x0 : 0u;
    ss->tm.y0 = o->win_w ? o->win_y0 : 0u;
    ss->tm.ww = o->win_w ? o->win_w : s->hs.W;
    ss->tm.wh = o->win_w ? o->win_h : s->hs.H;
    if (ss->tm.ww == 0 || ss->tm.wh == 0 || (uint64_t)ss->tm.x0 + ss->tm.ww > s->hs.W ||
        (uint64_t)ss->tm.y0 + ss->tm.wh > s->hs.H) {
        delete ss;
        return fail(PT_E_INVALID, "window outside the image");
    }
    ss->tm.tiles_x = (ss->tm.ww + 15u) / 16u;
    ss->tm.n_tiles = ss->tm.tiles_x * ((ss->tm.wh + 15u) / 16u);
    ss->tm.rank = o->rank;
    ss->tm.world = o->world;
    ss->gtiles = rank_tiles(ss->tm.n_tiles, ss->tm.tiles_x, o->rank, o->world);
    ss->n_tiles_local = (uint32_t)ss->gtiles.size();
    ss->n_slots = ss->n_tiles_local * 256u;
    ss->cam = make_cam(s);
    auto cleanup = [&](int code) {
        pt_session_free(ss);
        return code;
    };
    if (hipSetDevice(ss->dev) != hipSuccess) return cleanup(fail(PT_E_HIP, "hipSetDevice failed"));
    DevProps props;
    if ((rc = device_props(ss->dev, &props))) return cleanup(rc);
    const uint32_t cus = (uint32_t)props.cus;
    const size_t n = std::max<size_t>(ss->n_slots, 1);
    ss->st.depth = std::max<uint32_t>(ss->depth, 1u);
    ss->st.n_slots = ss->n_slots;
    // engine: the wavefront pipeline for the (filtered) replay traversal; the
    // megakernel for the exact DFS and the division-form replay (PT_TUNE engine=mega forces it)
    ss->wave = o->traversal == PT_TRAVERSAL_REPLAY;
    if (tune_str("engine") == "mega") ss->wave = false;
    std::vector<uint32_t> ord;   // wavefront: the local tiles' seeding order
    if (ss->wave) {
        ss->shade_grid = std::min<uint32_t>(cus * 8u, std::max(1u, ss->n_tiles_local));
        // path engine: PT_NQ query waves + 1 shade wave per workgroup, as many workgroups
        // per CU as its waves-per-SIMD occupancy holds (4 SIMDs per CU)
        ss->path_budget = (uint32_t)std::max(1, tune_int("budget", (int)ss->path_budget));
        // rounds end at one time for every wave (budget_us after the work ran out; 0: each
        // wave after `budget` trips of its own, also the mode of an explicit budget=N alone)
        // (at most 10 s: the device compares 32-bit clock differences as signed)
        ss->path_ticks = (uint32_t)std::min(10000000, std::max(0, tune_int("budget_us", tune_has("budget") ? 0 : 2500))) * 100u;
        // ... and the low-chain rounds' deadline: 5 ms (fewer rounds, each of which re-sorts and
        // re-takes the early launch's heaviest chains; with coop_grow 16 per CU, one GPU call,
        // 3 repeats of every rank (tools/gpu_r5_ab.sh, profiles/r05_ab): rank of 8 mean 83.5 ->
        // 80.2 ms per 256-spp pass, rank of 4 139.9 -> 137.6, of 2 259.2 -> 255.6, one GPU
        // 488.8 -> 486.3); with budget_us=0 (trip budgets) the path rounds' mode
        ss->low_ticks = tune_has("lowq_budget_us")
                            ? (uint32_t)std::min(10000000, std::max(1, tune_int("lowq_budget_us", 5000))) * 100u
                            : ss->path_ticks == 0 ? 0u : 500000u;
        const int wg_cu = std::max(1, (int)(PT_PATH_WAVES_PER_EU * 4u / (PT_NQ + 1u)));
        ss->path_grid = cus * (uint32_t)std::max(1, tune_int("wg_per_cu", wg_cu));
        // suspended-query records: Query | slot | aux stack, rounded to 16 B.  Only a
        // query lane suspends (one query at round end), and a pixel has at most one ray
        // in flight, so a round appends at most min(pixels, query lanes) of them: the
        // carry queue can never overflow.  The exact-DFS hand-over queues (ex, done, hid)
        // do NOT have that bound: a lane that hands its ray over goes on with another
        // chain of the round's supply, so a round can hand over a ray of every chain --
        // at most one per pixel (a chain that leaves for k_wexact leaves the round).
        // They hold n entries.
        ss->carry_words = ((uint32_t)(sizeof(pt::Query) / 4) + 1u + std::max<uint32_t>(s->auxw_stack, 1u) + 3u) & ~3u;
        ss->lane_cap = (uint32_t)std::min<uint64_t>(n, (uint64_t)ss->path_grid * PT_NQ * 64u);
        ss->carry_cap = ss->lane_cap;
        // a round whose chains are this few runs them to the end of the pass (a few
        // per query wave: rebalancing them costs more rounds than it saves)
        ss->path_runend = ss->path_grid * PT_NQ * 4u;
        ss->path_runend = (uint32_t)std::max(0, tune_int("runend", (int)ss->path_runend));
        // rounds with fewer chains than this run the end-of-pass (sparse) kernel
        ss->path_sparse = ss->path_grid * PT_NQ * 32u;
        ss->path_sparse = (uint32_t)std::max(0, tune_int("sparse", (int)ss->path_sparse));
        ss->sparse_steps = (uint32_t)std::max(1, tune_int("sparse_steps", (int)ss->sparse_steps));
        // a round whose chains are at most this many runs the cooperative engine (one
        // wave per chain) to the end of the pass; it needs a wave's aux stack to hold
        // a depth-first descent below its expansion limit, and lane 0's exact DFS stack
        // 49,152 on the 256-CU part (2 query waves per shade wave, hit-region query; rank-of-4 /
        // rank-of-8 per GPU, teams of 8, two runs each: 32 k 2,758-2,782 / 2,348-2,396, 49 k
        // 2,754-2,774 / 2,377-2,421, 65 k 2,731-2,763 / 2,318-2,338, 98 k 2,695-2,699 / 2,220-2,324,
        // 131 k 2,599-2,603 / 2,358-2,430 Mray/s)
        ss->coop_max = cus * 192u;
        ss->coop_max = (uint32_t)std::max(0, tune_int("coop", (int)ss->coop_max));
        ss->coop_grid = cus * 8u;
        // (a depth-first descent below the expansion limit adds at most 3 entries per level)
        const uint32_t reserve = 3u * (s->auxsl_depth + 2u);
        ss->coop_team = (uint32_t)tune_int("coop_team", (int)ss->coop_team);
        if (ss->coop_team != 8u && ss->coop_team != 16u && ss->coop_team != 32u) ss->coop_team = 64u;
        const uint32_t scap = ss->coop_team == 64u ? 448u : ss->coop_team == 32u ? 192u : QC_SCAP_MIN;
        if (scap < reserve + 64u || s->max_stack > scap) ss->coop_team = 64u;   // deep trees: whole-wave teams
        // (paths deeper than QC_FOLD keep their further fold records in HBM, planes and
        // emitters beyond QC_NPL / QC_NEM come from HBM: no scene limit besides the stacks)
        if (448u < reserve + 64u || s->max_stack > 448u)
            ss->coop_max = 0;
        else ss->coop_reserve = reserve;
        // with the cooperative engine the path engine never runs a round to the end:
        // its rounds stay budget-limited, so the host sees the chains fall below coop_max
        if (ss->coop_max && !tune_has("runend")) ss->path_runend = 0;
        // ... and the end-of-pass (sparse) path kernel, whose rounds are long, never runs
        // above the hand-over
        if (ss->coop_max && !tune_has("sparse")) ss->path_sparse = std::min(ss->path_sparse, ss->coop_max);
        ss->round_batch = (uint32_t)std::max(1, tune_int("round_batch", (int)ss->round_batch));
        ss->coop_order = tune_int("coop_order", 1) != 0;
        // the final launch's last chains to whole-wave teams: 16 per CU (4 per CU measured within
        // the spread of 0; 16 with the 5-ms low-round deadline above: see low_ticks)
        ss->coop_grow = (uint32_t)std::max(0, tune_int("coop_grow", (int)(cus * 16u)));
        // ... and, before that, its last coop_grow_mid chains to teams of 32 (0: no such stage; a
        // tree too deep for the teams-of-32 stack skips it)
        ss->coop_grow_mid = (uint32_t)std::max(0, tune_int("coop_grow_mid", 0));
        if (192u < reserve + 64u || s->max_stack > 192u) ss->coop_grow_mid = 0u;
        // Early cooperative launch (teams of 8, QC_WAVES waves per workgroup: 32 chains each):
        // the low-chain rounds leave each CU room for one more workgroup, which the heaviest
        // chains use from then on instead of waiting for the final hand-over
        ss->early_wg = (uint32_t)std::max(1, tune_int("early_wg", 1));
        ss->early_at = (uint32_t)std::max(0, tune_int("early_at", (int)(cus * 768u)));
        ss->early_k = (uint32_t)std::max(0, tune_int("early", 1));
        // lanes per chain of that launch: 8 (default) or 16 (half the chains, a shorter chain cycle)
        // (a scene beyond the LDS tables has only the teams-of-8 BIG instantiation)
        const bool big = ss->depth > QC_FOLD || s->planes.size() > QC_NPL || s->emitters.size() > QC_NEM;
        {
            const int st = tune_int("side_team", 8);
            ss->side_team = !big && (st == 16 || st == 32 || st == 64) ? (uint32_t)st : 8u;
            if (ss->side_team == 32u && (192u < reserve + 64u || s->max_stack > 192u)) ss->side_team = 8u;
            if (ss->side_team == 64u && (448u < reserve + 64u || s->max_stack > 448u)) ss->side_team = 8u;
        }
        if (ss->early_k == 1u) ss->early_k = cus * ss->early_wg * QC_WAVES * (64u / ss->side_team);   // early=1: what it holds
        if (!ss->coop_max || ss->coop_team != 8u) ss->early_k = 0;
        // a round's carry output also takes the early launch's yielded chains
        ss->carry_cap = (uint32_t)std::min<uint64_t>(n, (uint64_t)ss->lane_cap + ss->early_k);
        {
            static const char* keys[4] = {"probe_every", "probe_min", "aux_extra", "end_min"};
            static const char* lkeys[4] = {"lowq_probe_every", "lowq_probe_min", "lowq_aux_extra", "lowq_end_min"};
            for (int i = 0; i < 4; ++i) {
                const int lo = i == 0 || i == 3 ? 1 : 0;
                ss->mix[i] = (uint32_t)std::max(lo, tune_int(keys[i], (int)ss->mix[i]));
                // (the low rounds' end_min has a default of its own; the others follow the full rounds')
                ss->mix_low[i] = (uint32_t)std::max(lo, tune_int(lkeys[i], (int)(i == 3 ? ss->mix_low[i] : ss->mix[i])));
            }
            ss->mix[3] = std::min<uint32_t>(ss->mix[3], 64u);
            ss->mix_low[3] = std::min<uint32_t>(ss->mix_low[3], 64u);
            // Rounds that start with fewer than 768 chains per CU run on 2 path workgroups
            // per CU (PT_CMAX chains each) instead of 4: with that few chains the rounds are
            // bound by each chain's latency, and a query trip's instruction stream shares its
            // SIMD with fewer waves.  Rank-of-1 / 2 / 4 / 8 (rank 0, three interleaved
            // repeats, profiles/r03_lowq): +2.3 / +2 / +4 / +3-10 %; 150 k / 250 k chains
            // within 1 % at ranks of 1-4, and 300 k (every round of a rank of 8, the first
            // included) -25 % at rank-of-8.
            ss->lowq = (uint32_t)std::max(0, tune_int("lowq", (int)(cus * 768u)));
            ss->low_grid = std::min(ss->path_grid, cus * (uint32_t)std::max(1, tune_int("lowq_wg", 2)));
        }
        if (ss->n_tiles_local) {
            // seeding order of the pass: the local tiles sorted by the Z-order (Morton)
            // code of their tile coordinates
            std::vector<std::pair<uint64_t, uint32_t>> key(ss->n_tiles_local);
            for (uint32_t t = 0; t < ss->n_tiles_local; ++t) {
                const uint32_t gt = ss->gtiles[t];
                const uint32_t tx = gt % ss->tm.tiles_x, ty = gt / ss->tm.tiles_x;
                uint64_t m = 0;
                for (int b = 0; b < 16; ++b)
                    m |= (uint64_t)((tx >> b) & 1u) << (2 * b) | (uint64_t)((ty >> b) & 1u) << (2 * b + 1);
                key[t] = {m, t};
            }
            std::sort(key.begin(), key.end());
            ord.resize(ss->n_tiles_local);
            for (uint32_t t = 0; t < ss->n_tiles_local; ++t) ord[t] = key[t].second;
        }
    }
    // Every device buffer of the session in ONE allocation (sections at 256-B
    // offsets), and the two small host-made tables with one copy: session set-up is
    // a handful of runtime calls, whatever the pixel count.
    {
        size_t at = 0;
        auto sec = [&at](size_t bytes) {
            const size_t o = at;
            at = (at + std::max<size_t>(bytes, 16) + 255) & ~(size_t)255;
            return o;
        };
        const size_t tables = sec((ss->gtiles.size() + ord.size()) * 4);
        const size_t a_rec = sec(2 * n * sizeof(uint4)), a_fold = sec((size_t)ss->st.depth * n * sizeof(uint4));
        const size_t a_ctr = sec(8 * PT_CTR_COPIES * PT_CTR_STRIDE), a_out = sec(3 * n);
        // the window's framebuffer (pt_render's device-side gather; rank 0's session)
        const size_t a_fb = o->rank == 0 ? sec(3ull * ss->tm.ww * ss->tm.wh) : 0;
        size_t a_fq[2][3] = {{0, 0, 0}, {0, 0, 0}}, a_pid = 0, a_dq[2] = {0, 0}, a_ex[2] = {0, 0}, a_hid = 0;
        size_t a_carry = 0, a_ctl = 0, a_endq = 0, a_order = 0, a_side[6] = {0, 0, 0, 0, 0, 0};
        if (ss->wave) {
            for (int q = 0; q < 2; ++q)
                for (int k = 0; k < 3; ++k) a_fq[q][k] = sec(n * 16);
            a_pid = sec(2 * n * 4);
            for (int k = 0; k < 2; ++k) { a_dq[k] = sec(n * 16); a_ex[k] = sec(n * 16); }
            a_hid = sec(n * 4);
            a_carry = sec(2ull * ss->carry_cap * ss->carry_words * 4);
            a_ctl = sec(8 * PT_CTL_SET);
            a_endq = sec((size_t)ss->path_grid * PT_CMAX * sizeof(uint2));
            a_order = sec((n + 2 * PT_ORDER_BUCKETS) * 4);
            if (ss->early_k) {
                for (int k = 0; k < 3; ++k) a_side[k] = sec((size_t)ss->early_k * 16);
                a_side[3] = sec((size_t)ss->early_k * 4);
                a_side[4] = sec((size_t)ss->early_k * ss->carry_words * 4);
                a_side[5] = sec(8 * PT_CTL_SET);
            }
        }
        if (take_stream(ss->dev, &ss->stream) != hipSuccess) return cleanup(fail(PT_E_HIP, "stream creation failed"));
        // the early launch's stream and events: made on a helper thread beside the set-up and
        // the pass's first rounds (a stream's creation costs ~10 ms: neither on the set-up's
        // path nor in the pass), joined where the first early launch needs them
        if (ss->early_k) {
            const int dev = ss->dev;
            ss->side_th = std::thread([ss, dev] {
                ss->side_rc = hipSetDevice(dev);
                if (ss->side_rc == hipSuccess) ss->side_rc = take_stream(dev, &ss->side_stream, true);
                if (ss->side_rc == hipSuccess) ss->side_rc = hipEventCreateWithFlags(&ss->side_taken, hipEventDisableTiming);
                if (ss->side_rc == hipSuccess) ss->side_rc = hipEventCreateWithFlags(&ss->side_end, hipEventDisableTiming);
            });
        }
        void* p = nullptr;
        if (hipMalloc(&p, at) != hipSuccess) return cleanup(fail(PT_E_OOM, "device allocation failed (session buffers)"));
        ss->arena = static_cast<unsigned char*>(p);
        unsigned char* A = ss->arena;
        if (!ss->gtiles.empty()) {
            std::vector<uint32_t> t(ss->gtiles);
            t.insert(t.end(), ord.begin(), ord.end());
            if (hipMemcpy(A + tables, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
                return cleanup(fail(PT_E_HIP, "tile tables upload failed"));
            ss->tm.gtile = reinterpret_cast<const uint32_t*>(A + tables);
            if (!ord.empty()) ss->tile_order = reinterpret_cast<uint32_t*>(A + tables) + ss->gtiles.size();
        }
        ss->st.rec = reinterpret_cast<uint4*>(A + a_rec);
        ss->st.fold = reinterpret_cast<uint4*>(A + a_fold);
        ss->counters = reinterpret_cast<unsigned long long*>(A + a_ctr);
        ss->out = A + a_out;
        if (o->rank == 0) ss->fb = A + a_fb;
        if (ss->wave) {
            for (int q = 0; q < 2; ++q) {
                ss->fq[q].ro = reinterpret_cast<pt::F4*>(A + a_fq[q][0]);
                ss->fq[q].rd = reinterpret_cast<pt::F4*>(A + a_fq[q][1]);
                ss->fq[q].ri = reinterpret_cast<pt::F4*>(A + a_fq[q][2]);
                ss->fq[q].pid = reinterpret_cast<int*>(A + a_pid) + q * n;
            }
            ss->done = pt::DoneQ{reinterpret_cast<pt::F4*>(A + a_dq[0]), reinterpret_cast<pt::F4*>(A + a_dq[1]),
                                 reinterpret_cast<uint32_t*>(A + a_hid)};
            ss->ex = pt::RayQ{reinterpret_cast<pt::F4*>(A + a_ex[0]), reinterpret_cast<pt::F4*>(A + a_ex[1]), nullptr,
                              nullptr};
            ss->carry = reinterpret_cast<uint32_t*>(A + a_carry);
            ss->ctl = reinterpret_cast<uint32_t*>(A + a_ctl);
            ss->endq = reinterpret_cast<uint2*>(A + a_endq);
            ss->order = reinterpret_cast<uint32_t*>(A + a_order);
            if (ss->early_k) {
                ss->side.ro = reinterpret_cast<pt::F4*>(A + a_side[0]);
                ss->side.rd = reinterpret_cast<pt::F4*>(A + a_side[1]);
                ss->side.ri = reinterpret_cast<pt::F4*>(A + a_side[2]);
                ss->side.pid = reinterpret_cast<int*>(A + a_side[3]);
                ss->side_carry = reinterpret_cast<uint32_t*>(A + a_side[4]);
                ss->side_ctl = reinterpret_cast<uint32_t*>(A + a_side[5]);
            }
            if (hipHostMalloc(&ss->ctl_host, 64) != hipSuccess)
                return cleanup(fail(PT_E_OOM, "host allocation failed (round counters)"));
        }
        ss->arena_bytes = at;
    }
    if (hipMemsetAsync(ss->counters, 0, 8 * PT_CTR_COPIES * PT_CTR_STRIDE, ss->stream) != hipSuccess) return cleanup(fail(PT_E_HIP, "memset failed"));
    if (ss->n_tiles_local) {
        pt::InitParams ip;
        ip.tm = ss->tm;
        ip.st = ss->st;
        if (pt_launch_init(ip, ss->n_tiles_local, ss->stream) != hipSuccess)
            return cleanup(fail(PT_E_HIP, "k_init launch failed"));
    }
    *out = ss;
    return PT_OK;
}

int pt_session_layout(const pt_session* ss, uint32_t* n_tiles, uint64_t* packed_rgb_bytes) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (n_tiles) *n_tiles = ss->n_tiles_local;
    if (packed_rgb_bytes) *packed_rgb_bytes = 3ull * ss->n_slots;
    return PT_OK;
}

namespace {
double wall_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int trace_wave(pt_session* ss, uint32_t spp) {
    const DevScene& ds = *ss->ds;
    const pt_scene* s = ss->sc;
    pt::WaveParams wp;
    memset(&wp, 0, sizeof(wp));
    wp.S.aux = nullptr;
    wp.S.nodes = ds.nodes;
    wp.S.prims = ds.prims;
    wp.S.shade = ds.shade;
    wp.S.planes = ds.planes;
    wp.S.emitters = ds.emitters;
    wp.S.n_planes = (uint32_t)s->planes.size();
    wp.S.n_emitters = (uint32_t)s->emitters.size();
    wp.S.inv_emitters = s->emitters.empty() ? 0.f : 1.f / (float)s->emitters.size();
    wp.S.bg = pt::mk3(s->hs.bg[0], s->hs.bg[1], s->hs.bg[2]);
    wp.S.box_extent = s->box_extent;
    wp.S.anc_info = ds.anc_info;
    wp.S.anc = ds.anc;
    set_blob(wp.S, s, ds.blob);
    wp.top = ds.top;
    wp.n_top = ds.n_top;
    wp.n_aux = (uint32_t)s->auxsl.size();
    wp.cam = ss->cam;
    wp.tm = ss->tm;
    wp.st = ss->st;
    wp.fq[0] = ss->fq[0];
    wp.fq[1] = ss->fq[1];
    wp.done = ss->done;
    wp.ex = ss->ex;
    wp.endq = ss->endq;
    wp.cq[0] = ss->carry;
    wp.cq[1] = ss->carry + (size_t)ss->carry_cap * ss->carry_words;
    wp.carry_cap = ss->carry_cap;
    wp.carry_words = ss->carry_words;
    wp.ctl = ss->ctl;
    wp.counters = ss->counters;
    wp.depth = ss->depth;
    wp.target = (uint32_t)(ss->samples_done + spp);
    wp.n_tiles_local = ss->n_tiles_local;
    wp.max_stack = std::max<uint32_t>(s->max_stack, 1u);
    wp.aux_stack = std::max<uint32_t>(s->auxw_stack, 1u);
    wp.path = 1u;
    wp.path_budget = ss->path_budget;
    wp.path_ticks = ss->path_ticks;
    wp.path_runend = ss->path_runend;
    // Chains a workgroup may hold: 5/8 of the pixels' fair share, within
    // [256, PT_CMAX].  Below the share, about a third of the chains wait in the
    // queue and go to whichever workgroup drains first, instead of every
    // workgroup filling to its share and the costly ones finishing last
    // (1920x1080 on 1,024 workgroups: rank of 4 -> 319 instead of 478, +1 % over
    // three alternating pairs; ranks of 1 and 2 stay at 512, a rank of 8 at 256).
    {
        const uint64_t share = ((uint64_t)ss->n_slots + ss->path_grid - 1) / std::max(1u, ss->path_grid);
        wp.path_cap = (uint32_t)std::min<uint64_t>(PT_CMAX, std::max<uint64_t>(256u, share * 5u / 8u));
    }
    if (tune_has("cap")) wp.path_cap = std::min<uint32_t>(PT_CMAX, (uint32_t)std::max(64, tune_int("cap", 0)));
    wp.tile_order = ss->tile_order;
    wp.sparse_steps = ss->sparse_steps;
    wp.coop_reserve = ss->coop_reserve;
    // aux stack words per query lane (PT_TUNE lstack=N < PT_LSTACK: tests of the exact-DFS
    // hand-over of queries that outgrow it)
    // round-queue entries a query wave takes per pull: 32 (64 before round 3's low-chain
    // rounds): a workgroup fills closer to its chain cap in finer pulls; rank-of-1 / 2 / 4 / 8,
    // two calls: +0.5 / +0.5 / +3.5 / +3 % (8 and 16 the same at ranks of 1-4; profiles/r03_lowq)
    wp.batch = (uint32_t)std::min(64, std::max(1, tune_int("batch", 32)));
    wp.end_min = ss->mix[3];
    wp.lstack = std::min<uint32_t>(PT_LSTACK, (uint32_t)std::max(1, tune_int("lstack", (int)PT_LSTACK)));
    if (ss->on_progress && !ss->prog_host) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ss->prog_host), 8, hipHostMallocMapped | hipHostMallocCoherent));
        *ss->prog_host = 0ull;
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&ss->prog_dev), ss->prog_host, 0));
    }
    wp.progress = ss->on_progress ? ss->prog_dev : nullptr;
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, ss->stream));
    HIP_TRY(pt_launch_wave_start(wp, ss->stream));
    if (tune_int("roundlog", 0) >= 2) {
        HIP_TRY(hipStreamSynchronize(ss->stream));
        ss->roundlog_t = wall_ms();
        unsigned long long cc[PT_CTR_COPIES * PT_CTR_STRIDE];
        HIP_TRY(hipMemcpy(cc, ss->counters, sizeof(cc), hipMemcpyDeviceToHost));
        ss->roundlog_rays = 0;
        for (uint32_t x = 0; x < PT_CTR_COPIES; ++x) ss->roundlog_rays += cc[PT_CTR_STRIDE * x];
    }
    // rounds until no fresh ray and no suspended query is left; counts are
    // checked every few rounds (empty rounds are cheap, syncs are not free)
    // (the first round is counted alone: it ends once the pass's work is handed out, and
    // the cooperative engine may take over right after it)
    uint32_t p = 0, batch = ss->coop_max ? 1u : 4u;
    // end-of-pass kernel when the chains of the last counted round are few; before
    // the first count, the pass's pixels (at most one chain each) decide
    bool sparse = ss->n_slots < ss->path_sparse;
    // the cooperative engine once the chains are few (before the first count: the pixels)
    uint32_t chains = ss->n_slots;
    bool counted = false;
    for (uint32_t guard = 0;; ++guard) {
        if (chains <= ss->coop_max) {
            // The cooperative engine runs every remaining chain to the end of the pass.  A
            // launch of teams of 8 (the default) stops once all but ss->coop_grow of its chains
            // have ended and hands those -- the pass's slowest, whose chain cycle sets the
            // launch's end -- to a launch of whole-wave teams (the shortest cycle).
            // (a scene beyond the engine's LDS tables runs the BIG instantiation: teams of 8 or 64)
            const bool big = ss->depth > QC_FOLD || s->planes.size() > QC_NPL || s->emitters.size() > QC_NEM;
            uint32_t team = big && ss->coop_team != 64u ? 8u : ss->coop_team;
            for (;;) {
                // the next stage: teams of 8 -> (coop_grow_mid) teams of 32 -> (coop_grow) whole waves
                uint32_t keep = 0u, next_team = 64u;
                if (team == 8u && !big && ss->coop_grow_mid > ss->coop_grow && chains > ss->coop_grow_mid) {
                    keep = ss->coop_grow_mid;
                    next_team = 32u;
                } else if (team != 64u && ss->coop_grow && chains > ss->coop_grow) {
                    keep = ss->coop_grow;
                }
                const bool grow = keep != 0u;
                wp.parity = p;
                hipEvent_t i0, i1;
                HIP_TRY(hipEventCreate(&i0));
                HIP_TRY(hipEventCreate(&i1));
                ss->pending_isect.emplace_back(i0, i1);
                ss->pending_isect_coop.resize(ss->pending_isect.size(), false);
                ss->pending_isect_coop.back() = true;
                ss->isect_launches++;
                ss->coop_launches++;
                const uint32_t per_wg = QC_WAVES * (64u / team);   // chains per workgroup
                const uint32_t grid = std::max(1u, std::min(ss->coop_grid, (chains + per_wg - 1u) / per_wg));
                const bool cprof = tune_has("cprof");   // -DPT_CPROF builds: per-phase cycles on stderr
                if (cprof) {
                    if (!ss->wg_prof) HIP_TRY(hipMalloc(&ss->wg_prof, 512ull * ss->path_grid));
                    HIP_TRY(hipMemsetAsync(ss->wg_prof, 0, 512, ss->stream));
                    wp.wg_prof = ss->wg_prof;
                }
                if (ss->coop_order) {
                    const size_t cap = std::min<size_t>(std::max<size_t>(ss->n_slots, 1),
                                                        std::max<uint32_t>(ss->coop_max, 1u));
                    if (chains > cap) return fail(PT_E_HIP, "cooperative intake order: more chains than entries");
                    wp.order_cur = ss->order;
                    wp.order = ss->order + 2 * PT_ORDER_BUCKETS;
                    HIP_TRY(pt_launch_coop_order(wp, chains, ss->stream));
                }
                pt::WaveParams cp_ = wp;
                if (grow) {
                    // stop at the chain cycle after all but coop_grow chains have ended (its own
                    // C_ENDED); the rest go to the next launch's input as suspended queries
                    uint32_t* out = ss->ctl + PT_CTL_SET * (1u - p);
                    cp_.side_stop = out + pt::C_ENDED;
                    cp_.side_stop_n = keep;            // (against the launch's own item count: before
                    cp_.side_flags = PT_STOP_GROW |     //  the first count, `chains` is the slot count)
                                     (tune_int("grow_late", 0) ? PT_GROW_LATE : 0u);
                    cp_.yield_cq = wp.cq[1u - p];
                    cp_.yield_ctr = out + pt::C_CARRY;
                }
                HIP_TRY(pt_launch_coop(cp_, grid, team, big, ss->stream, i0, i1));
                wp.order = wp.order_cur = nullptr;
                if (cprof) {
                    unsigned long long cp[64];
                    HIP_TRY(hipMemcpyAsync(cp, wp.wg_prof, 512, hipMemcpyDeviceToHost, ss->stream));
                    HIP_TRY(hipStreamSynchronize(ss->stream));
                    float ms = 0.f;
                    HIP_TRY(hipEventElapsedTime(&ms, i0, i1));
                    const double cyc = (double)std::max(1ull, cp[5] + cp[6]) / (64.0 / team);
                    fprintf(stderr, "coop T=%u chains %u grid %u: %.2f ms, chain cycles %llu, chains %llu; cycles per chain "
                            "cycle: expand %.0f cand %.0f decide %.0f shade %.0f nextray %.0f; wave lifetime %.0f\n",
                            team, chains, grid, ms, cp[5], cp[6], cp[0] / cyc, cp[1] / cyc, cp[2] / cyc, cp[3] / cyc,
                            cp[4] / cyc, (double)cp[7] / (grid * (double)QC_WAVES));
                    // chains ending per 2^20-cycle bucket of their wave's lifetime
                    fprintf(stderr, "coop chain ends per 2^20 cycles:");
                    for (int i = 16; i < 64; ++i) fprintf(stderr, " %llu", cp[i]);
                    fprintf(stderr, "\n");
                    wp.wg_prof = nullptr;
                }
                ss->rounds++;
                p ^= 1u;
                HIP_TRY(hipMemcpyAsync(ss->ctl_host, ss->ctl + PT_CTL_SET * p, 8, hipMemcpyDeviceToHost, ss->stream));
                if (wp.progress) {
                    hipError_t e;
                    while ((e = hipStreamQuery(ss->stream)) == hipErrorNotReady) {
                        ss->on_progress(__atomic_load_n(ss->prog_host, __ATOMIC_RELAXED));
                        std::this_thread::sleep_for(std::chrono::microseconds(500));
                    }
                    HIP_TRY(e);
                }
                HIP_TRY(hipStreamSynchronize(ss->stream));
                const uint32_t left = ss->ctl_host[pt::C_CARRY] + ss->ctl_host[pt::C_FRESH];
                if (left == 0u) break;
                if (!grow) return fail(PT_E_HIP, "cooperative engine left chains behind");
                // the last chains: bigger teams
                chains = left;
                team = next_team;
                if (tune_int("roundlog", 0) >= 2) fprintf(stderr, "coop grow: %u chains to teams of %u\n", left, team);
            }
            break;
        }
        // The early cooperative launch, beside every low-chain round: the round's heaviest
        // chains (most samples left) run in a cooperative launch on the second stream while
        // the path round runs the others (through wp.pin); the launch stops at a chain cycle's
        // end once the round's path workgroups have all finished, its chains yielded to the
        // next round's carry queue, and the next round starts when both are done.
        // (only after a count: before the first one `chains` is the slot count, not the
        // queue's, and every pixel has the same samples left)
        bool side = false;
        // (test hook side_late: the side launch runs after the path round, on its stream --
        // every workgroup one that started after the round's end)
        pt::WaveParams late_sp;
        bool late = false;
        uint32_t late_grid = 0;
        if (ss->early_k && counted && chains < ss->early_at && chains > ss->coop_max) {
            const uint32_t k = std::min(ss->early_k, chains / 4u);
            const uint32_t grid = chains < ss->lowq && ss->low_grid ? ss->low_grid : ss->path_grid;
            if (k) {
                side = true;
                if (ss->side_th.joinable()) {
                    ss->side_th.join();
                    if (ss->side_rc != hipSuccess) return fail(PT_E_HIP, "side stream creation failed");
                }
                if (!ss->side_stream && take_stream(ss->dev, &ss->side_stream, true) != hipSuccess)
                    return fail(PT_E_HIP, "stream creation failed");
                wp.parity = p;
                wp.order_cur = ss->order;
                wp.order = ss->order + 2 * PT_ORDER_BUCKETS;
                HIP_TRY(pt_launch_coop_order(wp, chains, ss->stream));
                HIP_TRY(hipMemsetAsync(ss->side_ctl, 0, 8 * PT_CTL_SET, ss->stream));
                HIP_TRY(pt_launch_side_take(wp, k, ss->side, ss->side_carry, ss->side_ctl, ss->stream));
                // the round's output counters (its finished-workgroup count among them) are zero
                // before the side launch can look at them
                uint32_t* out = ss->ctl + PT_CTL_SET * (1u - p);
                HIP_TRY(hipMemsetAsync(out, 0, 4u * PT_CTL_SET, ss->stream));
                if (!ss->side_taken) HIP_TRY(hipEventCreateWithFlags(&ss->side_taken, hipEventDisableTiming));
                if (!ss->side_end) HIP_TRY(hipEventCreateWithFlags(&ss->side_end, hipEventDisableTiming));
                HIP_TRY(hipEventRecord(ss->side_taken, ss->stream));
                HIP_TRY(hipStreamWaitEvent(ss->side_stream, ss->side_taken, 0));
                pt::WaveParams sp = wp;
                sp.fq[0] = ss->side;
                sp.cq[0] = ss->side_carry;
                sp.ctl = ss->side_ctl;
                sp.parity = 0u;
                sp.order = sp.order_cur = nullptr;
                sp.pin = nullptr;
                sp.side_stop = out + pt::C_WGDONE;
                sp.side_stop_n = grid;
                sp.yield_cq = wp.cq[1u - p];
                sp.yield_ctr = out + pt::C_CARRY;
                sp.side_flags = (tune_int("side_late", 0) ? PT_SIDE_LATE : 0u) |
                                (tune_int("handon", 1) ? 0u : PT_SIDE_NO_HANDON);
                hipEvent_t i0, i1;
                HIP_TRY(hipEventCreate(&i0));
                HIP_TRY(hipEventCreate(&i1));
                ss->pending_isect.emplace_back(i0, i1);
                ss->pending_isect_coop.resize(ss->pending_isect.size(), false);
                ss->pending_isect_coop.back() = true;
                ss->isect_launches++;
                ss->coop_launches++;
                const bool big = ss->depth > QC_FOLD || s->planes.size() > QC_NPL || s->emitters.size() > QC_NEM;
                if (sp.side_flags & PT_SIDE_LATE) {
                    late = true;
                    late_sp = sp;
                    late_grid = ss->early_wg * (ss->coop_grid / 8u);
                    HIP_TRY(hipEventRecord(i0, ss->stream));   // (timed with the round)
                    HIP_TRY(hipEventRecord(i1, ss->stream));
                } else {
                    HIP_TRY(pt_launch_coop(sp, ss->early_wg * (ss->coop_grid / 8u), ss->side_team, big, ss->side_stream, i0, i1));
                    HIP_TRY(hipEventRecord(ss->side_end, ss->side_stream));
                }
                // the path round takes the other chains: items k .. chains of the order
                wp.pin = wp.order + k;
                wp.pin_n = chains - k;
                wp.order = wp.order_cur = nullptr;
                batch = 1u;   // (the next round reads what the side launch yields)
            }
        }
        for (uint32_t r = 0; r < batch; ++r) {
            wp.parity = p;
            const std::string wgps = tune_str("wgprof");
            const char* wgp = wgps.c_str();
            if (*wgp) {
                // diagnostics: per-round path workgroup timelines (32 u64 each) appended to the file
                const size_t wgb = 512ull * ss->path_grid;
                if (!ss->wg_prof) HIP_TRY(hipMalloc(&ss->wg_prof, wgb));
                HIP_TRY(hipMemsetAsync(ss->wg_prof, 0, wgb, ss->stream));
                wp.wg_prof = ss->wg_prof;
            }
            hipEvent_t i0, i1;
            HIP_TRY(hipEventCreate(&i0));
            HIP_TRY(hipEventCreate(&i1));
            ss->pending_isect.emplace_back(i0, i1);
            ss->isect_launches++;
            uint32_t grid = ss->path_grid;
            {
                const bool low = chains < ss->lowq;
                wp.path_ticks = low ? ss->low_ticks : ss->path_ticks;
                const uint32_t* m = low ? ss->mix_low : ss->mix;
                wp.probe_every = m[0];
                wp.probe_min = m[1];
                wp.aux_extra = m[2];
                wp.end_min = m[3];
                if (low && ss->low_grid) {
                    grid = ss->low_grid;
                    if (!tune_has("cap")) wp.path_cap = PT_CMAX;   // (an explicit cap=N stays)
                }
            }
            HIP_TRY(pt_launch_path_round(wp, grid, 64u, ss->stream, sparse, i0, i1));
            wp.pin = nullptr;   // (only the round beside the early launch skips its chains)
            if (late) {
                // (it yields into the round's output counters, which the round's own launch
                // zeroed: a side launch that could yield before that zeroing would lose items)
                const bool big = ss->depth > QC_FOLD || s->planes.size() > QC_NPL || s->emitters.size() > QC_NEM;
                HIP_TRY(pt_launch_coop(late_sp, late_grid, ss->side_team, big, ss->stream));
                HIP_TRY(hipEventRecord(ss->side_end, ss->stream));
                late = false;
            }
            if (wp.wg_prof) {
                uint32_t cnt[2][8];
                HIP_TRY(hipMemcpyAsync(cnt[0], ss->ctl + PT_CTL_SET * p, 32, hipMemcpyDeviceToHost, ss->stream));
                HIP_TRY(hipMemcpyAsync(cnt[1], ss->ctl + PT_CTL_SET * (1u - p), 32, hipMemcpyDeviceToHost, ss->stream));
                HIP_TRY(hipStreamSynchronize(ss->stream));
                fprintf(stderr, "round %u: in fresh %u carry %u -> out fresh %u carry %u exact %u\n", ss->rounds,
                        cnt[0][pt::C_FRESH], cnt[0][pt::C_CARRY], cnt[1][pt::C_FRESH], cnt[1][pt::C_CARRY],
                        cnt[1][pt::C_EXACT]);
                std::vector<unsigned long long> h(64ull * ss->path_grid);
                HIP_TRY(hipMemcpyAsync(h.data(), wp.wg_prof, h.size() * 8, hipMemcpyDeviceToHost, ss->stream));
                HIP_TRY(hipStreamSynchronize(ss->stream));
                if (FILE* f = fopen(wgp, "ab")) {
                    fwrite(h.data(), 8, h.size(), f);
                    fclose(f);
                }
            }
            ss->rounds++;
            p ^= 1u;
        }
        // (a side launch yields into this round's output: the count waits for it)
        if (side) HIP_TRY(hipStreamWaitEvent(ss->stream, ss->side_end, 0));
        HIP_TRY(hipMemcpyAsync(ss->ctl_host, ss->ctl + PT_CTL_SET * p, 8, hipMemcpyDeviceToHost, ss->stream));
        if (wp.progress) {
            // report the finished samples while the rounds run
            hipError_t e;
            while ((e = hipStreamQuery(ss->stream)) == hipErrorNotReady) {
                ss->on_progress(__atomic_load_n(ss->prog_host, __ATOMIC_RELAXED));
                std::this_thread::sleep_for(std::chrono::microseconds(500));
            }
            HIP_TRY(e);
        }
        HIP_TRY(hipStreamSynchronize(ss->stream));
        if (tune_int("roundlog", 0) >= 2) {
            // diagnostics: each round's chains, kind, wall time and rays (roundlog=3: also how
            // far behind the pass target the unfinished pixels are)
            const double now = wall_ms();
            unsigned long long cc[PT_CTR_COPIES * PT_CTR_STRIDE], rays = 0;
            HIP_TRY(hipMemcpy(cc, ss->counters, sizeof(cc), hipMemcpyDeviceToHost));
            for (uint32_t x = 0; x < PT_CTR_COPIES; ++x) rays += cc[PT_CTR_STRIDE * x];
            const double ms = now - ss->roundlog_t;
            fprintf(stderr, "round %u chains %u -> %u+%u (%s%s) %.2f ms rays %llu %.0f Mray/s", ss->rounds, chains,
                    ss->ctl_host[pt::C_FRESH], ss->ctl_host[pt::C_CARRY], chains < ss->lowq ? "low" : "full",
                    side ? "+side" : "", ms, rays - ss->roundlog_rays, (rays - ss->roundlog_rays) / ms / 1e3);
            ss->roundlog_rays = rays;
            if (tune_int("roundlog", 0) == 3) {
                std::vector<uint4> rec(2ull * ss->n_slots);
                HIP_TRY(hipMemcpy(rec.data(), ss->st.rec, rec.size() * sizeof(uint4), hipMemcpyDeviceToHost));
                std::vector<uint32_t> lag;
                for (uint32_t i = 0; i < ss->n_slots; ++i)
                    if (rec[2 * i].w < wp.target) lag.push_back(wp.target - rec[2 * i].w);
                std::sort(lag.begin(), lag.end());
                const size_t m = lag.size();
                fprintf(stderr, "; unfinished %zu lag p50 %u p90 %u p99 %u max %u", m, m ? lag[m / 2] : 0u,
                        m ? lag[m * 9 / 10] : 0u, m ? lag[m * 99 / 100] : 0u, m ? lag[m - 1] : 0u);
            }
            fprintf(stderr, "\n");
            ss->roundlog_t = wall_ms();
        }
        if (tune_int("dupcheck", 0)) {
            // diagnostics: every slot at most once in the next round's work (fresh rays + carry)
            const uint32_t nf = ss->ctl_host[pt::C_FRESH], nc = ss->ctl_host[pt::C_CARRY];
            std::vector<pt::F4> ro(nf);
            std::vector<uint32_t> cw((size_t)nc * ss->carry_words);
            if (nf) HIP_TRY(hipMemcpy(ro.data(), wp.fq[p].ro, nf * sizeof(pt::F4), hipMemcpyDeviceToHost));
            if (nc) HIP_TRY(hipMemcpy(cw.data(), wp.cq[p], cw.size() * 4, hipMemcpyDeviceToHost));
            std::vector<uint8_t> seen(ss->n_slots, 0);
            uint32_t dup = 0, bad = 0;
            auto see = [&](uint32_t slot) {
                if (slot >= ss->n_slots) { ++bad; return; }
                if (seen[slot]++) ++dup;
            };
            for (uint32_t i = 0; i < nf; ++i) see(pt::f2u(ro[i].w));
            for (uint32_t i = 0; i < nc; ++i) see(cw[(size_t)i * ss->carry_words + sizeof(pt::Query) / 4]);
            if (dup || bad)
                fprintf(stderr, "dupcheck: round %u (%s%s) fresh %u carry %u: %u duplicate slot(s), %u out of range\n",
                        ss->rounds, chains < ss->lowq ? "low" : "full", side ? "+side" : "", nf, nc, dup, bad);
        }
        if (ss->ctl_host[pt::C_FRESH] == 0u && ss->ctl_host[pt::C_CARRY] == 0u) break;
        if (guard > 100000u) return fail(PT_E_HIP, "wavefront rounds did not drain");
        chains = ss->ctl_host[pt::C_FRESH] + ss->ctl_host[pt::C_CARRY];
        counted = true;
        // near the cooperative hand-over every round is counted (the tail's rounds take ms)
        batch = chains > 4096u && chains > 4u * ss->coop_max ? ss->round_batch : (chains > 4096u ? 1u : 2u);
        sparse = chains < ss->path_sparse;
    }
    HIP_TRY(hipEventRecord(e1, ss->stream));
    ss->pending.emplace_back(e0, e1);
    ss->samples_done += spp;
    return PT_OK;
}
}  // namespace

// the statistics counters, summed over their per-XCD copies (after the stream's work)
static hipError_t read_counters(pt_session* ss, unsigned long long c[PT_CTR_STRIDE]) {
    unsigned long long cc[PT_CTR_COPIES * PT_CTR_STRIDE];
    // (on the session's stream: the null stream would also wait for other sessions' work)
    hipError_t e = hipMemcpyAsync(cc, ss->counters, sizeof(cc), hipMemcpyDeviceToHost, ss->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ss->stream);
    for (uint32_t k = 0; k < PT_CTR_STRIDE; ++k) c[k] = 0ull;
    if (e != hipSuccess) return e;
    for (uint32_t x = 0; x < PT_CTR_COPIES; ++x)
        for (uint32_t k = 0; k < PT_CTR_STRIDE; ++k) c[k] += cc[PT_CTR_STRIDE * x + k];
    return hipSuccess;
}

// run the coalesced trace() calls of the wavefront engine as one pass
static int flush_trace(pt_session* ss) {
    if (!ss->deferred_spp) return PT_OK;
    const uint32_t spp = ss->deferred_spp;
    ss->deferred_spp = 0;
    HIP_TRY(hipSetDevice(ss->dev));
    return trace_wave(ss, spp);
}

int pt_session_trace(pt_session* ss, uint32_t spp) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (spp == 0 || ss->n_tiles_local == 0) { ss->samples_done += spp; return PT_OK; }
    if (ss->wave) {
        // Consecutive calls are one pass: a pixel goes on with its next samples as soon
        // as it is done with the current ones, so only the last call waits for the
        // slowest pixel.  The pass runs at the next resolve / sync / stats.
        if (ss->deferred_spp > 0xffffffffu - spp) {
            const int rc = flush_trace(ss);
            if (rc) return rc;
        }
        ss->deferred_spp += spp;
        return PT_OK;
    }
    HIP_TRY(hipSetDevice(ss->dev));
    const DevScene& ds = *ss->ds;
    pt::TraceParams tp;
    const pt_scene* s = ss->sc;
    tp.S.aux = ss->traversal == PT_TRAVERSAL_EXACT ? nullptr : ds.aux;
    tp.cfg = replay_cfg(s);
    tp.S.nodes = ds.nodes;
    tp.S.prims = ds.prims;
    tp.S.shade = ds.shade;
    tp.S.planes = ds.planes;
    tp.S.emitters = ds.emitters;
    tp.S.n_planes = (uint32_t)s->planes.size();
    tp.S.n_emitters = (uint32_t)s->emitters.size();
    tp.S.inv_emitters = s->emitters.empty() ? 0.f : 1.f / (float)s->emitters.size();
    tp.S.bg = pt::mk3(s->hs.bg[0], s->hs.bg[1], s->hs.bg[2]);
    tp.S.box_extent = s->box_extent;
    tp.S.anc_info = ds.anc_info;
    tp.S.anc = ds.anc;
    tp.cam = ss->cam;
    tp.tm = ss->tm;
    tp.st = ss->st;
    tp.counters = ss->counters;
    tp.depth = ss->depth;
    tp.spp = spp;
    tp.n_tiles_local = ss->n_tiles_local;
    tp.wg_prof = nullptr;
    // kernel variant: filtered tests unless the division form was asked for; XCD-banded tile order
    const int variant = (ss->traversal == PT_TRAVERSAL_REPLAY ? 1 : 0) | 2;
    const std::string wgps = tune_str("wgprof");
    const char* wgp = wgps.c_str();
    if (*wgp) {
        if (!ss->wg_prof) HIP_TRY(hipMalloc(&ss->wg_prof, 32ull * std::max(ss->n_tiles_local, 1u)));
        HIP_TRY(hipMemsetAsync(ss->wg_prof, 0, 32ull * std::max(ss->n_tiles_local, 1u), ss->stream));
        tp.wg_prof = ss->wg_prof;
    }
    const uint32_t lds = 256u * 4u * lane_words(s, ss->traversal);
    if (lds > 160u * 1024u) return fail(PT_E_SCENE, "BVH too deep for the LDS traversal stack");
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, ss->stream));
    HIP_TRY(pt_launch_trace(tp, variant, lds, ss->stream));
    HIP_TRY(hipEventRecord(e1, ss->stream));
    if (tp.wg_prof) {
        // diagnostics: append this launch's per-workgroup timeline to the wgprof file
        std::vector<unsigned long long> h(4ull * ss->n_tiles_local);
        HIP_TRY(hipMemcpyAsync(h.data(), tp.wg_prof, h.size() * 8, hipMemcpyDeviceToHost, ss->stream));
        HIP_TRY(hipStreamSynchronize(ss->stream));
        if (FILE* f = fopen(wgp, "ab")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
    ss->pending.emplace_back(e0, e1);
    ss->samples_done += spp;
    return PT_OK;
}

int pt_session_resolve(pt_session* ss, uint8_t* dev_out, float* dev_radiance) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (ss->n_tiles_local == 0) return PT_OK;
    if (const int rc = flush_trace(ss)) return rc;
    HIP_TRY(hipSetDevice(ss->dev));
    pt::ResolveParams rp;
    rp.st = ss->st;
    rp.tm = ss->tm;
    rp.counters = ss->counters;
    rp.thr = ss->ds->thr;
    rp.out = dev_out ? dev_out : ss->out;
    rp.rad = dev_radiance;
    rp.samples = (uint32_t)ss->samples_done;
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, ss->stream));
    HIP_TRY(pt_launch_resolve(rp, ss->n_tiles_local, ss->stream));
    HIP_TRY(hipEventRecord(e1, ss->stream));
    HIP_TRY(hipStreamSynchronize(ss->stream));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess) ss->resolve_ms += ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    // pixels short of (or past) the samples so far: a chain was lost -- an error, not an image
    unsigned long long c[PT_CTR_STRIDE];
    HIP_TRY(read_counters(ss, c));
    if (c[pt::CTR_SHORT] != ss->short_seen) {
        const unsigned long long k = c[pt::CTR_SHORT] - ss->short_seen;
        ss->short_seen = c[pt::CTR_SHORT];
        if (tune_int("shortlog", 0)) {
            // diagnostics: how far the short pixels are from the target, and where they are
            std::vector<uint4> rec(2ull * ss->n_slots);
            if (hipMemcpy(rec.data(), ss->st.rec, rec.size() * sizeof(uint4), hipMemcpyDeviceToHost) == hipSuccess) {
                std::map<int, uint32_t> hist;
                uint32_t shown = 0;
                for (uint32_t i = 0; i < ss->n_slots; ++i) {
                    const uint32_t done = rec[2 * i].w, nv = rec[2 * i].z >> 8;
                    if (done == rp.samples || rec[2 * i + 1].w == 0xFFFFFFFFu) continue;
                    hist[(int)done - (int)rp.samples]++;
                    if (shown++ < 8)
                        fprintf(stderr, "short: slot %u pixel %u done %u nv %u\n", i, rec[2 * i + 1].w, done, nv);
                }
                for (auto& h : hist) fprintf(stderr, "short: done - samples = %d: %u pixels\n", h.first, h.second);
            }
        }
        return fail(PT_E_HIP, std::to_string(k) + " pixel(s) did not take exactly " + std::to_string(rp.samples) +
                                  " samples (a chain was lost)");
    }
    return PT_OK;
}

int pt_session_sync(pt_session* ss) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (const int rc = flush_trace(ss)) return rc;
    HIP_TRY(hipSetDevice(ss->dev));
    HIP_TRY(hipStreamSynchronize(ss->stream));
    return finish_pending(ss);
}

int pt_session_read_packed(pt_session* ss, uint8_t* host_out, size_t bytes) {
    if (!ss || !host_out) return fail(PT_E_INVALID, "null argument");
    if (bytes < 3ull * ss->n_slots) return fail(PT_E_INVALID, "buffer too small");
    if (ss->n_slots == 0) return PT_OK;
    HIP_TRY(hipSetDevice(ss->dev));
    HIP_TRY(hipMemcpyAsync(host_out, ss->out, 3ull * ss->n_slots, hipMemcpyDeviceToHost, ss->stream));
    HIP_TRY(hipStreamSynchronize(ss->stream));
    return PT_OK;
}

int pt_session_stats(pt_session* ss, pt_stats* st) {
    if (!ss || !st) return fail(PT_E_INVALID, "null argument");
    int rc = pt_session_sync(ss);
    if (rc) return rc;
    unsigned long long c[PT_CTR_STRIDE];
    HIP_TRY(read_counters(ss, c));
    memset(st, 0, sizeof(*st));
    st->rays = c[0];
    st->node_visits = c[1];
    st->prim_tests = c[2];
    st->plane_tests = c[3];
    st->errors = c[4];
    st->aux_visits = c[5];
    st->fallbacks = c[6];
    st->fallbacks_ray = c[7];
    st->samples = owned_pixels(ss) * ss->samples_done;
    st->kernel_ms = ss->kernel_ms;
    st->resolve_ms = ss->resolve_ms;
    st->node_bytes = sizeof(pt::Node);
    st->prim_bytes = sizeof(pt::Prim);
    // algorithmic bytes per counted unit: wavefront query = 4-wide aux node (128 B),
    // reference node record (32 B), primitive geometry (48 B: the 64-B compact record
    // adds the precomputed triangle normal, a layout choice, not counted)
    st->aux_bytes = ss->wave ? PT_AUXW * sizeof(pt::AuxSL) : sizeof(pt::AuxNode);
    if (ss->wave) st->prim_bytes = 48;
    st->isect_ms = ss->isect_ms;
    st->isect_launches = ss->isect_launches;
    st->rounds = ss->rounds;
    st->coop_rays = c[8];
    st->coop_node_visits = c[9];
    st->coop_prim_tests = c[10];
    st->coop_aux_visits = c[13];
    st->coop_ms = ss->coop_ms;
    st->coop_launches = ss->coop_launches;
    st->short_pixels = c[pt::CTR_SHORT];
    st->handed_on = c[pt::CTR_HANDON];
    return PT_OK;
}

void* pt_session_stream(pt_session* ss) {
    if (!ss) return nullptr;
    (void)flush_trace(ss);   // work ordered after the stream sees every trace() so far (errors: pt_last_error)
    return (void*)ss->stream;
}

void pt_session_free(pt_session* ss) {
    if (!ss) return;
    if (ss->side_th.joinable()) ss->side_th.join();
    (void)hipSetDevice(ss->dev);
    // both streams drained before any buffer goes (a side launch may still run after a
    // failed pass)
    if (ss->stream) (void)hipStreamSynchronize(ss->stream);
    if (ss->side_stream) (void)hipStreamSynchronize(ss->side_stream);
    finish_pending(ss);
    (void)hipFree(ss->arena);
    (void)hipFree(ss->rad); (void)hipFree(ss->wg_prof);
    if (ss->ctl_host) (void)hipHostFree(ss->ctl_host);
    if (ss->prog_host) (void)hipHostFree(ss->prog_host);
    if (ss->side_taken) (void)hipEventDestroy(ss->side_taken);
    if (ss->side_end) (void)hipEventDestroy(ss->side_end);
    if (ss->stream || ss->side_stream) {
        // back to the device's pools for the next session (no destroy/create per render)
        std::lock_guard<std::mutex> lk(g_spare_mu);
        if (ss->stream) g_spare_streams[ss->dev].push_back(ss->stream);
        if (ss->side_stream) g_spare_side[ss->dev].push_back(ss->side_stream);
    }
    delete ss;
}

int pt_unpack_tiles(uint32_t W, uint32_t H, uint32_t rank, uint32_t world, const uint8_t* packed, uint8_t* rgb) {
    if (!packed || !rgb || world == 0) return fail(PT_E_INVALID, "bad argument");
    const uint32_t tiles_x = (W + 15u) / 16u, n_tiles = tiles_x * ((H + 15u) / 16u);
    uint32_t lt = 0;
    for (uint32_t gt = 0; gt < n_tiles; ++gt) {
        if (pt::tile_owner(gt, tiles_x, world) != rank) continue;
        const uint32_t tx = gt % tiles_x, ty = gt / tiles_x;
        for (uint32_t j = 0; j < 16u; ++j) {
            const uint32_t y = ty * 16u + j;
            if (y >= H) break;
            const uint32_t x0 = tx * 16u, w = std::min(16u, W - x0);
            memcpy(rgb + ((size_t)y * W + x0) * 3, packed + ((size_t)lt * 256u + j * 16u) * 3, (size_t)w * 3);
        }
        ++lt;
    }
    return PT_OK;
}

int pt_unpack_tiles_f32(uint32_t W, uint32_t H, uint32_t rank, uint32_t world, const float* packed, float* rad) {
    if (!packed || !rad || world == 0) return fail(PT_E_INVALID, "bad argument");
    const uint32_t tiles_x = (W + 15u) / 16u, n_tiles = tiles_x * ((H + 15u) / 16u);
    uint32_t lt = 0;
    for (uint32_t gt = 0; gt < n_tiles; ++gt) {
        if (pt::tile_owner(gt, tiles_x, world) != rank) continue;
        const uint32_t tx = gt % tiles_x, ty = gt / tiles_x;
        for (uint32_t j = 0; j < 16u; ++j) {
            const uint32_t y = ty * 16u + j;
            if (y >= H) break;
            const uint32_t x0 = tx * 16u, w = std::min(16u, W - x0);
            memcpy(rad + ((size_t)y * W + x0) * 3, packed + ((size_t)lt * 256u + j * 16u) * 3, (size_t)w * 12);
        }
        ++lt;
    }
    return PT_OK;
}

// ------------------------------------------------------------- render -----
namespace {
// RCCL communicators over devices dev0 .. dev0+n-1, created once per process and
// device set (pt_gather_init may create one ahead of the render)
std::mutex g_comm_mu;
std::map<std::pair<int, int>, std::vector<ncclComm_t>> g_comms;
int comm_get(int dev0, int n, std::vector<ncclComm_t>** out) {
    // (caller holds g_comm_mu)
    auto key = std::make_pair(dev0, n);
    auto it = g_comms.find(key);
    if (it == g_comms.end()) {
        std::vector<int> devs(n);
        for (int g = 0; g < n; ++g) devs[g] = dev0 + g;
        std::vector<ncclComm_t> c(n);
        if (!rccl().ok) return fail(PT_E_RCCL, "librccl.so.1 not loadable");
        if (rccl().CommInitAll(c.data(), n, devs.data()) != ncclSuccess) return fail(PT_E_RCCL, "ncclCommInitAll failed");
        it = g_comms.emplace(key, c).first;
    }
    *out = &it->second;
    return PT_OK;
}

// Test-only (PT_TUNE same_device=1): pt_render(ngpu = n) runs its n sessions and
// host threads all on `device` -- the in-process multi-GPU path on one GPU.  RCCL
// cannot place two ranks on one device, so the framebuffer goes through the host.
bool same_device() { return tune_int("same_device", 0) != 0; }

// One process driving several GPUs: the packed u8 tiles of every session are
// gathered to the first device with one grouped ncclGather over xGMI
// (communicator cached per device set), then un-interleaved on the host.
int gather_rccl(const std::vector<pt_session*>& sess, int dev0, uint32_t W, uint32_t H, uint8_t* rgb,
                uint8_t* staging) {
    std::lock_guard<std::mutex> lk(g_comm_mu);
    const int n = (int)sess.size();
    std::vector<ncclComm_t>* cp = nullptr;
    if (const int rc = comm_get(dev0, n, &cp)) return rc;
    auto& c = *cp;
    size_t cap = 0;
    for (auto* x : sess) cap = std::max<size_t>(cap, 3ull * x->n_slots);
    cap = std::max<size_t>(cap, 16);
    // per-device staging buffers, released on every exit path (scope guard)
    struct Buffers {
        int dev0, n;
        std::vector<uint8_t*> send;
        uint8_t* recv = nullptr;
        Buffers(int d, int k) : dev0(d), n(k), send((size_t)k, nullptr) {}
        ~Buffers() {
            for (int g = 0; g < n; ++g)
                if (send[(size_t)g]) { (void)hipSetDevice(dev0 + g); (void)hipFree(send[(size_t)g]); }
            (void)hipSetDevice(dev0);
            if (recv) (void)hipFree(recv);
        }
    } buf(dev0, n);
    for (int g = 0; g < n; ++g) {
        HIP_TRY(hipSetDevice(dev0 + g));
        if (hipMalloc(&buf.send[(size_t)g], cap) != hipSuccess) return fail(PT_E_OOM, "gather buffer");
        if (sess[g]->n_slots)
            HIP_TRY(hipMemcpyAsync(buf.send[(size_t)g], sess[g]->out, 3ull * sess[g]->n_slots, hipMemcpyDeviceToDevice,
                                   sess[g]->stream));
        if (g == 0 && hipMalloc(&buf.recv, cap * n) != hipSuccess) return fail(PT_E_OOM, "gather buffer");
    }
    const Rccl& R = rccl();
    ncclResult_t r = R.GroupStart();
    for (int g = 0; g < n && r == ncclSuccess; ++g)
        r = R.Gather(buf.send[(size_t)g], g == 0 ? buf.recv : nullptr, cap, ncclUint8, 0, c[g], sess[g]->stream);
    if (r == ncclSuccess) r = R.GroupEnd();
    if (r != ncclSuccess) return fail(PT_E_RCCL, std::string("ncclGather: ") + R.GetErrorString(r));
    // the framebuffer on the first device: every window tile's source in the gathered blocks
    // (owner * cap + its rank among the owner's tiles * 768), un-tiled by one kernel, one copy out
    const uint32_t tiles_x = (W + 15u) / 16u, n_tiles = tiles_x * ((H + 15u) / 16u);
    std::vector<uint32_t> src(n_tiles), seen((size_t)n, 0u);
    for (uint32_t t = 0; t < n_tiles; ++t) {
        const uint32_t g = pt::tile_owner(t, tiles_x, (uint32_t)n);
        src[t] = (uint32_t)(g * cap + seen[g]++ * 768u);
    }
    if ((uint64_t)cap * n > 0xffffffffull) return fail(PT_E_INVALID, "gather buffer beyond 4 GB");
    HIP_TRY(hipSetDevice(dev0));
    uint32_t* dsrc = nullptr;
    HIP_TRY(hipMalloc(&dsrc, std::max<size_t>(n_tiles, 1) * 4));
    struct Free { uint32_t* p; ~Free() { (void)hipFree(p); } } free_src{dsrc};
    HIP_TRY(hipMemcpyAsync(dsrc, src.data(), n_tiles * 4ull, hipMemcpyHostToDevice, sess[0]->stream));
    HIP_TRY(pt_launch_untile(buf.recv, dsrc, tiles_x, W, H, staging ? staging : sess[0]->fb, sess[0]->stream));
    if (!staging) HIP_TRY(hipMemcpyAsync(rgb, sess[0]->fb, 3ull * W * H, hipMemcpyDeviceToHost, sess[0]->stream));
    for (int g = 0; g < n; ++g) {
        HIP_TRY(hipSetDevice(dev0 + g));
        HIP_TRY(hipStreamSynchronize(sess[g]->stream));
    }
    if (staging) memcpy(rgb, staging, 3ull * W * H);
    return PT_OK;
}
}  // namespace

int pt_gather_init(int device, int ngpu) {
    if (ngpu < 1 || device < 0) return fail(PT_E_INVALID, "bad device range");
    if (same_device()) return PT_OK;   // (test-only mode: host gather)
    std::lock_guard<std::mutex> lk(g_comm_mu);
    std::vector<ncclComm_t>* c = nullptr;
    return comm_get(device, ngpu, &c);
}

void pt_render_opts_default(pt_render_opts* o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->device = 0;
    o->ngpu = 1;
    o->traversal = PT_TRAVERSAL_REPLAY;
}

int pt_render(pt_scene* s, const pt_render_opts* opts, uint8_t* rgb, float* radiance, pt_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    auto ms_since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    if (!s) return fail(PT_E_INVALID, "null scene");
    pt_render_opts o;
    pt_render_opts_default(&o);
    if (opts) o = *opts;
    int rc = pt_scene_prepare(s);
    if (rc) return rc;
    const uint32_t S = o.samples ? o.samples : s->hs.samples;
    const uint32_t W = o.win_w ? o.win_w : s->hs.W, H = o.win_w ? o.win_h : s->hs.H;
    const int ngpu = std::max(1, o.ngpu);
    std::vector<pt_session*> sess((size_t)ngpu, nullptr);
    auto cleanup = [&](int code) {
        for (auto* x : sess) pt_session_free(x);
        return code;
    };
    // PT_TUNE same_device=1 (test-only): the ngpu sessions all on o.device, rendering
    // at once; same_device=2: the same, but the ranks render one after another once
    // every session is set up, so each rank's render time is its time alone on a GPU
    // (the per-rank phase times of PT_STATS=2 then project an ngpu-GPU run)
    const int same = tune_int("same_device", 0);
    // samples per trace call: one pass for all of them (a pass ends with its slowest
    // pixel, so every extra sync costs a tail).  The wavefront engine reports the
    // bar from inside the pass; the exact-traversal renderer takes ~20 passes.
    int last = 0;
    const bool wave = o.traversal == PT_TRAVERSAL_REPLAY && tune_str("engine") != "mega";
    const bool in_pass = o.progress && wave;
    const uint32_t chunk = o.spp_per_launch ? o.spp_per_launch
                           : o.progress && !in_pass ? std::max(1u, (S + 19u) / 20u) : std::max(S, 1u);
    // One host thread per GPU sets up its session (the device's scene upload and the
    // session buffers: devices in parallel) and drives it (the wavefront rounds sync
    // on their own stream) through the resolve; thread 0 reports progress.
    std::vector<int> trc((size_t)ngpu, PT_OK);
    std::vector<std::string> terr((size_t)ngpu);
    std::vector<float*> drads((size_t)ngpu, nullptr);
    struct Phase { double setup = 0, upload = 0, wait = 0, render = 0, resolve = 0; };
    std::vector<Phase> ph((size_t)ngpu);
    std::mutex turn_mu;
    std::condition_variable turn_cv;
    int created = 0, turn = 0;
    auto work = [&](int g) {
        Phase& f = ph[(size_t)g];
        auto t_g = std::chrono::steady_clock::now();
        pt_session_opts so;
        so.device = same ? o.device : o.device + g;
        so.rank = (uint32_t)g;
        so.world = (uint32_t)ngpu;
        so.traversal = o.traversal;
        so.win_x0 = o.win_x0;
        so.win_y0 = o.win_y0;
        so.win_w = o.win_w;
        so.win_h = o.win_h;
        int r = pt_session_create(s, &so, &sess[(size_t)g]);
        pt_session* x = sess[(size_t)g];
        if (!r) r = pt_session_sync(x);   // (the session's init kernel)
        if (!r && tune_int("inject_fail", -1) == g) r = fail(PT_E_INVALID, "injected failure (PT_TUNE inject_fail)");
        f.setup = ms_since(t_g);
        if (x) f.upload = x->upload_ms;
        if (same == 2) {
            // every session set up, then the ranks' renders one at a time, in rank order
            std::unique_lock<std::mutex> lk(turn_mu);
            ++created;
            turn_cv.notify_all();
            const auto tw = std::chrono::steady_clock::now();
            // (>=: every rank advances `turn` once, failed or not, so no rank can be skipped)
            turn_cv.wait(lk, [&] { return created == ngpu && turn >= g; });
            f.wait = ms_since(tw);
        }
        if (!r && same == 2 && tune_int("prespin_us", 0) > 0) {
            // (diagnostics: the device busy before this rank's render, outside its time)
            if (pt_launch_spin((uint32_t)tune_int("prespin_us", 0), 2048u, nullptr, x->stream) != hipSuccess)
                r = fail(PT_E_HIP, "spin kernel launch failed");
            if (!r) r = pt_session_sync(x);
        }
        const auto t_r = std::chrono::steady_clock::now();
        if (!r && g == 0 && in_pass) {
            const uint64_t total = owned_pixels(x) * S;
            x->on_progress = [&last, total](uint64_t k) { progress_bar(std::min(k, total), total, last); };
        }
        for (uint32_t done = 0; !r && done < S;) {
            const uint32_t k = std::min(chunk, S - done);
            r = pt_session_trace(x, k);
            if (!r && (o.progress || ngpu > 1)) r = pt_session_sync(x);
            done += k;
            if (!r && g == 0 && o.progress) progress_bar(done, S, last);
        }
        if (!r) r = pt_session_sync(x);
        f.render = ms_since(t_r);
        if (same == 2) {
            std::lock_guard<std::mutex> lk(turn_mu);
            ++turn;
            turn_cv.notify_all();
        }
        // resolve on the device (tonemap + quantise into the packed 8-bit tiles)
        const auto t_v = std::chrono::steady_clock::now();
        if (!r && radiance && x->n_slots) {
            if (hipMalloc(&x->rad, 12ull * x->n_slots) != hipSuccess) r = fail(PT_E_OOM, "radiance buffer");
            drads[(size_t)g] = x->rad;
        }
        if (!r) r = pt_session_resolve(x, nullptr, drads[(size_t)g]);
        f.resolve = ms_since(t_v);
        if (r) {
            trc[(size_t)g] = r;
            terr[(size_t)g] = pt_last_error();
        }
    };
    // a pinned staging buffer for the framebuffer's copy out (a device-to-pageable copy is
    // staged by the runtime at a fraction of the link's rate), allocated beside the render
    uint8_t* staging = nullptr;
    std::thread stage_th;
    if (rgb && W && H && tune_int("staging", 1))
        stage_th = std::thread([&staging, bytes = 3ull * W * H] {
            void* p = nullptr;
            if (hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess) staging = static_cast<uint8_t*>(p);
        });
    struct StageFree {
        std::thread& th;
        uint8_t*& p;
        ~StageFree() {
            if (th.joinable()) th.join();
            if (p) (void)hipHostFree(p);
        }
    } stage_free{stage_th, staging};
    if (ngpu == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < ngpu; ++g) th.emplace_back(work, g);
        for (auto& t : th) t.join();
    }
    for (int g = 0; g < ngpu; ++g)
        if (trc[(size_t)g]) return cleanup(fail(trc[(size_t)g], terr[(size_t)g]));
    // gather the packed 8-bit tiles: over RCCL to device `o.device` when ngpu > 1, else one copy
    pt_stats agg;
    memset(&agg, 0, sizeof(agg));
    const auto t_gather = std::chrono::steady_clock::now();
    if (rgb) {
        // PT_GATHER_AUTO: RCCL when ngpu > 1 (host fallback with a warning);
        // PT_GATHER_RCCL: RCCL at any ngpu, an error if it fails; PT_GATHER_HOST: never RCCL
        const bool try_rccl = !same && (o.gather == PT_GATHER_RCCL || (o.gather == PT_GATHER_AUTO && ngpu > 1));
        if (stage_th.joinable()) stage_th.join();
        if (try_rccl && (rc = gather_rccl(sess, o.device, W, H, rgb, staging)) == PT_OK) {
            agg.gather_rccl = 1;
        } else {
            if (o.gather == PT_GATHER_RCCL) return cleanup(rc);
            if (try_rccl) fprintf(stderr, "pt_render: RCCL gather unavailable (%s); gathering through the host\n",
                                  pt_last_error());
            if (ngpu == 1 && sess[0]->n_slots) {
                // one session owns every tile: un-tiled on its device, one copy out
                pt_session* x = sess[0];
                const uint32_t tiles_x = (W + 15u) / 16u;
                const double g0 = ms_since(t_gather);
                // (into the pinned staging buffer directly: the kernel's stores cross the link)
                if (hipSetDevice(x->dev) != hipSuccess ||
                    pt_launch_untile(x->out, nullptr, tiles_x, W, H, staging ? staging : x->fb, x->stream) != hipSuccess ||
                    (!staging && hipMemcpyAsync(rgb, x->fb, 3ull * W * H, hipMemcpyDeviceToHost, x->stream) != hipSuccess) ||
                    hipStreamSynchronize(x->stream) != hipSuccess)
                    return cleanup(fail(PT_E_HIP, "framebuffer copy failed"));
                const double g1 = ms_since(t_gather);
                if (staging) memcpy(rgb, staging, 3ull * W * H);
                if (getenv("PT_STATS") && atoi(getenv("PT_STATS")) >= 3)
                    fprintf(stderr, "gather ms: staging join %.1f untile+copy %.1f (%s) host copy %.1f\n", g0, g1 - g0,
                            staging ? "kernel into pinned" : "copy engine", ms_since(t_gather) - g1);
            }
            for (int g = 0; g < ngpu && ngpu > 1; ++g) {
                pt_session* x = sess[(size_t)g];
                if (!x->n_slots) continue;
                std::vector<uint8_t> packed(3ull * x->n_slots);
                if ((rc = pt_session_read_packed(x, packed.data(), packed.size()))) return cleanup(rc);
                pt_unpack_tiles(W, H, (uint32_t)g, (uint32_t)ngpu, packed.data(), rgb);
            }
        }
    }
    const double gather_ms = ms_since(t_gather);
    if (const char* e = getenv("PT_STATS"); e && atoi(e) >= 2) {
        // per-rank phase times (the CLI's PT_STATS=2): set-up = the device's scene upload (if
        // this session did it) + the session's buffers and init kernel
        for (int g = 0; g < ngpu; ++g) {
            pt_stats rs;
            if ((rc = pt_session_stats(sess[(size_t)g], &rs))) return cleanup(rc);
            fprintf(stderr, "pt_render rank %d/%d: setup_ms=%.1f scene_upload_ms=%.3f wait_ms=%.1f render_ms=%.1f "
                    "resolve_ms=%.1f isect_ms=%.1f coop_ms=%.1f coop_launches=%llu rounds=%llu rays=%llu "
                    "handed_on=%llu\n", g, ngpu, ph[(size_t)g].setup, ph[(size_t)g].upload, ph[(size_t)g].wait,
                    ph[(size_t)g].render, ph[(size_t)g].resolve, rs.isect_ms, rs.coop_ms,
                    (unsigned long long)rs.coop_launches, (unsigned long long)rs.rounds,
                    (unsigned long long)rs.rays, (unsigned long long)rs.handed_on);
        }
        fprintf(stderr, "pt_render gather_ms=%.1f path=%s\n", gather_ms, agg.gather_rccl ? "rccl" : "host");
    }
    for (int g = 0; g < ngpu; ++g) {
        pt_session* x = sess[(size_t)g];
        float* drad = drads[(size_t)g];
        if (radiance && x->n_slots) {
            std::vector<float> pr(3ull * x->n_slots);
            if (hipMemcpy(pr.data(), drad, pr.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
                return cleanup(fail(PT_E_HIP, "radiance readback failed"));
            pt_unpack_tiles_f32(W, H, (uint32_t)g, (uint32_t)ngpu, pr.data(), radiance);
        }
        pt_stats st;
        if ((rc = pt_session_stats(x, &st))) return cleanup(rc);
        agg.rays += st.rays; agg.node_visits += st.node_visits; agg.prim_tests += st.prim_tests;
        agg.plane_tests += st.plane_tests; agg.samples += st.samples; agg.errors += st.errors;
        agg.aux_visits += st.aux_visits; agg.fallbacks += st.fallbacks;
        agg.fallbacks_ray += st.fallbacks_ray;
        agg.short_pixels += st.short_pixels; agg.handed_on += st.handed_on;
        agg.isect_ms = std::max(agg.isect_ms, st.isect_ms);
        agg.isect_launches += st.isect_launches;
        agg.coop_rays += st.coop_rays; agg.coop_node_visits += st.coop_node_visits;
        agg.coop_prim_tests += st.coop_prim_tests; agg.coop_aux_visits += st.coop_aux_visits;
        agg.coop_ms = std::max(agg.coop_ms, st.coop_ms); agg.coop_launches += st.coop_launches;
        agg.rounds += st.rounds; agg.aux_bytes = st.aux_bytes;
        agg.kernel_ms = std::max(agg.kernel_ms, st.kernel_ms);
        agg.resolve_ms = std::max(agg.resolve_ms, st.resolve_ms);
        agg.node_bytes = st.node_bytes; agg.prim_bytes = st.prim_bytes;
    }
    if (o.progress) progress_bar(S, S, last);
    agg.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = agg;
    return cleanup(agg.errors ? fail(PT_E_INVALID, "exactness guard tripped (hit list overflow)") : PT_OK);
}

int pt_write_ppm(const char* path, uint32_t W, uint32_t H, const uint8_t* rgb) {
    if (!path || !rgb) return fail(PT_E_INVALID, "null argument");
    FILE* f = fopen(path, "wb");
    if (!f) return fail(PT_E_IO, std::string("cannot write ") + path);
    fprintf(f, "P6\n%u %u\n255\n", W, H);
    const size_t n = (size_t)W * H * 3;
    const bool ok = fwrite(rgb, 1, n, f) == n;
    if (fclose(f) != 0 || !ok) return fail(PT_E_IO, std::string("short write to ") + path);
    return PT_OK;
}

// ------------------------------------------------------------- selftests --
namespace {
struct HostStack {
    std::vector<uint32_t> v;
    uint32_t cap = 0xffffffffu;
    void setc(uint32_t i, uint32_t x, bool c) { if (c) set(i, x); }
    void set(uint32_t i, uint32_t x) { if (v.size() <= i) v.resize(i + 1); v[i] = x; }
    uint32_t get(uint32_t i) const { return v[i]; }
};
struct HostVStore {
    std::vector<uint32_t> v;
    void put(uint32_t k, uint32_t idm, float s1, float s2) {
        if (v.size() < 3 * (k + 1)) v.resize(3 * (k + 1));
        v[3 * k] = idm; v[3 * k + 1] = pt::f2u(s1); v[3 * k + 2] = pt::f2u(s2);
    }
    void get(uint32_t k, uint32_t& idm, float& s1, float& s2) const {
        idm = v[3 * k]; s1 = pt::u2f(v[3 * k + 1]); s2 = pt::u2f(v[3 * k + 2]);
    }
};
}  // namespace

int pt_selftest_ray_intersection(pt_scene* s, int32_t traversal, uint32_t n, const float* rays, int32_t* ids,
                                 float* hits, uint64_t* counters8) {
    int rc = pt_scene_prepare(s);
    if (rc) return rc;
    const pt::SceneView V = host_view(s, traversal);
    const pt::ReplayCfg cfg = replay_cfg(s);
    HostStack stk;
    pt::Counts C{};
    const bool coop = tune_str("qengine") == "coop";   // the cooperative engine's query (pt_coop.h)
    for (uint32_t i = 0; i < n; ++i) {
        pt::Ray r;
        r.o = pt::mk3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        r.d = pt::mk3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        pt::Hit h;
        int id;
        if (traversal == PT_TRAVERSAL_REPLAY) {
            pt::QCounts Q{0u, 0u, 0u, 0u};
            uint32_t ex = 0;
            id = coop ? pt::qc_query(V, r, stk, h, Q, ex) : pt::q_run(V, r, stk, h, Q, ex);
            if (Q.planes & 0x80000000u) return fail(PT_E_INVALID, "recomputed closest hit differs from the query's");
            C.rays++;
            C.nodes += Q.nodes; C.ptests += Q.ptests; C.planes += Q.planes; C.aux += Q.aux; C.fallbacks += ex;
        } else {
            id = pt::ray_intersection<false>(V, cfg, r, stk, h, C);
        }
        ids[i] = id;
        const bool ok = id != -1;
        hits[5 * i] = ok ? h.t : 0.f;
        hits[5 * i + 1] = ok ? h.n.x : 0.f;
        hits[5 * i + 2] = ok ? h.n.y : 0.f;
        hits[5 * i + 3] = ok ? h.n.z : 0.f;
        hits[5 * i + 4] = ok ? (h.interior ? 1.f : 0.f) : 0.f;
    }
    if (counters8) {
        const uint64_t c[8] = {C.rays, C.nodes, C.ptests, C.planes, C.errs, C.aux, C.fallbacks, 0};
        memcpy(counters8, c, sizeof(c));
    }
    return C.errs ? fail(PT_E_INVALID, "hit list overflow") : PT_OK;
}

int pt_selftest_render_host(pt_scene* s, int32_t traversal, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                            uint32_t spp, float* radiance) {
    int rc = pt_scene_prepare(s);
    if (rc) return rc;
    const pt::SceneView V = host_view(s, traversal);
    const pt::ReplayCfg cfg = replay_cfg(s);
    const pt::CamView cam = make_cam(s);
    const uint32_t S = spp ? spp : s->hs.samples;
    const uint32_t nt = std::max(1u, std::thread::hardware_concurrency());
    std::vector<std::thread> th;
    std::vector<uint32_t> errs(nt, 0);
    // diagnostics: PT_TUNE qstats=<file> dumps per-query {aux visits, node tests, prim tests, exact} (u32 x4)
    const std::string qpaths = tune_str("qstats");
    const char* qpath = qpaths.empty() ? nullptr : qpaths.c_str();
    std::vector<std::vector<std::array<uint32_t, 4>>> qlogs(nt);
    const bool coop = tune_str("qengine") == "coop";   // the cooperative engine's query (pt_coop.h)
    for (uint32_t t = 0; t < nt; ++t) {
        th.emplace_back([&, t]() {
            std::vector<std::array<uint32_t, 4>>* qlog = qpath ? &qlogs[t] : nullptr;
            HostStack stk;
            HostVStore vs;
            pt::Counts C{};
            for (uint64_t k = t; k < (uint64_t)w * h; k += nt) {
                const uint32_t x = x0 + (uint32_t)(k % w), y = y0 + (uint32_t)(k / w);
                pt::Rng R = pt::rng_seed(y * s->hs.W + x);
                pt::f3 sum = pt::mk3(0.f, 0.f, 0.f);
                for (uint32_t i = 0; i < S; ++i) {
                    const float fx = (float)x + pt::rng_uniform(R);
                    const float fy = (float)y + pt::rng_uniform(R);
                    const pt::Ray ray = pt::camera_ray(cam, fx, fy);
                    if (traversal == PT_TRAVERSAL_REPLAY) {
                        // the wavefront engine's query (pt_query.h state machine), run to completion
                        auto q = [&](const pt::Ray& rr, pt::Hit& hh, pt::Counts& cc) {
                            pt::QCounts Q{};
                            uint32_t ex = 0;
                            const int id = coop ? pt::qc_query(V, rr, stk, hh, Q, ex) : pt::q_run(V, rr, stk, hh, Q, ex);
                            cc.fallbacks += ex;
                            if (Q.planes & 0x80000000u) cc.errs |= 4u;   // recomputed hit differs (checked below)
#ifdef PT_QDIAG
                            if (qlog) qlog->push_back({Q.aux, Q.rc_acc | (Q.rc_rej << 16), Q.rc_walk, Q.cands | (Q.passes << 16)});
#else
                            if (qlog) qlog->push_back({Q.aux, Q.nodes, Q.ptests | (ex << 31), 0u});
#endif
                            return id;
                        };
                        sum = sum + pt::trace_path_with(V, q, ray, s->hs.depth, R, vs, C);
                    } else {
                        sum = sum + pt::trace_path<false>(V, cfg, ray, s->hs.depth, R, stk, vs, C);
                    }
                }
                const pt::f3 m = (1.f / (float)S) * sum;
                radiance[3 * k] = m.x; radiance[3 * k + 1] = m.y; radiance[3 * k + 2] = m.z;
            }
            errs[t] = C.errs;
        });
    }
    for (auto& x : th) x.join();
    if (qpath)
        if (FILE* f = fopen(qpath, "wb")) {
            for (auto& v : qlogs) fwrite(v.data(), 16, v.size(), f);
            fclose(f);
        }
    for (uint32_t e : errs)
        if (e) return fail(PT_E_INVALID, "hit list overflow");
    return PT_OK;
}

int pt_selftest_gamma_table(const pt_scene* s, float* thr256) {
    if (!s || !s->prepared || !thr256) return fail(PT_E_INVALID, "scene not prepared");
    memcpy(thr256, s->thr, sizeof(s->thr));
    return PT_OK;
}

}  // extern "C"
