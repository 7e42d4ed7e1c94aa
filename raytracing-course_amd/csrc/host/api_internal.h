// api_internal.h -- what libpt's host units share (internal; not part of the C ABI).
//
// The C ABI of include/pt.h is implemented across these units:
//   common.cpp    errors, PT_TUNE, the RCCL loader, stream pools, device properties,
//                 the scene's device copy, pt_device_init
//   scene_api.cpp Scene::Load / InitScene equivalents: parse, reference BVH, aux BVH,
//                 the query blob (pt_scene_*)
//   session.cpp   tile sessions: set-up, the megakernel pass, resolve, stats (pt_session_*)
//   rounds.cpp    the wavefront pass: path rounds, early / final cooperative launches
//   render.cpp    Scene::Render equivalent: per-GPU threads, the RCCL / host gather, PPM
//   selftest.cpp  host execution of the device query / integrator code (tests only)
#pragma once
#include "pt.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <utility>
#include <vector>

#include "../device/pt_coop.h"
#include "../device/pt_kernels.h"
#include "pt_scene.h"

#pragma GCC visibility push(hidden)

namespace pti {

// the message of the last failure on this thread (pt_last_error)
int fail(int code, const std::string& msg);
const std::string& last_error();

// PT_TUNE="key=value,..." (the keys are listed in common.cpp and INTEGRATION.md)
std::string tune_str(const char* key);
bool tune_has(const char* key);
int tune_int(const char* key, int def);
// PT_STATS=N (the CLI's phase reports): N, or 0 when unset
int stats_level();

// RCCL, loaded on first use (dlopen): only the multi-GPU gather needs it
struct Rccl {
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclGather) Gather = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    bool ok = false;
};
const Rccl& rccl();

// streams: per-device pools (pt_device_init makes one ahead of time; sessions take
// streams from the pools and give them back).  side = the early cooperative launch's
// stream, from a pool of greatest-priority streams (common.cpp has the reason).
hipError_t take_stream(int dev, hipStream_t* s, bool side = false);
void give_stream(int dev, hipStream_t s, bool side);

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

// device properties, queried once per device
struct DevProps { bool ok = false; int cus = 0; char arch[64] = {0}; double props_ms = 0.0; };
int device_props(int dev, DevProps* out);
int check_device(int dev);
int ensure_device_scene(pt_scene* s, int dev, bool mega, DevScene** out, double* upload_ms);
void free_device_scene(DevScene& d);

// scene views (scene_api.cpp)
pt::ReplayCfg replay_cfg(const pt_scene* s);
uint32_t lane_words(const pt_scene* s, int traversal);
void set_blob(pt::SceneView& v, const pt_scene* s, const pt::F4* blob);
pt::SceneView host_view(const pt_scene* s, int traversal);
pt::CamView make_cam(const pt_scene* s);

// fn(begin, end, part) over [0, n) in at most `parts` contiguous chunks, one thread each
// (host preparation loops whose items are independent).  A thread that cannot be
// started leaves its chunk to the calling thread.
template <class F>
void parallel_chunks(size_t n, unsigned parts, F fn) {
    parts = std::max(1u, std::min<unsigned>(parts, (unsigned)((n + 8191) / 8192)));
    if (parts == 1) { fn((size_t)0, n, 0u); return; }
    std::vector<std::thread> th;
    std::vector<unsigned> here;
    for (unsigned k = 0; k < parts; ++k) {
        try {
            th.emplace_back(fn, n * k / parts, n * (k + 1) / parts, k);
        } catch (const std::system_error&) {
            here.push_back(k);
        }
    }
    for (unsigned k : here) fn(n * k / parts, n * (k + 1) / parts, k);
    for (auto& t : th) t.join();
}
unsigned prep_threads();

// sessions (session.cpp, rounds.cpp)
double wall_ms();
int finish_pending(pt_session* ss);
std::vector<uint32_t> rank_tiles(uint32_t n_tiles, uint32_t tiles_x, uint32_t rank, uint32_t world);
uint64_t owned_pixels(const pt_session* ss);
hipError_t read_counters(pt_session* ss, unsigned long long c[PT_CTR_STRIDE]);
int flush_trace(pt_session* ss);
int trace_wave(pt_session* ss, uint32_t spp);
// the hand-off site named `name` (PT_HO_*: "suspend", "flush", "ringout", "exact", "side_take",
// "side_yield", "side_handon", "grow_yield", "grow_handon"), or -1
int handoff_site(const char* name);
// a scene beyond the cooperative engine's LDS tables (RAY_DEPTH > QC_FOLD, more than
// QC_NPL planes or QC_NEM emitters) runs its BIG instantiation
bool coop_big(const pt_session* ss);

static_assert(pt::HO_SUSPEND == PT_HO_SUSPEND && pt::HO_FLUSH == PT_HO_FLUSH && pt::HO_RINGOUT == PT_HO_RINGOUT &&
                  pt::HO_EXACT == PT_HO_EXACT && pt::HO_SIDE_TAKE == PT_HO_SIDE_TAKE &&
                  pt::HO_SIDE_YIELD == PT_HO_SIDE_YIELD && pt::HO_SIDE_HANDON == PT_HO_SIDE_HANDON &&
                  pt::HO_GROW_YIELD == PT_HO_GROW_YIELD && pt::HO_GROW_HANDON == PT_HO_GROW_HANDON &&
                  pt::HO_N == PT_HO_N && PT_HO_N <= 12 && pt::CTR_HO + PT_HO_N <= PT_CTR_STRIDE,
              "hand-off sites: device and ABI numbering differ");

}  // namespace pti

#define HIP_TRY(expr)                                                                                 \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return pti::fail(PT_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_));       \
    } while (0)

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
    std::map<int, std::unique_ptr<pti::DevEntry>> dev;
    std::mutex mu;                    // the image and the device map (not the uploads)
};

struct pt_session {
    pt_scene* sc = nullptr;
    int dev = 0;
    const pti::DevScene* ds = nullptr;   // the scene's copy on this device
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
    uint32_t coop_team = 4;       // lanes per chain in the cooperative engine (pure-coop rate, teams of
                                  // 64 / 32 / 16 / 8: 283 / 392 / 572 / 815 Mray/s; the final launch in
                                  // teams of 4 against 8, rank 0 of 1 / 8: 475.9 / 74.7 ms against
                                  // 476.3 / 79.2, means of 5 interleaved runs, profiles/r06_coop/team4)
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

#pragma GCC visibility pop
