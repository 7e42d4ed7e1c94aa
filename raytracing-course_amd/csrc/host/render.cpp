// render.cpp -- Scene::Render equivalent (pt_render): one host thread and one session
// per GPU, the device tonemap, the framebuffer gather (one grouped ncclGather over
// xGMI to the first device, or through the host), the P6 write.
#include <stdio.h>
#include <string.h>

#include <condition_variable>
#include "api_internal.h"

namespace pti {
namespace {

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

// RCCL communicators over devices dev0 .. dev0+n-1, created once per process and
// device set (pt_gather_init may create one ahead of the render), with the gather's
// device buffers: made by the first render that gathers over the set and kept (grown
// when a later render needs more), so consecutive renders allocate nothing
struct CommSet {
    std::vector<ncclComm_t> c;
    std::vector<uint8_t*> send;   // per device: cap bytes (its rank's packed tiles)
    uint8_t* recv = nullptr;      // first device: n x cap bytes (the gathered blocks)
    uint32_t* src = nullptr;      // first device: per window tile, its source in recv
    size_t cap = 0, src_n = 0;
};
std::mutex g_comm_mu;
std::map<std::pair<int, int>, CommSet> g_comms;
int comm_get(int dev0, int n, CommSet** out) {
    // (caller holds g_comm_mu)
    auto key = std::make_pair(dev0, n);
    auto it = g_comms.find(key);
    if (it == g_comms.end()) {
        std::vector<int> devs(n);
        for (int g = 0; g < n; ++g) devs[g] = dev0 + g;
        std::vector<ncclComm_t> c(n);
        if (!rccl().ok) return fail(PT_E_RCCL, "librccl.so.1 not loadable");
        if (rccl().CommInitAll(c.data(), n, devs.data()) != ncclSuccess) return fail(PT_E_RCCL, "ncclCommInitAll failed");
        CommSet cs;
        cs.c = c;
        cs.send.assign((size_t)n, nullptr);
        it = g_comms.emplace(key, std::move(cs)).first;
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
// (communicator and buffers cached per device set), then un-tiled there by one
// kernel into the caller's framebuffer.  *allocs = the device allocations made.
int gather_rccl(const std::vector<pt_session*>& sess, int dev0, uint32_t W, uint32_t H, uint8_t* rgb,
                uint8_t* staging, uint64_t* allocs) {
    if (tune_int("inject_rccl", 0)) return fail(PT_E_RCCL, "injected RCCL gather failure (PT_TUNE inject_rccl)");
    std::lock_guard<std::mutex> lk(g_comm_mu);
    const int n = (int)sess.size();
    CommSet* cs = nullptr;
    if (const int rc = comm_get(dev0, n, &cs)) return rc;
    size_t cap = 0;
    for (auto* x : sess) cap = std::max<size_t>(cap, 3ull * x->n_slots);
    cap = std::max<size_t>(cap, 16);
    if ((uint64_t)cap * n > 0xffffffffull) return fail(PT_E_INVALID, "gather buffer beyond 4 GB");
    const uint32_t tiles_x = (W + 15u) / 16u, n_tiles = tiles_x * ((H + 15u) / 16u);
    if (cap > cs->cap) {
        // (grown: the old buffers go, new ones of the size this render needs)
        for (int g = 0; g < n; ++g) {
            HIP_TRY(hipSetDevice(dev0 + g));
            if (cs->send[(size_t)g]) (void)hipFree(cs->send[(size_t)g]);
            cs->send[(size_t)g] = nullptr;
            if (g == 0 && cs->recv) (void)hipFree(cs->recv);
            if (g == 0) cs->recv = nullptr;
        }
        cs->cap = 0;
        for (int g = 0; g < n; ++g) {
            HIP_TRY(hipSetDevice(dev0 + g));
            if (hipMalloc(&cs->send[(size_t)g], cap) != hipSuccess) return fail(PT_E_OOM, "gather buffer");
            ++*allocs;
        }
        HIP_TRY(hipSetDevice(dev0));
        if (hipMalloc(&cs->recv, cap * n) != hipSuccess) return fail(PT_E_OOM, "gather buffer");
        ++*allocs;
        cs->cap = cap;
    }
    if (n_tiles > cs->src_n) {
        HIP_TRY(hipSetDevice(dev0));
        if (cs->src) (void)hipFree(cs->src);
        cs->src = nullptr;
        cs->src_n = 0;
        if (hipMalloc(&cs->src, std::max<size_t>(n_tiles, 1) * 4) != hipSuccess) return fail(PT_E_OOM, "gather buffer");
        ++*allocs;
        cs->src_n = n_tiles;
    }
    for (int g = 0; g < n; ++g) {
        HIP_TRY(hipSetDevice(dev0 + g));
        if (sess[g]->n_slots)
            HIP_TRY(hipMemcpyAsync(cs->send[(size_t)g], sess[g]->out, 3ull * sess[g]->n_slots, hipMemcpyDeviceToDevice,
                                   sess[g]->stream));
    }
    const Rccl& R = rccl();
    ncclResult_t r = R.GroupStart();
    for (int g = 0; g < n && r == ncclSuccess; ++g)
        r = R.Gather(cs->send[(size_t)g], g == 0 ? cs->recv : nullptr, cs->cap, ncclUint8, 0, cs->c[g], sess[g]->stream);
    if (r == ncclSuccess) r = R.GroupEnd();
    if (r != ncclSuccess) return fail(PT_E_RCCL, std::string("ncclGather: ") + R.GetErrorString(r));
    // the framebuffer on the first device: every window tile's source in the gathered blocks
    // (owner * cap + its rank among the owner's tiles * 768), un-tiled by one kernel, one copy out
    std::vector<uint32_t> src(n_tiles), seen((size_t)n, 0u);
    for (uint32_t t = 0; t < n_tiles; ++t) {
        const uint32_t g = pt::tile_owner(t, tiles_x, (uint32_t)n);
        src[t] = (uint32_t)(g * cs->cap + seen[g]++ * 768u);
    }
    HIP_TRY(hipSetDevice(dev0));
    HIP_TRY(hipMemcpyAsync(cs->src, src.data(), n_tiles * 4ull, hipMemcpyHostToDevice, sess[0]->stream));
    HIP_TRY(pt_launch_untile(cs->recv, cs->src, tiles_x, W, H, staging ? staging : sess[0]->fb, sess[0]->stream));
    if (!staging) HIP_TRY(hipMemcpyAsync(rgb, sess[0]->fb, 3ull * W * H, hipMemcpyDeviceToHost, sess[0]->stream));
    for (int g = 0; g < n; ++g) {
        HIP_TRY(hipSetDevice(dev0 + g));
        HIP_TRY(hipStreamSynchronize(sess[g]->stream));
    }
    if (staging) memcpy(rgb, staging, 3ull * W * H);
    return PT_OK;
}
}  // namespace
}  // namespace pti

using namespace pti;

extern "C" {

int pt_gather_init(int device, int ngpu) {
    if (ngpu < 1 || device < 0) return fail(PT_E_INVALID, "bad device range");
    if (same_device()) return PT_OK;   // (test-only mode: host gather)
    std::lock_guard<std::mutex> lk(g_comm_mu);
    CommSet* c = nullptr;
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
    if (rgb && W && H && tune_int("staging", 1)) {
        try {
            stage_th = std::thread([&staging, bytes = 3ull * W * H] {
                void* p = nullptr;
                if (hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess) staging = static_cast<uint8_t*>(p);
            });
        } catch (const std::system_error&) {
            // (no thread: the copy out goes through the device framebuffer instead)
        }
    }
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
        for (int g = 0; g < ngpu; ++g) {
            try {
                th.emplace_back(work, g);
            } catch (const std::system_error&) {
                // a rank whose thread cannot start fails; it still counts as set up and
                // rendered, so the ranks of same_device=2 waiting for their turn go on
                trc[(size_t)g] = fail(PT_E_INVALID, "cannot start the host thread of rank " + std::to_string(g));
                terr[(size_t)g] = pt_last_error();
                std::lock_guard<std::mutex> lk(turn_mu);
                ++created;
                ++turn;
                turn_cv.notify_all();
            }
        }
        for (auto& t : th) t.join();
    }
    for (int g = 0; g < ngpu; ++g)
        if (trc[(size_t)g]) return cleanup(fail(trc[(size_t)g], terr[(size_t)g]));
    // gather the packed 8-bit tiles: over RCCL to device `o.device` when ngpu > 1, else one copy
    pt_stats agg;
    memset(&agg, 0, sizeof(agg));
    const auto t_gather = std::chrono::steady_clock::now();
    if (rgb) {
        // PT_GATHER_AUTO: RCCL when ngpu > 1 (host fallback with a warning, the reason in
        // pt_last_error); PT_GATHER_RCCL: RCCL at any ngpu, an error if it fails;
        // PT_GATHER_HOST: never RCCL.  (PT_TUNE inject_rccl=1: the AUTO fail-over at any ngpu)
        const bool auto_rccl = ngpu > 1 || tune_int("inject_rccl", 0) != 0;
        const bool try_rccl = !same && (o.gather == PT_GATHER_RCCL || (o.gather == PT_GATHER_AUTO && auto_rccl));
        if (stage_th.joinable()) stage_th.join();
        if (try_rccl && (rc = gather_rccl(sess, o.device, W, H, rgb, staging, &agg.gather_allocs)) == PT_OK) {
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
        for (int k = 0; k < PT_HO_N; ++k) agg.handoff[k] += st.handoff[k];
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

}  // extern "C"
