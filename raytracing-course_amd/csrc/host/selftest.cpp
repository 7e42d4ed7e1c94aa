// selftest.cpp -- host execution of the device query and integrator code (pt_query.h,
// pt_coop.h, pt_trace.h) for the CPU tests; never used by pt_render.
#include <stdio.h>
#include <string.h>

#include <array>
#include "api_internal.h"

namespace pti {
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
}  // namespace pti

using namespace pti;

extern "C" {

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
