// pt_trace.h -- closest-hit query and path integrator of the hw5 render loop,
// restated for one-ray-per-lane execution on gfx950.
//
// Traversal = the reference's recursive BVH_t::Intersect_ (src/bvh.cpp:185-225)
// turned into an iterative, left-first DFS with an explicit stack, keeping its
// exact pruning semantics (not the simplified "global bound" variant):
//   * a node is skipped iff its slab test misses or (bound < t_entry && !interior);
//   * a right child's bound is the best hit found in its left sibling's
//     subtree if there was one, else the parent's bound -- so the bound can
//     RISE (leaf hits are not clipped to their boxes).
// Encoding: a stack entry is (right child | hits-found-at-push << 24); leaf
// hits are appended to a small monotone "suffix minimum" list, so the best
// hit inside a just-finished left subtree is the first list entry whose
// sequence number is >= the entry's; if no hit was found there, the running
// bound is provably unchanged (every pop inside that subtree restored it).
//
// Integrator = src/scene.cpp:83-178 made iterative.  The reference folds
// c_k = E_k + f_k(c_{k+1}) from the deepest vertex back; the per-vertex
// factors are kept in a small per-lane record stack and folded in that same
// order, so the float result is bit-identical (no forward-throughput
// reassociation).
#pragma once
#include "pt_core.h"

namespace pt {

struct Counts {
    uint64_t rays;        // Scene::RayIntersection calls (SURVEY §8d "Mray/s" numerator)
    uint64_t nodes;       // BVH node records fetched + slab-tested
    uint64_t ptests;      // leaf primitive tests
    uint64_t planes;      // plane tests
    uint32_t errs;        // hit-list overflow (must stay 0; the result is then not exact)
};

struct CamView {
    f3 pos, right, up, fwd;
    float tx, ty;         // (float)tan((double)(fov/2)) and (tx*H)/W, precomputed on the host
    float W, H;           // (float)width, (float)height
};

// src/scene.cpp:180-187 (direction is NOT normalised)
PT_HD Ray camera_ray(const CamView& c, float x, float y) {
    const float nx = (2.f * x / c.W - 1.f) * c.tx;
    const float ny = -1.f * (2.f * y / c.H - 1.f) * c.ty;
    Ray r;
    r.o = c.pos;
    r.d = nx * c.right + ny * c.up + 1.f * c.fwd;
    return r;
}

#define PT_HITLIST 6

// Exact reference traversal.  `stk` provides push(i, v) / get(i) of u32.
template <class Stack>
PT_HD int bvh_exact(const SceneView& S, const Ray& ray, float cb, Stack& stk, Hit& best, Counts& C) {
    int best_id = -1;
    best.t = PT_INF;
    float ms_t[PT_HITLIST];
    uint32_t ms_q[PT_HITLIST];
    uint32_t msn = 0;
    uint32_t nh = 0;
    uint32_t sp = 0;
    uint32_t node = 0;
    for (;;) {
        const Node nd = S.nodes[node];
        C.nodes++;
        const f3 c = mk3(nd.a.x, nd.a.y, nd.a.z);
        const f3 s = mk3(nd.a.w, nd.b.x, nd.b.y);
        float t;
        uint32_t interior;
        // AABB_t::Intersect: IntersectBox(ray + -1*center, s)  (src/bvh.cpp:89-93)
        const bool hit = slab(ray.o + -1.f * c, ray.d, s, t, interior);
        bool descend = false;
        if (hit && !(cb < t && !interior)) {
            const uint32_t ref = f2u(nd.b.z), cnt = f2u(nd.b.w);
            if (cnt != 0u) {
                // leaf: first-min over its primitives (strict <), src/bvh.cpp:205-213
                Hit lb;
                lb.t = PT_INF;
                int lid = -1;
                for (uint32_t i = ref; i < ref + cnt; ++i) {
                    Hit h;
                    C.ptests++;
                    if (prim_intersect(S.prims[i], ray, h) && h.t < lb.t) { lb = h; lid = (int)i; }
                }
                if (lid >= 0) {
                    // append to the monotone suffix-minimum list
                    uint32_t keep = 0;
#pragma unroll
                    for (int k = 0; k < PT_HITLIST; ++k)
                        if ((uint32_t)k < msn && ms_t[k] < lb.t) keep = (uint32_t)k + 1u;
                    if (keep == PT_HITLIST) {
                        // overflow: drop the oldest entry (never seen in practice; counted)
#pragma unroll
                        for (int k = 0; k + 1 < PT_HITLIST; ++k) { ms_t[k] = ms_t[k + 1]; ms_q[k] = ms_q[k + 1]; }
                        keep = PT_HITLIST - 1;
                        C.errs |= 1u;
                    }
#pragma unroll
                    for (int k = 0; k < PT_HITLIST; ++k)
                        if ((uint32_t)k == keep) { ms_t[k] = lb.t; ms_q[k] = nh; }
                    msn = keep + 1u;
                    nh++;
                    if (nh >= 255u) C.errs |= 2u;
                    if (lb.t < best.t) { best = lb; best_id = lid; }
                }
            } else {
                stk.push(sp++, ref | (nh << 24));
                node = node + 1u;
                descend = true;
            }
        }
        if (descend) continue;
        if (sp == 0u) break;
        const uint32_t e = stk.get(--sp);
        node = e & 0x00ffffffu;
        const uint32_t hs = e >> 24;
        if (hs != nh) {
            // hits inside the finished left subtree: bound = their minimum
            bool found = false;
#pragma unroll
            for (int k = 0; k < PT_HITLIST; ++k)
                if (!found && (uint32_t)k < msn && ms_q[k] >= hs) { cb = ms_t[k]; found = true; }
        }
    }
    return best_id;
}

// src/scene.cpp:46-77: planes first (strict <), then the BVH bounded by the plane t
template <class Stack>
PT_HD int ray_intersection(const SceneView& S, const Ray& ray, Stack& stk, Hit& out, Counts& C) {
    int id = -1;
    float closest = PT_INF;
    for (uint32_t k = 0; k < S.n_planes; ++k) {
        const uint32_t pi = S.planes[k];
        Hit h;
        C.planes++;
        if (prim_intersect(S.prims[pi], ray, h) && h.t < closest) { closest = h.t; out = h; id = (int)pi; }
    }
    Hit bh;
    const int bid = bvh_exact(S, ray, closest, stk, bh, C);
    if (bid != -1 && bh.t < closest) { out = bh; id = bid; }
    return id;
}

// per-vertex fold record modes
enum : uint32_t { V_TERM = 0u, V_DIFFUSE = 1u, V_COL = 2u, V_IDENT = 3u };

// One camera sample: src/scene.cpp:189-203 (inner) + RayTrace :83-178.
// `vs` provides put(k, idmode, s1, s2) / get(k, idmode, s1, s2) for k < depth.
template <class Stack, class VStore>
PT_HD f3 trace_path(const SceneView& S, Ray ray, uint32_t depth, Rng& R, Stack& stk, VStore& vs, Counts& C) {
    const float eps = 1e-4f;  // Scene::eps, include/scene.h:56
    uint32_t nv = 0;
    f3 leaf = mk3(0.f, 0.f, 0.f);
    for (uint32_t rem = depth;; --rem) {
        if (rem == 0u) { leaf = mk3(0.f, 0.f, 0.f); break; }
        C.rays++;
        Hit h;
        const int id = ray_intersection(S, ray, stk, h, C);
        if (id == -1) { leaf = S.bg; break; }
        const Shade sh = S.shade[id];
        const uint32_t mat = f2u(sh.s1.w);
        const f3 p = ray.o + h.t * ray.d;
        const f3 n = h.n;
        if (mat == M_DIFFUSE) {
            const f3 p_outer = p + eps * n;
            const f3 dir = sample_mix(S, R, p_outer, n);
            const float cosv = dot(dir, n);
            if (cosv <= 0.f) { vs.put(nv++, (uint32_t)id | (V_TERM << 30), 0.f, 0.f); break; }
            const float pw = pdf_mix(S, p_outer, n, dir);
            vs.put(nv++, (uint32_t)id | (V_DIFFUSE << 30), cosv, 1.f / pw);
            ray.o = p + eps * dir;
            ray.d = dir;
        } else if (mat == M_METALLIC) {
            const f3 rd = reflect(n, normalize(ray.d));
            vs.put(nv++, (uint32_t)id | (V_COL << 30), 1.f, 1.f);
            ray.o = p + eps * rd;
            ray.d = rd;
        } else if (mat == M_DIELECTRIC) {
            float eta1 = 1.f, eta2 = sh.s0.w;
            if (h.interior) { const float tt = eta1; eta1 = eta2; eta2 = tt; }
            const f3 dir = -1.f * normalize(ray.d);
            const float cosn = dot(n, dir);
            const float sin2 = (float)((double)(eta1 / eta2) * sqrt((double)smax(0.f, 1.f - cosn * cosn)));
            bool refl;
            if (fabs((double)sin2) > 1.0) {
                refl = true;                                  // total internal reflection
            } else {
                const float q = (eta1 - eta2) / (eta1 + eta2);
                const float r0 = (float)((double)q * (double)q);             // pow(q, 2.)
                const float rr = (float)((double)r0 + (double)(1.f - r0) * pow5_cr((double)(1.f - cosn)));
                refl = rng_uniform(R) < rr;
            }
            if (refl) {
                const f3 rd = reflect(n, normalize(ray.d));
                vs.put(nv++, (uint32_t)id | (V_IDENT << 30), 1.f, 1.f);
                ray.o = p + eps * rd;
                ray.d = rd;
            } else {
                const float cos2 = (float)sqrt((double)(1.f - sin2 * sin2));
                const float k = eta1 / eta2;
                const f3 rd = k * (-1.f * dir) + (k * cosn - cos2) * n;
                vs.put(nv++, (uint32_t)id | ((h.interior ? V_IDENT : V_COL) << 30), 1.f, 1.f);
                ray.o = p + eps * rd;
                ray.d = rd;
            }
        } else {
            vs.put(nv++, (uint32_t)id | (V_TERM << 30), 0.f, 0.f);   // unknown material: other = 0
            break;
        }
    }
    // backward fold: L = E_k + ((A_k * L) * s1_k) * s2_k, deepest vertex first
    f3 L = leaf;
    while (nv > 0u) {
        --nv;
        uint32_t idm;
        float s1, s2;
        vs.get(nv, idm, s1, s2);
        const uint32_t id = idm & 0x3fffffffu, mode = idm >> 30;
        const Shade sh = S.shade[id];
        const f3 E = mk3(sh.s1.x, sh.s1.y, sh.s1.z);
        f3 other;
        if (mode == V_TERM) {
            other = mk3(0.f, 0.f, 0.f);
        } else {
            const f3 col = mk3(sh.s0.x, sh.s0.y, sh.s0.z);
            f3 A;
            if (mode == V_DIFFUSE) A = col / PT_PI_F;
            else if (mode == V_COL) A = col;
            else A = mk3(1.f, 1.f, 1.f);
            other = ((A * L) * s1) * s2;
        }
        L = E + other;
    }
    return L;
}

}  // namespace pt
