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
    uint64_t aux;         // auxiliary BVH node visits (candidate replay)
    uint64_t fallbacks;   // rays that took the exact stack DFS although replay was enabled
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

// Exact reference traversal.  `stk` is per-lane word memory: set(i, v) / get(i).
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
            if (!(cnt & PT_NODE_INTERIOR)) {
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
                stk.set(sp++, ref | (nh << 24));
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

// ---------------------------------------------------------------------------
// Candidate replay: the same traversal semantics, evaluated only where they can
// matter.  A reference leaf can contribute a hit only if its own slab test
// passes, so (1) the auxiliary BVH enumerates every leaf whose exact slab test
// passes (conservative fast box tests, then the exact test), (2) the leaves are
// processed in reference preorder (= the DFS order of BVH_t::Intersect_), and
// (3) for each one the root->leaf path is replayed with the reference's tests
// and bounds: a node is skipped iff slab miss or (bound < t_entry && !interior);
// going right at node a sets bound = min{hits in leaves (a, right(a))} if any,
// else keeps bound(a).  Subtrees without candidates return no hit in the
// reference, so they change neither the result nor any bound.  Result and
// pruning are therefore identical to the full recursion (proof: DESIGN.md §4).
// Per-lane word memory `L`: [0, as) aux traversal stack, [as, as+cap) candidates.
#define PT_REPLAY_HITS 6   // recorded replay hits before a query hands over to the exact DFS

struct ReplayCfg {
    uint32_t as;    // aux stack words
    uint32_t cap;   // candidate list words per pass
};

// conservative ray/box test on an inflated auxiliary box (o*inv precomputed)
PT_HD bool aux_box(float lx, float ly, float lz, float hx, float hy, float hz, f3 inv, f3 oinv) {
    const float ax = fmaf(lx, inv.x, -oinv.x), bx = fmaf(hx, inv.x, -oinv.x);
    const float ay = fmaf(ly, inv.y, -oinv.y), by = fmaf(hy, inv.y, -oinv.y);
    const float az = fmaf(lz, inv.z, -oinv.z), bz = fmaf(hz, inv.z, -oinv.z);
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    return tn <= tf && tf >= 0.f;
}

// exact reference slab test of node `n` (AABB_t::Intersect, src/bvh.cpp:89-93)
PT_HD bool node_slab(const Node& nd, const Ray& ray, float& t, uint32_t& interior) {
    const f3 c = mk3(nd.a.x, nd.a.y, nd.a.z);
    const f3 s = mk3(nd.a.w, nd.b.x, nd.b.y);
    return slab(ray.o + -1.f * c, ray.d, s, t, interior);
}

// Filtered exact node test.  Decides exactly what node_slab + the reference's
// prune rule decide -- hit iff !(t1 > t2) && !(t2 < 0); pruned iff
// bound < t1 && !(t1 < 0) -- but evaluates the six quotients (+-s - o)/d as
// (+-s - o) * rinv with rinv = 1/d (IEEE, once per ray) instead of six IEEE
// divisions.  Both quotient forms are within 1.5 ulp of the real quotient
// (rinv rel. error <= 2^-24, product rounding <= 2^-24; the IEEE quotient
// <= 2^-24), min/max selection is monotone in both, so every compared value
// is within E = |v| 2^-20 + 1e-30 of its exact counterpart.  A decision whose
// operands are closer than that margin is re-done with the exact division
// (slab()).  Requires replay_ok_ray(ray) (finite, non-tiny d: |rinv| < 1e30).
// Returns true iff the node is entered (hit and not pruned).
// exact = true: always the IEEE-division form (rays with near-zero direction components).
// approximate slab interval of a (center, half-size) box: the reference's
// numerators (same IEEE ops) times the per-ray reciprocal
PT_HD void slab_approx(F4 a, F4 b, const Ray& ray, f3 rinv, float& t1, float& t2) {
    const f3 c = mk3(a.x, a.y, a.z);
    const f3 s = mk3(a.w, b.x, b.y);
    const f3 o = ray.o + -1.f * c;                 // src/bvh.cpp:92 (same IEEE adds)
    const f3 nlo = -1.f * s - o, nhi = s - o;      // src/primitives.cpp:71-72 numerators
    const float ax = nlo.x * rinv.x, bx = nhi.x * rinv.x;
    const float ay = nlo.y * rinv.y, by = nhi.y * rinv.y;
    const float az = nlo.z * rinv.z, bz = nhi.z * rinv.z;
    t1 = smax(smax(smin(ax, bx), smin(ay, by)), smin(az, bz));
    t2 = smin(smin(smax(ax, bx), smax(ay, by)), smax(az, bz));
}

// node_enter's decision from the approximate interval: 0 = not entered,
// 1 = entered, 2 = too close to call (redo with the exact division)
// (evaluated as a chain of selects, last test first: no branches)
PT_HD uint32_t enter_decide(float t1, float t2, float bound) {
    const float e1 = fabsf(t1) * 0x1p-20f + 1e-30f, e2 = fabsf(t2) * 0x1p-20f + 1e-30f;
    const float d12 = t1 - t2;
    const float eb = 2.f * e1 + fabsf(bound) * 0x1p-22f;
    uint32_t v = bound < t1 ? 0u : 1u;
    v = fabsf(bound - t1) > eb ? v : 2u;
    v = t1 < 0.f ? 1u : v;                                      // interior: never pruned
    v = fabsf(t1) > e1 ? v : 2u;
    v = t2 < 0.f ? 0u : v;                                      // box behind the ray
    v = fabsf(t2) > e2 ? v : 2u;
    v = d12 > 0.f ? 0u : v;                                     // t1 > t2: miss
    v = (e1 < 1e20f && e2 < 1e20f) && fabsf(d12) > 2.f * (e1 + e2) ? v : 2u;
    return v;
}

// the exact decision (IEEE division, the reference's slab)
PT_HD bool enter_exact(F4 a, F4 b, const Ray& ray, float bound) {
    const f3 c = mk3(a.x, a.y, a.z);
    const f3 s = mk3(a.w, b.x, b.y);
    float t;
    uint32_t in;
    if (!slab(ray.o + -1.f * c, ray.d, s, t, in)) return false;
    return !(bound < t && !in);
}

PT_HD bool node_enter(const Node& nd, const Ray& ray, f3 rinv, float bound, bool exact = false) {
    float t1, t2;
    slab_approx(nd.a, nd.b, ray, rinv, t1, t2);
    const uint32_t v = exact ? 2u : enter_decide(t1, t2, bound);
    if (v == 2u) return enter_exact(nd.a, nd.b, ray, bound);
    return v == 1u;
}

// conservative inflated-box test for rays with near-zero direction components
// (|d_k| <= 1e-30): such an axis bounds no t, the origin must lie in the slab;
// other axes as aux_box.  Covers every box the exact (inf/NaN) slab test can
// enter: with o_k outside the slab by more than the inflation margin the exact
// quotients are both huge of one sign (t beyond any bound, or exit < 0).
PT_HD bool aux_box_par(float lx, float ly, float lz, float hx, float hy, float hz, const Ray& r, f3 inv, f3 oinv) {
    const float lo[3] = {lx, ly, lz}, hi[3] = {hx, hy, hz};
    const float o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    const float iv[3] = {inv.x, inv.y, inv.z}, oi[3] = {oinv.x, oinv.y, oinv.z};
    float tn = -INFINITY, tf = INFINITY;
    bool inside = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (!(fabsf(d[k]) > 1e-30f)) {
            inside = inside && lo[k] <= o[k] && o[k] <= hi[k];
        } else {
            const float a = fmaf(lo[k], iv[k], -oi[k]), b = fmaf(hi[k], iv[k], -oi[k]);
            tn = fmaxf(tn, fminf(a, b));
            tf = fminf(tf, fmaxf(a, b));
        }
    }
    return inside && tn <= tf && tf >= 0.f;
}

PT_HD bool replay_ok_ray(const Ray& r) {
    // rays with a (near-)zero or non-finite direction component, or a non-finite
    // origin, take the exact stack DFS (NaN/inf slab semantics)
    const float m = 1e-30f, big = 3e38f;
    return fabsf(r.d.x) > m && fabsf(r.d.y) > m && fabsf(r.d.z) > m && fabsf(r.d.x) < big &&
           fabsf(r.d.y) < big && fabsf(r.d.z) < big && fabsf(r.o.x) < big && fabsf(r.o.y) < big &&
           fabsf(r.o.z) < big;
}

// returns best hit id (-1 none); sets `fallback` when the exact DFS must be used instead.
// FAST: filtered node tests (node_enter) and one flat replay loop over all
// (candidate, ancestor) steps; otherwise the IEEE-division reference form.
template <bool FAST, class Mem>
PT_HD int bvh_replay(const SceneView& S, const ReplayCfg& cfg, const Ray& ray, float P, Mem& L, Hit& best,
                     Counts& C, bool& fallback) {
    fallback = false;
    int best_id = -1;
    best.t = PT_INF;
    const f3 inv = mk3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
    const f3 oinv = mk3(ray.o.x * inv.x, ray.o.y * inv.y, ray.o.z * inv.z);
    uint32_t h_idx[PT_REPLAY_HITS];
    float h_t[PT_REPLAY_HITS];
    uint32_t nh = 0;
    uint32_t lb = 0;  // every candidate below lb has been processed
    for (;;) {
        // ---- pass: collect the `cap` smallest candidate leaves >= lb (unsorted), track overflow
        uint32_t n = 0, mx = 0, mxpos = 0;
        bool overflow = false;
        uint32_t sp = 0;
        uint32_t node = 0;
        for (;;) {
            const AuxNode an = S.aux[node];
            C.aux++;
            const uint32_t c0 = f2u(an.d.x), c1 = f2u(an.d.y);
            const bool h0 = c0 != 0xffffffffu && aux_box(an.a.x, an.a.y, an.a.z, an.a.w, an.b.x, an.b.y, inv, oinv);
            const bool h1 = c1 != 0xffffffffu && aux_box(an.b.z, an.b.w, an.c.x, an.c.y, an.c.z, an.c.w, inv, oinv);
            uint32_t next = 0xffffffffu;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const bool hk = k == 0 ? h0 : h1;
                const uint32_t code = k == 0 ? c0 : c1;
                if (!hk) continue;
                if (code & 0x80000000u) {
                    const uint32_t leaf = code & 0x7fffffffu;
                    if (leaf < lb) continue;
                    C.nodes++;
                    if (FAST) {
                        if (!node_enter(S.nodes[leaf], ray, inv, PT_INF)) continue;
                    } else {
                        float t;
                        uint32_t in;
                        if (!node_slab(S.nodes[leaf], ray, t, in)) continue;
                    }
                    if (n < cfg.cap) {
                        L.set(cfg.as + n, leaf);
                        if (leaf > mx || n == 0) { mx = leaf; mxpos = n; }
                        ++n;
                    } else {
                        overflow = true;
                        if (leaf < mx) {   // keep the cap smallest: replace the largest
                            L.set(cfg.as + mxpos, leaf);
                            mx = 0;
                            for (uint32_t q = 0; q < n; ++q) {
                                const uint32_t v = L.get(cfg.as + q);
                                if (v >= mx) { mx = v; mxpos = q; }
                            }
                        }
                    }
                } else if (next == 0xffffffffu) {
                    next = code;
                } else {
                    L.set(sp++, code);
                }
            }
            if (next != 0xffffffffu) { node = next; continue; }
            if (sp == 0u) break;
            node = L.get(--sp);
        }
        if (n == 0u) break;
        // ---- sort the candidates (insertion sort, ascending preorder index)
        for (uint32_t i = 1; i < n; ++i) {
            const uint32_t v = L.get(cfg.as + i);
            uint32_t j = i;
            while (j > 0u) {
                const uint32_t u = L.get(cfg.as + j - 1u);
                if (u <= v) break;
                L.set(cfg.as + j, u);
                --j;
            }
            L.set(cfg.as + j, v);
        }
        // ---- replay root -> candidate paths in preorder
        uint32_t skip = lb;
        if (FAST) {
            // one flat loop: each iteration tests one node of the current candidate's root path
            uint32_t k = 0, cand = 0;
            while (k < n && (cand = L.get(cfg.as + k)) < skip) ++k;
            uint32_t a = 0;
            float bound = P;
            while (k < n) {
                const Node nd = S.nodes[a];
                C.nodes++;
                const uint32_t ref = f2u(nd.b.z), info = f2u(nd.b.w);
                bool next_cand = false;
                if (!node_enter(nd, ray, inv, bound)) {
                    skip = (info & PT_NODE_INTERIOR) ? (info & 0x7fffffffu) : a + 1u;
                    next_cand = true;
                } else if (a == cand) {
                    // leaf reached: first-min over its primitives (src/bvh.cpp:205-213)
                    Hit lbh;
                    lbh.t = PT_INF;
                    int lid = -1;
                    for (uint32_t i = ref; i < ref + info; ++i) {
                        Hit h;
                        C.ptests++;
                        if (prim_intersect(S.prims[i], ray, h) && h.t < lbh.t) { lbh = h; lid = (int)i; }
                    }
                    if (lid >= 0) {
                        if (nh == PT_REPLAY_HITS) { fallback = true; return -1; }
#pragma unroll
                        for (int q = 0; q < PT_REPLAY_HITS; ++q)
                            if ((uint32_t)q == nh) { h_idx[q] = cand; h_t[q] = lbh.t; }
                        ++nh;
                        if (lbh.t < best.t) { best = lbh; best_id = lid; }
                    }
                    skip = cand + 1u;
                    next_cand = true;
                } else if (cand < ref) {
                    a = a + 1u;                      // left child: same bound
                } else {
                    // right child: bound = best hit of the left sibling's subtree, if any
                    float m = bound;
                    bool any = false;
#pragma unroll
                    for (int q = 0; q < PT_REPLAY_HITS; ++q) {
                        if ((uint32_t)q < nh && h_idx[q] > a && h_idx[q] < ref) {
                            if (!any || h_t[q] < m) m = h_t[q];
                            any = true;
                        }
                    }
                    bound = m;
                    a = ref;
                }
                if (next_cand) {
                    ++k;
                    while (k < n && (cand = L.get(cfg.as + k)) < skip) ++k;
                    a = 0;
                    bound = P;
                }
            }
        } else {
            for (uint32_t k = 0; k < n; ++k) {
                const uint32_t cand = L.get(cfg.as + k);
                if (cand < skip) continue;
                uint32_t a = 0;
                float bound = P;
                for (;;) {
                    const Node nd = S.nodes[a];
                    C.nodes++;
                    float t;
                    uint32_t in;
                    const bool hit = node_slab(nd, ray, t, in);
                    const uint32_t ref = f2u(nd.b.z), info = f2u(nd.b.w);
                    if (!hit || (bound < t && !in)) {
                        skip = (info & PT_NODE_INTERIOR) ? (info & 0x7fffffffu) : a + 1u;
                        break;
                    }
                    if (a == cand) {
                        // leaf reached: first-min over its primitives (src/bvh.cpp:205-213)
                        Hit lbh;
                        lbh.t = PT_INF;
                        int lid = -1;
                        for (uint32_t i = ref; i < ref + info; ++i) {
                            Hit h;
                            C.ptests++;
                            if (prim_intersect(S.prims[i], ray, h) && h.t < lbh.t) { lbh = h; lid = (int)i; }
                        }
                        if (lid >= 0) {
                            if (nh == PT_REPLAY_HITS) { fallback = true; return -1; }
#pragma unroll
                            for (int q = 0; q < PT_REPLAY_HITS; ++q)
                                if ((uint32_t)q == nh) { h_idx[q] = cand; h_t[q] = lbh.t; }
                            ++nh;
                            if (lbh.t < best.t) { best = lbh; best_id = lid; }
                        }
                        skip = cand + 1u;
                        break;
                    }
                    if (cand < ref) {
                        a = a + 1u;                      // left child: same bound
                    } else {
                        // right child: bound = best hit of the left sibling's subtree, if any
                        float m = bound;
                        bool any = false;
#pragma unroll
                        for (int q = 0; q < PT_REPLAY_HITS; ++q) {
                            if ((uint32_t)q < nh && h_idx[q] > a && h_idx[q] < ref) {
                                if (!any || h_t[q] < m) m = h_t[q];
                                any = true;
                            }
                        }
                        bound = m;
                        a = ref;
                    }
                }
            }
        }
        if (!overflow) break;
        const uint32_t last = L.get(cfg.as + n - 1u) + 1u;
        lb = skip > last ? skip : last;
    }
    return best_id;
}

// src/scene.cpp:46-77: planes first (strict <), then the BVH bounded by the plane t
template <bool FAST, class Stack>
PT_HD int ray_intersection(const SceneView& S, const ReplayCfg& cfg, const Ray& ray, Stack& stk, Hit& out,
                           Counts& C) {
    int id = -1;
    float closest = PT_INF;
    for (uint32_t k = 0; k < S.n_planes; ++k) {
        const uint32_t pi = S.planes[k];
        Hit h;
        C.planes++;
        if (prim_intersect(S.prims[pi], ray, h) && h.t < closest) { closest = h.t; out = h; id = (int)pi; }
    }
    Hit bh;
    int bid;
    bool fallback = true;
    if (S.aux && replay_ok_ray(ray)) bid = bvh_replay<FAST>(S, cfg, ray, closest, stk, bh, C, fallback);
    if (fallback) {
        if (S.aux) C.fallbacks++;
        bid = bvh_exact(S, ray, closest, stk, bh, C);
    }
    if (bid != -1 && bh.t < closest) { out = bh; id = bid; }
    return id;
}

// per-vertex fold record modes
enum : uint32_t { V_TERM = 0u, V_DIFFUSE = 1u, V_COL = 2u, V_IDENT = 3u };

// One path vertex of RayTrace (src/scene.cpp:91-177) after a closest hit:
// consumes the vertex's random numbers, returns its fold record
// (idm = prim id | mode << 30, factors s1, s2) and whether the path continues
// with `ray` set to the child ray.  Shared by the megakernel integrator and
// the wavefront shade kernel.
// `em` = the emitter records (EmitGlobal or a copy), `sh` = the prim's shading record.
template <class EM>
PT_HD bool shade_vertex_e(const SceneView& S, const EM& em, const Shade& sh, Rng& R, Ray& ray, const Hit& h, int id,
                          uint32_t& idm, float& s1, float& s2) {
    const float eps = 1e-4f;  // Scene::eps, include/scene.h:56
    const uint32_t mat = f2u(sh.s1.w);
    const f3 p = ray.o + h.t * ray.d;
    const f3 n = h.n;
    if (mat == M_DIFFUSE) {
        const f3 p_outer = p + eps * n;
        const f3 dir = sample_mix_e(S, em, R, p_outer, n);
        const float cosv = dot(dir, n);
        if (cosv <= 0.f) { idm = (uint32_t)id | (V_TERM << 30); s1 = s2 = 0.f; return false; }
        const float pw = pdf_mix_e(S, em, p_outer, n, dir);
        idm = (uint32_t)id | (V_DIFFUSE << 30);
        s1 = cosv;
        s2 = 1.f / pw;
        ray.o = p + eps * dir;
        ray.d = dir;
        return true;
    }
    if (mat == M_METALLIC) {
        const f3 rd = reflect(n, normalize(ray.d));
        idm = (uint32_t)id | (V_COL << 30);
        s1 = s2 = 1.f;
        ray.o = p + eps * rd;
        ray.d = rd;
        return true;
    }
    if (mat == M_DIELECTRIC) {
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
        s1 = s2 = 1.f;
        if (refl) {
            const f3 rd = reflect(n, normalize(ray.d));
            idm = (uint32_t)id | (V_IDENT << 30);
            ray.o = p + eps * rd;
            ray.d = rd;
        } else {
            const float cos2 = (float)sqrt((double)(1.f - sin2 * sin2));
            const float k = eta1 / eta2;
            const f3 rd = k * (-1.f * dir) + (k * cosn - cos2) * n;
            idm = (uint32_t)id | ((h.interior ? V_IDENT : V_COL) << 30);
            ray.o = p + eps * rd;
            ray.d = rd;
        }
        return true;
    }
    idm = (uint32_t)id | (V_TERM << 30);   // unknown material: other = 0
    s1 = s2 = 0.f;
    return false;
}
PT_HD bool shade_vertex(const SceneView& S, Rng& R, Ray& ray, const Hit& h, int id, uint32_t& idm, float& s1,
                        float& s2) {
    return shade_vertex_e(S, EmitGlobal{S}, S.shade[id], R, ray, h, id, idm, s1, s2);
}

// backward fold of one vertex record with its shading record: L = E_k + ((A_k * L) * s1_k) * s2_k
PT_HD f3 fold_vertex_sh(const Shade& sh, f3 L, uint32_t idm, float s1, float s2) {
    const uint32_t mode = idm >> 30;
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
    return E + other;
}
PT_HD f3 fold_vertex(const SceneView& S, f3 L, uint32_t idm, float s1, float s2) {
    return fold_vertex_sh(S.shade[idm & 0x3fffffffu], L, idm, s1, s2);
}

// One camera sample: src/scene.cpp:189-203 (inner) + RayTrace :83-178.
// `vs` provides put(k, idmode, s1, s2) / get(k, idmode, s1, s2) for k < depth.
// `isect(ray, hit, counts)` is the closest-hit query (Scene::RayIntersection).
template <class Isect, class VStore>
PT_HD f3 trace_path_with(const SceneView& S, Isect&& isect, Ray ray, uint32_t depth, Rng& R, VStore& vs, Counts& C) {
    uint32_t nv = 0;
    f3 leaf = mk3(0.f, 0.f, 0.f);
    for (uint32_t rem = depth;; --rem) {
        if (rem == 0u) { leaf = mk3(0.f, 0.f, 0.f); break; }
        C.rays++;
        Hit h;
        const int id = isect(ray, h, C);
        if (id == -1) { leaf = S.bg; break; }
        uint32_t idm;
        float s1, s2;
        const bool cont = shade_vertex(S, R, ray, h, id, idm, s1, s2);
        vs.put(nv++, idm, s1, s2);
        if (!cont) break;
    }
    // backward fold, deepest vertex first
    f3 L = leaf;
    while (nv > 0u) {
        --nv;
        uint32_t idm;
        float s1, s2;
        vs.get(nv, idm, s1, s2);
        L = fold_vertex(S, L, idm, s1, s2);
    }
    return L;
}

template <bool FAST, class Stack, class VStore>
PT_HD f3 trace_path(const SceneView& S, const ReplayCfg& cfg, Ray ray, uint32_t depth, Rng& R, Stack& stk, VStore& vs,
                    Counts& C) {
    return trace_path_with(
        S, [&](const Ray& r, Hit& h, Counts& c) { return ray_intersection<FAST>(S, cfg, r, stk, h, c); }, ray, depth, R,
        vs, C);
}

}  // namespace pt
