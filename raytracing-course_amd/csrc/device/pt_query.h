// pt_query.h -- the closest-hit query of the wavefront renderer as a per-lane
// state machine (Scene::RayIntersection, src/scene.cpp:46-77, with the
// reference BVH semantics of src/bvh.cpp:181-225 reproduced by candidate
// replay; see pt_trace.h for the replay argument).
//
// Built for a persistent, refilling intersection kernel: every call of
// q_step() advances ONE lane by one node visit, so lanes whose rays need many
// visits (the candidate tail: p99 ~25 leaves) no longer hold the other 63
// lanes of their wave -- an idle lane simply takes the next ray.
//
//   * auxiliary BVH: stackless BVH2 in DFS preorder with skip links
//     (AuxSL, 32 B): internal = conservative inflated box; leaf = the
//     reference leaf's own exact (center, half-size), tested with the filtered
//     exact test node_enter() -- one dependent load per visit, no stack.
//   * candidates: the PT_QK smallest reference-leaf indices of the pass, kept
//     sorted in registers by a min/max insertion network (no LDS, no dynamic
//     register indexing); more than PT_QK -> further passes above the last
//     processed index (rare).
//   * replay: one reference node per step, root -> candidate, with the
//     reference's pruning and right-child bounds.
// Rays the replay cannot take (non-finite or near-zero direction
// components) or whose replay hit list overflows are flagged for the exact
// stack DFS (bvh_exact) in a separate pass.
#pragma once
#include "pt_trace.h"

namespace pt {

#ifndef PT_QK
#define PT_QK 16
#endif
#ifndef PT_AUXW
#define PT_AUXW 4               // auxiliary BVH width (nodes = PT_AUXW AuxSL entries)
#endif

// stackless auxiliary node (32 B):
//   internal: a = {lo.x, lo.y, lo.z, hi.x}, b = {hi.y, hi.z, u32 skip, 0xffffffff}
//   leaf:     a = {c.x, c.y, c.z, s.x},     b = {s.y, s.z, u32 skip (= own index + 1), u32 reference leaf}
// (c, s) of a leaf are bit-identical copies of the reference node's record.
struct AuxSL { F4 a, b; };
#define PT_AUX_INTERNAL 0xffffffffu

enum : uint32_t { Q_AUX = 0u, Q_REPLAY = 1u, Q_DONE = 2u, Q_EXACT = 3u };
// replay step kinds: each issues one round of independent loads
enum : uint32_t { R_CAND = 0u, R_LEAF = 1u, R_WALK_E = 2u, R_WALK_N = 3u };

struct QHits {                  // replay hit list (reference leaf index, leaf first-min t)
    uint32_t idx[PT_REPLAY_HITS];
    float t[PT_REPLAY_HITS];
};

struct Query {
    Ray ray;
    f3 inv;                     // 1/d (IEEE, once per ray)
    float P;                    // closest plane t (the BVH bound at the root)
    // small state packed into one register
    uint32_t phase : 2;         // Q_*
    uint32_t walk : 2;          // Q_REPLAY step kind: R_CAND, R_LEAF, R_WALK_E, R_WALK_N
    uint32_t par : 1;           // near-zero direction component: exact node tests, robust aux boxes
    uint32_t robust : 1;        // leaf check: the ray crosses the leaf box robustly (t1c, mc valid)
    uint32_t known : 1;         // walk: the segment bound is known (below the LCA with the last hit)
    uint32_t overflow : 1;      // aux pass dropped candidates above the kept PT_QK
    uint32_t nh : 3;            // recorded replay hits (<= PT_REPLAY_HITS)
    uint32_t sp : 7;            // Q_AUX: pending aux nodes on the per-lane stack
    uint32_t pos : 7;           // walk: position reached in the ancestor list
    uint32_t len : 7;           // walk: ancestor list length
    uint32_t node;              // Q_AUX: aux node
    uint32_t lb;                // every candidate below lb has been processed
    uint32_t cand, skip, last;
    float bound;
    float dl;                   // certification margin (t units, see q_leaf_certain)
    uint32_t lref, lcnt;        // the candidate leaf's primitive range
    uint32_t off;               // walk: ancestor list offset
    uint32_t e[4];              // walk: the entries under test (0xffffffff = none)
    uint32_t astar;             // walk: deepest ancestor at or above that LCA seen so far
    float t1c, mc;              // leaf check: approximate entry and certification margin
    uint32_t c[PT_QK];          // sorted candidates of this pass (0xffffffff = empty)
    QHits H;
    float bt;                   // best BVH leaf hit so far (first strict minimum)
    float res_t;                // result so far (plane, then BVH hits that beat it): t and prim;
    int res_id;                 // the normal is recomputed from the prim by the consumer
};
static_assert(PT_REPLAY_HITS < 8, "nh is a 3-bit field");

struct QCounts {
    uint32_t nodes, aux, ptests, planes;
#ifdef PT_QDIAG
    uint32_t cands, passes, steps;
#endif
};

// planes (src/scene.cpp:50-57), then the BVH set-up
PT_HD void q_init(const SceneView& S, const Ray& ray, Query& q, QCounts& C) {
    q.ray = ray;
    q.res_id = -1;
    q.res_t = PT_INF;
    float closest = PT_INF;
    for (uint32_t k = 0; k < S.n_planes; ++k) {
        const uint32_t pi = S.planes[k];
        Hit h;
        C.planes++;
        if (plane_intersect(S.prims[pi], ray, h) && h.t < closest) { closest = h.t; q.res_t = h.t; q.res_id = (int)pi; }
    }
    q.P = closest;
    q.bt = PT_INF;
    q.nh = 0;
    q.lb = 0;
    q.overflow = 0;
    q.node = 0;
    q.sp = 0;
#pragma unroll
    for (int i = 0; i < PT_QK; ++i) q.c[i] = 0xffffffffu;
    // non-finite rays: exact stack DFS (their NaN/inf slab semantics are not replayed)
    const float big = 3e38f;
    if (!(fabsf(ray.o.x) < big && fabsf(ray.o.y) < big && fabsf(ray.o.z) < big && fabsf(ray.d.x) < big &&
          fabsf(ray.d.y) < big && fabsf(ray.d.z) < big)) {
        q.phase = Q_EXACT;
        return;
    }
    q.par = replay_ok_ray(ray) ? 0u : 1u;
    q.inv = mk3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
    const float om = fmaxf(fmaxf(fabsf(ray.o.x), fabsf(ray.o.y)), fabsf(ray.o.z));
    const float dm = fminf(fminf(fabsf(ray.d.x), fabsf(ray.d.y)), fabsf(ray.d.z));
    q.dl = q.par ? INFINITY : 0x1p-18f * (S.box_extent + om) / dm;
    q.phase = Q_AUX;
}

PT_HD void q_insert(Query& q, uint32_t v) {
#pragma unroll
    for (int i = 0; i < PT_QK; ++i) {
        const uint32_t lo = q.c[i] < v ? q.c[i] : v;
        v = q.c[i] < v ? v : q.c[i];
        q.c[i] = lo;
    }
    if (v != 0xffffffffu) q.overflow = 1u;   // a candidate above the kept PT_QK was dropped
}

PT_HD uint32_t q_pop(Query& q) {
    const uint32_t v = q.c[0];
#pragma unroll
    for (int i = 0; i + 1 < PT_QK; ++i) q.c[i] = q.c[i + 1];
    q.c[PT_QK - 1] = 0xffffffffu;
    return v;
}

// next candidate >= skip, or end of pass (-> next pass / done)
PT_HD void q_next_candidate(Query& q) {
    for (;;) {
        const uint32_t v = q_pop(q);
        if (v == 0xffffffffu) break;
        q.last = v;
        if (v >= q.skip) {
            q.cand = v;
            q.walk = R_CAND;
            q.phase = Q_REPLAY;
            return;
        }
    }
    if (q.overflow) {
        // candidates above the last processed one were dropped: another aux pass
        q.lb = q.skip > q.last + 1u ? q.skip : q.last + 1u;
        q.overflow = 0;
        q.node = 0;
        q.sp = 0;
        q.phase = Q_AUX;
        return;
    }
    q.phase = Q_DONE;
}

// leaf reached: first-min over its primitives (src/bvh.cpp:205-213), hit bookkeeping
// returns false when the replay hit list is full (the ray then takes the exact DFS)
PT_HD bool q_leaf_hit(const SceneView& S, Query& q, uint32_t a, uint32_t ref, uint32_t cnt, QCounts& C) {
    Hit lbh;
    lbh.t = PT_INF;
    int lid = -1;
    for (uint32_t i = ref; i < ref + cnt; ++i) {
        Hit h;
        C.ptests++;
        if (bvh_prim_intersect(S.prims[i], q.ray, h) && h.t < lbh.t) { lbh = h; lid = (int)i; }
    }
    if (lid >= 0) {
        if (q.nh == PT_REPLAY_HITS) return false;
#pragma unroll
        for (int k = 0; k < PT_REPLAY_HITS; ++k)
            if ((uint32_t)k == q.nh) { q.H.idx[k] = a; q.H.t[k] = lbh.t; }
        ++q.nh;
        // BVH result = first strict minimum; it replaces the plane hit iff strictly closer
        if (lbh.t < q.bt) {
            q.bt = lbh.t;
            if (lbh.t < q.P) { q.res_t = lbh.t; q.res_id = lid; }
        }
    }
    return true;
}

// min of the recorded hits strictly inside (a, r) (the left subtree of a when
// r is a's right child); at least one exists when called with a = a*
PT_HD float q_bound_between(const Query& q, uint32_t a, uint32_t r) {
    float m = q.P;
    bool any = false;
#pragma unroll
    for (int k = 0; k < PT_REPLAY_HITS; ++k) {
        if ((uint32_t)k < q.nh && q.H.idx[k] > a && q.H.idx[k] < r) {
            if (!any || q.H.t[k] < m) m = q.H.t[k];
            any = true;
        }
    }
    return m;
}

// Candidate leaf check before any root-path replay.  Every bound the replay
// can carry is P or a minimum over earlier hits, so it lies in [lo, hi] =
// [min, max](P, recorded hits).
//  * certain accept: the ray crosses the leaf box robustly (slab interval
//    longer than 2 margins, exit beyond the margin) and lo >= entry + margin.
//    Every ancestor's box contains the leaf's (the reference builds them as
//    exact min/max unions); their stored (center, half-size) records and the
//    float slab evaluation move interval ends by at most the margin
//    dl = 2^-18 (X + |o|max) / |d|min + 2^-18 |t| (X = scene box extent;
//    rounding of c/s <= 2^-23 X each, of o and the numerators <= 2^-24 each,
//    quotients 2^-24 relative, the multiply-by-reciprocal form 2^-20; >= 4x
//    headroom).  So every ancestor is hit with entry <= leaf entry + margin
//    <= its bound (or is interior): no ancestor prunes and the leaf is entered.
//  * certain reject: the leaf's own exact test fails even against hi (its
//    actual bound is <= hi): it is not entered whatever its ancestors do.
// Returns 1 = accept, 0 = reject, 2 = undecided (replay the root path).
PT_HD uint32_t q_leaf_certain(Query& q, const Node& nd) {
    float lo = q.P, hi = q.P;
#pragma unroll
    for (int k = 0; k < PT_REPLAY_HITS; ++k)
        if ((uint32_t)k < q.nh) { lo = fminf(lo, q.H.t[k]); hi = fmaxf(hi, q.H.t[k]); }
    const f3 c = mk3(nd.a.x, nd.a.y, nd.a.z);
    const f3 s = mk3(nd.a.w, nd.b.x, nd.b.y);
    const f3 o = q.ray.o + -1.f * c;
    const f3 nlo = -1.f * s - o, nhi = s - o;
    const float ax = nlo.x * q.inv.x, bx = nhi.x * q.inv.x;
    const float ay = nlo.y * q.inv.y, by = nhi.y * q.inv.y;
    const float az = nlo.z * q.inv.z, bz = nhi.z * q.inv.z;
    const float t1 = smax(smax(smin(ax, bx), smin(ay, by)), smin(az, bz));
    const float t2 = smin(smin(smax(ax, bx), smax(ay, by)), smax(az, bz));
    const float m = q.dl + (fabsf(t1) + fabsf(t2)) * 0x1p-18f;
    q.t1c = t1;
    q.mc = m;
    q.robust = (!q.par && t1 + m <= t2 - m && t2 - m >= 0.f) ? 1u : 0u;
    if (q.robust && lo >= t1 + m) return 1u;
    if (!node_enter(nd, q.ray, q.inv, hi, q.par != 0u)) return 0u;
    return 2u;
}

// Advance one node visit.  Precondition: phase is Q_AUX or Q_REPLAY.
// `stk` = per-lane word memory for the pending aux nodes (set/get).
template <class Mem>
PT_HD void q_step(const SceneView& S, const AuxSL* aux, uint32_t n_aux, Query& q, QCounts& C, Mem& stk) {
#ifdef PT_QDIAG
    C.steps++;
#endif
    if (q.phase == Q_AUX) {
        // one wide node: PT_AUXW child entries (independent loads)
        AuxSL e[PT_AUXW];
#pragma unroll
        for (int k = 0; k < PT_AUXW; ++k) e[k] = aux[q.node * PT_AUXW + k];
        C.aux++;
        const f3 oinv = mk3(q.ray.o.x * q.inv.x, q.ray.o.y * q.inv.y, q.ray.o.z * q.inv.z);
        uint32_t next = 0xffffffffu;
#pragma unroll
        for (int k = 0; k < PT_AUXW; ++k) {
            const uint32_t code = f2u(e[k].b.w);
            if (code == 0xffffffffu) continue;
            if (code & 0x80000000u) {
                const uint32_t leaf = code & 0x7fffffffu;
                if (leaf < q.lb) continue;
                Node nd;
                nd.a = e[k].a;
                nd.b = e[k].b;
                if (node_enter(nd, q.ray, q.inv, PT_INF, q.par != 0u)) {
#ifdef PT_QDIAG
                    C.cands++;
#endif
                    q_insert(q, leaf);
                }
            } else if (q.par ? aux_box_par(e[k].a.x, e[k].a.y, e[k].a.z, e[k].a.w, e[k].b.x, e[k].b.y, q.ray, q.inv,
                                           oinv)
                             : aux_box(e[k].a.x, e[k].a.y, e[k].a.z, e[k].a.w, e[k].b.x, e[k].b.y, q.inv, oinv)) {
                if (next == 0xffffffffu) next = code;
                else stk.set(q.sp++, code);
            }
        }
        if (next == 0xffffffffu && q.sp > 0u) next = stk.get(--q.sp);
        if (next != 0xffffffffu) {
            q.node = next;
            return;
        }
#ifdef PT_QDIAG
        C.passes++;
#endif
        // aux pass complete: replay the candidates in reference preorder
        q.skip = q.lb;
        q_next_candidate(q);
        return;
    }
    // Q_REPLAY.  One round of independent loads per step (the wave waits for
    // its slowest lane's chain, so no step may chain two memory round trips).
    bool reject = false;
    if (q.walk == R_CAND) {
        // the candidate's own leaf record (+ where its ancestor list is)
        const Node nd = S.nodes[q.cand];
        const uint32_t info = S.anc_info[q.cand];
        C.nodes++;
        q.lref = f2u(nd.b.z);
        q.lcnt = f2u(nd.b.w);
        const uint32_t v = q_leaf_certain(q, nd);
        if (v == 1u) {
            q.walk = R_LEAF;
            return;
        }
        if (v == 0u) {
            reject = true;
        } else {
            // undecided: test the root path below a* = LCA(last recorded hit, cand).
            // Ancestors at or above a* were entered on that hit's path (same
            // node, same bound: both depend only on earlier hits) -- they are the
            // list entries <= the hit.  Below a* no left subtree holds a hit, so
            // the bound is constant: B = min{hits in (a*, right child of a*)}.
            // Each remaining ancestor, then the leaf itself (entry len), is
            // tested with B.
            q.off = info & 0x03ffffffu;
            q.len = info >> 26;
            q.pos = 0u;
            q.known = q.nh == 0u ? 1u : 0u;   // no earlier hit: the bound is P on the whole path
            q.bound = q.P;
            q.astar = 0u;
            q.walk = R_WALK_E;
            return;
        }
    } else if (q.walk == R_LEAF) {
        // leaf entered: its primitives (src/bvh.cpp:205-213)
        if (!q_leaf_hit(S, q, q.cand, q.lref, q.lcnt, C)) {
            q.phase = Q_EXACT;
            return;
        }
    } else if (q.walk == R_WALK_E) {
        // next 4 path entries (position len is the leaf itself)
        uint32_t hlast = 0u;   // last recorded hit (unrolled select: no dynamic register indexing)
#pragma unroll
        for (int k = 0; k < PT_REPLAY_HITS; ++k)
            if ((uint32_t)k + 1u == q.nh) hlast = q.H.idx[k];
        bool any = false, accept = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t at = q.pos + (uint32_t)j;
            uint32_t e = at < q.len ? S.anc[q.off + at] : (at == q.len ? q.cand : 0xffffffffu);
            if (e != 0xffffffffu && !accept && !q.known) {
                if (e <= hlast) {
                    q.astar = e;          // entered on the last hit's path
                    e = 0xffffffffu;
                } else {
                    q.bound = q_bound_between(q, q.astar, e);
                    q.known = 1u;
                    if (q.robust && q.bound >= q.t1c + q.mc) accept = true;   // whole segment certain
                }
            }
            if (accept) e = 0xffffffffu;
            q.e[j] = e;
            any = any || e != 0xffffffffu;
        }
        if (accept) {
            q.walk = R_LEAF;
            return;
        }
        if (any) {
            q.walk = R_WALK_N;
        } else {
            q.pos += 4u;              // all at or above a*
        }
        return;
    } else {
        // R_WALK_N: the records of the pending entries, tested with B
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (q.e[j] == 0xffffffffu || reject) continue;
            C.nodes++;
            if (!node_enter(S.nodes[q.e[j]], q.ray, q.inv, q.bound, q.par != 0u)) reject = true;
        }
        if (!reject) {
            q.pos += 4u;
            q.walk = q.pos > q.len ? R_LEAF : R_WALK_E;   // past the leaf: entered
            return;
        }
    }
    (void)reject;
    q.skip = q.cand + 1u;
    q_next_candidate(q);
}

// exact stack DFS for the rays the replay leaves (planes again + bvh_exact:
// the replay may already have replaced the plane result)
template <class Stack>
PT_HD int q_exact(const SceneView& S, const Ray& ray, Stack& stk, Hit& out, QCounts& C) {
    SceneView E = S;
    E.aux = nullptr;
    Counts X{};
    const ReplayCfg cfg{0u, 0u};
    const int id = ray_intersection<false>(E, cfg, ray, stk, out, X);
    C.nodes += (uint32_t)X.nodes;
    C.ptests += (uint32_t)X.ptests;
    C.planes += (uint32_t)X.planes;
    return id;
}

// whole query on one thread (host tests / reference form of the state machine)
template <class Stack>
PT_HD int q_run(const SceneView& S, const AuxSL* aux, uint32_t n_aux, const Ray& ray, Stack& stk, Hit& out,
                QCounts& C, uint32_t& exact_used) {
    Query q;
    q_init(S, ray, q, C);
    while (q.phase == Q_AUX || q.phase == Q_REPLAY) q_step(S, aux, n_aux, q, C, stk);
    exact_used = q.phase == Q_EXACT ? 1u : 0u;
    if (exact_used) return q_exact(S, ray, stk, out, C);
    if (q.res_id >= 0) {
        // the consumer's form: the hit recomputed from its primitive (identical operations)
        const bool ok = prim_intersect(S.prims[q.res_id], ray, out);
        if (!ok || f2u(out.t) != f2u(q.res_t)) C.planes |= 0x80000000u;   // must never happen (tests check)
    }
    return q.res_id;
}

}  // namespace pt
