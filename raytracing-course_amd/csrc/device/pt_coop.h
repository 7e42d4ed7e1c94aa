// pt_coop.h -- the closest-hit query of the cooperative engine: ONE wave per
// ray, for the end of a pass, when a few thousand pixels' chains are all that
// is left and each chain's latency, not the chip's issue rate, sets the time.
//
// Semantics: Scene::RayIntersection (src/scene.cpp:46-77) with the reference
// recursion BVH_t::Intersect_ (src/bvh.cpp:185-225), as in pt_query.h, but
// reorganised so that almost every load of a query is independent of the
// others and can be issued by its own lane:
//
//  1. Enumerate every reference leaf whose (conservative, inflated) wide aux
//     box the ray crosses.  Order does not matter here, so the aux BVH is
//     expanded breadth-first, up to 64 nodes per round (one per lane).
//  2. Per candidate leaf, independent of any bound: its exact slab test
//     against no bound (a leaf whose box the ray misses is never entered,
//     src/bvh.cpp:188-192) and the first strict minimum over its primitives
//     (src/bvh.cpp:205-213: t < INF, first index on ties).
//  3. Only leaves with a primitive hit can change anything: an entered leaf
//     without one returns id -1, which changes neither the result nor the
//     bound its parent hands to the right child (src/bvh.cpp:216-223).  So the
//     hitting leaves are decided alone, in reference preorder (the recursion's
//     DFS order): a leaf is entered iff every node of its root path passes the
//     reference test, hit && !(bound < t && !interior), with the bound the
//     recursion carries there -- P at the root; at a right child the minimum
//     over the entered hits of its left sibling's subtree if there is one,
//     else the parent's bound (left child = parent + 1 in the preorder layout,
//     src/bvh.cpp:170-176).  The root path of every leaf is precomputed
//     (SceneView::anc_info / anc), so the whole path is one round of loads,
//     one node per lane.
//  4. The BVH result is the first strict minimum over the entered hits in
//     preorder; it replaces the plane hit iff strictly closer (scene.cpp:70-74).
//
// qc_run() is the same algorithm on one thread (host tests, PT_TUNE
// qengine=coop in the self-tests); qc_team() / qc_pool() in pt_wcoop.hip are the wave forms.
#pragma once
#include "pt_query.h"

namespace pt {

// exact slab hit test of a reference node record, no bound (a node with this
// false is never entered); filtered like node_enter: decided from the
// reciprocal-form interval when the margins allow, else by the IEEE division
// form (slab()).  exact = true: always the division form.
PT_HD bool qc_slab_hit(const Node& nd, const Ray& ray, f3 rinv, bool exact) {
    if (!exact) {
        float t1, t2;
        slab_approx(nd.a, nd.b, ray, rinv, t1, t2);
        const float e1 = fabsf(t1) * 0x1p-20f + 1e-30f, e2 = fabsf(t2) * 0x1p-20f + 1e-30f;
        const float d12 = t1 - t2;
        uint32_t v = 1u;
        v = t2 < 0.f ? 0u : v;                   // box behind the ray
        v = fabsf(t2) > e2 ? v : 2u;
        v = d12 > 0.f ? 0u : v;                  // t1 > t2: miss
        v = (e1 < 1e20f && e2 < 1e20f) && fabsf(d12) > 2.f * (e1 + e2) ? v : 2u;
        if (v != 2u) return v == 1u;
    }
    float t;
    uint32_t in;
    return node_slab(nd, ray, t, in);
}

// the bound the recursion carries at node v of a root path (v's parent `prev`,
// bound there `b`): a right child's bound is the minimum over the entered hits
// strictly inside (prev, v) -- its left sibling's subtree -- if there is one.
// `rec_idx/rec_t` = the entered hits so far, in preorder.
template <class Rec>
PT_HD float qc_child_bound(const Rec& rec, uint32_t nrec, uint32_t prev, uint32_t v, float b) {
    if (v == prev + 1u) return b;   // left child: the parent's bound
    float m = b;
    bool any = false;
    for (uint32_t r = 0; r < nrec; ++r) {
        const uint32_t i = rec.idx(r);
        if (i > prev && i < v) {
            const float t = rec.t(r);
            if (!any || t < m) m = t;
            any = true;
        }
    }
    return m;
}

// is hitting leaf c entered? (its whole root path passes with the carried bounds)
template <class Rec>
PT_HD bool qc_path_entered(const SceneView& S, const Ray& ray, f3 inv, bool par, float P, uint32_t c,
                           const Rec& rec, uint32_t nrec, QCounts& C) {
    const uint32_t info = S.anc_info[c];
    const uint32_t off = info & 0x03ffffffu, len = info >> 26;
    float b = P;
    uint32_t prev = 0u;
    for (uint32_t j = 0; j < len; ++j) {
        const uint32_t v = S.anc[off + j];
        if (j > 0u) b = qc_child_bound(rec, nrec, prev, v, b);
        C.nodes++;
        if (!node_enter(S.nodes[v], ray, inv, b, par)) return false;
        prev = v;
    }
    return true;
}

// one thread, whole query.  Returns the closest prim (-1 none); `exact` is set
// (and -1 returned) when the ray needs the exact stack DFS instead (non-finite
// components).  M = word memory (aux node stack).
template <class Mem>
PT_HD int qc_run(const SceneView& S, const Ray& ray, float P, int pid, F4 pre, Mem& M, QCounts& C, bool& exact,
                 float& res_t) {
    exact = pre.w != pre.w;
    res_t = P;
    if (exact) return -1;
    const bool par = signbit(pre.w);
    const f3 inv = mk3(pre.x, pre.y, pre.z);
    const f3 oinv = mk3(ray.o.x * inv.x, ray.o.y * inv.y, ray.o.z * inv.z);
    // 1-2: candidates and their bound-free leaf results
    struct HitLeaf { uint32_t c; float t; int lid; };
    HitLeaf hl[64];
    uint32_t nh = 0;
    uint32_t sp = 0;
    M.set(sp++, 0u);
    while (sp) {
        const uint32_t node = M.get(--sp);
        C.aux++;
        for (uint32_t k = 0; k < PT_AUXW; ++k) {
            const uint32_t o = S.o_aux + (node * PT_AUXW + k) * (uint32_t)sizeof(AuxSL);
            const F4 ea = blob_piece(S, o), eb = blob_piece(S, o + 16u);
            const uint32_t code = f2u(eb.w);
            if (code == 0xffffffffu) continue;
            const bool h = aux_entry_hit(ea, eb, ray, inv, oinv, pre.w);
            if (!h) continue;
            if (!(code & 0x80000000u)) {
                M.set(sp++, code);
                continue;
            }
            const uint32_t c = code & 0x7fffffffu;
            const Node nd = S.nodes[c];
            C.nodes++;
            if (!qc_slab_hit(nd, ray, inv, par)) continue;
            const uint32_t ref = f2u(nd.b.z), cnt = f2u(nd.b.w);
            float lt = PT_INF;
            int lid = -1;
            for (uint32_t i = ref; i < ref + cnt; ++i) {
                Hit hh;
                C.ptests++;
                if (bvh_prim_intersect(S.prims[i], ray, hh) && hh.t < lt) { lt = hh.t; lid = (int)i; }
            }
            if (lid < 0) continue;
            if (nh == 64u) { exact = true; return -1; }
            hl[nh++] = HitLeaf{c, lt, lid};
        }
    }
    // 3: the hitting leaves in preorder
    for (uint32_t i = 1; i < nh; ++i)
        for (uint32_t j = i; j > 0u && hl[j - 1].c > hl[j].c; --j) {
            const HitLeaf x = hl[j]; hl[j] = hl[j - 1]; hl[j - 1] = x;
        }
    struct Rec {
        uint32_t i_[64];
        float t_[64];
        PT_HD uint32_t idx(uint32_t r) const { return i_[r]; }
        PT_HD float t(uint32_t r) const { return t_[r]; }
    } rec;
    uint32_t nrec = 0;
    float bt = PT_INF;
    int res = pid;
    for (uint32_t k = 0; k < nh; ++k) {
        if (!qc_path_entered(S, ray, inv, par, P, hl[k].c, rec, nrec, C)) continue;
        rec.i_[nrec] = hl[k].c;
        rec.t_[nrec] = hl[k].t;
        ++nrec;
        // 4: first strict minimum; replaces the plane hit iff strictly closer
        if (hl[k].t < bt) {
            bt = hl[k].t;
            if (hl[k].t < P) { res_t = hl[k].t; res = hl[k].lid; }
        }
    }
    return res;
}

// whole RayIntersection on one thread with the cooperative algorithm (host
// self-tests): planes, qc_run, the exact DFS for the rays it hands back, and the
// consumer's recomputed hit (checked against the query's t)
template <class Stack>
PT_HD int qc_query(const SceneView& S, const Ray& ray, Stack& stk, Hit& out, QCounts& C, uint32_t& exact_used) {
    float P;
    int pid;
    q_planes(S, ray, P, pid);
    C.planes += S.n_planes;
    bool ex = false;
    float rt;
    const int id = qc_run(S, ray, P, pid, q_prep(S, ray), stk, C, ex, rt);
    exact_used = ex ? 1u : 0u;
    if (ex) return q_exact(S, ray, stk, out, C);
    if (id >= 0) {
        const bool ok = prim_intersect(S.prims[id], ray, out);
        if (!ok || f2u(out.t) != f2u(rt)) C.planes |= 0x80000000u;   // must never happen (tests check)
    }
    return id;
}

}  // namespace pt
