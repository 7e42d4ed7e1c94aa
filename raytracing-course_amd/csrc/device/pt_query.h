// pt_query.h -- the closest-hit query of the wavefront renderer as a per-lane
// state machine (Scene::RayIntersection, src/scene.cpp:46-77, with the
// reference BVH semantics of src/bvh.cpp:181-225 reproduced by candidate
// replay; the argument is in DESIGN.md §2 and at each step below).
//
// Built for a persistent, refilling intersection kernel: every q_step()
// advances ONE lane by one step, so the rays with long candidate lists do not
// hold the other lanes of their wave -- an idle lane takes the next ray.
//
// Memory discipline (the kernel is bound by the latency of dependent
// L2/Infinity-Cache loads): a step is  addresses -> ONE batch of eight
// independent 16-B loads -> compute.  Every phase expresses its reads as up to
// eight 16-B pieces of one "blob" (all query arrays, 16-B aligned, 32-bit byte
// offsets), so lanes in different phases share one round trip per step
// instead of serialising one per phase and one per guarded load.
//
//   * auxiliary BVH: 4-wide, nodes of 4 x 32-B entries (one step), conservative
//     inflated boxes; pending items (aux nodes and candidate leaves) on a
//     per-lane LDS stack.
//   * probe: each candidate leaf the aux pass meets is probed at once -- its
//     bundle (node record + first primitive, one step), then any further
//     primitives, one per step: the first strict minimum over its primitives,
//     which does not depend on any bound.  Only leaves with a primitive hit can
//     change the result or a bound (src/bvh.cpp:205-223), so only they join the
//     hitting-leaf list (PT_QHK, sorted by reference index = preorder; more ->
//     another pass above the last decided leaf).
//   * decision per hitting leaf, in preorder: its leaf record (certain accept /
//     certain reject), else its ancestor list below the LCA with the last
//     recorded hit, 4 entries then their 4 records per step.
// Rays with non-finite components, or a list full of entered hits with another
// hit to add, take the exact stack DFS (bvh_exact) in a separate pass.
#pragma once
#include "pt_trace.h"

namespace pt {

#ifndef PT_AUXW
#define PT_AUXW 4               // auxiliary BVH width (nodes = PT_AUXW AuxSL entries)
#endif

// Query-blob form of a wide aux entry (32 B, the AuxSL slot): two boxes in
// binary16, each rounded outward, then {range, code}:
//   w0..w2: the subtree's own box  (lo.x | lo.y << 16, lo.z | hi.x << 16, hi.y | hi.z << 16)
//   w3..w5: the subtree's hit region (same packing; +-inf halves: unbounded)
//   w6: internal entry -- its leaf range; leaf entry -- the leaf's bundle ordinal
//   w7: code (internal child node, 0x80000000 | reference leaf, 0xffffffff empty)
// A reference leaf matters only if its own box is crossed (else it is never
// entered) AND one of its primitives is hit, which can only happen inside its
// hit region (host/scene_api.cpp leaf_hit_region: a plain triangle is only ever hit
// on its copy moved onto the plane through the origin, widened there for the
// edge tests' rounding).  A subtree holds such a leaf only if the ray crosses
// both the union of its own boxes and the union of its hit regions, so an entry
// is taken iff both tests pass.  The computed hit point lies within ~22u (2|o| +
// 3X) of the ray (u = 2^-24, X = scene box extent), so the hit-region test is
// widened per ray by PT_LEAF_MARGIN x dl, where dl = 2^-18 (X + |o|max) / |d|min
// (q_prep) is 64u (X + |o|) per unit of t: ~60x headroom.  Rays with a
// near-zero direction component test the own boxes only (robust form).
#define PT_LEAF_MARGIN 64.f

PT_HD float h16(uint32_t bits) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(bits & 0xffffu)); }

// slab interval of the ray against a box given by its binary16 halves
PT_HD void aux_slab16(uint32_t w0, uint32_t w1, uint32_t w2, f3 inv, f3 oinv, float& tn, float& tf) {
    const float ax = fmaf(h16(w0), inv.x, -oinv.x), bx = fmaf(h16(w1 >> 16), inv.x, -oinv.x);
    const float ay = fmaf(h16(w0 >> 16), inv.y, -oinv.y), by = fmaf(h16(w2), inv.y, -oinv.y);
    const float az = fmaf(h16(w1), inv.z, -oinv.z), bz = fmaf(h16(w2 >> 16), inv.z, -oinv.z);
    tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
}

// is the entry (ea, eb) taken?  dlw = the q_prep record's w (dl; negative: a
// near-zero direction component)
PT_HD bool aux_entry_hit(const F4& ea, const F4& eb, const Ray& ray, f3 inv, f3 oinv, float dlw) {
    if (signbit(dlw))
        return aux_box_par(h16(f2u(ea.x)), h16(f2u(ea.x) >> 16), h16(f2u(ea.y)), h16(f2u(ea.y) >> 16),
                           h16(f2u(ea.z)), h16(f2u(ea.z) >> 16), ray, inv, oinv);
    float tn, tf, un, uf;
    aux_slab16(f2u(ea.x), f2u(ea.y), f2u(ea.z), inv, oinv, tn, tf);
    aux_slab16(f2u(ea.w), f2u(eb.x), f2u(eb.y), inv, oinv, un, uf);
    const float mt = PT_LEAF_MARGIN * dlw;
    return tn <= tf && tf >= 0.f && (!(mt < INFINITY) || (un - mt <= uf + mt && uf + mt >= 0.f));
}

// wide aux entry, host form (AuxSL, 32 B; the array k_wcamera's costly-class test
// reads): a = {lo.xyz, hi.x}, b = {hi.y, hi.z, range, code} with the own box in f32;
// the query blob holds the dual binary16 form above with the same range and code:
//   internal entry: range = (max reference leaf of the subtree >> S, rounded up) << 16 | (min >> S)
//   (S = SceneView::aux_rshift; annotate_aux_ranges in host/aux_bvh.cpp)
//   leaf entry (code = 0x80000000 | reference leaf): range = the leaf's ordinal (its bundle)
// stackless auxiliary node (32 B):
//   internal: a = {lo.x, lo.y, lo.z, hi.x}, b = {hi.y, hi.z, u32 skip, 0xffffffff}
//   leaf:     a = {c.x, c.y, c.z, s.x},     b = {s.y, s.z, u32 skip (= own index + 1), u32 reference leaf}
// (c, s) of a leaf are bit-identical copies of the reference node's record.
struct AuxSL { F4 a, b; };
#define PT_AUX_INTERNAL 0xffffffffu

enum : uint32_t { Q_AUX = 0u, Q_REPLAY = 1u, Q_DONE = 2u, Q_EXACT = 3u, Q_DECIDE = 4u };
// replay step kinds: each issues one round of independent loads
enum : uint32_t { R_CAND = 0u, R_WALK_E = 1u, R_WALK_N = 2u };
#define PT_RKINDS 3u

// compact primitive records of the query (64 B, blob section o_qprim, same index
// as the full 80-B records):
//   plain triangle (pos = +0, rotation = (0,0,0,1) exactly): {a.xyz, T_TRIANGLE}, {b.xyz, n.x}, {c.xyz, n.y},
//                           {n.z, -, -, -} with n = normalize(cross(b - a, c - a)) (host, same operations)
//   box / ellipsoid:        {size.xyz, type}, {pos.xyz, rot.x}, {rot.yzw, -}, {-}
//   anything else:          {-, -, -, type | PT_QP_FULL} -> full record
#define PT_QPRIM_BYTES 64u
#define PT_QP_FULL 0x100u

// the full Prim a compact record stands for (bit-identical fields, so
// bvh_prim_intersect performs exactly the reference operations)
PT_HD Prim qprim_expand(const F4& r0, const F4& r1, const F4& r2) {
    Prim P;
    const uint32_t type = f2u(r0.w);
    if (type == T_TRIANGLE) {
        P.p0 = F4{0.f, 0.f, 0.f, r0.w};
        P.p1 = F4{0.f, 0.f, 0.f, 1.f};
        P.p2 = F4{r0.x, r0.y, r0.z, 0.f};
        P.p3 = F4{r1.x, r1.y, r1.z, r2.x};
        P.p4 = F4{r2.y, r2.z, 0.f, 0.f};
    } else {
        P.p0 = F4{r1.x, r1.y, r1.z, r0.w};
        P.p1 = F4{r1.w, r2.x, r2.y, r2.z};
        P.p2 = F4{r0.x, r0.y, r0.z, 0.f};
        P.p3 = F4{0.f, 0.f, 0.f, 0.f};
        P.p4 = F4{0.f, 0.f, 0.f, 0.f};
    }
    return P;
}

// leaf bundle (96 B, blob section o_bundle, one per reference leaf, numbered in
// the order the wide aux nodes hold the leaves; the number -- the leaf's
// "ordinal" -- is carried in its wide aux entry's b.z): the first three pieces of
// the compact record of the leaf's first primitive, then {leaf node index, first
// prim, prim count, the record's n.z}, then the leaf's node record box {c.xyz,
// s.x}, {s.y, s.z, -, -} (the probe prices its certain accept, q_leaf_accept_t)
#define PT_BUNDLE_BYTES 96u
#define PT_LEAFQ 0x80000000u    // Q_AUX item: a candidate leaf to probe (| its ordinal)

#ifndef PT_QHK
#define PT_QHK 6                // hitting-leaf list: entered hits of earlier passes + this pass's undecided ones
#endif

struct Query {
    Ray ray;
    f3 inv;                     // 1/d (IEEE, once per ray)
    float P;                    // closest plane t (the BVH bound at the root)
    // small state packed into two registers
    uint32_t phase : 3;         // Q_* (Q_DECIDE only inside q_exec)
    uint32_t walk : 2;          // Q_REPLAY step kind: R_CAND, R_WALK_E, R_WALK_N
    uint32_t par : 1;           // near-zero direction component: exact node tests, robust aux boxes
    uint32_t robust : 1;        // leaf check: the ray crosses the leaf box robustly (t1c, mc valid)
    uint32_t known : 1;         // walk: the segment bound is known (below the LCA with the last hit)
    uint32_t overflow : 1;      // this pass dropped hitting leaves above the list's largest one
    uint32_t sp : 7;            // Q_AUX: pending aux items on the per-lane stack
    uint32_t pos : 7;           // walk: position reached in the ancestor list
    uint32_t len : 7;           // walk: ancestor list length
    uint32_t nh : 4;            // hitting leaves in the list (<= PT_QHK)
    uint32_t ne : 4;            // ... of which the first ne are decided and entered (the recorded hits)
    uint32_t cid : 10;          // k_wpath: the chain's entry in its workgroup's LDS pixel table
    uint32_t spare : 13;        // (fills the word: a narrower unit is accessed bytewise, which keeps
                                //  the whole Query out of registers)
    uint32_t node;              // Q_AUX: aux node, or PT_LEAFQ | ordinal of the leaf being probed
    uint32_t lb;                // every hitting leaf below lb has been decided
    uint32_t cand;              // probe: its leaf; Q_REPLAY: the hitting leaf being decided (hidx[ne])
    float dl;                   // certification margin (t units, see q_leaf_certain)
    // the probe's state (Q_AUX) and the decision's (Q_REPLAY) share registers: li is 0
    // whenever an aux pass starts (q_init_pre, q_pass_done)
    union {
        struct {
            uint32_t lref, lcnt;        // probe: the leaf's primitive range
            uint32_t li;                // probe: primitives tested (bit 31: this step = full record)
            float lt;                   // probe: leaf first-min t so far
            int lid;                    // probe: its primitive (-1 none)
            float lacc;                 // probe: the leaf's certain-accept threshold
        };
        struct {
            uint32_t off;               // walk: ancestor list offset
            uint32_t e[4];              // walk: the entries under test (0xffffffff = none)
            uint32_t astar;             // walk: deepest ancestor at or above that LCA seen so far
            float bound;                // walk: the segment's bound
            float t1c, mc;              // leaf check: approximate entry and certification margin
        };
    };
    uint32_t hidx[PT_QHK];      // hitting leaves (reference index, sorted; 0xffffffff = empty)
    float ht[PT_QHK];           // ... their first-min t
    int hid[PT_QHK];            // ... and its primitive
    float hacc[PT_QHK];         // ... and its certain-accept threshold (q_leaf_accept_t)
    float bt;                   // best BVH leaf hit so far (first strict minimum)
    float res_t;                // result so far (plane, then BVH hits that beat it): t and prim;
    int res_id;                 // the normal is recomputed from the prim by the consumer
};
static_assert(PT_QHK < 16, "nh and ne are 4-bit fields");
#define PT_QUERY_SP_MAX 127u    // Query::sp is a 7-bit field: pt_scene_prepare rejects deeper aux stacks

struct QCounts {
    uint32_t nodes, aux, ptests, planes;
#ifdef PT_QDIAG
    uint32_t cands, passes, steps, rc_acc, rc_rej, rc_walk;
#endif
};

// planes (src/scene.cpp:50-57), then the BVH set-up
// the planes part of RayIntersection (src/scene.cpp:50-57): closest plane t and
// its prim (-1 none).  Run by the ray's producer (camera / shade kernels), so
// the query kernel starts at the BVH.
// `pl(k, pi)` = the k-th plane's record and prim index (PlanesGlobal, or a copy)
struct PlanesGlobal {
    const SceneView& S;
    PT_HD Prim operator()(uint32_t k, uint32_t& pi) const { pi = S.planes[k]; return S.prims[pi]; }
};
template <class PL>
PT_HD void q_planes_e(const SceneView& S, const PL& pl, const Ray& ray, float& P, int& pid) {
    P = PT_INF;
    pid = -1;
    for (uint32_t k = 0; k < S.n_planes; ++k) {
        uint32_t pi;
        const Prim pr = pl(k, pi);
        Hit h;
        bool ok;
        if (f2u(pr.p1.x) == 0u && f2u(pr.p1.y) == 0u && f2u(pr.p1.z) == 0u && f2u(pr.p1.w) == 0x3f800000u) {
            // identity rotation: the local ray equals (o - pos, d) up to the sign of
            // zero components, which changes neither the accept decision nor t
            // (a signed zero only matters in a sum that is exactly zero, where
            // every test below fails either way); the normal is not needed here
            Ray lr;
            lr.o = ray.o + -1.f * mk3(pr.p0.x, pr.p0.y, pr.p0.z);
            lr.d = ray.d;
            ok = isect_plane(lr, mk3(pr.p2.x, pr.p2.y, pr.p2.z), h);
        } else {
            ok = plane_intersect(pr, ray, h);
        }
        if (ok && h.t < P) { P = h.t; pid = (int)pi; }
    }
}
PT_HD void q_planes(const SceneView& S, const Ray& ray, float& P, int& pid) { q_planes_e(S, PlanesGlobal{S}, ray, P, pid); }

// Per-ray set-up a query needs, computed once by the ray's producer (so the
// IEEE divisions run on the producer's full wave, not on the few lanes a query
// wave refills): {1/d.xyz, dl}; dl < 0 (sign bit) marks a ray with a
// near-zero direction component (par), NaN a non-finite ray (exact stack DFS:
// its NaN/inf slab semantics are not replayed).
PT_HD F4 q_prep(const SceneView& S, const Ray& ray) {
    const float big = 3e38f;
    if (!(fabsf(ray.o.x) < big && fabsf(ray.o.y) < big && fabsf(ray.o.z) < big && fabsf(ray.d.x) < big &&
          fabsf(ray.d.y) < big && fabsf(ray.d.z) < big))
        return F4{0.f, 0.f, 0.f, __builtin_nanf("")};
    const bool par = !replay_ok_ray(ray);
    const float om = fmaxf(fmaxf(fabsf(ray.o.x), fabsf(ray.o.y)), fabsf(ray.o.z));
    const float dm = fminf(fminf(fabsf(ray.d.x), fabsf(ray.d.y)), fabsf(ray.d.z));
    // non-par: dm > 1e-30 and a positive numerator, so dl is +finite or +inf
    const float dl = par ? -INFINITY : 0x1p-18f * (S.box_extent + om) / dm;
    return F4{1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z, dl};
}

// BVH query set-up for a ray whose plane result (P, pid) and q_prep record are known
PT_HD void q_init_pre(const Ray& ray, float P, int pid, F4 pre, Query& q) {
    q.ray = ray;
    q.res_id = pid;
    q.res_t = P;
    q.P = P;
    q.bt = PT_INF;
    q.nh = 0;
    q.ne = 0;
    q.lb = 0;
    q.overflow = 0;
    q.node = 0;
    q.sp = 0;
    q.li = 0;
#pragma unroll
    for (int i = 0; i < PT_QHK; ++i) q.hidx[i] = 0xffffffffu;
    q.inv = mk3(pre.x, pre.y, pre.z);
    q.par = signbit(pre.w) ? 1u : 0u;
    q.dl = fabsf(pre.w);
    q.phase = pre.w != pre.w ? Q_EXACT : Q_AUX;
}

PT_HD void q_init(const SceneView& S, const Ray& ray, float P, int pid, Query& q) {
    q_init_pre(ray, P, pid, q_prep(S, ray), q);
}

// hidx[k] / ht[k] / hid[k] for a lane-varying k < PT_QHK: an unrolled select
// chain.  Its default is not an element, so the optimiser cannot fold the chain
// into a dynamically indexed load (which would keep the whole Query in scratch).
template <class T>
PT_HD T q_sel(const T (&a)[PT_QHK], uint32_t k, T dflt) {
    T v = dflt;
#pragma unroll
    for (int i = 0; i < PT_QHK; ++i)
        if ((uint32_t)i == k) v = a[i];
    return v;
}

// A probed leaf with a primitive hit joins the list, sorted by reference index.
// Entered hits of earlier passes lie below lb <= c, so they never move; with
// the list full the largest entry (undecided: it is above c >= lb) or c itself
// drops out and another pass follows.  Returns false when every slot holds an
// entered hit (the exact DFS takes the ray).
PT_HD bool q_add_hit(Query& q, uint32_t c, float t, int id, float acc) {
    if (q.ne == PT_QHK) return false;
#pragma unroll
    for (int k = 0; k < PT_QHK; ++k) {
        const bool sw = q.hidx[k] > c;   // empty slots hold 0xffffffff
        const uint32_t xi = q.hidx[k];
        const float xt = q.ht[k];
        const int xd = q.hid[k];
        const float xa = q.hacc[k];
        if (sw) {
            q.hidx[k] = c; q.ht[k] = t; q.hid[k] = id; q.hacc[k] = acc;
            c = xi; t = xt; id = xd; acc = xa;
        }
    }
    if (c != 0xffffffffu) q.overflow = 1u;   // a hitting leaf above the kept ones dropped out
    else q.nh = q.nh + 1u;
    return true;
}

// every hitting leaf of the pass is decided: another pass above lb, or done
PT_HD void q_pass_done(Query& q) {
    if (q.overflow) {
        if (q.ne == PT_QHK) {
            q.phase = Q_EXACT;
            return;
        }
        q.overflow = 0;
        q.node = 0;
        q.sp = 0;
        q.li = 0;
        q.phase = Q_AUX;
        return;
    }
    q.phase = Q_DONE;
}

// hitting leaf hidx[ne] (= cand) is entered: it becomes a recorded hit
// (src/bvh.cpp:205-213 + the recursion's fold: the BVH result is the first
// strict minimum over entered hits in preorder; it replaces the plane hit iff
// strictly closer, src/scene.cpp:68-74)
PT_HD void q_record_entered(Query& q) {
    const float t = q_sel(q.ht, q.ne, PT_INF);
    const int id = q_sel(q.hid, q.ne, -1);
    if (t < q.bt) {
        q.bt = t;
        if (t < q.P) { q.res_t = t; q.res_id = id; }
    }
    q.ne = q.ne + 1u;
    q.lb = q.cand + 1u;
}

// the next undecided hitting leaf is decided at the end of the step (q_decide)
PT_HD void q_next_decision(Query& q) { q.phase = Q_DECIDE; }

PT_HD void q_entered(Query& q) {
    q_record_entered(q);
    q_next_decision(q);
}

// End of a step that left the lane at a decision (phase Q_DECIDE; one place in
// the code): hitting leaves whose precomputed certain accept holds (q_leaf_certain's
// first case: lo = min(P, recorded hits) = min(P, bt) >= the threshold the probe
// computed, q_leaf_accept_t) are entered here; the first other one gets the leaf
// check (R_CAND), or the pass is done.
PT_HD void q_decide(Query& q) {
#pragma unroll 1
    while (q.ne < q.nh) {
        q.cand = q_sel(q.hidx, q.ne, 0xffffffffu);
        if (!(fminf(q.P, q.bt) >= q_sel(q.hacc, q.ne, PT_INF))) {
            q.walk = R_CAND;
            q.phase = Q_REPLAY;
            return;
        }
        q_record_entered(q);
    }
    q_pass_done(q);
}

// hitting leaf hidx[ne] is not entered: it leaves the list (an unentered leaf
// changes neither the result nor any bound)
PT_HD void q_rejected(Query& q) {
#pragma unroll
    for (int k = 0; k + 1 < PT_QHK; ++k) {
        if ((uint32_t)k >= q.ne) {
            q.hidx[k] = q.hidx[k + 1];
            q.ht[k] = q.ht[k + 1];
            q.hid[k] = q.hid[k + 1];
            q.hacc[k] = q.hacc[k + 1];
        }
    }
    q.hidx[PT_QHK - 1] = 0xffffffffu;
    q.nh = q.nh - 1u;
    q.lb = q.cand + 1u;
    q_next_decision(q);
}

// min of the recorded hits strictly inside (a, r) (the left subtree of a when
// r is a's right child); at least one exists when called with a = a*
PT_HD float q_bound_between(const Query& q, uint32_t a, uint32_t r) {
    float m = q.P;
    bool any = false;
#pragma unroll
    for (int k = 0; k < PT_QHK; ++k) {
        if ((uint32_t)k < q.ne && q.hidx[k] > a && q.hidx[k] < r) {
            if (!any || q.ht[k] < m) m = q.ht[k];
            any = true;
        }
    }
    return m;
}

// The certain-accept threshold of a leaf (q_leaf_certain's first case, computed by
// the probe from the bundle's copy of the leaf's node record, the same floats and
// operations): the leaf is entered whenever lo = min(P, recorded hits) >= it;
// +inf if the ray does not cross the leaf box robustly.
PT_HD float q_leaf_accept_t(const Query& q, const F4& na, const F4& nb) {
    const f3 c = mk3(na.x, na.y, na.z);
    const f3 s = mk3(na.w, nb.x, nb.y);
    const f3 o = q.ray.o + -1.f * c;
    const f3 nlo = -1.f * s - o, nhi = s - o;
    const float ax = nlo.x * q.inv.x, bx = nhi.x * q.inv.x;
    const float ay = nlo.y * q.inv.y, by = nhi.y * q.inv.y;
    const float az = nlo.z * q.inv.z, bz = nhi.z * q.inv.z;
    const float t1 = smax(smax(smin(ax, bx), smin(ay, by)), smin(az, bz));
    const float t2 = smin(smin(smax(ax, bx), smax(ay, by)), smax(az, bz));
    const float m = q.dl + (fabsf(t1) + fabsf(t2)) * 0x1p-18f;
    const bool robust = !q.par && t1 + m <= t2 - m && t2 - m >= 0.f;
    return robust ? t1 + m : INFINITY;
}

// Hitting-leaf check before any root-path replay.  Every bound the replay
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
    for (int k = 0; k < PT_QHK; ++k)
        if ((uint32_t)k < q.ne) { lo = fminf(lo, q.ht[k]); hi = fmaxf(hi, q.ht[k]); }
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
    // certain reject: node_enter's decision against hi on the same quotients (its
    // slab_approx is this computation); exact division when too close to call
    uint32_t v = q.par ? 2u : enter_decide(t1, t2, hi);
    if (v == 2u) v = enter_exact(nd.a, nd.b, q.ray, hi) ? 1u : 0u;
    return v == 0u ? 0u : 2u;
}

// ---- step = addresses -> one batch of 8 x 16-B loads -> compute -------------

// byte offsets (into S.blob) of the 8 pieces this lane's next step reads
PT_HD void q_addr(const SceneView& S, const Query& q, uint32_t off[8]) {
    uint32_t b0, b1, b2;
    if (q.phase == Q_AUX) {
        if (!(q.node & PT_LEAFQ)) {
            const uint32_t b = S.o_aux + q.node * (uint32_t)(PT_AUXW * sizeof(AuxSL));
#pragma unroll
            for (int k = 0; k < 8; ++k) off[k] = b + 16u * (uint32_t)k;
            return;
        }
        if (q.li == 0u) {
            // the leaf's bundle (first primitive + primitive range + leaf box): 6 pieces
            b0 = S.o_bundle + PT_BUNDLE_BYTES * (q.node & 0x7fffffffu);
#pragma unroll
            for (int k = 0; k < 8; ++k) off[k] = b0 + 16u * (uint32_t)(k < 6 ? k : 5);
            return;
        }
        if (q.li & 0x80000000u) {
            // a full primitive record: 5 pieces
            b0 = S.o_prim + 80u * (q.lref + (q.li & 0x7fffffffu));
#pragma unroll
            for (int k = 0; k < 8; ++k) off[k] = b0 + 16u * (uint32_t)(k < 5 ? k : 4);
            return;
        }
        // the leaf's next compact primitive: 4 pieces
        b0 = S.o_qprim + PT_QPRIM_BYTES * (q.lref + q.li);
#pragma unroll
        for (int k = 0; k < 8; ++k) off[k] = b0 + 16u * (uint32_t)(k < 4 ? k : 3);
        return;
    } else if (q.walk == R_CAND) {
        b0 = S.o_nodes + 32u * q.cand;
        b1 = b0 + 16u;
        b2 = S.o_ainfo + 16u * (q.cand >> 2);     // the 16 B holding anc_info[cand]
    } else if (q.walk == R_WALK_E) {
        b0 = S.o_anc + 4u * (q.off + q.pos);      // 4 entries (lists padded to 16 B)
        b1 = b0;
        b2 = b0;
    } else {
        // R_WALK_N: the records of the 4 pending entries (none -> node 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t e = q.e[j] == 0xffffffffu ? 0u : q.e[j];
            off[2 * j] = S.o_nodes + 32u * e;
            off[2 * j + 1] = off[2 * j] + 16u;
        }
        return;
    }
    off[0] = b0; off[1] = b1; off[2] = b2;
#pragma unroll
    for (int k = 3; k < 8; ++k) off[k] = b0;
}

// Q_AUX: the next item of the aux pass (top of the lane's stack), or the end
// of the pass: its hitting leaves are decided next
template <class Mem>
PT_HD void q_aux_next(Query& q, Mem& stk, uint32_t next) {
    if (next == 0xffffffffu && q.sp > 0u) next = stk.get(--q.sp);
    if (next != 0xffffffffu) {
        q.node = next;
        return;
    }
    q_next_decision(q);
}

// Diagnostics builds (PT_QPROF, device only): each step kind's branch stamps the
// shader clock on entry into qp[kind] (this lane's copy; the caller takes the
// wave's and attributes the time to the kinds in program order).
#if defined(PT_QPROF) && defined(__HIP_DEVICE_COMPILE__)
#define PT_QPROF_DEV 1
#define QP_STAMP(i) do { uint64_t t_; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); qp[i] = (uint32_t)t_; } while (0)
#define QP_ARG , uint32_t* qp
#else
#define QP_STAMP(i) (void)0
#define QP_ARG
#endif
// The aux-node step kind (one wide node: PT_AUXW child entries); ends in the next
// aux item, the end of the pass (Q_DECIDE) or the exact DFS.
template <class Mem>
PT_HD void q_exec_aux(const SceneView& S, Query& q, QCounts& C, Mem& stk, const F4 r[8]) {
    C.aux++;
    const f3 oinv = mk3(q.ray.o.x * q.inv.x, q.ray.o.y * q.inv.y, q.ray.o.z * q.inv.z);
    // all PT_AUXW slab tests first, branch-free (the robust form only when a lane
    // of the wave needs it); then the bookkeeping per entry
    // both boxes of each entry (own box, hit region: see PT_LEAF_MARGIN),
    // branch-free; the robust own-box form only when a lane of the wave needs it
    const float mt = PT_LEAF_MARGIN * q.dl;
    const bool mwide = !(mt < INFINITY);
    bool hit[PT_AUXW];
#pragma unroll
    for (int k = 0; k < PT_AUXW; ++k) {
        const F4 ea = r[2 * k], eb = r[2 * k + 1];
        float tn, tf, un, uf;
        aux_slab16(f2u(ea.x), f2u(ea.y), f2u(ea.z), q.inv, oinv, tn, tf);
        aux_slab16(f2u(ea.w), f2u(eb.x), f2u(eb.y), q.inv, oinv, un, uf);
        hit[k] = tn <= tf && tf >= 0.f && (mwide || (un - mt <= uf + mt && uf + mt >= 0.f));
    }
    if (pt_any(q.par != 0u)) {
#pragma unroll
        for (int k = 0; k < PT_AUXW; ++k) {
            const F4 ea = r[2 * k];
            if (q.par)
                hit[k] = aux_box_par(h16(f2u(ea.x)), h16(f2u(ea.x) >> 16), h16(f2u(ea.y)), h16(f2u(ea.y) >> 16),
                                     h16(f2u(ea.z)), h16(f2u(ea.z) >> 16), q.ray, q.inv, oinv);
        }
    }
    uint32_t next = 0xffffffffu;
    // the largest listed hitting leaf when the list is full (else none): a leaf
    // above it could only join the list to drop out again
    const uint32_t hmax = q.hidx[PT_QHK - 1];
    // (bookkeeping in locals and selects: the packed fields are written once, and a
    // stack push is one store whatever the entry -- no per-entry exec-mask branches)
    uint32_t sp = q.sp;
    bool ovf = false;
#pragma unroll
    for (int k = 0; k < PT_AUXW; ++k) {
        // every entry's box is conservative: a reference leaf passing it is a
        // candidate, probed next (its own slab test is decided only if one of
        // its primitives is hit: a leaf failing it is never entered,
        // src/bvh.cpp:188-198)
        const uint32_t code = f2u(r[2 * k + 1].w);
        const uint32_t rng = f2u(r[2 * k + 1].z);   // leaf: its ordinal; internal: its leaf range
        const bool h = hit[k] && code != 0xffffffffu;
        const bool isleaf = (code & 0x80000000u) != 0u;
        const uint32_t lidx = code & 0x7fffffffu;
        // a subtree is skipped when all its leaves lie below lb (decided in an
        // earlier pass), or above the largest listed hitting leaf of a full
        // list: it could only add hits the list would drop, so another pass follows
        const bool above = isleaf ? lidx > hmax
                                  : (hmax != 0xffffffffu && ((rng & 0xffffu) << S.aux_rshift) > hmax);
        const bool fresh = isleaf ? lidx >= q.lb : ((rng >> 16) << S.aux_rshift) >= q.lb;
        ovf = ovf || (h && fresh && above);
        const bool take = h && fresh && !above;
        const uint32_t item = isleaf ? (PT_LEAFQ | rng) : code;
        const bool first = take && next == 0xffffffffu;
        const bool push = take && !first;
        next = first ? item : next;
        stk.setc(sp, item, push && sp < stk.cap);
        sp += push ? 1u : 0u;   // (past the stack's capacity: the exact DFS below)
    }
    if (ovf) q.overflow = 1u;
    if (sp > stk.cap) {
        q.phase = Q_EXACT;   // the pending items do not fit the stack: exact DFS (same result)
        return;
    }
    q.sp = sp;
#ifdef PT_QDIAG
    if (next == 0xffffffffu && q.sp == 0u) C.passes++;
    if (q.sp > C.steps) C.steps = q.sp;   // (diagnostics: the deepest aux stack of the query)
#endif
    q_aux_next(q, stk, next);
}

template <class Mem>
PT_HD void q_exec_kind(const SceneView& S, Query& q, QCounts& C, Mem& stk, const F4 r[8] QP_ARG) {
    if (q.phase == Q_AUX && !(q.node & PT_LEAFQ)) {
        QP_STAMP(0);
        q_exec_aux(S, q, C, stk, r);
        return;
    }
    if (q.phase == Q_AUX) {
        QP_STAMP(1);
        // probe a candidate leaf: the first strict minimum over its primitives
        // (src/bvh.cpp:205-213), independent of any bound.  Every record form goes
        // through ONE test of each primitive kind (a wave runs each kind's code once
        // whatever mix of forms its lanes hold), and only t is computed: the
        // consumer recomputes the closest hit's normal and side.
        if (q.li == 0u) {
            // its bundle: its first primitive and the primitive range
            q.cand = f2u(r[3].x);
            q.lref = f2u(r[3].y);
            q.lcnt = f2u(r[3].z);
            q.lt = PT_INF;
            q.lid = -1;
            q.lacc = q_leaf_accept_t(q, r[4], r[5]);
#ifdef PT_QDIAG
            C.cands++;
#endif
            if (q.lcnt == 0u) {
                q_aux_next(q, stk, 0xffffffffu);
                return;
            }
        }
        const bool full = (q.li & 0x80000000u) != 0u;   // this step holds the full 80-B record
        const uint32_t cty = f2u(r[0].w);
        if (!full && (cty & PT_QP_FULL)) {
            q.li |= 0x80000000u;                        // not representable compactly: full record next step
            return;
        }
        // the primitive (a compact record expands to the same bits)
        Prim pr = qprim_expand(r[0], r[1], r[2]);
        if (full) { pr.p0 = r[0]; pr.p1 = r[1]; pr.p2 = r[2]; pr.p3 = r[3]; pr.p4 = r[4]; }
        const uint32_t ty = f2u(pr.p0.w);
        // A plain triangle (compact: pos = +0, identity rotation) is tested on the world
        // ray: the world->local rotation changes at most the sign of zero components,
        // which changes neither the accept decision nor t (a signed zero only matters in
        // a sum that is exactly zero, where every compare here is false either way).  The
        // same holds for the rotation of any record whose rotation is exactly (0,0,0,1)
        // (only t is wanted here, not the normal): its local ray is (o - pos, d).  Other
        // records go to local space exactly as Primitive::Intersect does.
        Ray lr = q.ray;
        if (full || cty != T_TRIANGLE) {
            const f3 pos = mk3(pr.p0.x, pr.p0.y, pr.p0.z);
            lr.o = q.ray.o + -1.f * pos;
            const bool ident = f2u(pr.p1.x) == 0u && f2u(pr.p1.y) == 0u && f2u(pr.p1.z) == 0u &&
                               f2u(pr.p1.w) == 0x3f800000u;
            if (!ident) {
                q4 qq;
                qq.x = pr.p1.x; qq.y = pr.p1.y; qq.z = pr.p1.z; qq.w = pr.p1.w;
                const q4 cq = conj(qq);
                lr.o = qrot(cq, lr.o);
                lr.d = qrot(cq, q.ray.d);
            }
        }
        const f3 pa = mk3(pr.p2.x, pr.p2.y, pr.p2.z);
        bool ok;
        float t = 0.f;
        uint32_t in;
        if (ty == T_TRIANGLE) {
            const f3 pb = mk3(pr.p3.x, pr.p3.y, pr.p3.z), pc = mk3(pr.p3.w, pr.p4.x, pr.p4.y);
            // a compact record carries the triangle's normal (n.z: in the bundle's header
            // piece, or the record's fourth piece)
            f3 n = mk3(r[1].w, r[2].w, q.li == 0u ? r[3].w : r[3].x);
            if (full) n = normalize(cross(pb - pa, pc - pa));
            Hit h;
            ok = isect_triangle_n(lr, pa, pb, pc, n, h);
            t = h.t;
        } else if (ty == T_BOX) {
            ok = slab(lr.o, lr.d, pa, t, in);
        } else {
            ok = ellipsoid_root(lr, pa, t, in);
        }
        const uint32_t li = q.li & 0x7fffffffu;
        C.ptests++;
        if (ok && t < q.lt) { q.lt = t; q.lid = (int)(q.lref + li); }
        q.li = li + 1u;
        if (q.li < q.lcnt) return;
        q.li = 0u;
        if (q.lid >= 0 && !q_add_hit(q, q.cand, q.lt, q.lid, q.lacc)) {
            q.phase = Q_EXACT;
            return;
        }
        q_aux_next(q, stk, 0xffffffffu);
        return;
    }
    // Q_REPLAY: is hitting leaf hidx[ne] (= cand) entered?
    if (q.walk == R_CAND) {
        QP_STAMP(2);
        // its own leaf record (+ where its ancestor list is)
        Node nd;
        nd.a = r[0];
        nd.b = r[1];
        const uint32_t k4 = q.cand & 3u;
        const uint32_t info = f2u(k4 == 0u ? r[2].x : k4 == 1u ? r[2].y : k4 == 2u ? r[2].z : r[2].w);
        C.nodes++;
        const uint32_t v = q_leaf_certain(q, nd);
#ifdef PT_QDIAG
        if (v == 1u) C.rc_acc++; else if (v == 0u) C.rc_rej++; else C.rc_walk++;
#endif
        if (v == 1u) {
            q_entered(q);
            return;
        }
        if (v == 0u) {
            q_rejected(q);
            return;
        }
        // undecided: test the root path below a* = LCA(last recorded hit, cand).
        // Ancestors at or above a* were entered on that hit's path (same
        // node, same bound: both depend only on earlier hits) -- they are the
        // list entries <= the hit.  Below a* no left subtree holds a hit, so
        // the bound is constant: B = min{hits in (a*, right child of a*)}.
        // Each remaining ancestor, then the leaf itself (the list's last
        // entry), is tested with B.
        q.off = info & 0x03ffffffu;
        q.len = info >> 26;
        q.pos = 0u;
        q.known = q.ne == 0u ? 1u : 0u;   // no earlier hit: the bound is P on the whole path
        q.bound = q.P;
        q.astar = 0u;
        q.walk = R_WALK_E;
        return;
    }
    if (q.walk == R_WALK_E) {
        QP_STAMP(3);
        // next 4 list entries (ancestors, then the leaf; 0xffffffff = padding)
        const uint32_t hlast = q_sel(q.hidx, q.ne - 1u, 0u);   // last recorded hit (none: 0)
        bool any = false, accept = false;
        const uint32_t ent[4] = {f2u(r[0].x), f2u(r[0].y), f2u(r[0].z), f2u(r[0].w)};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t e = q.pos + (uint32_t)j < q.len ? ent[j] : 0xffffffffu;
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
            q_entered(q);
            return;
        }
        if (any) q.walk = R_WALK_N;
        else q.pos += 4u;                // all at or above a*
        return;
    }
    // R_WALK_N: the records of the pending entries, tested with B
    QP_STAMP(4);
    bool reject = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (q.e[j] == 0xffffffffu) continue;
        Node nd;
        nd.a = r[2 * j];
        nd.b = r[2 * j + 1];
        C.nodes++;
        if (!node_enter(nd, q.ray, q.inv, q.bound, q.par != 0u)) reject = true;
    }
    if (reject) {
        q_rejected(q);
        return;
    }
    q.pos += 4u;
    if (q.pos >= q.len) q_entered(q);   // the leaf (last entry) was entered too
    else q.walk = R_WALK_E;
}

// one step's compute: the step kind's transition, then the precomputed accepts
template <class Mem>
PT_HD void q_exec(const SceneView& S, Query& q, QCounts& C, Mem& stk, const F4 r[8] QP_ARG) {
#ifdef PT_QPROF_DEV
    q_exec_kind(S, q, C, stk, r, qp);
#else
    q_exec_kind(S, q, C, stk, r);
#endif
    if (q.phase == Q_DECIDE) q_decide(q);
}

PT_HD F4 blob_piece(const SceneView& S, uint32_t off) {
    return *reinterpret_cast<const F4*>(reinterpret_cast<const unsigned char*>(S.blob) + off);
}

// Advance one step.  Precondition: phase is Q_AUX or Q_REPLAY.
// `stk` = per-lane word memory for the pending aux nodes (set/get).
// Every lane loads 8 pieces (q_addr repeats a step's last piece): loading only
// the distinct ones measured -5 % (the exec-mask branches cost more than the
// repeated loads, which hit the same line).
template <class Mem>
PT_HD void q_step(const SceneView& S, Query& q, QCounts& C, Mem& stk) {
    uint32_t off[8];
    q_addr(S, q, off);
    F4 r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = blob_piece(S, off[k]);
#ifdef PT_QPROF_DEV
    uint32_t qp[5];
    q_exec(S, q, C, stk, r, qp);
#else
    q_exec(S, q, C, stk, r);
#endif
}

// One aux-node step only (a lane whose next step is an aux node: phase Q_AUX, node
// not a leaf); the decisions a pass end leaves are resolved as in q_exec.
template <class Mem>
PT_HD void q_aux_step(const SceneView& S, Query& q, QCounts& C, Mem& stk) {
    const uint32_t b = S.o_aux + q.node * (uint32_t)(PT_AUXW * sizeof(AuxSL));
    F4 r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = blob_piece(S, b + 16u * (uint32_t)k);
    q_exec_aux(S, q, C, stk, r);
    if (q.phase == Q_DECIDE) q_decide(q);
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
PT_HD int q_run(const SceneView& S, const Ray& ray, Stack& stk, Hit& out, QCounts& C, uint32_t& exact_used) {
    Query q;
    float P;
    int pid;
    q_planes(S, ray, P, pid);
    C.planes += S.n_planes;
    q_init(S, ray, P, pid, q);
    while (q.phase == Q_AUX || q.phase == Q_REPLAY) q_step(S, q, C, stk);
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
