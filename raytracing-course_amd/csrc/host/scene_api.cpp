// scene_api.cpp -- Scene::Load / InitScene equivalents (pt_scene_*): the parse
// (scene_load.cpp), the reference BVH (bvh_build.cpp), the auxiliary BVHs
// (aux_bvh.cpp), and the device layouts built from them: node and primitive
// records, ancestor lists, leaf hit regions and the one query blob the kernels read.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <array>
#include <cmath>
#include <fstream>
#include <stdexcept>
#include "api_internal.h"

namespace pti {

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

}  // namespace

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

}  // namespace pti

using namespace pti;

extern "C" {

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
        // PT_TUNE prepstats=1 (or PT_STATS=3): per-stage times on stderr
        const bool stats = tune_int("prepstats", 0) != 0 || stats_level() >= 3;
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

}  // extern "C"
