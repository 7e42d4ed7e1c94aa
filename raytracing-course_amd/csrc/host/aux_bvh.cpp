// aux_bvh.cpp -- auxiliary spatial BVH over the reference tree's LEAF boxes.
//
// Used only to enumerate, per ray, the reference leaves whose box the ray's
// line meets (the "candidates"); the exact reference traversal is then
// replayed over those candidates alone (pt_trace.h: bvh_replay).  Its boxes
// are the reference leaf boxes inflated outward (relative + absolute margin)
// so that the fast, inverse-direction box test is conservative with respect
// to the reference's exact center/half-size slab test; every candidate is
// re-checked with that exact test before it is used.
//
// Build: binned SAH (32 bins) over the own-box and hit-region centroids, BVH2,
// one reference leaf per auxiliary leaf slot, nodes in DFS preorder.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <stdexcept>
#include <vector>

#include "pt_scene.h"

namespace pth {
namespace {

struct Box {
    float lo[3], hi[3];
};

inline void grow(Box& b, const Box& o) {
    for (int a = 0; a < 3; ++a) {
        b.lo[a] = std::min(b.lo[a], o.lo[a]);
        b.hi[a] = std::max(b.hi[a], o.hi[a]);
    }
}
inline Box empty_box() {
    Box b;
    for (int a = 0; a < 3; ++a) { b.lo[a] = INFINITY; b.hi[a] = -INFINITY; }
    return b;
}
inline float area(const Box& b) {
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    if (!(dx >= 0.f)) return 0.f;
    return dx * dy + dx * dz + dy * dz;
}
// outward inflation: |x| * 2^-16 + 2^-17 (~1.5e-5 relative, 7.6e-6 absolute)
inline float down(float x) { return (float)((double)x - fabs((double)x) * 1.52587890625e-05 - 7.62939453125e-06); }
inline float up(float x) { return (float)((double)x + fabs((double)x) * 1.52587890625e-05 + 7.62939453125e-06); }

struct Builder {
    std::vector<Box> box;        // per item (reference leaf)
    std::vector<Box> reg;        // per item: where its primitives can be hit (its own box when unbounded)
    std::vector<float> cen[6];   // centroids of box (0-2) and reg (3-5)
    std::vector<uint32_t> item;  // reference leaf node index per item
    std::atomic<uint32_t> max_depth{0};

    static void set_child(pt::AuxNode& n, int k, const Box& b, uint32_t code) {
        float* f = reinterpret_cast<float*>(&n);
        // layout: a = {c0.lo.xyz, c0.hi.x}, b = {c0.hi.yz, c1.lo.xy}, c = {c1.lo.z, c1.hi.xyz}, d = {code0, code1, -, -}
        if (k == 0) {
            f[0] = b.lo[0]; f[1] = b.lo[1]; f[2] = b.lo[2]; f[3] = b.hi[0]; f[4] = b.hi[1]; f[5] = b.hi[2];
        } else {
            f[6] = b.lo[0]; f[7] = b.lo[1]; f[8] = b.lo[2]; f[9] = b.hi[0]; f[10] = b.hi[1]; f[11] = b.hi[2];
        }
        uint32_t* u = reinterpret_cast<uint32_t*>(&n);
        u[12 + k] = code;
    }

    // returns the child code of the subtree over items [b, e) and its bounds; its
    // nodes go to `out` in preorder (codes local to `out`).  Subtrees work on
    // disjoint item ranges: a large one's first half is built on another thread
    // into its own vector and spliced in front of the second (same preorder).
    uint32_t build(uint32_t b, uint32_t e, Box& bounds, uint32_t depth, std::vector<pt::AuxNode>& out, int spawn) {
        bounds = empty_box();
        for (uint32_t i = b; i < e; ++i) grow(bounds, box[i]);
        if (e - b == 1) return 0x80000000u | item[b];
        for (uint32_t m = max_depth.load(); m < depth + 1 && !max_depth.compare_exchange_weak(m, depth + 1);) {
        }
        // binned SAH over six split axes, the own-box and the hit-region centroids.
        // A subtree is entered when the ray crosses both its unions (pt_query.h
        // PT_LEAF_MARGIN), so a side's cost is its count x area(own)^0.6 x
        // area(region)^0.4 (aux visits per query on c3: own area alone 5.31,
        // exponent 0.2 / 0.3 / 0.4 / 0.5 / 0.6 on the region: 5.17 / 5.08 / 5.04 /
        // 5.17 / 5.90; area sum 6.29, minimum 5.31)
        constexpr int naxes = 6;
        float clo[6], chi[6];
        for (int a = 0; a < naxes; ++a) { clo[a] = INFINITY; chi[a] = -INFINITY; }
        for (uint32_t i = b; i < e; ++i)
            for (int a = 0; a < naxes; ++a) { clo[a] = std::min(clo[a], cen[a][i]); chi[a] = std::max(chi[a], cen[a][i]); }
        constexpr int NB = 32;
        auto measure = [](const Box& x, const Box& y) -> float { return powf(area(x), 0.6f) * powf(area(y), 0.4f); };
        float best_cost = INFINITY;
        int best_axis = -1, best_split = 0;
        for (int a = 0; a < naxes; ++a) {
            const float ext = chi[a] - clo[a];
            if (!(ext > 0.f)) continue;
            Box bb[NB], rb[NB];
            uint32_t cnt[NB] = {0};
            for (int k = 0; k < NB; ++k) bb[k] = rb[k] = empty_box();
            const float sc = NB / ext;
            for (uint32_t i = b; i < e; ++i) {
                int k = (int)((cen[a][i] - clo[a]) * sc);
                k = std::min(std::max(k, 0), NB - 1);
                grow(bb[k], box[i]);
                grow(rb[k], reg[i]);
                cnt[k]++;
            }
            Box lb[NB], lr[NB];
            uint32_t lc[NB];
            Box acc = empty_box(), accr = empty_box();
            uint32_t c = 0;
            for (int k = 0; k < NB; ++k) { grow(acc, bb[k]); grow(accr, rb[k]); c += cnt[k]; lb[k] = acc; lr[k] = accr; lc[k] = c; }
            acc = empty_box();
            accr = empty_box();
            c = 0;
            for (int k = NB - 1; k >= 1; --k) {
                grow(acc, bb[k]);
                grow(accr, rb[k]);
                c += cnt[k];
                // (an empty bin k - 1 gives the same partition as split k - 1)
                if (lc[k - 1] == 0 || c == 0 || cnt[k - 1] == 0) continue;
                const float cost = measure(lb[k - 1], lr[k - 1]) * (float)lc[k - 1] + measure(acc, accr) * (float)c;
                if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = k; }
            }
        }
        uint32_t mid;
        if (best_axis < 0) {
            mid = b + (e - b) / 2;  // all centroids coincide: median split by index
        } else {
            const float ext = chi[best_axis] - clo[best_axis];
            const float sc = NB / ext;
            uint32_t i = b, j = e;
            while (i < j) {
                int k = (int)((cen[best_axis][i] - clo[best_axis]) * sc);
                k = std::min(std::max(k, 0), NB - 1);
                if (k < best_split) { ++i; continue; }
                --j;
                std::swap(box[i], box[j]);
                std::swap(reg[i], reg[j]);
                std::swap(item[i], item[j]);
                for (int a = 0; a < 6; ++a) std::swap(cen[a][i], cen[a][j]);
            }
            mid = i;
            if (mid == b || mid == e) mid = b + (e - b) / 2;
        }
        const uint32_t self = (uint32_t)out.size();
        out.emplace_back();
        Box b0, b1;
        uint32_t c0, c1;
        if (spawn > 0 && e - b >= 8192u) {
            std::vector<pt::AuxNode> v0, v1;
            std::thread t([&] { c0 = build(b, mid, b0, depth + 1, v0, spawn - 1); });
            c1 = build(mid, e, b1, depth + 1, v1, spawn - 1);
            t.join();
            const auto splice = [&out](const std::vector<pt::AuxNode>& v, uint32_t code) {
                const uint32_t off = (uint32_t)out.size();
                for (pt::AuxNode n : v) {
                    uint32_t* u = reinterpret_cast<uint32_t*>(&n);
                    for (int k = 12; k < 14; ++k)
                        if (!(u[k] & 0x80000000u)) u[k] += off;   // internal child (0xFFFFFFFF has the bit)
                    out.push_back(n);
                }
                return (code & 0x80000000u) ? code : code + off;
            };
            c0 = splice(v0, c0);
            c1 = splice(v1, c1);
        } else {
            c0 = build(b, mid, b0, depth + 1, out, 0);
            c1 = build(mid, e, b1, depth + 1, out, 0);
        }
        set_child(out[self], 0, b0, c0);
        set_child(out[self], 1, b1, c1);
        return self;
    }
};

}  // namespace

void build_aux_bvh(const std::vector<HNode>& nodes, const std::vector<float>& regions, std::vector<pt::AuxNode>& out,
                   uint32_t& max_depth) {
    out.clear();
    Builder B;
    for (uint32_t i = 0; i < (uint32_t)nodes.size(); ++i) {
        const HNode& n = nodes[i];
        if (n.left != 0xFFFFFFFFu) continue;
        Box bx, rg;
        for (int a = 0; a < 3; ++a) { bx.lo[a] = down(n.mn[a]); bx.hi[a] = up(n.mx[a]); }
        rg = bx;
        if (6ull * i + 5 < regions.size() && regions[6ull * i] <= regions[6ull * i + 3])
            for (int a = 0; a < 3; ++a) { rg.lo[a] = regions[6ull * i + a]; rg.hi[a] = regions[6ull * i + 3 + a]; }
        B.box.push_back(bx);
        B.reg.push_back(rg);
        for (int a = 0; a < 3; ++a) {
            B.cen[a].push_back(0.5f * (bx.lo[a] + bx.hi[a]));
            B.cen[3 + a].push_back(0.5f * (rg.lo[a] + rg.hi[a]));
        }
        B.item.push_back(i);
    }
    if (B.item.empty()) throw std::runtime_error("no BVH leaves");
    Box root;
    if (B.item.size() == 1) {
        pt::AuxNode n;
        memset(&n, 0, sizeof(n));
        Builder::set_child(n, 0, B.box[0], 0x80000000u | B.item[0]);
        Builder::set_child(n, 1, empty_box(), 0xFFFFFFFFu);
        out.push_back(n);
        max_depth = 1;
        return;
    }
    // subtrees of >= 8192 items fork down to depth 4 (at most 16 threads)
    B.build(0, (uint32_t)B.item.size(), root, 0, out, 4);
    max_depth = B.max_depth;
}

}  // namespace pth

namespace pth {

// Stackless preorder form of the auxiliary BVH (pt_query.h AuxSL): every node
// carries its own box and the index one past its subtree (skip link).
// Internal boxes are the inflated (conservative) child boxes of the pair
// tree; leaves carry the reference leaf's exact (center, half-size) record,
// so the query's leaf test IS the reference slab test.
void build_aux_stackless(const std::vector<pt::AuxNode>& pairs, const std::vector<pt::Node>& dnodes,
                         std::vector<pt::AuxSL>& out, uint32_t& max_depth) {
    out.clear();
    max_depth = 0;
    auto child = [&](const pt::AuxNode& n, int k, float lo[3], float hi[3]) {
        const float* f = reinterpret_cast<const float*>(&n) + 6 * k;
        for (int a = 0; a < 3; ++a) { lo[a] = f[a]; hi[a] = f[3 + a]; }
        return reinterpret_cast<const uint32_t*>(&n)[12 + k];
    };
    struct Item { uint32_t code; float lo[3], hi[3]; uint32_t depth; };
    // explicit preorder walk; skip links are patched when a subtree closes
    std::vector<std::pair<uint32_t, uint32_t>> open;  // (out index of internal node, depth)
    std::vector<Item> st;
    {
        Item r;
        r.code = 0;  // aux pair node 0 = root (internal unless the tree is a single leaf pair)
        float l0[3], h0[3], l1[3], h1[3];
        const uint32_t c1 = child(pairs[0], 1, l1, h1);
        child(pairs[0], 0, l0, h0);
        for (int a = 0; a < 3; ++a) {
            r.lo[a] = c1 == 0xFFFFFFFFu ? l0[a] : std::min(l0[a], l1[a]);
            r.hi[a] = c1 == 0xFFFFFFFFu ? h0[a] : std::max(h0[a], h1[a]);
        }
        r.depth = 0;
        st.push_back(r);
    }
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        // close every open internal node that is not an ancestor of this item
        while (!open.empty() && open.back().second >= it.depth) {
            const uint32_t idx = open.back().first;
            reinterpret_cast<uint32_t*>(&out[idx])[6] = (uint32_t)out.size();
            open.pop_back();
        }
        max_depth = std::max(max_depth, it.depth + 1);
        pt::AuxSL n;
        uint32_t* u = reinterpret_cast<uint32_t*>(&n);
        float* f = reinterpret_cast<float*>(&n);
        if (it.code & 0x80000000u) {
            const uint32_t leaf = it.code & 0x7fffffffu;
            const pt::Node& r = dnodes[leaf];
            f[0] = r.a.x; f[1] = r.a.y; f[2] = r.a.z; f[3] = r.a.w; f[4] = r.b.x; f[5] = r.b.y;
            u[6] = (uint32_t)out.size() + 1u;
            u[7] = leaf;
            out.push_back(n);
            continue;
        }
        f[0] = it.lo[0]; f[1] = it.lo[1]; f[2] = it.lo[2]; f[3] = it.hi[0]; f[4] = it.hi[1]; f[5] = it.hi[2];
        u[6] = 0;
        u[7] = PT_AUX_INTERNAL;
        open.emplace_back((uint32_t)out.size(), it.depth);
        out.push_back(n);
        const pt::AuxNode& p = pairs[it.code];
        for (int k = 1; k >= 0; --k) {  // push right first: left child is visited next (index + 1)
            Item c;
            c.code = child(p, k, c.lo, c.hi);
            if (c.code == 0xFFFFFFFFu) continue;
            c.depth = it.depth + 1;
            st.push_back(c);
        }
    }
    while (!open.empty()) {
        reinterpret_cast<uint32_t*>(&out[open.back().first])[6] = (uint32_t)out.size();
        open.pop_back();
    }
}

}  // namespace pth

namespace pth {

// Wide (W-ary) form of the auxiliary BVH for the wavefront query: the binary
// pair tree collapsed greedily (the child with the largest weight -- box and
// hit-region areas, below -- is replaced by its two children until W children
// or only leaves remain).
// Node n = entries [n*W, n*W + W) in the AuxSL layout; entry code:
// internal child node index, 0x80000000 | reference leaf, or 0xffffffff
// (empty); every box is the conservative inflated box of its subtree.
void build_aux_wide(const std::vector<pt::AuxNode>& pairs, const std::vector<pt::Node>& dnodes, uint32_t W,
                    std::vector<pt::AuxSL>& out, uint32_t& max_depth, uint32_t& max_stack,
                    const std::vector<float>& regions) {
    struct Ch { uint32_t code; float lo[3], hi[3]; };
    // each pair child's hit-region union (a leaf without one: its own box), bottom-up over the
    // preorder pair tree, for the collapse's weight
    const bool use_reg = !regions.empty();
    std::vector<Box> preg(use_reg ? 2 * pairs.size() : 0);
    auto child = [&](const pt::AuxNode& n, int k) {
        Ch c;
        const float* f = reinterpret_cast<const float*>(&n) + 6 * k;
        for (int a = 0; a < 3; ++a) { c.lo[a] = f[a]; c.hi[a] = f[3 + a]; }
        c.code = reinterpret_cast<const uint32_t*>(&n)[12 + k];
        return c;
    };
    if (use_reg) {
        for (size_t n = pairs.size(); n-- > 0;) {
            for (int k = 0; k < 2; ++k) {
                const Ch c = child(pairs[n], k);
                Box r = empty_box();
                if (c.code == 0xFFFFFFFFu) {
                } else if (c.code & 0x80000000u) {
                    const size_t i = 6ull * (c.code & 0x7FFFFFFFu);
                    if (i + 5 < regions.size() && regions[i] <= regions[i + 3])
                        for (int a = 0; a < 3; ++a) { r.lo[a] = regions[i + a]; r.hi[a] = regions[i + 3 + a]; }
                    else
                        for (int a = 0; a < 3; ++a) { r.lo[a] = c.lo[a]; r.hi[a] = c.hi[a]; }
                } else {
                    if (c.code <= n || c.code >= pairs.size()) throw std::runtime_error("aux pair tree: child before its parent");
                    r = preg[2 * c.code];
                    grow(r, preg[2 * c.code + 1]);
                }
                preg[2 * n + k] = r;
            }
        }
    }
    // the collapse opens the child a ray is likeliest to enter: the split cost's measure
    // (area(own)^0.6 x area(region)^0.4, build_aux_bvh), or the own box's area alone (no
    // regions).  tools/aux_quality.py on c3 (24 windows of 32x32, 2 spp, 202 k queries): aux
    // visits per query 4.754 by own area, 4.710 by the measure (region exponent 0.1 / 0.25 /
    // 0.55 / 0.7 / 1: 4.733 / 4.717 / 4.749 / 4.789 / 5.397; an optimal collapse under the same
    // cost, a dynamic program over the pair tree, 4.714: the greedy one is kept)
    auto weight = [&](const Ch& c) {
        const float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
        const float own = dx * dy + dx * dz + dy * dz;
        if (!use_reg) return own;
        const Box& r = preg[2 * c.code];
        Box u = r;
        grow(u, preg[2 * c.code + 1]);
        return powf(own, 0.6f) * powf(area(u), 0.4f);
    };
    out.clear();
    max_depth = 0;
    // BFS over wide nodes: (pair-tree internal code, wide node index, depth)
    std::vector<std::pair<uint32_t, uint32_t>> todo;  // pair node code -> wide node index
    std::vector<uint32_t> depth_of;
    out.resize(W);
    depth_of.push_back(1);
    todo.emplace_back(0u, 0u);
    for (size_t qi = 0; qi < todo.size(); ++qi) {
        const uint32_t pc = todo[qi].first, wn = todo[qi].second;
        std::vector<Ch> ch;
        ch.push_back(child(pairs[pc], 0));
        const Ch c1 = child(pairs[pc], 1);
        if (c1.code != 0xFFFFFFFFu) ch.push_back(c1);
        for (;;) {
            if (ch.size() >= W) break;
            int best = -1;
            float ba = -1.f;
            for (int k = 0; k < (int)ch.size(); ++k)
                if (!(ch[k].code & 0x80000000u) && weight(ch[k]) > ba) { ba = weight(ch[k]); best = k; }
            if (best < 0) break;
            const pt::AuxNode& p = pairs[ch[best].code];
            const Ch a = child(p, 0), b = child(p, 1);
            ch[best] = a;
            if (b.code != 0xFFFFFFFFu) ch.push_back(b);
        }
        max_depth = std::max(max_depth, depth_of[wn]);
        for (uint32_t k = 0; k < W; ++k) {
            pt::AuxSL e;
            memset(&e, 0, sizeof(e));
            uint32_t* u = reinterpret_cast<uint32_t*>(&e);
            float* f = reinterpret_cast<float*>(&e);
            if (k >= ch.size()) {
                u[7] = 0xFFFFFFFFu;
            } else if (ch[k].code & 0x80000000u) {
                // reference leaf: its inflated (conservative) box, like an internal child;
                // the exact test of the leaf record happens in the replay's candidate step
                f[0] = ch[k].lo[0]; f[1] = ch[k].lo[1]; f[2] = ch[k].lo[2];
                f[3] = ch[k].hi[0]; f[4] = ch[k].hi[1]; f[5] = ch[k].hi[2];
                u[7] = ch[k].code;
            } else {
                f[0] = ch[k].lo[0]; f[1] = ch[k].lo[1]; f[2] = ch[k].lo[2];
                f[3] = ch[k].hi[0]; f[4] = ch[k].hi[1]; f[5] = ch[k].hi[2];
                const uint32_t nn = (uint32_t)(out.size() / W);
                out.resize(out.size() + W);
                depth_of.push_back(depth_of[wn] + 1);
                todo.emplace_back(ch[k].code, nn);
                u[7] = nn;
            }
            out[(size_t)wn * W + k] = e;
        }
    }
    // stack bound: a visit pushes at most W-1 entries beyond the one it continues with
    max_stack = (W - 1) * max_depth + 1;
}

// Reference-leaf index range of every entry's subtree, packed into the entry's
// spare word (AuxSL b.z): (max >> shift, rounded up) << 16 | (min >> shift).
// The query skips a subtree whose leaves all lie below the pass's lower bound
// (already processed in an earlier pass), or -- with its candidate list full --
// all lie above the list's largest kept candidate (flagging another pass), so a
// ray with many candidates does not re-walk the whole aux tree in every pass.
void annotate_aux_ranges(std::vector<pt::AuxSL>& out, uint32_t W, uint32_t n_ref_nodes, uint32_t& shift) {
    shift = 0;
    const uint64_t top = n_ref_nodes ? n_ref_nodes - 1u : 0u;
    while (((top + (1ull << shift) - 1) >> shift) > 0xffffull) ++shift;
    const size_t nn = out.size() / W;
    std::vector<uint32_t> lo(nn, 0xFFFFFFFFu), hi(nn, 0u);
    for (size_t n = nn; n-- > 0;) {
        for (uint32_t k = 0; k < W; ++k) {
            uint32_t* u = reinterpret_cast<uint32_t*>(&out[n * W + k]);
            const uint32_t code = u[7];
            if (code == 0xFFFFFFFFu) continue;
            uint32_t mn, mx;
            if (code & 0x80000000u) {
                mn = mx = code & 0x7FFFFFFFu;
            } else {
                if (code <= n || code >= nn) throw std::runtime_error("aux wide tree: child before its parent");
                mn = lo[code];
                mx = hi[code];
            }
            lo[n] = std::min(lo[n], mn);
            hi[n] = std::max(hi[n], mx);
            const uint32_t mxq = (uint32_t)(((uint64_t)mx + (1ull << shift) - 1) >> shift);
            u[6] = (mxq << 16) | (mn >> shift);
        }
    }
}

}  // namespace pth
