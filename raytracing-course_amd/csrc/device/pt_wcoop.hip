// pt_wcoop.hip -- the cooperative engine k_wcoop: at the end of a pass,
// and beside the low-chain path rounds, a TEAM of lanes per remaining chain runs the
// closest-hit query (pt_coop.h's algorithm) and the team's first lane shades.
#include "pt_wave.h"

namespace pt {

// ---- cooperative engine (end of a pass) ---------------------------------------
// k_wcoop<T>: a TEAM of T lanes per pixel chain (64/T chains per wave), run to the
// end of the pass.  With few chains left, the path engine's lanes idle while every
// chain waits on its own long sequence of dependent steps and ring hand-offs; here
// a chain's query is spread over its team's lanes (pt_coop.h: breadth-first aux
// expansion, every candidate leaf and its primitives at once, root paths a block
// of nodes per round) and the team's first lane shades the result itself, with
// the pixel's state in registers and its fold records in LDS for the chain's
// whole life, so nothing waits in a ring.  The teams of a wave run their chain
// cycles in step (query, then shading), so one instruction stream shades 64/T
// chains.
enum : uint32_t { QH_IDX = 0u, QH_T, QH_LID, QH_NX, QH_NY, QH_NZ, QH_IN, QH_INFO, QH_N };
template <uint32_t T>
struct QcTeamLds {
    // aux stack words per chain (also the leader's exact DFS stack): a whole-wave team's own;
    // smaller teams share their wave's pool (QcPoolLds), SCAP words per chain
    // (teams of 4: 64, so that their wave's pool -- 16 chains -- stays at 1,024 words)
    static constexpr uint32_t SCAP = T == 64u ? 448u : T == 32u ? 192u : T == 4u ? 64u : QC_SCAP_MIN;
    static constexpr uint32_t CCAP = 5u * T;                    // candidates (< T + 4 T at any time)
    static constexpr uint32_t HCAP = T >= 32u ? 32u : T == 16u ? 16u : T == 8u ? 12u : 8u;   // hitting leaves per
                                    // query (more: the exact DFS); LDS fits 3 WGs per CU (teams of 4: 2)
    uint32_t stk[T == 64u ? SCAP : 1u];
    uint32_t cand[T == 64u ? CCAP : 1u];
    uint32_t hl[QH_N][HCAP];       // hitting leaves: index, first-min t, its prim, hit normal and side,
                                   // ancestor-list info
    uint32_t perm[HCAP];           // their preorder: perm[k] = the entry of the k-th smallest index
    uint32_t r_idx[HCAP], r_t[HCAP];   // entered hits so far (preorder)
    Shade fold_sh[QC_FOLD];        // the chain's fold records: the vertex prim's shading record ...
    uint4 fold[QC_FOLD];           // ... and {idm, s1, s2, -}
    uint4 sum;                     // the pixel's sum.rgb and global index (rec[2 slot + 1]) while the team
                                   // owns it (touched at path ends only: registers would spill)
};
// per wave, teams of T < 64 (qc_pool): the chains' pending aux nodes and candidate
// leaves, (chain << SH | node / leaf ordinal) items, and each chain's ray
template <uint32_t T>
struct QcPoolLds {
    static constexpr uint32_t CPW = 64u / T;                    // chains per wave
    static constexpr uint32_t SH = CPW > 8u ? 28u : 29u;        // item = chain << SH | node (host: nodes < 2^SH)
    static constexpr uint32_t MASK = (1u << SH) - 1u;
    static constexpr uint32_t SW = QcTeamLds<T>::SCAP * CPW;    // pending nodes (chain c's exact DFS stack after
                                                                // the query: words [c SCAP, (c + 1) SCAP))
    static constexpr uint32_t CW = 128u;                        // candidates (< 64 + 64 at any time)
    uint32_t stk[SW];
    uint32_t cand[CW];
    F4 ray[CPW][4];                // {o.xyz, pre.w}, {d.xyz, -}, {1/d}, {o / d}
    uint32_t nh[CPW];              // hitting leaves found (may pass HCAP: then the exact DFS)
    uint32_t ovf[CPW];             // the chain takes the exact DFS (its items are skipped)
};
template <>
struct QcPoolLds<64u> {
    uint32_t unused;
};
// per workgroup: the records every chain cycle reads, copied once per launch
struct QcScene {
    Prim pl[QC_NPL];               // planes (q_planes order) and their prim indices
    Prim em[QC_NEM];               // emitters
    AuxSL top[QC_TOPN * PT_AUXW];  // aux nodes 0..QC_TOPN-1
    uint32_t pl_id[QC_NPL];
};
// the first QC_NPL planes / QC_NEM emitters from the LDS copy, any further ones
// (BIG: a scene beyond the tables) from HBM
template <bool BIG>
struct PlanesLds {
    const QcScene& Q;
    const SceneView& S;
    __device__ Prim operator()(uint32_t k, uint32_t& pi) const {
        if (!BIG || k < QC_NPL) {
            pi = Q.pl_id[k];
            return Q.pl[k];
        }
        pi = S.planes[k];
        return S.prims[pi];
    }
};
template <bool BIG>
struct EmitLds {
    const QcScene& Q;
    const SceneView& S;
    __device__ Prim operator()(uint32_t k) const { return !BIG || k < QC_NEM ? Q.em[k] : S.prims[S.emitters[k]]; }
};

// bvh_prim_intersect from the compact record (pt_query.h): a plain triangle (pos = +0,
// rotation exactly (0,0,0,1)) is tested on the world ray -- the world->local transform
// changes at most the sign of zero components, which changes neither the decision nor
// t, nor the sign of dn that picks the normal's side (pt_query.h probe) -- and its
// normal goes through the same last step, normalize(qrot(rotation, n)), so the Hit
// has the full test's bits; other records expand to the full form.
__device__ __forceinline__ bool qc_prim_hit_rec(const SceneView& S, uint32_t i, F4 r0, F4 r1, F4 r2, F4 r3,
                                                const Ray& ray, Hit& h) {
    const uint32_t ty = f2u(r0.w);
    if (ty == T_TRIANGLE) {
        if (!isect_triangle_n(ray, mk3(r0.x, r0.y, r0.z), mk3(r1.x, r1.y, r1.z), mk3(r2.x, r2.y, r2.z),
                              mk3(r1.w, r2.w, r3.x), h))
            return false;
        q4 q;
        q.x = 0.f; q.y = 0.f; q.z = 0.f; q.w = 1.f;
        h.n = normalize(qrot(q, h.n));
        return true;
    }
    if (ty & PT_QP_FULL) return bvh_prim_intersect(S.prims[i], ray, h);
    return bvh_prim_intersect(qprim_expand(r0, r1, r2), ray, h);
}
__device__ __forceinline__ bool qc_prim_hit(const SceneView& S, uint32_t i, const Ray& ray, Hit& h) {
    const uint32_t o = S.o_qprim + PT_QPRIM_BYTES * i;
    return qc_prim_hit_rec(S, i, blob_piece(S, o), blob_piece(S, o + 16u), blob_piece(S, o + 32u),
                           blob_piece(S, o + 48u), ray, h);
}

// k_wcoop's work counters: per wave in LDS, one LDS add per wave and counting site (a
// lane-private counter costs a VGPR for the kernel's life; the engine sits at the
// 3-waves-per-SIMD limit)
// (no plane-test counter: every counted ray tests every plane, so the plane tests are the
// rays x n_planes, formed in 64 bits at the end -- a 32-bit LDS count of them could wrap)
enum : uint32_t { LC_RAYS = 0u, LC_NODES, LC_PTESTS, LC_YIELD, LC_AUX, LC_FALLB, LC_HANDED, LC_N = 8u };
__device__ __forceinline__ void lc_add(uint32_t* lc, uint32_t k, bool c, uint32_t w = 1u) {
    const unsigned long long m = __ballot(c);
    if (m && lane_id() == (uint32_t)__ffsll((long long)m) - 1u) atomicAdd(lc + k, (uint32_t)__popcll(m) * w);
}

#ifdef PT_CPROF
// diagnostics build: per-phase shader cycles of the cooperative engine (summed per wave)
#define QC_T0() uint64_t qc_t = __builtin_amdgcn_s_memtime()
#define QC_TICK(i) do { const uint64_t n_ = __builtin_amdgcn_s_memtime(); cp[i] += n_ - qc_t; qc_t = n_; } while (0)
#define QC_CP_ARG , uint64_t* cp
#define QC_CP_PASS , cp
#else
#define QC_T0() (void)0
#define QC_TICK(i) (void)0
#define QC_CP_ARG
#define QC_CP_PASS
#endif

// Phases 3-5 of the query, per team (team-uniform arguments; dec = this team decides):
// the hitting leaves L.hl[0, nh) in reference preorder, each decided on its root path
// with the bound the recursion carries there; the result as qc_team's.
template <uint32_t T>
__device__ __forceinline__ int qc_decide(const SceneView& S, QcTeamLds<T>& L, bool on, bool dec, uint32_t nh,
                                         const Ray& ray, float P, int pid, uint32_t* lc, Hit& hit,
                                         bool& bvh QC_CP_ARG) {
    QC_T0();
    const uint32_t lane = lane_id(), tl = lane % T, tbase = lane - tl;
    const unsigned long long tmask = T == 64u ? ~0ull : (((1ull << T) - 1ull) << tbase);
    // 3. the hitting leaves in reference preorder (distinct indices: rank = count below)
    for (uint32_t i0 = 0;; i0 += T) {
        const bool srt = dec && i0 < nh;
        if (__ballot(srt) == 0ull) break;
        const bool act = srt && i0 + tl < nh;
        const uint32_t c = act ? L.hl[QH_IDX][i0 + tl] : 0u;
        uint32_t rank = 0u;
        for (uint32_t j = 0; __ballot(srt && j < nh) != 0ull; ++j)
            if (srt && j < nh) rank += L.hl[QH_IDX][j] < c ? 1u : 0u;
        if (act) L.perm[rank] = i0 + tl;
    }
    // 4. decide them in order: lane j of the team holds nodes j, j + T, ... of the
    //    leaf's root path with their exact slab results (the reference's division form)
    constexpr uint32_t NB = 64u / T;            // path blocks (a root path has at most 63 nodes)
    constexpr uint32_t NG = NB < 4u ? NB : 4u;  // blocks loaded together
    uint32_t nrec = 0u;
    float bt = PT_INF;
    int res = pid, resk = -1;
    for (uint32_t kk = 0;; ++kk) {
        const bool dk = dec && kk < nh;
        if (__ballot(dk) == 0ull) break;
        const uint32_t ke = dk ? L.perm[kk] : 0u;   // the kk-th hitting leaf in preorder
        const uint32_t info = dk ? L.hl[QH_INFO][ke] : 0u;
        const uint32_t off = info & 0x03ffffffu, len = dk ? info >> 26 : 0u;
        float carry = P;          // the bound at the previous block's last node
        uint32_t vlast = 0u;      // that node
        bool fail = false;
        for (uint32_t g = 0; g < NB; g += NG) {
            if (__ballot(g * T < len) == 0ull) break;
            uint32_t v[NG], hf[NG];
            float tq[NG];
#pragma unroll
            for (uint32_t b = 0; b < NG; ++b) {
                const uint32_t j = (g + b) * T + tl;
                v[b] = j < len ? S.anc[off + j] : 0u;
            }
#pragma unroll
            for (uint32_t b = 0; b < NG; ++b) {
                const bool pon = (g + b) * T + tl < len;
                const Node nd = S.nodes[v[b]];
                float t = 0.f;
                uint32_t in = 0u;
                const bool hs = pon && node_slab(nd, ray, t, in);
                tq[b] = t;
                hf[b] = (hs ? 1u : 0u) | (in << 1);
                lc_add(lc, LC_NODES, pon);
            }
#pragma unroll
            for (uint32_t b = 0; b < NG; ++b) {
                if (__ballot((g + b) * T < len) == 0ull) break;
                const uint32_t j = (g + b) * T + tl;
                const bool pon = j < len;
                const uint32_t up = __shfl(v[b], (int)(lane == 0u ? 0u : lane - 1u), 64);
                const uint32_t prev = tl == 0u ? vlast : up;
                // the carried bound: at a right child the minimum over the entered hits of its
                // left sibling's subtree (prev, v), if any; else the parent's (scan down the path)
                const bool rc = pon && j > 0u && v[b] != prev + 1u;
                float m = 0.f;
                bool any = false;
                for (uint32_t r = 0; __ballot(r < nrec) != 0ull; ++r) {
                    if (r < nrec) {
                        const uint32_t ri = L.r_idx[r];
                        const float rt = u2f(L.r_t[r]);
                        if (rc && ri > prev && ri < v[b]) {
                            if (!any || rt < m) m = rt;
                            any = true;
                        }
                    }
                }
                const unsigned long long dm = __ballot(any) & tmask;
                const unsigned long long below = dm & ((2ull << lane) - 1ull);
                const int src = below ? 63 - __clzll((long long)below) : (int)lane;
                const float mb = __shfl(m, src, 64);
                const float bound = below ? mb : carry;
                // src/bvh.cpp:188-198: slab miss, or pruned by the bound (not interior)
                const bool ok = !pon || ((hf[b] & 1u) && !(bound < tq[b] && !(hf[b] & 2u)));
                fail = fail || (__ballot(!ok) & tmask) != 0ull;
                carry = __shfl(bound, (int)(tbase + T - 1u), 64);
                vlast = __shfl(v[b], (int)(tbase + T - 1u), 64);
            }
        }
        if (dk && !fail) {
            // 5. entered: record; first strict minimum; replaces the plane iff closer
            const float lt = u2f(L.hl[QH_T][ke]);
            if (tl == 0u) {
                L.r_idx[nrec] = L.hl[QH_IDX][ke];
                L.r_t[nrec] = f2u(lt);
            }
            ++nrec;
            if (lt < bt) {
                bt = lt;
                if (lt < P) {
                    res = (int)L.hl[QH_LID][ke];
                    resk = (int)ke;
                }
            }
        }
    }
    QC_TICK(2);
    if (resk >= 0) {
        bvh = true;
        hit.t = u2f(L.hl[QH_T][resk]);
        hit.n = mk3(u2f(L.hl[QH_NX][resk]), u2f(L.hl[QH_NY][resk]), u2f(L.hl[QH_NZ][resk]));
        hit.interior = L.hl[QH_IN][resk];
    }
    return on ? res : -1;
}

// The query of one ray per team (every argument team-uniform; `on` = this team has
// a query).  `reserve` = 3 (aux depth + 2): above SCAP - reserve pending nodes the
// expansion takes fewer nodes per round, so a depth-first descent still fits.
// Returns the closest prim (-1 none) and, for a BVH result, `hit` = its intersection
// (t, n, side, from the same bvh_prim_intersect the consumer would repeat); `bvh`
// tells which.  `exact` set = hand the ray to the exact DFS.
template <uint32_t T>
__device__ int qc_team(const SceneView& S, const QcScene& Q, QcTeamLds<T>& L, bool on, const Ray& ray, float P,
                       int pid, F4 pre, uint32_t reserve, uint32_t* lc, bool& exact, Hit& hit, bool& bvh QC_CP_ARG) {
    QC_T0();
    constexpr uint32_t SCAP = QcTeamLds<T>::SCAP, HCAP = QcTeamLds<T>::HCAP;
    const uint32_t lane = lane_id(), tl = lane % T, tbase = lane - tl;
    const unsigned long long tmask = T == 64u ? ~0ull : (((1ull << T) - 1ull) << tbase);
    bvh = false;
    const uint32_t slim = SCAP - reserve;
    exact = on && pre.w != pre.w;
    const bool run = on && !exact;
    const bool par = signbit(pre.w);
    const f3 inv = mk3(pre.x, pre.y, pre.z);
    const f3 oinv = mk3(ray.o.x * inv.x, ray.o.y * inv.y, ray.o.z * inv.z);
    uint32_t ns = run ? 1u : 0u, nc = 0u, nh = 0u;
    bool ovf = false;
    if (tl == 0u && run) L.stk[0] = 0u;
    for (;;) {
        // 2. candidate leaves, T at a time (the rest once the expansion is over):
        //    bound-free slab test, then the first strict minimum over the primitives;
        //    the leaf's ancestor-list info is fetched alongside its record
        for (;;) {
            const bool want = run && !ovf && (nc >= T || (ns == 0u && nc > 0u));
            if (__ballot(want) == 0ull) break;
            QC_TICK(0);
            const uint32_t take = want ? (nc < T ? nc : T) : 0u;
            nc -= take;
            const bool act = tl < take;
            // a candidate is its leaf's bundle (pt_query.h: the leaf's node box, its primitive
            // range and its first primitive's compact record): the slab test and the first
            // primitive's test take one round of independent loads
            const uint32_t ord = act ? L.cand[nc + tl] : 0u;
            const uint32_t bo = S.o_bundle + PT_BUNDLE_BYTES * ord;
            const F4 b0 = blob_piece(S, bo), b1 = blob_piece(S, bo + 16u), b2 = blob_piece(S, bo + 32u),
                     b3 = blob_piece(S, bo + 48u), b4 = blob_piece(S, bo + 64u), b5 = blob_piece(S, bo + 80u);
            const uint32_t c = f2u(b3.x);          // the reference leaf
            const uint32_t ainfo = act ? S.anc_info[c] : 0u;
            Node nd;
            nd.a = b4;                             // the leaf's node record: {c.xyz, s.x}, {s.y, s.z, first, count}
            nd.b = F4{b5.x, b5.y, b3.y, b3.z};
            lc_add(lc, LC_NODES, act);
            const bool hb = act && qc_slab_hit(nd, ray, inv, par);
            const uint32_t ref = f2u(b3.y), cnt = hb ? f2u(b3.z) : 0u;
            Hit best;
            best.t = PT_INF;
            best.n = mk3(0.f, 0.f, 0.f);
            best.interior = 0u;
            int lid = -1;
            lc_add(lc, LC_PTESTS, cnt != 0u);
            if (cnt) {
                Hit hh;
                if (qc_prim_hit_rec(S, ref, b0, b1, b2, F4{b3.w, 0.f, 0.f, 0.f}, ray, hh)) { best = hh; lid = (int)ref; }
            }
            for (uint32_t i = 1; __ballot(i < cnt) != 0ull; ++i) {
                lc_add(lc, LC_PTESTS, i < cnt);
                if (i < cnt) {
                    Hit hh;
                    if (qc_prim_hit(S, ref + i, ray, hh) && hh.t < best.t) { best = hh; lid = (int)(ref + i); }
                }
            }
            const unsigned long long m = __ballot(lid >= 0) & tmask;
            const uint32_t nm = (uint32_t)__popcll(m);
            if (want) {
                if (nh + nm > HCAP) {
                    ovf = true;
                } else if (lid >= 0) {
                    const uint32_t j = nh + lanes_below(m);
                    L.hl[QH_IDX][j] = c;
                    L.hl[QH_T][j] = f2u(best.t);
                    L.hl[QH_LID][j] = (uint32_t)lid;
                    L.hl[QH_NX][j] = f2u(best.n.x);
                    L.hl[QH_NY][j] = f2u(best.n.y);
                    L.hl[QH_NZ][j] = f2u(best.n.z);
                    L.hl[QH_IN][j] = best.interior;
                    L.hl[QH_INFO][j] = ainfo;
                }
                nh += nm;
            }
            QC_TICK(1);
        }
        const bool expand = run && !ovf && ns > 0u;
        if (__ballot(expand) == 0ull) break;
        uint32_t k = slim > ns ? (slim - ns) / 3u : 0u;
        k = k < 1u ? 1u : k;
        // 1. breadth-first expansion of the wide aux BVH: QC_EPL nodes per PT_AUXW team
        //    lanes, a lane per entry of each (a round's instructions test QC_EPL entries,
        //    their loads issued together: the round's latency is one load's)
        constexpr uint32_t KN = T / PT_AUXW * QC_EPL;
        k = k > KN ? KN : k;
        k = k > ns ? ns : k;
        if (!expand) k = 0u;
        if (ns + 3u * k > SCAP) { ovf = true; k = 0u; }   // cannot happen with the host's reserve (checked)
        ns -= k;
        {
            const uint32_t e = tl % PT_AUXW;
            F4 ea[QC_EPL], eb[QC_EPL];
            bool act[QC_EPL];
#pragma unroll
            for (uint32_t j = 0; j < QC_EPL; ++j) {
                const uint32_t ni = tl / PT_AUXW + j * (T / PT_AUXW);
                act[j] = ni < k;
                const uint32_t node = act[j] ? L.stk[ns + ni] : 0u;
                lc_add(lc, LC_AUX, act[j] && e == 0u);
                if (node < QC_TOPN) {
                    ea[j] = Q.top[node * PT_AUXW + e].a;
                    eb[j] = Q.top[node * PT_AUXW + e].b;
                } else {
                    const uint32_t b = S.o_aux + (node * PT_AUXW + e) * (uint32_t)sizeof(AuxSL);
                    ea[j] = blob_piece(S, b);
                    eb[j] = blob_piece(S, b + 16u);
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < QC_EPL; ++j) {
                const uint32_t code = f2u(eb[j].w);
                bool h = act[j] && code != 0xffffffffu;
                if (h) h = aux_entry_hit(ea[j], eb[j], ray, inv, oinv, pre.w);
                const bool leaf = h && (code & 0x80000000u) != 0u;
                const bool inner = h && (code & 0x80000000u) == 0u;
                const unsigned long long mi = __ballot(inner) & tmask, ml = __ballot(leaf) & tmask;
                if (inner) L.stk[ns + lanes_below(mi)] = code;
                if (leaf) L.cand[nc + lanes_below(ml)] = f2u(eb[j].z);   // (a leaf entry's range: its bundle)
                ns += (uint32_t)__popcll(mi);
                nc += (uint32_t)__popcll(ml);
            }
        }
    }
    QC_TICK(0);
    if (ovf) exact = true;
    return qc_decide<T>(S, L, on, run && !ovf, nh, ray, P, pid, lc, hit, bvh QC_CP_PASS);
}

// The query for teams of T < 64 lanes, phases 1-2 pooled over the wave: the 64/T
// chains' aux expansions share one stack of (chain, node) items and one list of
// (chain, leaf) candidates, so every round expands up to 16 pending nodes (a lane
// per entry) and tests up to 64 candidates, of whichever chains have them.  A team
// of 8 lanes alone expands 2 nodes per round, and the wave's teams run in step, so
// its rounds followed its slowest chain's work; pooled they follow the chains' sum
// (and the depth).  Which leaves are collected does not depend on the order, and the
// hitting leaves go to their team's list (L.hl, any order: qc_decide sorts them),
// so the result is qc_team's.  The lanes that take an item read its chain's ray from
// the pool (W.ray).  `reserve` as for qc_team, over the pool.
template <uint32_t T>
__device__ int qc_pool(const SceneView& S, const QcScene& Q, QcPoolLds<T>& W, QcTeamLds<T>* Lw, bool on,
                       const Ray& ray, float P, int pid, F4 pre, uint32_t reserve, uint32_t* lc, bool& exact, Hit& hit,
                       bool& bvh QC_CP_ARG) {
    QC_T0();
    constexpr uint32_t SW = QcPoolLds<T>::SW, HCAP = QcTeamLds<T>::HCAP;
    constexpr uint32_t KN = 64u / PT_AUXW;      // nodes per expansion round
    const uint32_t lane = lane_id(), tl = lane % T, team = lane / T;
    bvh = false;
    exact = on && pre.w != pre.w;
    const bool run = on && !exact;
    if (tl == 0u) {
        // the chain's ray and query set-up, for the lanes that take its items
        W.ray[team][0] = F4{ray.o.x, ray.o.y, ray.o.z, pre.w};
        W.ray[team][1] = F4{ray.d.x, ray.d.y, ray.d.z, 0.f};
        W.ray[team][2] = F4{pre.x, pre.y, pre.z, 0.f};
        W.ray[team][3] = F4{ray.o.x * pre.x, ray.o.y * pre.y, ray.o.z * pre.z, 0.f};
        W.nh[team] = 0u;
        W.ovf[team] = 0u;
    }
    // every running chain's root node
    const unsigned long long mr = __ballot(run && tl == 0u);
    if (run && tl == 0u) W.stk[lanes_below(mr)] = team << QcPoolLds<T>::SH;
    uint32_t ns = (uint32_t)__popcll(mr), nc = 0u;   // wave-uniform
    bool wovf = false;                               // the pool overflowed: every chain takes the exact DFS
    const uint32_t slim = SW - reserve;
    for (;;) {
        // 2. candidate leaves, 64 at a time (the rest once the expansion is over): the
        //    bundle's bound-free slab test and first-primitive test in one round of
        //    loads, then the leaf's further primitives
        while (nc >= 64u || (ns == 0u && nc > 0u)) {
            QC_TICK(0);
            const uint32_t take = nc < 64u ? nc : 64u;
            nc -= take;
            const uint32_t item = lane < take ? W.cand[nc + lane] : 0u;
            const uint32_t ch = item >> QcPoolLds<T>::SH;
            const bool act = lane < take && W.ovf[ch] == 0u;
            const F4 q0 = W.ray[ch][0], q1 = W.ray[ch][1], q2 = W.ray[ch][2];
            Ray ir;
            ir.o = mk3(q0.x, q0.y, q0.z);
            ir.d = mk3(q1.x, q1.y, q1.z);
            const f3 iinv = mk3(q2.x, q2.y, q2.z);
            const uint32_t ord = act ? item & QcPoolLds<T>::MASK : 0u;
            const uint32_t bo = S.o_bundle + PT_BUNDLE_BYTES * ord;
            const F4 b0 = blob_piece(S, bo), b1 = blob_piece(S, bo + 16u), b2 = blob_piece(S, bo + 32u),
                     b3 = blob_piece(S, bo + 48u), b4 = blob_piece(S, bo + 64u), b5 = blob_piece(S, bo + 80u);
            const uint32_t c = f2u(b3.x);          // the reference leaf
            const uint32_t ainfo = act ? S.anc_info[c] : 0u;
            Node nd;
            nd.a = b4;                             // the leaf's node record: {c.xyz, s.x}, {s.y, s.z, first, count}
            nd.b = F4{b5.x, b5.y, b3.y, b3.z};
            lc_add(lc, LC_NODES, act);
            const bool hb = act && qc_slab_hit(nd, ir, iinv, signbit(q0.w));
            const uint32_t ref = f2u(b3.y), cnt = hb ? f2u(b3.z) : 0u;
            Hit best;
            best.t = PT_INF;
            best.n = mk3(0.f, 0.f, 0.f);
            best.interior = 0u;
            int lid = -1;
            lc_add(lc, LC_PTESTS, cnt != 0u);
            if (cnt) {
                Hit hh;
                if (qc_prim_hit_rec(S, ref, b0, b1, b2, F4{b3.w, 0.f, 0.f, 0.f}, ir, hh)) { best = hh; lid = (int)ref; }
            }
            for (uint32_t i = 1; __ballot(i < cnt) != 0ull; ++i) {
                lc_add(lc, LC_PTESTS, i < cnt);
                if (i < cnt) {
                    Hit hh;
                    if (qc_prim_hit(S, ref + i, ir, hh) && hh.t < best.t) { best = hh; lid = (int)(ref + i); }
                }
            }
            if (lid >= 0) {
                // (distinct leaves: the list's order is free)
                const uint32_t j = atomicAdd(&W.nh[ch], 1u);
                if (j < HCAP) {
                    QcTeamLds<T>& H = Lw[ch];
                    H.hl[QH_IDX][j] = c;
                    H.hl[QH_T][j] = f2u(best.t);
                    H.hl[QH_LID][j] = (uint32_t)lid;
                    H.hl[QH_NX][j] = f2u(best.n.x);
                    H.hl[QH_NY][j] = f2u(best.n.y);
                    H.hl[QH_NZ][j] = f2u(best.n.z);
                    H.hl[QH_IN][j] = best.interior;
                    H.hl[QH_INFO][j] = ainfo;
                } else {
                    W.ovf[ch] = 1u;                // more hitting leaves than the list: the exact DFS
                }
            }
            QC_TICK(1);
        }
        if (ns == 0u) break;
        // 1. expansion: the KN most recent pending nodes (with few free words the pool
        //    is expanded depth-first, so a descent fits the reserve), a lane per entry
        uint32_t k = slim > ns ? (slim - ns) / 3u : 0u;
        k = k < 1u ? 1u : k;
        k = k > KN ? KN : k;
        k = k > ns ? ns : k;
        if (ns + 3u * k > SW) {                    // cannot happen with the host's reserve (checked)
            wovf = true;
            break;
        }
        ns -= k;
        const uint32_t ni = lane / PT_AUXW, e = lane % PT_AUXW;
        const uint32_t item = ni < k ? W.stk[ns + ni] : 0u;
        const uint32_t ch = item >> QcPoolLds<T>::SH, node = item & QcPoolLds<T>::MASK;
        const bool act = ni < k && W.ovf[ch] == 0u;
        lc_add(lc, LC_AUX, act && e == 0u);
        F4 ea, eb;
        if (node < QC_TOPN) {
            ea = Q.top[node * PT_AUXW + e].a;
            eb = Q.top[node * PT_AUXW + e].b;
        } else {
            const uint32_t bo = S.o_aux + (node * PT_AUXW + e) * (uint32_t)sizeof(AuxSL);
            ea = blob_piece(S, bo);
            eb = blob_piece(S, bo + 16u);
        }
        const F4 q0 = W.ray[ch][0], q1 = W.ray[ch][1], q2 = W.ray[ch][2], q3 = W.ray[ch][3];
        Ray ir;
        ir.o = mk3(q0.x, q0.y, q0.z);
        ir.d = mk3(q1.x, q1.y, q1.z);
        const uint32_t code = f2u(eb.w);
        bool h = act && code != 0xffffffffu;
        if (h) h = aux_entry_hit(ea, eb, ir, mk3(q2.x, q2.y, q2.z), mk3(q3.x, q3.y, q3.z), q0.w);
        const bool leaf = h && (code & 0x80000000u) != 0u;
        const bool inner = h && (code & 0x80000000u) == 0u;
        const unsigned long long mi = __ballot(inner), ml = __ballot(leaf);
        if (inner) W.stk[ns + lanes_below(mi)] = ch << QcPoolLds<T>::SH | code;
        if (leaf) W.cand[nc + lanes_below(ml)] = ch << QcPoolLds<T>::SH | f2u(eb.z);   // (a leaf entry's range: its bundle)
        ns += (uint32_t)__popcll(mi);
        nc += (uint32_t)__popcll(ml);
    }
    QC_TICK(0);
    const uint32_t nh = W.nh[team];
    const bool ovf = run && (wovf || W.ovf[team] != 0u || nh > HCAP);
    if (ovf) exact = true;
    return qc_decide<T>(S, Lw[team], on, run && !ovf, nh, ray, P, pid, lc, hit, bvh QC_CP_PASS);
}

// the chain's pixel state while a team owns it (its first lane's registers; the sum
// and the global pixel index in the team's LDS, QcTeamLds::sum)
struct CoopPixel {
    Rng R;
    uint32_t nv, done;
};

// shade_item for the cooperative engine (a team's first lane): the same vertex /
// fold / next sample logic (src/scene.cpp:91-203), with the pixel state in
// registers, the fold records in LDS and the hit handed over by the query
template <bool BIG, class TL>
__device__ __forceinline__ bool coop_shade(const WaveParams& P, const QcScene& Q, TL& L, CoopPixel& px,
                                           uint32_t slot, Ray& ray, int id, const Hit& h, bool& sdone) {
    bool emit = false;
    uint32_t end = PE_LIVE;
    if (id < 0) {
        end = PE_MISS;
    } else {
        uint32_t idm;
        float s1, s2;
        const Shade sh = P.S.shade[id];
        const bool cont = shade_vertex_e(P.S, EmitLds<BIG>{Q, P.S}, sh, px.R, ray, h, id, idm, s1, s2);
        if (!BIG || px.nv < QC_FOLD) {
            L.fold_sh[px.nv] = sh;
            L.fold[px.nv] = make_uint4(idm, f2u(s1), f2u(s2), 0u);
        } else {
            // a path deeper than the LDS records: the rest in the slot's HBM fold records
            P.st.fold[(size_t)slot * P.st.depth + px.nv] = make_uint4(idm, f2u(s1), f2u(s2), 0u);
        }
        ++px.nv;
        if (!cont) end = PE_TERM;
        else if (px.nv >= P.depth) end = PE_CUT;   // RayTrace(.., 0) = 0
        else emit = true;
    }
    sdone = end != PE_LIVE;
    if (end != PE_LIVE) {
        // path over: backward fold (deepest vertex first), src/scene.cpp:198 sum += ...
        f3 Lr = end == PE_MISS ? P.S.bg : mk3(0.f, 0.f, 0.f);
        for (uint32_t k = px.nv; k > 0u; --k) {
            if (!BIG || k - 1u < QC_FOLD) {
                const uint4 f = L.fold[k - 1u];
                Lr = fold_vertex_sh(L.fold_sh[k - 1u], Lr, f.x, u2f(f.y), u2f(f.z));
            } else {
                const uint4 f = P.st.fold[(size_t)slot * P.st.depth + (k - 1u)];
                Lr = fold_vertex_sh(P.S.shade[f.x & 0x3fffffffu], Lr, f.x, u2f(f.y), u2f(f.z));
            }
        }
        const uint4 sp = L.sum;
        const f3 sum = mk3(u2f(sp.x), u2f(sp.y), u2f(sp.z)) + Lr;   // src/scene.cpp:198 sum += ...
        L.sum = make_uint4(f2u(sum.x), f2u(sum.y), f2u(sum.z), sp.w);
        px.done += 1u;
        px.nv = 0u;
        if (px.done < P.target) {
            const WaveParams& K = karg<WaveParams>();   // (read here: see end_item)
            ray = camera_sample(K.cam, px.R, sp.w % K.tm.W, sp.w / K.tm.W);
            emit = true;
        }
    }
    return emit;
}

#ifndef QC_WAVES_PER_EU
#define QC_WAVES_PER_EU 3
#endif
// BIG: a scene beyond the LDS tables (RAY_DEPTH > QC_FOLD, more than QC_NPL planes
// or QC_NEM emitters): the rest of them from HBM (a separate instantiation, so the
// common case carries none of that code)
// (teams of 4: 70 KB of LDS per workgroup, 2 per CU, so 2 waves per SIMD)
template <uint32_t T, bool BIG>
__global__ void __launch_bounds__(64u * QC_WAVES) __attribute__((amdgpu_waves_per_eu(T == 4u ? 2u : QC_WAVES_PER_EU, T == 4u ? 2u : QC_WAVES_PER_EU)))
k_wcoop(WaveParams P) {
    __shared__ QcTeamLds<T> Ls[QC_WAVES * (64u / T)];
    __shared__ QcPoolLds<T> Pool[T < 64u ? QC_WAVES : 1u];   // (teams of T < 64: the wave's query pool)
    __shared__ QcScene Q;
    const uint32_t lane = lane_id(), tl = lane % T, tbase = lane - tl;
    QcTeamLds<T>& L = Ls[(threadIdx.x >> 6) * (64u / T) + lane / T];
    __shared__ uint32_t Lc[QC_WAVES][LC_N];
    uint32_t* lc = Lc[threadIdx.x >> 6];
    if (lane < LC_N) lc[lane] = 0u;
    {
        // this launch's copies: the first planes and emitters, the aux BVH's top nodes
        F4* q = reinterpret_cast<F4*>(&Q);
        const uint32_t npl = (P.S.n_planes < QC_NPL ? P.S.n_planes : QC_NPL) * 5u;
        const uint32_t nem = (P.S.n_emitters < QC_NEM ? P.S.n_emitters : QC_NEM) * 5u;
        const uint32_t ntop = (P.n_aux < QC_TOPN * PT_AUXW ? P.n_aux : QC_TOPN * PT_AUXW) * 2u;
        for (uint32_t i = threadIdx.x; i < npl; i += blockDim.x)
            q[i] = reinterpret_cast<const F4*>(P.S.prims + P.S.planes[i / 5u])[i % 5u];
        for (uint32_t i = threadIdx.x; i < nem; i += blockDim.x)
            q[QC_NPL * 5u + i] = reinterpret_cast<const F4*>(P.S.prims + P.S.emitters[i / 5u])[i % 5u];
        for (uint32_t i = threadIdx.x; i < ntop; i += blockDim.x)
            q[(QC_NPL + QC_NEM) * 5u + i] = P.S.blob[P.S.o_aux / 16u + i];   // (the query-blob form)
        if (threadIdx.x < P.S.n_planes && threadIdx.x < QC_NPL) Q.pl_id[threadIdx.x] = P.S.planes[threadIdx.x];
        __syncthreads();
    }
    const uint32_t* in = P.ctl + PT_CTL_SET * P.parity;
    uint32_t* out = P.ctl + PT_CTL_SET * (1u - P.parity);
    const uint32_t n_carry = in[C_CARRY], n_total = in[C_FRESH] + n_carry;
    const RayQ FQ = P.fq[P.parity];
    uint32_t prog = 0u;   // finished samples not yet reported (wave-uniform)
    // the stop count: side_stop_n finished path workgroups, or (the final launch's hand-over
    // to whole-wave teams) all but side_stop_n of this launch's work items ended
    // (the late-workgroup test hooks: a stop count of 0, so the loop holds no flag test)
    const bool late = (P.side_flags & PT_SIDE_LATE) || ((P.side_flags & PT_GROW_LATE) && (blockIdx.x & 1u));
    // (test hook side_stop_now: no stop test at the top; the loop leaves after its first chain cycle)
    const uint32_t stop_n = (P.side_flags & PT_SIDE_STOP_NOW) ? 0xffffffffu
                            : late ? 0u
                            : !(P.side_flags & PT_STOP_GROW) ? P.side_stop_n
                            : n_total > P.side_stop_n ? n_total - P.side_stop_n : 0xffffffffu;
#ifdef PT_CPROF
    // expansion, candidates, decisions, shading, next ray, chain cycles, chains, wave lifetime
    uint64_t cp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t cp_start = __builtin_amdgcn_s_memtime();
#endif
    bool have = false, exhausted = false, stopped = false;
    uint32_t slot = 0u;
    Ray ray;
    ray.o = ray.d = mk3(0.f, 0.f, 0.f);
    float Pt = PT_INF;
    int pid = -1;
    F4 pre = F4{0.f, 0.f, 0.f, 0.f};
    CoopPixel px;
    px.R.x = 0u;
    px.R.saved = 0.f;
    px.R.saved_ok = 0u;
    px.nv = px.done = 0u;
    for (;;) {
        if (P.side_stop) {
            // beside a path round: once its workgroups have all finished, the chains leave at
            // this chain cycle's end (after the loop: the yield's registers stay out of it)
            uint32_t fin = 0u;
            if (lane == 0u) fin = __hip_atomic_load(P.side_stop, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            fin = __builtin_amdgcn_readfirstlane(fin);
            if (fin >= stop_n) {
                stopped = true;
                break;
            }
        }
        // teams without a chain take the next one (queue order: carry, then fresh)
        const bool need = !have && !exhausted;
        if (__ballot(need) != 0ull) {
            uint32_t gi = wave_append(out + C_HEADS, need && tl == 0u);
            gi = __shfl(gi, (int)tbase, 64);
            if (need) {
                if (gi >= n_total) {
                    exhausted = true;
                } else {
                    if (P.order) gi = P.order[gi];   // the pixels furthest from the target first
                    have = true;
#ifdef PT_CPROF
                    if (tl == 0u) cp[6]++;
#endif
                    if (gi < n_carry) {
                        // a query suspended by the path engine: restarted from its ray (a query is a
                        // function of the ray alone; its ray and plane tests were counted when taken)
                        const uint32_t* w = P.cq[P.parity] + (size_t)gi * P.carry_words;
                        ray = reinterpret_cast<const Query*>(w)->ray;
                        slot = w[sizeof(Query) / 4u];
                        q_planes_e(P.S, PlanesLds<BIG>{Q, P.S}, ray, Pt, pid);
                        pre = q_prep(P.S, ray);
                    } else {
                        const uint32_t fi = gi - n_carry;
                        const F4 o = FQ.ro[fi], d = FQ.rd[fi];
                        ray.o = mk3(o.x, o.y, o.z);
                        ray.d = mk3(d.x, d.y, d.z);
                        slot = f2u(o.w);
                        Pt = d.w;
                        pid = FQ.pid[fi];
                        pre = FQ.ri[fi];
                        lc_add(lc, LC_RAYS, tl == 0u);
                    }
                    // the pixel's state for the chain's life: RNG / vertices / samples and the
                    // sum in the first lane's registers, the current path's fold records in LDS
                    const PixelHot hot = load_hot(P.st, slot);
                    px.R = hot.R;
                    px.nv = hot.nv;
                    px.done = hot.done;
                    if (tl == 0u) L.sum = P.st.rec[2u * slot + 1u];
                    // the current path's vertices so far (written by the path engine; any
                    // beyond QC_FOLD stay in HBM; teams of 4: a lane takes two)
                    for (uint32_t v = tl; v < hot.nv && (!BIG || v < QC_FOLD); v += T) {
                        const uint4 f = P.st.fold[(size_t)slot * P.st.depth + opaque_v(v)];
                        L.fold[v] = f;
                        L.fold_sh[v] = P.S.shade[f.x & 0x3fffffffu];
                    }
                }
            }
        }
        if (__ballot(have) == 0ull) break;
        bool ex, bvh;
        Hit h;
        int id;
        if constexpr (T < 64u)
            id = qc_pool<T>(P.S, Q, Pool[threadIdx.x >> 6], &Ls[(threadIdx.x >> 6) * (64u / T)], have, ray, Pt, pid, pre,
                            P.coop_reserve, lc, ex, h, bvh QC_CP_PASS);
        else
            id = qc_team<T>(P.S, Q, L, have, ray, Pt, pid, pre, P.coop_reserve, lc, ex, h, bvh QC_CP_PASS);
        bool emit = false, sdone = false;
        QC_T0();
        if (tl == 0u && have) {
            if (ex) {
                // the exact stack DFS (non-finite rays, too many hitting leaves)
                // (its stack: the team's own, or its chain's slice of the wave's pool)
                uint32_t* xs = L.stk;
                if constexpr (T < 64u) xs = Pool[threadIdx.x >> 6].stk + (lane / T) * QcTeamLds<T>::SCAP;
                LdsMemN<1u> stk{xs};
                QCounts Cx{0u, 0u, 0u, 0u};
                id = q_exact(P.S, ray, stk, h, Cx);
                atomicAdd(lc + LC_NODES, Cx.nodes);
                atomicAdd(lc + LC_PTESTS, Cx.ptests);
                atomicAdd(lc + LC_FALLB, 1u);
            } else if (id >= 0 && !bvh) {
                // the plane hit (its record from the LDS copy)
                Prim pr = P.S.prims[id];
                for (uint32_t k = 0; k < P.S.n_planes && (!BIG || k < QC_NPL); ++k)
                    if (Q.pl_id[k] == (uint32_t)id) pr = Q.pl[k];
                (void)prim_intersect(pr, ray, h);
            }
            emit = coop_shade<BIG>(P, Q, L, px, slot, ray, id, h, sdone);
        }
        prog += (uint32_t)__popcll(__ballot(sdone));
        lc_add(lc, LC_RAYS, emit);
        emit = __shfl(emit ? 1 : 0, (int)tbase, 64) != 0;
        QC_TICK(3);
        {
            // chains that end here (their pixel reached the target): counted for the final
            // launch's stop (one atomic per wave)
            const unsigned long long me = __ballot(have && !emit && tl == 0u);
            if (P.side_stop && me && lane == (uint32_t)__ffsll((long long)me) - 1u)
                atomicAdd(out + C_ENDED, (uint32_t)__popcll(me));
        }
        if (have && !emit) {
#ifdef PT_CPROF
            // when the chains end: a histogram over 2^20-cycle buckets of the wave's lifetime
            if (tl == 0u && P.wg_prof) {
                const uint64_t bk = (__builtin_amdgcn_s_memtime() - cp_start) >> 20;
                atomicAdd(P.wg_prof + 16 + (bk < 47u ? bk : 47u), 1ull);
            }
#endif
            // the pixel has reached the pass target: its state back to HBM
            if (tl == 0u) {
                PixelHot hot;
                hot.R = px.R;
                hot.nv = px.nv;
                hot.done = px.done;
                store_hot(P.st, slot, hot);
                P.st.rec[2u * slot + 1u] = L.sum;
            }
            have = false;
        }
        if (__ballot(have) != 0ull) {
            // the chains' next rays (the first lanes'), plane tests and query set-up on every lane
            ray.o = mk3(__shfl(ray.o.x, (int)tbase, 64), __shfl(ray.o.y, (int)tbase, 64), __shfl(ray.o.z, (int)tbase, 64));
            ray.d = mk3(__shfl(ray.d.x, (int)tbase, 64), __shfl(ray.d.y, (int)tbase, 64), __shfl(ray.d.z, (int)tbase, 64));
            if (have) {
                q_planes_e(P.S, PlanesLds<BIG>{Q, P.S}, ray, Pt, pid);
                pre = q_prep(P.S, ray);
            }
#ifdef PT_CPROF
            if (have && tl == 0u) cp[5]++;
#endif
        }
        QC_TICK(4);
        if (karg<WaveParams>().side_flags & PT_SIDE_STOP_NOW) {
            stopped = true;
            break;
        }
        // (the wave's 32-bit visit counters go to the 64-bit statistics before they could wrap:
        // a chain cycle adds far less than 2^31)
        if (lane == 0u && (lc[LC_NODES] | lc[LC_PTESTS] | lc[LC_AUX]) >= 0x80000000u) {
            unsigned long long* ctr = ctr_copy(karg<WaveParams>().counters);
            atomicAdd(ctr + 9, (unsigned long long)lc[LC_NODES]);
            atomicAdd(ctr + 1, (unsigned long long)lc[LC_NODES]);
            atomicAdd(ctr + 10, (unsigned long long)lc[LC_PTESTS]);
            atomicAdd(ctr + 2, (unsigned long long)lc[LC_PTESTS]);
            atomicAdd(ctr + 13, (unsigned long long)lc[LC_AUX]);
            atomicAdd(ctr + 5, (unsigned long long)lc[LC_AUX]);
            lc[LC_NODES] = lc[LC_PTESTS] = lc[LC_AUX] = 0u;
        }
        if (P.progress && prog >= 256u) {
            if (lane == 0u)
                __hip_atomic_fetch_add(P.progress, (unsigned long long)prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            prog = 0u;
        }
    }
    if (stopped) {
        // A launch beside a path round that stopped: each team's next query, as a
        // suspended query at its start, to the round's next carry queue (a resumed query is
        // not counted again: its ray was counted when first taken), its pixel state and the
        // current path's fold records to HBM (the path engine continues the path from there)
        // (hand-off site HO_SIDE_YIELD, or HO_GROW_YIELD for the final launch's grow stop;
        // PT_TUNE drop=side_yield / grow_yield loses them instead)
        const bool drop = P.drop == 1u + ((P.side_flags & PT_STOP_GROW) ? HO_GROW_YIELD : HO_SIDE_YIELD);
        lc_add(lc, LC_YIELD, have && tl == 0u);
        const uint32_t k = wave_append(P.yield_ctr, have && tl == 0u && !drop);
        // (k < carry_cap always: the host sizes the stops to the carry queue; a yield past it
        // would be a lost chain, which the resolve reports, never a write past the queue)
        if (have && tl == 0u && !drop && k < P.carry_cap) {
            Query q;
            q_init_pre(ray, Pt, pid, pre, q);
            uint32_t* w = P.yield_cq + (size_t)k * P.carry_words;
            *reinterpret_cast<Query*>(w) = q;
            w[sizeof(Query) / 4u] = slot;
            PixelHot hot;
            hot.R = px.R;
            hot.nv = px.nv;
            hot.done = px.done;
            store_hot(P.st, slot, hot);
            P.st.rec[2u * slot + 1u] = L.sum;
        }
        const uint32_t nv = __shfl(px.nv, (int)tbase, 64);
        for (uint32_t v = tl; have && v < nv && (!BIG || v < QC_FOLD); v += T) P.st.fold[(size_t)slot * P.st.depth + v] = L.fold[v];
        have = false;
    }
    if (stopped && !(P.side_flags & PT_SIDE_NO_HANDON)) {
        // ... then the work items no team took (a
        // workgroup that started only after the round's end -- the launch shares the
        // device with the path round and anything else on it) go to the next round as
        // they are, their pixels' records untouched in HBM (a fresh ray is counted
        // here, as the intake would have)
        for (;;) {
            uint32_t gi = wave_append(out + C_HEADS, true);
            const bool on = gi < n_total;
            if (__ballot(on) == 0ull) break;
            // (through the intake order, as the teams take them: the final launch's grow stop
            // runs with one, and a workgroup that starts late finds items no team took)
            const uint32_t* order = karg<WaveParams>().order;
            if (on && order) gi = order[gi];
            Ray r;
            float rp = PT_INF;
            int rid = -1;
            F4 rpre = F4{0.f, 0.f, 0.f, 0.f};
            uint32_t rslot = 0u;
            if (on && gi < n_carry) {
                const uint32_t* w = P.cq[P.parity] + (size_t)gi * P.carry_words;
                r = reinterpret_cast<const Query*>(w)->ray;
                rslot = w[sizeof(Query) / 4u];
                q_planes_e(P.S, PlanesLds<BIG>{Q, P.S}, r, rp, rid);
                rpre = q_prep(P.S, r);
            } else if (on) {
                const uint32_t fi = gi - n_carry;
                const F4 o = FQ.ro[fi], d = FQ.rd[fi];
                r.o = mk3(o.x, o.y, o.z);
                r.d = mk3(d.x, d.y, d.z);
                rslot = f2u(o.w);
                rp = d.w;
                rid = FQ.pid[fi];
                rpre = FQ.ri[fi];
            }
            lc_add(lc, LC_RAYS, on && gi >= n_carry);
            lc_add(lc, LC_HANDED, on);
            // (hand-off site HO_SIDE_HANDON, or HO_GROW_HANDON; PT_TUNE drop=side_handon /
            // grow_handon: the items taken here are lost instead)
            const bool keep = on && P.drop != 1u + ((P.side_flags & PT_STOP_GROW) ? HO_GROW_HANDON : HO_SIDE_HANDON);
            const uint32_t k2 = wave_append(P.yield_ctr, keep);
            if (keep && k2 < P.carry_cap) {
                Query q;
                q_init_pre(r, rp, rid, rpre, q);
                uint32_t* w = P.yield_cq + (size_t)k2 * P.carry_words;
                *reinterpret_cast<Query*>(w) = q;
                w[sizeof(Query) / 4u] = rslot;
            }
        }
    }
    if (P.progress && lane == 0u && prog)
        __hip_atomic_fetch_add(P.progress, (unsigned long long)prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // the wave's counters (LDS) to this XCD's statistics copy: the totals, and this engine's
    // share (pt_stats coop_*)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0u) {
        unsigned long long* ctr = ctr_copy(P.counters);
        const uint32_t v[LC_N] = {lc[0], lc[1], lc[2], lc[3], lc[4], lc[5], lc[6], lc[7]};
        const bool grow = (P.side_flags & PT_STOP_GROW) != 0u;
        const uint32_t to[LC_N] = {0u, 1u, 2u, CTR_HO + (grow ? HO_GROW_YIELD : HO_SIDE_YIELD), 5u, 6u, CTR_HANDON, 0u};
        for (uint32_t k = 0; k < LC_HANDED + 1u; ++k)
            if (v[k]) atomicAdd(ctr + to[k], (unsigned long long)v[k]);
        if (v[LC_HANDED]) atomicAdd(ctr + CTR_HO + (grow ? HO_GROW_HANDON : HO_SIDE_HANDON), (unsigned long long)v[LC_HANDED]);
        if (v[LC_RAYS] && P.S.n_planes) atomicAdd(ctr + 3, (unsigned long long)v[LC_RAYS] * P.S.n_planes);
        if (v[LC_RAYS]) atomicAdd(ctr + 8, (unsigned long long)v[LC_RAYS]);
        if (v[LC_NODES]) atomicAdd(ctr + 9, (unsigned long long)v[LC_NODES]);
        if (v[LC_PTESTS]) atomicAdd(ctr + 10, (unsigned long long)v[LC_PTESTS]);
        if (v[LC_AUX]) atomicAdd(ctr + 13, (unsigned long long)v[LC_AUX]);
    }
#ifdef PT_CPROF
    // (per team first lanes: chain counts; cycle sums are per wave, counted by lane 0)
    cp[7] = __builtin_amdgcn_s_memtime() - cp_start;
    if (P.wg_prof && tl == 0u) {
        for (int i = 5; i < 7; ++i) atomicAdd(P.wg_prof + i, (unsigned long long)cp[i]);
        if (lane == 0u) {
            for (int i = 0; i < 5; ++i) atomicAdd(P.wg_prof + i, (unsigned long long)cp[i]);
            atomicAdd(P.wg_prof + 7, (unsigned long long)cp[7]);
        }
    }
#endif
}

}  // namespace pt

extern "C++" {
hipError_t pt_preload_kernels_coop() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(pt::k_wcoop<8u, false>));
}

hipError_t pt_launch_coop(pt::WaveParams p, uint32_t grid, uint32_t team, bool big, hipStream_t s, hipEvent_t e0,
                          hipEvent_t e1) {
    hipError_t e = hipMemsetAsync(p.ctl + PT_CTL_SET * (1u - p.parity), 0, 4u * PT_CTL_SET, s);
    if (e != hipSuccess) return e;
    p.path = 1u;
    if (e0 && (e = hipEventRecord(e0, s)) != hipSuccess) return e;
    if (big) {
        // (a scene beyond the LDS tables: teams of 8, or whole waves for deep trees)
        if (team == 64u) hipLaunchKernelGGL((pt::k_wcoop<64u, true>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
        else hipLaunchKernelGGL((pt::k_wcoop<8u, true>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    } else if (team == 8u) hipLaunchKernelGGL((pt::k_wcoop<8u, false>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    else if (team == 4u) hipLaunchKernelGGL((pt::k_wcoop<4u, false>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    else if (team == 16u) hipLaunchKernelGGL((pt::k_wcoop<16u, false>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    else if (team == 32u) hipLaunchKernelGGL((pt::k_wcoop<32u, false>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    else hipLaunchKernelGGL((pt::k_wcoop<64u, false>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    if (e1 && (e = hipEventRecord(e1, s)) != hipSuccess) return e;
    return hipGetLastError();
}
}
