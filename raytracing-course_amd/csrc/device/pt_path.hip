// pt_path.hip -- the path engine k_wpath: persistent, warp-specialised
// workgroups of PT_NQ query waves and one shade wave; a pixel's chain keeps going
// inside the kernel through LDS rings.  pt_wave.h has the pass's outline.
#include "pt_wave.h"

namespace pt {

// ---- path engine -------------------------------------------------------------
// k_wpath: persistent and warp-specialised.  A workgroup is PT_NQ query waves
// plus one shade wave.  A pixel's chain (its one ray in flight) is always in
// exactly one place: a query lane, the done ring (query finished, waiting to be
// shaded), a shade lane, or the ray ring (its next ray, waiting for a query
// lane).  Query lanes refill from the ray ring first and from the round's work
// (suspended queries, then fresh rays) second, so a chain keeps going inside the
// kernel instead of advancing one query per round -- with fewer pixels than
// lanes (a rank of a multi-GPU render, the end of a pass) the lanes stay busy.
// Once the round's work is used up a query wave keeps its chains going until the
// round's deadline (`path_ticks` after the first wave found the work used up: all
// waves stop together; or `path_budget` more trips of its own), then suspends its
// queries to the carry queue; the
// shade wave, last out, hands the remaining chains' next rays to the fresh queue
// of the next round.  Rounds then only rebalance chains between workgroups.
//
// LDS accessors with the address space spelled out (a reference to a __shared__ member is a

// The shade wave's halves of shade_item, with the pixel record in the workgroup's
// LDS table (entry cid, PathLds::H) instead of HBM.  vertex_item: the vertex
// (src/scene.cpp:91-177) and its fold record; true with `ray` = the child ray, or
// false when the path ended (the miss, or the vertex ends it), `miss` telling how.
// end_item: the backward fold into the sum (src/scene.cpp:198) and the next sample's
// camera ray, run later in a batch of ended paths; false = the pixel reached the
// pass target (its record is then written back to HBM).  A pixel has one chain, and
// its next sample starts only from end_item, so its operations keep shade_item's order.
template <class EM>
__device__ __forceinline__ bool vertex_item(const WaveParams& P, const EM& em, uint4* H, uint32_t cid, uint32_t slot,
                                            Ray& ray, uint32_t hid, bool& miss) {
    PixelHot hot = hot_unpack(lds_get(H, cid));
    uint32_t nv = hot.nv;
    Rng R = hot.R;
    bool live = false;
    miss = hid == 0xffffffffu;
    if (!miss) {
        Hit h;
        (void)prim_intersect(P.S.prims[hid], ray, h);
        uint32_t idm;
        float s1, s2;
        const bool cont = shade_vertex_e(P.S, em, P.S.shade[hid], R, ray, h, (int)hid, idm, s1, s2);
        HbmVStore vs = fold_store(P.st, slot);
        vs.put(nv, idm, s1, s2);
        ++nv;
        live = cont && nv < P.depth;   // RayTrace(.., 0) = 0
    }
    hot.nv = nv;
    hot.R = R;
    lds_put(H, cid, hot_pack(hot));
    return live;
}
__device__ __forceinline__ bool end_item(const WaveParams& P, uint4* H, uint32_t cid, uint32_t slot, bool miss,
                                         Ray& ray) {
    PixelHot hot = hot_unpack(lds_get(H, cid));
    Rng R = hot.R;
    f3 L = miss ? P.S.bg : mk3(0.f, 0.f, 0.f);
    HbmVStore vs = fold_store(P.st, slot);
    for (uint32_t k = hot.nv; k > 0u; --k) {
        uint32_t idm;
        float s1, s2;
        vs.get(k - 1u, idm, s1, s2);
        L = fold_vertex(P.S, L, idm, s1, s2);
    }
    uint32_t pix;
    const f3 sum = load_sum_pix(P.st, slot, pix);
    store_sum(P.st, slot, sum + L, pix);
    hot.done += 1u;
    hot.nv = 0u;
    bool emit = false;
    if (hot.done < P.target) {
        // (the camera block read here, not held in SGPRs across the shade wave's loop)
        const WaveParams& K = karg<WaveParams>();
        ray = camera_sample(K.cam, R, pix % K.tm.W, pix / K.tm.W);
        emit = true;
    }
    hot.R = R;
    if (emit) lds_put(H, cid, hot_pack(hot));
    else store_hot(P.st, slot, hot);   // the pixel leaves the workgroup
    return emit;
}

// Rings: entries and positions in LDS, ordered by workgroup-scope release/acquire
// fences.  Every ring has ONE producer, which publishes its entries in order, so a
// consumer takes a contiguous range: the ray ring is written by the shade wave, and
// each query wave has its own done ring.  At most PT_CMAX chains are resident per
// workgroup and a chain has at most one ring entry, so the ray ring (PT_CMAX
// entries) never overflows; a done ring (PT_DQN entries) is flow-controlled by its
// consumer's head.  No entry is overwritten before it has been read.
struct PathLds {
    uint32_t rq_head;             // next ray-ring entry to take (query waves, CAS)
    uint32_t rq_tail;             // ray-ring entries published (shade wave)
    uint32_t resident;            // chains held by this workgroup
    uint32_t leaked;              // chains handed to the exact DFS (their table entries stay taken)
    uint32_t qw_done;             // query waves that have left
    uint32_t f_head;              // pixel-table entries taken from the free ring (query waves, atomic)
    uint32_t dq_tail[PT_NQ];      // done-ring entries published, per query wave
    uint32_t dq_head[PT_NQ];      // done-ring entries read by the shade wave (free space for the producer)
    // The resident chains' pixel records (rec[2 slot]: RNG, vertex count, samples
    // done): a chain takes an entry when it joins the workgroup (query wave intake)
    // and its record lives here, not in HBM, until it leaves -- its pixel reaches the
    // pass target (the shade wave writes it back and frees the entry), or the round
    // ends or the exact DFS takes its ray (written back, the entry stays taken).
    uint4 H[PT_CMAX];
    uint16_t F[PT_CMAX];          // free entries (ring: taken at f_head, returned by the shade wave)
    F4 rq_ro[PT_CMAX];            // ray ring: {o.xyz, slot}
    F4 rq_rd[PT_CMAX];            //           {d.xyz, P}
    F4 rq_ri[PT_CMAX];            //           q_prep record
    int rq_pid[PT_CMAX];          //           closest plane
    uint16_t rq_cid[PT_CMAX];     //           pixel-table entry
    F4 dq_ro[PT_NQ][PT_DQN];      // done rings: {o.xyz, slot}
    F4 dq_rd[PT_NQ][PT_DQN];      //             {d.xyz, u32 closest prim | 0xffffffff}
    uint16_t dq_cid[PT_NQ][PT_DQN];   //         pixel-table entry
    uint32_t stk[(PT_LSTACK + 1u) * 64u * PT_NQ];   // query lanes' aux stacks, [word][lane] (+ a trash word)
    // the shade wave's copies of the first planes and emitters (any further ones: HBM);
    // a plane's record carries its prim index in p2.w (unused by a plane)
    F4 pl[QC_NPL * 5u];
    F4 em[QC_NEM * 5u];
};
static_assert(PT_CMAX <= 1024u, "Query::cid is a 10-bit field");
// k_wpath's occupancy (PT_PATH_WAVES_PER_EU waves per SIMD, 4 SIMDs per CU) assumes
// that many workgroups fit the CU's 160 KB of LDS: a bigger ring, stack or table
// would silently drop a workgroup per CU (every tuning number assumes 4)
static_assert((PT_PATH_WAVES_PER_EU * 4u / (PT_NQ + 1u)) * sizeof(PathLds) <= 160u * 1024u,
              "PathLds no longer fits PT_PATH_WAVES_PER_EU*4/(PT_NQ+1) workgroups per CU");
// the first QC_NPL planes / QC_NEM emitters from the workgroup's LDS copy, any further ones from HBM
struct PlanesPath {
    const PathLds& L;
    const SceneView& S;
    __device__ Prim operator()(uint32_t k, uint32_t& pi) const {
        if (k < QC_NPL) {
            Prim p;
            p.p0 = lds_get(L.pl, 5u * k); p.p1 = lds_get(L.pl, 5u * k + 1u); p.p2 = lds_get(L.pl, 5u * k + 2u);
            p.p3 = lds_get(L.pl, 5u * k + 3u); p.p4 = lds_get(L.pl, 5u * k + 4u);
            pi = f2u(p.p2.w);
            p.p2.w = 0.f;
            return p;
        }
        pi = S.planes[k];
        return S.prims[pi];
    }
};
struct EmitPath {
    const PathLds& L;
    const SceneView& S;
    __device__ Prim operator()(uint32_t k) const {
        if (k < QC_NEM) {
            Prim p;
            p.p0 = lds_get(L.em, 5u * k); p.p1 = lds_get(L.em, 5u * k + 1u); p.p2 = lds_get(L.em, 5u * k + 2u);
            p.p3 = lds_get(L.em, 5u * k + 3u); p.p4 = lds_get(L.em, 5u * k + 4u);
            return p;
        }
        return S.prims[S.emitters[k]];
    }
};



#ifndef PT_PATH_REFILL_MIN
#define PT_PATH_REFILL_MIN 8u      // idle lanes before a query wave refills (any, once the round's work is out;
                                   // 4 / 16 measured -1 % / -1.5 % in round 3)
#endif
#define PT_NOWORK 0xffffffffu
#define PT_CAPPED 0xfffffffeu

// SPARSE: the kernel of the rounds at the end of a pass (few chains, heavy queries:
// bound by each chain's latency, not by issue): a trip runs every step kind and
// up to P.sparse_steps steps.  A separate instantiation, so its registers do not
// weigh on the main kernel.
template <bool SPARSE>
__device__ __forceinline__ void path_query_wave(const WaveParams& P, PathLds& L, uint32_t qw) {
    LdsMemN<64u * PT_NQ> stk{L.stk + 64u * qw + lane_id(), P.lstack, PT_LSTACK};
    const uint32_t p = P.parity;
    const uint32_t* in = P.ctl + PT_CTL_SET * p;
    uint32_t* out = P.ctl + PT_CTL_SET * (1u - p);
    const uint32_t n_carry = in[C_CARRY], n_total = P.pin ? P.pin_n : in[C_FRESH] + n_carry;
    const uint32_t n_waves = gridDim.x * PT_NQ;
    // Rounds exist to rebalance chains between workgroups.  Once the round's chains
    // fit in the query lanes (the tail of a pass: only the slowest pixels are left)
    // suspending gains nothing and costs a round: run them to the end.
    const uint32_t budget = n_total <= P.path_runend ? 0xffffffffu : P.path_budget;
    uint32_t bsz = n_total / n_waves;
    bsz = bsz < 1u ? 1u : (bsz > P.batch ? P.batch : bsz);   // queue indices a wave takes per atomic
    const RayQ FQ = P.fq[p];
    const uint32_t xcc = xcc_id();
    uint32_t xs = 0u;                 // XCD batch counters found empty
    uint32_t bbase = 0u, bleft = 0u;  // this wave's batch of the round's work not yet handed out
    bool exhausted = false;
    uint32_t wpost = 0u;              // trips since the round's work ran out
    uint32_t deadline = 0u;           // the round's end (path_ticks mode; 0 = not read yet)
    uint32_t trip = 0u;
    uint32_t ptrip = 0u;              // trips since the last probe turn
    const uint32_t wq = qw;                 // this query wave's done ring
    uint32_t rr = 0u;                       // replay step kind served last
    uint32_t dq_res = 0u;                   // done-ring entries written and published
    bool active = false;
    uint32_t slot = 0u;
    Query q;
    QCounts C{0u, 0u, 0u, 0u};
    // wave-level counters (scalar registers; per-lane ones would cost VGPRs)
    // (the plane tests are rays x n_planes: every ray taken was plane-tested by its producer;
    // exact-DFS hand-offs per wave and launch stay far below 2^32)
    uint64_t rays = 0u;
    uint32_t fallbacks = 0u, init_exact = 0u;
    QProf pf;                         // (diagnostics builds only: PT_WPROF)
    for (;;) {
        const unsigned long long idle = __ballot(!active);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        pf.trip(nidle, L, wq);
        if (!exhausted && (++trip & 15u) == 0u) {
            // A wave whose lanes stay busy with its workgroup's chains does not pull,
            // so it would never find the round's work used up and would run its
            // chains to the end of the pass: look at the 8 batch counters instead.
            bool used = true;
            if (lane_id() < 8u) {
                const uint32_t h = __hip_atomic_load(out + C_HEADS + 32u * lane_id(), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                used = (8ull * h + lane_id()) * bsz >= n_total;
            }
            exhausted = __ballot(!used) == 0ull;
        }
        if (exhausted && bleft == 0u) {
            bool over;
            if (budget == 0xffffffffu) {
                over = false;
            } else if (karg<WaveParams>().path_ticks) {
                // One deadline for the whole round: the trip counts of workgroups with heavy
                // and light chains differ, so a per-wave trip budget ends them at different
                // times and the first ones out wait for the last (a round of a rank of 8:
                // query waves tripping ~75 % of the round's span)
                if (deadline == 0u) {
                    uint32_t d = 0u;
                    if (lane_id() == 0u) {
                        const uint32_t want = ((uint32_t)__builtin_amdgcn_s_memrealtime() + karg<WaveParams>().path_ticks) | 1u;
                        const uint32_t old = atomicCAS(out + C_DEADLINE, 0u, want);
                        d = old ? old : want;
                    }
                    deadline = __builtin_amdgcn_readfirstlane(d);
                }
                over = (int32_t)((uint32_t)__builtin_amdgcn_s_memrealtime() - deadline) >= 0;
            } else {
                over = wpost >= budget;
            }
            if (over) {
                // the round is over for this wave: suspend its running queries (hand-off site
                // HO_SUSPEND; PT_TUNE drop=suspend loses them instead)
                const WaveParams& K0 = karg<WaveParams>();
                const bool drop = K0.drop == 1u + HO_SUSPEND;
                if (active && !drop) {
                    const WaveParams& K = karg<WaveParams>();
                    const uint32_t k = wave_append(K.ctl + PT_CTL_SET * (1u - K.parity) + C_CARRY, true);
                    uint32_t* w = K.cq[1u - K.parity] + (size_t)k * K.carry_words;
                    *reinterpret_cast<Query*>(w) = q;
                    uint32_t* tail = w + sizeof(Query) / 4u;
                    tail[0] = slot;
                    for (uint32_t j = 0; j < q.sp; ++j) tail[1u + j] = stk.get(j);
                    K.st.rec[2u * slot] = lds_get(L.H, (uint32_t)q.cid);   // the chain leaves the workgroup
                }
                const uint32_t ns = (uint32_t)__popcll(__ballot(active));
                if (lane_id() == 0u && ns) {
                    atomicSub(&L.resident, ns);
                    atomicAdd(ctr_copy(K0.counters) + CTR_HO + HO_SUSPEND, (unsigned long long)ns);
                }
                pf.exit_budget();
                break;
            }
            if (nidle == 64u && lds_read(L.resident) == 0u) break;   // no chain left anywhere
            ++wpost;
        }
        if (nidle >= PT_PATH_REFILL_MIN || nidle == 64u || (nidle > 0u && exhausted)) {
            // refill: this wave's batch leftovers, then the ray ring, then new batches
            const uint32_t pos = lanes_below(idle);   // this idle lane's rank
            uint32_t given = 0u, src = 0u, gi = 0u;   // src 1 = work item gi, 2 = ray-ring entry gi
            {
                const uint32_t take = nidle < bleft ? nidle : bleft;
                if (!active && pos < take) { src = 1u; gi = bbase + pos; }
                bbase += take;
                bleft -= take;
                given = take;
            }
            if (given < nidle) {
                uint32_t h = 0u, take = 0u;
                if (lane_id() == 0u) {
                    for (;;) {
                        h = lds_read(L.rq_head);
                        const uint32_t t = lds_read(L.rq_tail), want = nidle - given;
                        take = t - h < want ? t - h : want;
                        if (take == 0u || atomicCAS(&L.rq_head, h, h + take) == h) break;
                    }
                }
                h = __builtin_amdgcn_readfirstlane(h);
                take = __builtin_amdgcn_readfirstlane(take);
                if (!active && pos >= given && pos < given + take) { src = 2u; gi = (h + pos - given) % PT_CMAX; }
                given += take;
                pf.ring(take);
            }
            while (given < nidle && !exhausted) {
                uint32_t v = PT_NOWORK, cnt = 0u;
                if (lane_id() == 0u) {
                    if (atomicAdd(&L.resident, bsz) + bsz + lds_read(L.leaked) > P.path_cap) {
                        atomicSub(&L.resident, bsz);   // workgroup full: its chains first
                        v = PT_CAPPED;
                    } else {
                        while (xs < 8u) {
                            const uint32_t y = (xcc + xs) & 7u;
                            const uint64_t b = 8ull * atomicAdd(out + C_HEADS + 32u * y, 1u) + y;
                            if (b * bsz < n_total) { v = (uint32_t)(b * bsz); break; }
                            ++xs;
                        }
                        if (v == PT_NOWORK) {
                            atomicSub(&L.resident, bsz);
                        } else {
                            cnt = n_total - v < bsz ? n_total - v : bsz;
                            if (cnt < bsz) atomicSub(&L.resident, bsz - cnt);
                        }
                    }
                }
                v = __builtin_amdgcn_readfirstlane(v);
                xs = __builtin_amdgcn_readfirstlane(xs);
                cnt = __builtin_amdgcn_readfirstlane(cnt);
                if (v == PT_CAPPED) break;
                if (v == PT_NOWORK) { exhausted = true; break; }
                bbase = v;
                bleft = cnt;
                pf.pulled(cnt);
                const uint32_t take = nidle - given < bleft ? nidle - given : bleft;
                if (!active && pos >= given && pos < given + take) { src = 1u; gi = bbase + pos - given; }
                bbase += take;
                bleft -= take;
                given += take;
            }
            // chains joining the workgroup (src 1: the round's work) take a pixel-table
            // entry from the free ring (there are enough: the entries taken never exceed
            // resident + leaked <= path_cap <= PT_CMAX); ray-ring chains bring theirs
            const unsigned long long mjoin = __ballot(src == 1u);
            uint32_t fh = 0u;
            if (mjoin) {
                if (lane_id() == 0u) fh = atomicAdd(&L.f_head, (uint32_t)__popcll(mjoin));
                fh = __builtin_amdgcn_readfirstlane(fh);
            }
            if (src != 0u) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            uint32_t cid = 0u;
            if (src == 1u) cid = lds_get(L.F, (fh + lanes_below(mjoin)) % PT_CMAX);
            if (src == 2u) cid = lds_get(L.rq_cid, gi);
            if (src == 1u) {
                const uint32_t* pin = karg<WaveParams>().pin;
                if (pin) gi = pin[gi];   // (the early cooperative launch took the other items)
            }
            bool took = false;   // a fresh ray (not a resumed query) started in this lane
            if (src == 1u && gi < n_carry) {
                // resume a suspended query: state, slot, then its aux stack into LDS
                const WaveParams& K = karg<WaveParams>();
                const uint32_t* w = K.cq[K.parity] + (size_t)gi * K.carry_words;
                q = *reinterpret_cast<const Query*>(w);
                const uint32_t* tail = w + sizeof(Query) / 4u;
                slot = tail[0];
                for (uint32_t k = 0; k < q.sp; ++k) stk.set(k, tail[1u + k]);
                lds_put(L.H, cid, K.st.rec[2u * slot]);   // its pixel record, for its stay here
                active = true;
            } else if (src != 0u) {
                // a fresh ray of the round, or a chain's next ray from the ray ring
                F4 o, d, pre;
                int pid;
                if (src == 1u) {
                    const uint32_t fi = gi - n_carry;
                    o = FQ.ro[fi];
                    d = FQ.rd[fi];
                    pid = FQ.pid[fi];
                    pre = FQ.ri[fi];
                } else {
                    o = lds_get(L.rq_ro, gi);
                    d = lds_get(L.rq_rd, gi);
                    pid = lds_get(L.rq_pid, gi);
                    pre = lds_get(L.rq_ri, gi);
                }
                Ray ray;
                ray.o = mk3(o.x, o.y, o.z);
                ray.d = mk3(d.x, d.y, d.z);
                slot = f2u(o.w);
                took = true;
                pf.query_start();
                q_init_pre(ray, d.w, pid, pre, q);
                if (src == 1u) lds_put(L.H, cid, P.st.rec[2u * slot]);   // its pixel record, for its stay here
                active = true;
            }
            if (src != 0u) q.cid = cid;
            const uint32_t ntook = (uint32_t)__popcll(__ballot(took));
            rays += ntook;
            init_exact += (uint32_t)__popcll(__ballot(took && q.phase == Q_EXACT));
        }
        if (__ballot(active) == 0ull) {
            pf.sleep();
            __builtin_amdgcn_s_sleep(2);   // nothing to run: chains are being shaded (no `continue`:
        }                                  // a second back edge costs ~30 VGPRs)
        pf.refill_end(active);
        if constexpr (SPARSE) {
#pragma unroll 1
            for (uint32_t it = 0; it < P.sparse_steps; ++it) {
                const bool run = active && (q.phase == Q_AUX || q.phase == Q_REPLAY);
                if (__ballot(run) == 0ull) break;
                if (run) q_step(P.S, q, C, stk);
            }
        } else {
            // One replay step kind per trip besides the aux steps (the kinds' code paths
            // would otherwise all be issued every trip): round-robin over the kinds present.
            uint32_t kind = active && q.phase == Q_REPLAY ? 1u + q.walk : active && q.phase == Q_AUX ? 0u : 7u;
            uint32_t present = 0u;
#pragma unroll
            for (uint32_t k = 1; k <= PT_RKINDS; ++k)
                if (__ballot(kind == k) != 0ull) present |= 1u << k;
            uint32_t pick = 0u;
#pragma unroll
            for (uint32_t j = 1; j <= PT_RKINDS; ++j) {
                const uint32_t c = (rr + j - 1u) % PT_RKINDS + 1u;
                if (pick == 0u && ((present >> c) & 1u)) pick = c;
            }
            if (pick) rr = pick;
            // candidate probes (the aux pass's leaf steps) run on every probe_every-th trip,
            // or whenever probe_min lanes wait for one: the probe code is issued for the
            // whole wave, so a trip that carries it for a few lanes costs every lane
            const bool want_probe = kind == 0u && (q.node & PT_LEAFQ) != 0u;
            const bool turn = ++ptrip >= P.probe_every;
            const bool probe_go = turn || (uint32_t)__popcll(__ballot(want_probe)) >= P.probe_min;
            if (turn) ptrip = 0u;
            if (want_probe && !probe_go) kind = 7u;
            pf.kinds(kind == 0u, pick != 0u, kind == 0u || kind == pick);
            pf.kind_mix(kind == 0u ? ((q.node & PT_LEAFQ) ? 1u : 0u) : kind == pick ? kind + 1u : 7u);
            if (kind == 0u || kind == pick) q_step(P.S, q, C, stk);
            // aux_extra more aux-node steps in the same trip for the lanes whose next step is one
#pragma unroll 1
            for (uint32_t x = 0; x < P.aux_extra; ++x) {
                const bool a2 = active && q.phase == Q_AUX && !(q.node & PT_LEAFQ);
                if (__ballot(a2) == 0ull) break;
                pf.extra_aux((uint32_t)__popcll(__ballot(a2)));
                if (a2) q_aux_step(P.S, q, C, stk);
            }
        }
        pf.step_end();
        // finished queries -> this wave's done ring, in lane order, as far as it has room
        // (the shade wave recomputes t, n and side from the prim); the others wait in
        // their lanes (phase Q_DONE) for the next trip
        const uint32_t room = PT_DQN - (dq_res - __builtin_amdgcn_readfirstlane(lds_read(L.dq_head[wq])));
        const unsigned long long mfin = __ballot(active && q.phase == Q_DONE);
        const uint32_t rank = lanes_below(mfin);
        const bool fin = active && q.phase == Q_DONE && rank < room;
        const uint32_t nfin = (uint32_t)__popcll(mfin) < room ? (uint32_t)__popcll(mfin) : room;
        const uint32_t dq_at = dq_res;
        dq_res += nfin;
        fallbacks += (uint32_t)__popcll(__ballot(active && q.phase == Q_EXACT));
        if (active) {
            if (fin) {
                const uint32_t j = wq * PT_DQN + (dq_at + rank) % PT_DQN;
                lds_put(&L.dq_ro[0][0], j, F4{q.ray.o.x, q.ray.o.y, q.ray.o.z, u2f(slot)});
                lds_put(&L.dq_rd[0][0], j,
                        F4{q.ray.d.x, q.ray.d.y, q.ray.d.z, u2f(q.res_id < 0 ? 0xffffffffu : (uint32_t)q.res_id)});
                lds_put(&L.dq_cid[0][0], j, (uint16_t)q.cid);
                active = false;
                pf.query_done();
            } else if (q.phase == Q_EXACT) {
                // rare: the exact stack DFS after this kernel; the chain leaves the workgroup
                // (hand-off site HO_EXACT, counted with the fallbacks; PT_TUNE drop=exact)
                const WaveParams& K = karg<WaveParams>();
                if (K.drop != 1u + HO_EXACT) {
                    const uint32_t k = atomicAdd(K.ctl + PT_CTL_SET * (1u - K.parity) + C_EXACT, 1u);
                    K.ex.ro[k] = F4{q.ray.o.x, q.ray.o.y, q.ray.o.z, u2f(slot)};
                    K.ex.rd[k] = F4{q.ray.d.x, q.ray.d.y, q.ray.d.z, u2f(k)};
                    K.st.rec[2u * slot] = lds_get(L.H, (uint32_t)q.cid);   // (k_wshade shades it from HBM)
                }
                atomicAdd(&L.leaked, 1u);   // (its table entry stays taken for the round)
                atomicSub(&L.resident, 1u);
                active = false;
            }
        }
        if (nfin) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane_id() == 0u) lds_write(L.dq_tail[wq], dq_res);
        }
        pf.done_end();
    }
    unsigned long long* ctr = ctr_copy(P.counters);
    wave_add_u64(ctr + 1, C.nodes);
    wave_add_u64(ctr + 2, C.ptests);
    wave_add_u64(ctr + 5, C.aux);
    if (lane_id() == 0u) {
        if (rays) atomicAdd(ctr + 0, (unsigned long long)rays);
        if (rays && P.S.n_planes) atomicAdd(ctr + 3, (unsigned long long)rays * P.S.n_planes);
        if (fallbacks) atomicAdd(ctr + 6, (unsigned long long)fallbacks);
        if (fallbacks) atomicAdd(ctr + CTR_HO + HO_EXACT, (unsigned long long)fallbacks);
        if (init_exact) atomicAdd(ctr + 7, (unsigned long long)init_exact);
    }
    pf.store(P.wg_prof, rays);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane_id() == 0u) atomicAdd(&L.qw_done, 1u);
}

__device__ __forceinline__ void path_shade_wave(const WaveParams& P, PathLds& L) {
    uint32_t* out = P.ctl + PT_CTL_SET * (1u - P.parity);
    const RayQ N = P.fq[1u - P.parity];
    const uint32_t lane = lane_id();
    uint32_t head[PT_NQ];             // done rings consumed (this wave only)
#pragma unroll
    for (uint32_t w = 0; w < PT_NQ; ++w) head[w] = 0u;
    uint32_t tail = 0u;               // ray ring published
    uint32_t f_tail = PT_CMAX;        // pixel-table free ring: entries returned (this wave only)
    SProf pf;                         // (diagnostics builds only: PT_WPROF)
    uint32_t prog = 0u;               // finished samples not yet added to P.progress
    // ended paths waiting for their fold (this wave's own queue: {slot | miss << 31, table entry})
    uint2* endq = P.endq + (size_t)blockIdx.x * PT_CMAX;
    uint32_t e_head = 0u, e_tail = 0u;
    if (karg<WaveParams>().side_flags & PT_SHADE_HOLD) {
        // (test hook: the query waves of a round with a budget leave by themselves)
        const WaveParams& K = karg<WaveParams>();
        const uint32_t* in = K.ctl + PT_CTL_SET * K.parity;
        const uint32_t n_total = K.pin ? K.pin_n : in[C_FRESH] + in[C_CARRY];
        if (n_total > K.path_runend)
            while (__builtin_amdgcn_readfirstlane(lds_read(L.qw_done)) != PT_NQ) __builtin_amdgcn_s_sleep(2);
    }
    for (;;) {
        // published entries of the done rings (ring indices are compile-time: no scratch)
        uint32_t av[PT_NQ], total = 0u;
#pragma unroll
        for (uint32_t w = 0; w < PT_NQ; ++w) {
            av[w] = __builtin_amdgcn_readfirstlane(lds_read(L.dq_tail[w])) - head[w];
            total += av[w];
        }
        Ray ray;
        uint32_t slot = 0u, cid = 0u;
        bool emit = false, sdone = false, have = false;
        pf.begin();
        const uint32_t pend = e_tail - e_head;
        if (pend >= P.end_min || (total == 0u && pend > 0u)) {
            // a batch of ended paths: folds, sums, the next samples' camera rays
            const uint32_t n = pend < 64u ? pend : 64u;
            have = lane < n;
            if (have) {
                const uint2 v = endq[(e_head + lane) % PT_CMAX];
                slot = v.x & 0x7fffffffu;
                cid = v.y;
                emit = end_item(P, L.H, cid, slot, (v.x >> 31) != 0u, ray);
                sdone = true;
            }
            e_head += n;
        } else if (total == 0u) {
            if (lds_read(L.qw_done) == PT_NQ) {
                // every query wave has left (and published): one more look, then done
                uint32_t left = 0u;
#pragma unroll
                for (uint32_t w = 0; w < PT_NQ; ++w) left += lds_read(L.dq_tail[w]) - head[w];
                if (__builtin_amdgcn_readfirstlane(left) == 0u) break;   // (no ended path waits: see above)
                continue;
            }
            pf.spin();
            __builtin_amdgcn_s_sleep(1);
            continue;
        } else {
            // up to 64 of them: a fair share of each ring first (a full ring holds back its
            // producer's finished queries), then the rest in ring order
            uint32_t take[PT_NQ], n = 0u;
#pragma unroll
            for (uint32_t w = 0; w < PT_NQ; ++w) {
                take[w] = av[w] < 64u / PT_NQ ? av[w] : 64u / PT_NQ;
                n += take[w];
            }
#pragma unroll
            for (uint32_t w = 0; w < PT_NQ; ++w) {
                const uint32_t x = av[w] - take[w] < 64u - n ? av[w] - take[w] : 64u - n;
                take[w] += x;
                n += x;
            }
            pf.batch(n);
            // this lane's entry: ring w, position head[w] + (lane - entries of the rings before w)
            uint32_t j = 0u, before = 0u;
#pragma unroll
            for (uint32_t w = 0; w < PT_NQ; ++w) {
                if (lane >= before && lane < before + take[w]) j = w * PT_DQN + (head[w] + lane - before) % PT_DQN;
                before += take[w];
            }
#pragma unroll
            for (uint32_t w = 0; w < PT_NQ; ++w) head[w] += take[w];
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            have = lane < n;
            F4 o = F4{0.f, 0.f, 0.f, 0.f}, d = o;
            if (have) {
                o = lds_get(&L.dq_ro[0][0], j);
                d = lds_get(&L.dq_rd[0][0], j);
                cid = lds_get(&L.dq_cid[0][0], j);
            }
            // the entries are in registers: their slots go back to the producers
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
            for (uint32_t w = 0; w < PT_NQ; ++w)
                if (lane == w) lds_write(L.dq_head[w], head[w]);
            pf.read_done();
            bool miss = false;
            if (have) {
                slot = f2u(o.w);
                ray.o = mk3(o.x, o.y, o.z);
                ray.d = mk3(d.x, d.y, d.z);
                emit = vertex_item(P, EmitPath{L, P.S}, L.H, cid, slot, ray, f2u(d.w), miss);
            }
            // ended paths wait for a fold batch of their own (appended in lane order)
            const bool ended = have && !emit;
            const unsigned long long me = __ballot(ended);
            if (ended) endq[(e_tail + lanes_below(me)) % PT_CMAX] = make_uint2(slot | (miss ? 0x80000000u : 0u), cid);
            e_tail += (uint32_t)__popcll(me);
            have = have && emit;   // (an ended path is not gone: its pixel waits for the fold)
            pf.shaded();
        }
        // finished samples for the host's progress bar: a system-scope add per ~4 k
        prog += (uint32_t)__popcll(__ballot(sdone));
        if (prog >= 4096u) {
            unsigned long long* pg = karg<WaveParams>().progress;
            if (pg && lane == 0u) __hip_atomic_fetch_add(pg, (unsigned long long)prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (pg) prog = 0u;
        }
        const bool flush = __builtin_amdgcn_readfirstlane(lds_read(L.qw_done)) == PT_NQ;
        const unsigned long long me = __ballot(emit);
        // pixels done with this pass (end_item wrote their records back): their table entries are free
        const bool fin = have && !emit;
        const unsigned long long mf = __ballot(fin);
        uint32_t gone = (uint32_t)__popcll(mf);
        if (fin) lds_put(L.F, (f_tail + lanes_below(mf)) % PT_CMAX, (uint16_t)cid);
        f_tail += gone;
        if (flush) {
            // no query wave left to take it: the next round's fresh queue (the chain leaves
            // the workgroup with its pixel record; hand-off site HO_FLUSH, PT_TUNE drop=flush)
            const WaveParams& K = karg<WaveParams>();
            const bool keep = emit && K.drop != 1u + HO_FLUSH;
            const uint32_t k = wave_append(K.ctl + PT_CTL_SET * (1u - K.parity) + C_FRESH, keep);
            if (keep) {
                push_ray(K, K.fq[1u - K.parity], k, ray, slot);
                K.st.rec[2u * slot] = lds_get(L.H, cid);
            }
            // (counted here: a count carried through the loop would hold a register for its life)
            if (lane == 0u && me) atomicAdd(ctr_copy(K.counters) + CTR_HO + HO_FLUSH, (unsigned long long)__popcll(me));
            gone += (uint32_t)__popcll(me);
        } else {
            if (emit) {
                // the next ray into the LDS ray ring (RayQ form: push_ray's plane test and set-up)
                const uint32_t e = (tail + lanes_below(me)) % PT_CMAX;
                float pt;
                int pid;
                q_planes_e(P.S, PlanesPath{L, P.S}, ray, pt, pid);
                lds_put(L.rq_ro, e, F4{ray.o.x, ray.o.y, ray.o.z, u2f(slot)});
                lds_put(L.rq_rd, e, F4{ray.d.x, ray.d.y, ray.d.z, pt});
                lds_put(L.rq_pid, e, pid);
                lds_put(L.rq_ri, e, q_prep(P.S, ray));
                lds_put(L.rq_cid, e, (uint16_t)cid);
            }
            tail += (uint32_t)__popcll(me);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0u) lds_write(L.rq_tail, tail);
        }
        // (the freed table entries are written before the decrement that lets a query wave take them)
        if (gone) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0u && gone) atomicSub(&L.resident, gone);
        pf.end();
    }
    pf.store(P.wg_prof);
    if (P.progress && prog && lane == 0u)
        __hip_atomic_fetch_add(P.progress, (unsigned long long)prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // the ray ring's leftovers (no query wave takes from it any more) -> next round, with
    // their pixel records (hand-off site HO_RINGOUT, PT_TUNE drop=ringout)
    const uint32_t h = lds_read(L.rq_head);
    if (lane == 0u && tail != h) atomicAdd(ctr_copy(P.counters) + CTR_HO + HO_RINGOUT, (unsigned long long)(tail - h));
    const uint32_t ring_end = karg<WaveParams>().drop == 1u + HO_RINGOUT ? h : tail;
    for (uint32_t b = h; b < ring_end; b += 64u) {
        const uint32_t i = b + lane;
        const bool has = i < ring_end;
        // (the append first: ring values held across its atomic would live in scratch)
        const uint32_t k = wave_append(out + C_FRESH, has);
        if (has) {
            const uint32_t e = i % PT_CMAX;
            const F4 ro = lds_get(L.rq_ro, e);
            N.ro[k] = ro;
            N.rd[k] = lds_get(L.rq_rd, e);
            N.pid[k] = lds_get(L.rq_pid, e);
            N.ri[k] = lds_get(L.rq_ri, e);
            P.st.rec[2u * f2u(ro.w)] = lds_get(L.H, (uint32_t)lds_get(L.rq_cid, e));
        }
    }
}

// The end-of-pass (sparse) kernel runs few chains, bound by their latency, not by
// occupancy: it is held to 2 waves per SIMD (256 VGPRs, no spills; 2 workgroups per CU
// run at a time, the grid's others start as those finish and find the round's work taken)
template <bool SPARSE>
__global__ void __launch_bounds__(PT_PATH_WG)
__attribute__((amdgpu_waves_per_eu(SPARSE ? 2u : PT_PATH_WAVES_PER_EU, SPARSE ? 2u : PT_PATH_WAVES_PER_EU)))
k_wpath(WaveParams P) {
    __shared__ PathLds L;
    {
        // the first planes and emitters (the shade wave's plane tests and light sampling)
        const uint32_t npl = (P.S.n_planes < QC_NPL ? P.S.n_planes : QC_NPL) * 5u;
        const uint32_t nem = (P.S.n_emitters < QC_NEM ? P.S.n_emitters : QC_NEM) * 5u;
        for (uint32_t i = threadIdx.x; i < npl; i += blockDim.x) {
            const uint32_t pi = P.S.planes[i / 5u];
            F4 v = reinterpret_cast<const F4*>(P.S.prims + pi)[i % 5u];
            if (i % 5u == 2u) v.w = u2f(pi);
            lds_put(L.pl, i, v);
        }
        for (uint32_t i = threadIdx.x; i < nem; i += blockDim.x)
            lds_put(L.em, i, reinterpret_cast<const F4*>(P.S.prims + P.S.emitters[i / 5u])[i % 5u]);
    }
    if (threadIdx.x == 0u) {
        L.rq_head = L.rq_tail = L.resident = L.qw_done = L.leaked = L.f_head = 0u;
    }
    if (threadIdx.x < PT_NQ) L.dq_tail[threadIdx.x] = L.dq_head[threadIdx.x] = 0u;
    for (uint32_t i = threadIdx.x; i < PT_CMAX; i += blockDim.x) lds_put(L.F, i, (uint16_t)i);   // every entry free
    wprof_start(P.wg_prof);
    __syncthreads();
    // waves 0 .. PT_NQ-1 query, wave PT_NQ shades
    const uint32_t wave = threadIdx.x >> 6;
    if (wave == PT_NQ) path_shade_wave(P, L);
    else path_query_wave<SPARSE>(P, L, wave);
    // the round's finished workgroups (an early cooperative launch beside this round stops
    // once all are done: WaveParams::side_stop)
    __syncthreads();
    if (threadIdx.x == 0u)
        __hip_atomic_fetch_add(P.ctl + PT_CTL_SET * (1u - P.parity) + C_WGDONE, 1u, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace pt

extern "C++" {
hipError_t pt_preload_kernels_path() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(pt::k_wpath<false>));
}

hipError_t pt_launch_path_round(pt::WaveParams p, uint32_t path_grid, uint32_t shade_grid, hipStream_t s, bool sparse,
                                hipEvent_t e0, hipEvent_t e1) {
    hipError_t e = hipMemsetAsync(p.ctl + PT_CTL_SET * (1u - p.parity), 0, 4u * PT_CTL_SET, s);
    if (e != hipSuccess) return e;
    p.path = 1u;
    if (e0 && (e = hipEventRecord(e0, s)) != hipSuccess) return e;
    if (sparse)
        hipLaunchKernelGGL(pt::k_wpath<true>, dim3(path_grid), dim3(PT_PATH_WG), 0, s, p);
    else
        hipLaunchKernelGGL(pt::k_wpath<false>, dim3(path_grid), dim3(PT_PATH_WG), 0, s, p);
    if (e1 && (e = hipEventRecord(e1, s)) != hipSuccess) return e;
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return pt_launch_exact_shade(p, shade_grid, s);
}
}
