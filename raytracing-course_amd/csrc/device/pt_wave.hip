// pt_wave.hip -- wavefront form of the hw5 render loop on gfx950.
//
// A pass advances every owned pixel by `target` samples (src/scene.cpp:
// 189-203) through rounds of launches on one stream:
//
//   k_wcamera   (pass start) the first sample's 2 jitter draws and camera
//               ray (src/scene.cpp:180-199) of every pixel -> fresh queue
//   round r (parity p):
//     k_wpath   the path engine (below): persistent query waves + a shade
//               wave per workgroup; a pixel's chain (its one ray in flight)
//               keeps going inside the kernel; once the round's work is used
//               up, running queries are suspended (state + LDS stack to the
//               carry queue) and resume next round
//     k_wexact  the rare rays handed to the exact stack DFS
//     k_wshade  shades k_wexact's results: the vertex (shade_vertex: material
//               logic and random draws) and its fold record, then either the
//               child ray, or -- path over -- the backward fold into the pixel
//               sum and the next sample's camera ray
//
// Every pixel has at most one ray in flight and consumes its random stream
// in the reference order (jitter, then vertex by vertex), so results are
// bit-identical however the rounds interleave pixels.  The host loops rounds
// until the fresh and carry queues are empty.  Compiled with
// -ffp-contract=off (pt_core.h).
#include <hip/hip_runtime.h>

#include "pt_devutil.h"
#include "pt_kernels.h"
#include "pt_coop.h"
#include "pt_query.h"
#include "pt_wprof.h"

namespace pt {

// enqueue a fresh ray with its plane result (RayIntersection's plane loop)
__device__ __forceinline__ void push_ray(const WaveParams& P, const RayQ& Q, uint32_t qi, const Ray& ray,
                                         uint32_t slot) {
    float pt;
    int pid;
    q_planes(P.S, ray, pt, pid);
    Q.ro[qi] = F4{ray.o.x, ray.o.y, ray.o.z, u2f(slot)};
    Q.rd[qi] = F4{ray.d.x, ray.d.y, ray.d.z, pt};
    Q.pid[qi] = pid;
    Q.ri[qi] = q_prep(P.S, ray);
}

// A value the optimiser must treat as new at this point: a loop-invariant expression
// built from it (a per-lane address) is then not hoisted into a VGPR held across the
// whole persistent loop, where it would spill
template <class T>
__device__ __forceinline__ T opaque_v(T v) { asm volatile("" : "+v"(v)); return v; }
// The launch's parameter block read where it is used: scalar loads from the kernarg
// segment at each use (its pointer is opaque there, so nothing is hoisted), for the
// parameters of a persistent loop's rare branches, which would otherwise hold SGPRs
// (and spill them to VGPR lanes) for the loop's whole life.  Its callers' kernels
// (k_wpath, k_wshade, k_wcoop) take the block as their only argument, at offset 0.
template <class K>
__device__ __forceinline__ const K& karg() {
#if defined(__HIP_DEVICE_COMPILE__)
    auto p = __builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *reinterpret_cast<const K*>(p);
#else
    __builtin_unreachable();   // (host pass: never called)
#endif
}
// a pixel's next camera sample, its jitter draws and camera ray (src/scene.cpp:189-196):
// x = pix % W, y = pix / W
__device__ __forceinline__ Ray camera_sample(const CamView& cam, Rng& R, uint32_t x, uint32_t y) {
    const float fx = (float)x + rng_uniform(R);
    const float fy = (float)y + rng_uniform(R);
    return camera_ray(cam, fx, fy);
}

// One finished query of a pixel's chain (src/scene.cpp:91-177 for the vertex,
// :198 for the fold): the vertex and its fold record -- or the miss -- and, at
// path end, the backward fold into the pixel sum.  Returns true with `ray` set
// to the chain's next ray (the child, or the next sample's camera ray); false
// when the pixel has reached this pass's target.  `ray` enters as the query ray.
// `sdone` returns whether a sample of the pixel ended here.
template <class EM>
__device__ __forceinline__ bool shade_item(const WaveParams& P, const EM& em, uint32_t slot, Ray& ray, uint32_t hid,
                                           bool& sdone) {
    bool emit = false;
    PixelHot hot = load_hot(P.st, slot);     // one 16-B load: RNG, vertex count, samples done
    uint32_t nv = hot.nv;
    uint32_t end = PE_LIVE;
    Rng R = hot.R;
    if (hid == 0xffffffffu) {
        end = PE_MISS;
    } else {
        // the closest hit's t, normal and side: recomputed from its primitive
        // (the query's own test, same operations -> same bits)
        Hit h;
        (void)prim_intersect(P.S.prims[hid], ray, h);
        uint32_t idm;
        float s1, s2;
        const bool cont = shade_vertex_e(P.S, em, P.S.shade[hid], R, ray, h, (int)hid, idm, s1, s2);
        HbmVStore vs = fold_store(P.st, slot);
        vs.put(nv, idm, s1, s2);
        ++nv;
        if (!cont) end = PE_TERM;
        else if (nv >= P.depth) end = PE_CUT;   // RayTrace(.., 0) = 0
        else emit = true;
    }
    sdone = end != PE_LIVE;
    if (end != PE_LIVE) {
        // path over: backward fold (deepest vertex first), src/scene.cpp:198 sum += ...
        f3 L = end == PE_MISS ? P.S.bg : mk3(0.f, 0.f, 0.f);
        HbmVStore vs = fold_store(P.st, slot);
        for (uint32_t k = nv; k > 0u; --k) {
            uint32_t idm;
            float s1, s2;
            vs.get(k - 1u, idm, s1, s2);
            L = fold_vertex(P.S, L, idm, s1, s2);
        }
        uint32_t pix;
        const f3 sum = load_sum_pix(P.st, slot, pix);
        store_sum(P.st, slot, sum + L, pix);   // src/scene.cpp:198 sum += RayTrace(...)
        const uint32_t done = hot.done + 1u;
        hot.done = done;
        nv = 0u;
        if (done < P.target) {
            // the pixel's next sample: jitter draws + camera ray
            const WaveParams& K = karg<WaveParams>();   // (read here: see end_item)
            ray = camera_sample(K.cam, R, pix % K.tm.W, pix / K.tm.W);
            emit = true;
        }
    }
    hot.nv = nv;
    hot.R = R;
    store_hot(P.st, slot, hot);               // one 16-B store
    return emit;
}

__global__ void __launch_bounds__(256) k_wcamera(WaveParams P) {
    // blocks append in about block order: the queue follows tile_order (Z-order of
    // the tiles, so the pixels resident together form compact image regions)
    const uint32_t t = P.tile_order ? P.tile_order[blockIdx.x] : blockIdx.x;
    const uint32_t slot = t * 256u + threadIdx.x;
    uint32_t x, y;
    const bool ok = slot_pixel(P.tm, t, threadIdx.x, x, y);
    bool want = false;
    Ray ray;
    if (ok) {
        PixelHot hot = load_hot(P.st, slot);
        Rng R = hot.R;
        uint32_t done = hot.done;
        if (P.depth == 0u) {
            // RayTrace(.., 0) = 0: only the jitter draws and sum += 0 per sample
            f3 sum = load_sum(P.st, slot);
            for (; done < P.target; ++done) {
                (void)camera_sample(P.cam, R, x, y);
                sum = sum + mk3(0.f, 0.f, 0.f);
            }
            store_sum(P.st, slot, sum, y * P.tm.W + x);
        } else if (done < P.target) {
            ray = camera_sample(P.cam, R, x, y);
            want = true;
        }
        hot.R = R;
        hot.done = done;
        hot.nv = 0u;
        store_hot(P.st, slot, hot);
    }
    // Pull order of the pass: pixels whose camera ray enters the BVH's boxes first
    // (the costly ones -- a pass ends with its slowest pixel, and pixels are pulled
    // as capacity frees up), the others after them (k_wcamera_merge).
    bool front = false;
    if (want) {
        // the (conservative) boxes of the aux BVH's top two levels: tighter than the
        // reference root box (root entries +2.6 % over it, two levels +2.5 % more)
        const f3 rinv = mk3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
        const f3 oinv = mk3(ray.o.x * rinv.x, ray.o.y * rinv.y, ray.o.z * rinv.z);
        for (uint32_t k = 0; k < PT_AUXW && k < P.n_top; ++k) {
            const AuxSL e = P.top[k];
            const uint32_t code = f2u(e.b.w);
            if (code == 0xffffffffu || !aux_box(e.a.x, e.a.y, e.a.z, e.a.w, e.b.x, e.b.y, rinv, oinv)) continue;
            if (code & 0x80000000u) {
                front = true;
                continue;
            }
            for (uint32_t j = 0; j < PT_AUXW; ++j) {   // one level down
                const AuxSL c = P.top[code * PT_AUXW + j];   // (code = 1 + k in the host's top copy)
                front = front || (f2u(c.b.w) != 0xffffffffu && aux_box(c.a.x, c.a.y, c.a.z, c.a.w, c.b.x, c.b.y, rinv, oinv));
            }
        }
    }
    __shared__ uint32_t agg[5];
    uint32_t* ctl = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t qf = block_append<4u>(ctl + C_FRONT, want && front, agg);
    const uint32_t qb = block_append<4u>(ctl + C_BACK, want && !front, agg);
    if (want) push_ray(P, front ? P.fq[P.parity] : P.fq[1u - P.parity], front ? qf : qb, ray, slot);
}

// the back class after the front one: fq[1-p][0, n_back) -> fq[p][n_front + i]
__global__ void __launch_bounds__(256) k_wcamera_merge(WaveParams P) {
    uint32_t* ctl = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t nf = ctl[C_FRONT], nb = ctl[C_BACK];
    const RayQ A = P.fq[P.parity], B = P.fq[1u - P.parity];
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nb; i += gridDim.x * 256u) {
        A.ro[nf + i] = B.ro[i];
        A.rd[nf + i] = B.rd[i];
        A.pid[nf + i] = B.pid[i];
        A.ri[nf + i] = B.ri[i];
    }
    if (blockIdx.x == 0u && threadIdx.x == 0u) ctl[C_FRESH] = nf + nb;
}

#define PT_SUSPENDED 0xfffffffeu   // done.id of a query suspended to the next round

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
// generic pointer, which the compiler may otherwise lower to flat instructions)
#if defined(__HIP_DEVICE_COMPILE__)
#define PT_LDS __attribute__((address_space(3)))
#else
#define PT_LDS
#endif
__device__ __forceinline__ uint32_t lds_read(const uint32_t& v) { return *(const volatile PT_LDS uint32_t*)&v; }
__device__ __forceinline__ void lds_write(uint32_t& v, uint32_t x) { *(volatile PT_LDS uint32_t*)&v = x; }
template <class T>
__device__ __forceinline__ T lds_get(const T* a, uint32_t i) { return ((const PT_LDS T*)a)[i]; }
template <class T>
__device__ __forceinline__ void lds_put(T* a, uint32_t i, const T& v) { ((PT_LDS T*)a)[i] = v; }

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
                // the round is over for this wave: suspend its running queries
                if (active) {
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
                if (lane_id() == 0u && ns) atomicSub(&L.resident, ns);
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
            if (kind == 0u || kind == pick) q_step(P.S, q, C, stk);
            // aux_extra more aux-node steps in the same trip for the lanes whose next step is one
#pragma unroll 1
            for (uint32_t x = 0; x < P.aux_extra; ++x) {
                const bool a2 = active && q.phase == Q_AUX && !(q.node & PT_LEAFQ);
                if (__ballot(a2) == 0ull) break;
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
                const WaveParams& K = karg<WaveParams>();
                const uint32_t k = atomicAdd(K.ctl + PT_CTL_SET * (1u - K.parity) + C_EXACT, 1u);
                K.ex.ro[k] = F4{q.ray.o.x, q.ray.o.y, q.ray.o.z, u2f(slot)};
                K.ex.rd[k] = F4{q.ray.d.x, q.ray.d.y, q.ray.d.z, u2f(k)};
                K.st.rec[2u * slot] = lds_get(L.H, (uint32_t)q.cid);   // (k_wshade shades it from HBM)
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
            // the workgroup with its pixel record)
            const WaveParams& K = karg<WaveParams>();
            const uint32_t k = wave_append(K.ctl + PT_CTL_SET * (1u - K.parity) + C_FRESH, emit);
            if (emit) {
                push_ray(K, K.fq[1u - K.parity], k, ray, slot);
                K.st.rec[2u * slot] = lds_get(L.H, cid);
            }
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
    // their pixel records
    const uint32_t h = lds_read(L.rq_head);
    for (uint32_t b = h; b < tail; b += 64u) {
        const uint32_t i = b + lane;
        const bool has = i < tail;
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
    static constexpr uint32_t SCAP = T == 64u ? 448u : T == 32u ? 192u : QC_SCAP_MIN;   // aux stack (also the
                                                                                      // leader's exact DFS stack)
    static constexpr uint32_t CCAP = 5u * T;                    // candidates (< T + 4 T at any time)
    static constexpr uint32_t HCAP = T >= 32u ? 32u : T == 16u ? 16u : 12u;   // hitting leaves per query (more: the
                                                                              // exact DFS); LDS fits 3 WGs per CU
    uint32_t stk[SCAP];
    uint32_t cand[CCAP];
    uint32_t hl[QH_N][HCAP];       // hitting leaves: index, first-min t, its prim, hit normal and side,
                                   // ancestor-list info
    uint32_t perm[HCAP];           // their preorder: perm[k] = the entry of the k-th smallest index
    uint32_t r_idx[HCAP], r_t[HCAP];   // entered hits so far (preorder)
    Shade fold_sh[QC_FOLD];        // the chain's fold records: the vertex prim's shading record ...
    uint4 fold[QC_FOLD];           // ... and {idm, s1, s2, -}
    uint4 sum;                     // the pixel's sum.rgb and global index (rec[2 slot + 1]) while the team
                                   // owns it (touched at path ends only: registers would spill)
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
enum : uint32_t { LC_RAYS = 0u, LC_NODES, LC_PTESTS, LC_SPARE, LC_AUX, LC_FALLB, LC_HANDED, LC_N = 8u };
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
    const uint32_t slim = SCAP - reserve;
    bvh = false;
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
    const bool dec = run && !ovf;
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
template <uint32_t T, bool BIG>
__global__ void __launch_bounds__(64u * QC_WAVES) __attribute__((amdgpu_waves_per_eu(QC_WAVES_PER_EU, QC_WAVES_PER_EU)))
k_wcoop(WaveParams P) {
    __shared__ QcTeamLds<T> Ls[QC_WAVES * (64u / T)];
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
    const uint32_t stop_n = late ? 0u
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
                    if (tl < hot.nv && (!BIG || tl < QC_FOLD)) {
                        // the current path's vertices so far (written by the path engine; any
                        // beyond QC_FOLD stay in HBM)
                        const uint4 f = P.st.fold[(size_t)slot * P.st.depth + opaque_v(tl)];
                        L.fold[tl] = f;
                        L.fold_sh[tl] = P.S.shade[f.x & 0x3fffffffu];
                    }
                }
            }
        }
        if (__ballot(have) == 0ull) break;
        bool ex, bvh;
        Hit h;
        int id = qc_team<T>(P.S, Q, L, have, ray, Pt, pid, pre, P.coop_reserve, lc, ex, h, bvh QC_CP_PASS);
        bool emit = false, sdone = false;
        QC_T0();
        if (tl == 0u && have) {
            if (ex) {
                // the exact stack DFS (non-finite rays, too many hitting leaves)
                LdsMemN<1u> stk{L.stk};
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
        const uint32_t k = wave_append(P.yield_ctr, have && tl == 0u);
        // (k < carry_cap always: the host sizes the stops to the carry queue; a yield past it
        // would be a lost chain, which the resolve reports, never a write past the queue)
        if (have && tl == 0u && k < P.carry_cap) {
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
        if (have && tl < nv && (!BIG || tl < QC_FOLD)) P.st.fold[(size_t)slot * P.st.depth + tl] = L.fold[tl];
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
            const uint32_t k2 = wave_append(P.yield_ctr, on);
            if (on && k2 < P.carry_cap) {
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
        const uint32_t to[LC_N] = {0u, 1u, 2u, 3u, 5u, 6u, CTR_HANDON, 0u};
        for (uint32_t k = 0; k < LC_HANDED + 1u; ++k)
            if (v[k]) atomicAdd(ctr + to[k], (unsigned long long)v[k]);
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

// The cooperative engine's intake order.  Its launch runs until the pixel with the
// most work left reaches the pass target, and a chain keeps its team to the end, so
// with more chains than teams (a hand-over at 49 k chains, 24.6 k resident teams
// of 8) the chains that wait for a team must be the ones with the least left.  A
// counting sort of the round's work items (suspended queries, then fresh rays) by
// their pixels' remaining samples, in PT_ORDER_BUCKETS buckets, most first.
__device__ __forceinline__ uint32_t coop_order_bucket(const WaveParams& P, uint32_t gi, uint32_t n_carry) {
    const uint32_t slot = gi < n_carry ? P.cq[P.parity][(size_t)gi * P.carry_words + sizeof(Query) / 4u]
                                       : f2u(P.fq[P.parity].ro[gi - n_carry].w);
    const uint32_t done = P.st.rec[2u * slot].w;
    const uint32_t rem = done < P.target ? P.target - done : 0u;
    const uint64_t b = (uint64_t)rem * PT_ORDER_BUCKETS / ((uint64_t)P.target + 1u);
    return PT_ORDER_BUCKETS - 1u - (uint32_t)b;   // bucket 0 = the most samples left
}
__global__ void __launch_bounds__(256) k_coop_hist(WaveParams P) {
    __shared__ uint32_t h[PT_ORDER_BUCKETS];
    const uint32_t* in = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t n_carry = in[C_CARRY], n = in[C_FRESH] + n_carry;
    h[threadIdx.x] = 0u;
    __syncthreads();
    for (uint32_t gi = blockIdx.x * 256u + threadIdx.x; gi < n; gi += gridDim.x * 256u)
        atomicAdd(&h[coop_order_bucket(P, gi, n_carry)], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(P.order_cur + PT_ORDER_BUCKETS + threadIdx.x, h[threadIdx.x]);
}
__global__ void __launch_bounds__(256) k_coop_scatter(WaveParams P) {
    __shared__ uint32_t base[PT_ORDER_BUCKETS];
    const uint32_t* in = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t n_carry = in[C_CARRY], n = in[C_FRESH] + n_carry;
    if (threadIdx.x == 0u) {
        // (every block scans the 256 counts itself)
        uint32_t t = 0u;
        for (uint32_t b = 0; b < PT_ORDER_BUCKETS; ++b) {
            base[b] = t;
            t += P.order_cur[PT_ORDER_BUCKETS + b];
        }
    }
    __syncthreads();
    for (uint32_t gi = blockIdx.x * 256u + threadIdx.x; gi < n; gi += gridDim.x * 256u) {
        const uint32_t b = coop_order_bucket(P, gi, n_carry);
        P.order[base[b] + atomicAdd(P.order_cur + b, 1u)] = gi;
    }
}

// The early cooperative launch's queue (pt_launch_side_take): item j < k of the
// intake order, a fresh ray copied as it is, a suspended query as a restart record
// (the cooperative engine restarts a query from its ray and slot alone).  side_ctl's
// C_CARRY / C_FRESH count the two kinds as they are appended (the launch's round
// counters: carry records first in its work numbering, as in every round).
__global__ void __launch_bounds__(256) k_side_take(WaveParams P, uint32_t k, RayQ side, uint32_t* side_carry,
                                                   uint32_t* side_ctl) {
    const uint32_t* in = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t n_carry = in[C_CARRY];
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    const bool on = j < k;
    const uint32_t gi = on ? P.order[j] : 0u;
    const bool carry = on && gi < n_carry;
    const uint32_t kc = wave_append(side_ctl + C_CARRY, carry);
    const uint32_t kf = wave_append(side_ctl + C_FRESH, on && !carry);
    if (carry) {
        const uint32_t* w = P.cq[P.parity] + (size_t)gi * P.carry_words;
        uint32_t* d = side_carry + (size_t)kc * P.carry_words;
        *reinterpret_cast<Ray*>(d) = reinterpret_cast<const Query*>(w)->ray;
        d[sizeof(Query) / 4u] = w[sizeof(Query) / 4u];
    } else if (on) {
        const RayQ& F = P.fq[P.parity];
        const uint32_t fi = gi - n_carry;
        side.ro[kf] = F.ro[fi];
        side.rd[kf] = F.rd[fi];
        side.pid[kf] = F.pid[fi];
        side.ri[kf] = F.ri[fi];
    }
}

// The rays the path engine hands back (Q_EXACT: an aux stack deeper than the
// engine's LDS stack, a hitting-leaf list full of entered hits, non-finite
// components); 64-lane workgroups, one ray per lane, stack in LDS.  The replay
// first, with a stack as deep as the wide aux tree needs (a ray that only
// overflowed the engine's 16 words -- the common case -- costs its ~100 aux
// steps, not a whole reference DFS of ~10^4 node visits, tens of ms on one lane),
// then the exact stack DFS for what the replay cannot take (q_run).
__global__ void __launch_bounds__(64) k_wexact(WaveParams P) {
    extern __shared__ uint32_t lds_stack[];
    uint32_t* out = P.ctl + PT_CTL_SET * (1u - P.parity);
    const uint32_t n = out[C_EXACT];
    const uint32_t words = P.max_stack > P.aux_stack ? P.max_stack : P.aux_stack;
    LdsMemN<64u> stk{lds_stack + threadIdx.x, words, words};   // (+ a trash word)
    QCounts C{0u, 0u, 0u, 0u};
    uint32_t err = 0u;
    for (uint32_t k = blockIdx.x * 64u + threadIdx.x; k < n; k += gridDim.x * 64u) {
        const F4 o = P.ex.ro[k], d = P.ex.rd[k];
        Ray ray;
        ray.o = mk3(o.x, o.y, o.z);
        ray.d = mk3(d.x, d.y, d.z);
        Hit h;
        uint32_t used = 0u;
        const int id = q_run(P.S, ray, stk, h, C, used);
        // q_run flags a recomputed hit that differs from the query's in the plane count's
        // top bit (must never happen): an exactness error, not plane tests
        err += C.planes >> 31;
        C.planes = 0u;   // (the path engine counted this ray's plane tests when it took it)
        const uint32_t j = f2u(d.w);   // the ray's work index
        P.done.ro[j] = o;
        P.done.rd[j] = F4{d.x, d.y, d.z, 0.f};
        P.done.id[j] = id < 0 ? 0xffffffffu : (uint32_t)id;
    }
    unsigned long long* ctr = ctr_copy(P.counters);
    wave_add_u64(ctr + 1, C.nodes);
    wave_add_u64(ctr + 2, C.ptests);
    wave_add_u64(ctr + 4, err);
}

__global__ void __launch_bounds__(256) k_wshade(WaveParams P) {
    __shared__ uint32_t agg[5];
    uint32_t* out = P.ctl + PT_CTL_SET * (1u - P.parity);
    // the exact-DFS results of this round (the path engine shades everything else itself)
    const uint32_t n = out[C_EXACT];
    const RayQ N = P.fq[1u - P.parity];
    const uint32_t stride = gridDim.x * 256u;
    // grid-stride with a block-uniform trip count (the block-aggregated append needs every thread)
    for (uint32_t base = blockIdx.x * 256u; base < n; base += stride) {
        const uint32_t i = base + threadIdx.x;
        bool emit = false, sdone = false;
        Ray ray;
        uint32_t slot = 0u;
        const uint32_t hid = i < n ? P.done.id[i] : PT_SUSPENDED;
        if (hid != PT_SUSPENDED) {
            const F4 o = P.done.ro[i], d = P.done.rd[i];
            slot = f2u(o.w);
            ray.o = mk3(o.x, o.y, o.z);
            ray.d = mk3(d.x, d.y, d.z);
            emit = shade_item(P, EmitGlobal{P.S}, slot, ray, hid, sdone);
        }
        if (P.progress) {
            const uint32_t nd = (uint32_t)__popcll(__ballot(sdone));
            if (nd && (threadIdx.x & 63u) == 0u)
                __hip_atomic_fetch_add(P.progress, (unsigned long long)nd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const uint32_t qn = block_append<4u>(out + C_FRESH, emit, agg);
        if (emit) push_ray(P, N, qn, ray, slot);
    }
}

}  // namespace pt

extern "C++" {
// load this file's code object onto the current device (no launch)
hipError_t pt_preload_kernels_wave() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(pt::k_wpath<false>));
}

hipError_t pt_launch_wave_start(pt::WaveParams p, hipStream_t s) {
    hipError_t e = hipMemsetAsync(p.ctl, 0, 4u * 2u * PT_CTL_SET, s);
    if (e != hipSuccess) return e;
    p.parity = 0u;
    hipLaunchKernelGGL(pt::k_wcamera, dim3(p.n_tiles_local), dim3(256), 0, s, p);
    hipLaunchKernelGGL(pt::k_wcamera_merge, dim3(p.n_tiles_local < 1024u ? p.n_tiles_local : 1024u), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t pt_launch_coop_order(pt::WaveParams p, uint32_t n, hipStream_t s) {
    hipError_t e = hipMemsetAsync(p.order_cur, 0, 2u * PT_ORDER_BUCKETS * 4u, s);
    if (e != hipSuccess) return e;
    const uint32_t grid = n / 256u + 1u < 1024u ? n / 256u + 1u : 1024u;
    hipLaunchKernelGGL(pt::k_coop_hist, dim3(grid), dim3(256), 0, s, p);
    hipLaunchKernelGGL(pt::k_coop_scatter, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t pt_launch_side_take(pt::WaveParams p, uint32_t k, pt::RayQ side, uint32_t* side_carry, uint32_t* side_ctl,
                               hipStream_t s) {
    if (k == 0u) return hipSuccess;
    hipLaunchKernelGGL(pt::k_side_take, dim3((k + 255u) / 256u), dim3(256), 0, s, p, k, side, side_carry, side_ctl);
    return hipGetLastError();
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
    else if (team == 16u) hipLaunchKernelGGL((pt::k_wcoop<16u, false>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    else if (team == 32u) hipLaunchKernelGGL((pt::k_wcoop<32u, false>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    else hipLaunchKernelGGL((pt::k_wcoop<64u, false>), dim3(grid), dim3(64u * QC_WAVES), 0, s, p);
    if (e1 && (e = hipEventRecord(e1, s)) != hipSuccess) return e;
    return hipGetLastError();
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
    const uint32_t xw = p.max_stack > p.aux_stack ? p.max_stack : p.aux_stack;
    const uint32_t exact_lds = 64u * 4u * ((xw ? xw : 1u) + 1u);
    hipLaunchKernelGGL(pt::k_wexact, dim3(64), dim3(64), exact_lds, s, p);
    hipLaunchKernelGGL(pt::k_wshade, dim3(shade_grid), dim3(256), 0, s, p);
    return hipGetLastError();
}

}
