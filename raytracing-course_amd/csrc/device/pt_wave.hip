// pt_wave.hip -- wavefront form of the hw5 render loop on gfx950.
//
// One camera sample of every owned pixel = a short pipeline of launches on
// one stream (no host round trips; counts stay on the device):
//
//   k_wcamera        per pixel: the sample's 2 jitter draws, the camera ray
//                    (src/scene.cpp:189-199), appended to queue 0
//   for b < RAY_DEPTH:
//     k_wisect       persistent, per-lane refilling closest-hit query
//                    (pt_query.h): lanes pull rays in wave batches, one node
//                    visit per loop trip, so the candidate tail of a few rays
//                    never idles the rest of the wave
//     k_wexact       the rare rays the replay hands back (exact stack DFS)
//     k_wshade       per ray: the vertex's material logic and random draws
//                    (shade_vertex), its fold record, and the child ray
//                    appended to queue b+1 (wave-aggregated append)
//   k_wfold          per pixel: backward fold of the vertex records
//                    (bit-identical to the reference recursion) into the sum
//
// Each pixel's random stream is consumed in exactly the reference order: a
// pixel has at most one ray in flight and its draws happen in camera, then
// shade b = 0, 1, ... order.  Compiled with -ffp-contract=off (pt_core.h).
#include <hip/hip_runtime.h>

#include "pt_devutil.h"
#include "pt_kernels.h"
#include "pt_query.h"

namespace pt {

__global__ void __launch_bounds__(256) k_wcamera(WaveParams P) {
    const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
    uint32_t x, y;
    const bool ok = slot_pixel(P.tm, blockIdx.x, threadIdx.x, x, y);
    Ray ray;
    if (ok) {
        Rng R;
        R.x = P.st.rng_x[slot];
        R.saved = P.st.rng_saved[slot];
        R.saved_ok = P.st.rng_flag[slot];
        const float fx = (float)x + rng_uniform(R);
        const float fy = (float)y + rng_uniform(R);
        ray = camera_ray(P.cam, fx, fy);
        P.st.rng_x[slot] = R.x;
        P.st.rng_flag[slot] = R.saved_ok;
        P.st.rng_saved[slot] = R.saved;
        P.pstate[slot] = P.depth ? (PE_LIVE << 8) : (PE_CUT << 8);
    }
    const bool want = ok && P.depth > 0u;
    const uint32_t qi = wave_append(P.ctl + 0, want);
    if (want) {
        P.q[0].ro[qi] = F4{ray.o.x, ray.o.y, ray.o.z, u2f(slot)};
        P.q[0].rd[qi] = F4{ray.d.x, ray.d.y, ray.d.z, 0.f};
    }
}

__device__ __forceinline__ void write_hit(const WaveParams& P, uint32_t qi, int id, const Hit& h) {
    if (id < 0) {
        P.hits.id[qi] = 0xffffffffu;
        return;
    }
    P.hits.th[qi] = F4{h.t, h.n.x, h.n.y, h.n.z};
    P.hits.id[qi] = (uint32_t)id | (h.interior ? 0x80000000u : 0u);
}

#define PT_BATCH 64u
#define PT_REFILL_MIN 16u

__global__ void __launch_bounds__(256) k_wisect(WaveParams P) {
    extern __shared__ uint32_t lds_stack[];
    LdsMem stk{lds_stack + threadIdx.x};
    const uint32_t b = P.bounce;
    const uint32_t count = P.ctl[b];
    uint32_t* head = P.ctl + P.depth + 1u + b;
    const WaveQueue Q = P.q[b & 1u];
    // wave-uniform batch of queue indices
    uint32_t bbase = 0u, bleft = 0u;
    bool exhausted = false;
    bool active = false;
    uint32_t qi = 0u;
    Query q;
    QCounts C{0u, 0u, 0u, 0u};
    uint32_t rays = 0u, fallbacks = 0u, init_exact = 0u;
    for (;;) {
        const unsigned long long idle = __ballot(!active);
        uint32_t nidle = (uint32_t)__popcll(idle);
        if (!exhausted && (nidle >= PT_REFILL_MIN || nidle == 64u)) {
            uint32_t rank = lanes_below(idle);
            bool fresh = false;
            while (nidle > 0u) {
                if (bleft == 0u) {
                    uint32_t v = 0u;
                    if (lane_id() == 0u) v = atomicAdd(head, PT_BATCH);
                    v = __builtin_amdgcn_readfirstlane(v);
                    if (v >= count) { exhausted = true; break; }
                    bbase = v;
                    bleft = count - v < PT_BATCH ? count - v : PT_BATCH;
                }
                const uint32_t take = nidle < bleft ? nidle : bleft;
                if (!active && !fresh) {
                    if (rank < take) { qi = bbase + rank; fresh = true; }
                    else rank -= take;
                }
                bbase += take;
                bleft -= take;
                nidle -= take;
            }
            if (fresh) {
                const F4 o = Q.ro[qi], d = Q.rd[qi];
                Ray ray;
                ray.o = mk3(o.x, o.y, o.z);
                ray.d = mk3(d.x, d.y, d.z);
                rays++;
                q_init(P.S, ray, q, C);
                if (q.phase == Q_EXACT) init_exact++;
                active = true;
            }
        }
        if (__ballot(active) == 0ull) break;
        if (active) {
            if (q.phase == Q_AUX || q.phase == Q_REPLAY) q_step(P.S, P.aux, P.n_aux, q, C, stk);
            if (q.phase == Q_DONE) {
                write_hit(P, qi, q.res_id, q.res);
                active = false;
            } else if (q.phase == Q_EXACT) {
                const uint32_t k = atomicAdd(P.ctl + 2u * (P.depth + 1u) + b, 1u);
                P.fb[k] = qi;
                fallbacks++;
                active = false;
            }
        }
    }
    wave_add_u64(P.counters + 0, rays);
    wave_add_u64(P.counters + 1, C.nodes);
    wave_add_u64(P.counters + 2, C.ptests);
    wave_add_u64(P.counters + 3, C.planes);
    wave_add_u64(P.counters + 5, C.aux);
    wave_add_u64(P.counters + 6, fallbacks);
    wave_add_u64(P.counters + 7, init_exact);
}

// exact stack DFS for the handed-back rays; 64-lane workgroups, stack in LDS
__global__ void __launch_bounds__(64) k_wexact(WaveParams P) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t b = P.bounce;
    const uint32_t n = P.ctl[2u * (P.depth + 1u) + b];
    const WaveQueue Q = P.q[b & 1u];
    LdsMemN<64u> stk{lds_stack + threadIdx.x};
    QCounts C{0u, 0u, 0u, 0u};
    for (uint32_t k = blockIdx.x * 64u + threadIdx.x; k < n; k += gridDim.x * 64u) {
        const uint32_t qi = P.fb[k];
        const F4 o = Q.ro[qi], d = Q.rd[qi];
        Ray ray;
        ray.o = mk3(o.x, o.y, o.z);
        ray.d = mk3(d.x, d.y, d.z);
        Hit h;
        const int id = q_exact(P.S, ray, stk, h, C);
        write_hit(P, qi, id, h);
    }
    wave_add_u64(P.counters + 1, C.nodes);
    wave_add_u64(P.counters + 2, C.ptests);
    wave_add_u64(P.counters + 3, C.planes);
}

__global__ void __launch_bounds__(256) k_wshade(WaveParams P) {
    const uint32_t b = P.bounce;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const bool in = i < P.ctl[b];
    bool cont = false;
    Ray ray;
    uint32_t slot = 0u;
    if (in) {
        const WaveQueue Q = P.q[b & 1u];
        const F4 o = Q.ro[i], d = Q.rd[i];
        slot = f2u(o.w);
        ray.o = mk3(o.x, o.y, o.z);
        ray.d = mk3(d.x, d.y, d.z);
        const uint32_t hid = P.hits.id[i];
        const uint32_t nv = P.pstate[slot] & 0xffu;
        if (hid == 0xffffffffu) {
            P.pstate[slot] = nv | (PE_MISS << 8);
        } else {
            const F4 th = P.hits.th[i];
            Hit h;
            h.t = th.x;
            h.n = mk3(th.y, th.z, th.w);
            h.interior = hid >> 31;
            const int id = (int)(hid & 0x7fffffffu);
            Rng R;
            R.x = P.st.rng_x[slot];
            R.saved = P.st.rng_saved[slot];
            R.saved_ok = P.st.rng_flag[slot];
            uint32_t idm;
            float s1, s2;
            cont = shade_vertex(P.S, R, ray, h, id, idm, s1, s2);
            P.st.rng_x[slot] = R.x;
            P.st.rng_saved[slot] = R.saved;
            P.st.rng_flag[slot] = R.saved_ok;
            HbmVStore vs{P.vscratch + slot, P.st.n_slots};
            vs.put(nv, idm, s1, s2);
            uint32_t end = PE_LIVE;
            if (!cont) end = PE_TERM;
            else if (b + 1u >= P.depth) { end = PE_CUT; cont = false; }   // RayTrace(.., 0) = 0
            P.pstate[slot] = (nv + 1u) | (end << 8);
        }
    }
    const uint32_t qn = wave_append(P.ctl + b + 1u, cont);
    if (cont) {
        const WaveQueue N = P.q[(b + 1u) & 1u];
        N.ro[qn] = F4{ray.o.x, ray.o.y, ray.o.z, u2f(slot)};
        N.rd[qn] = F4{ray.d.x, ray.d.y, ray.d.z, 0.f};
    }
}

__global__ void __launch_bounds__(256) k_wfold(WaveParams P) {
    const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
    uint32_t x, y;
    if (!slot_pixel(P.tm, blockIdx.x, threadIdx.x, x, y)) return;
    const uint32_t ps = P.pstate[slot];
    uint32_t nv = ps & 0xffu;
    f3 L = (ps >> 8) == PE_MISS ? P.S.bg : mk3(0.f, 0.f, 0.f);
    HbmVStore vs{P.vscratch + slot, P.st.n_slots};
    while (nv > 0u) {
        --nv;
        uint32_t idm;
        float s1, s2;
        vs.get(nv, idm, s1, s2);
        L = fold_vertex(P.S, L, idm, s1, s2);
    }
    // src/scene.cpp:198: sum += RayTrace(...)
    P.st.sum[slot] = P.st.sum[slot] + L.x;
    P.st.sum[P.st.n_slots + slot] = P.st.sum[P.st.n_slots + slot] + L.y;
    P.st.sum[2u * P.st.n_slots + slot] = P.st.sum[2u * P.st.n_slots + slot] + L.z;
}

}  // namespace pt

extern "C++" {
hipError_t pt_launch_wave_sample(pt::WaveParams p, uint32_t isect_grid, hipStream_t s) {
    const uint32_t nt = p.n_tiles_local;
    const uint32_t D = p.depth;
    hipError_t e = hipMemsetAsync(p.ctl, 0, 4u * (3u * (D + 1u)), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pt::k_wcamera, dim3(nt), dim3(256), 0, s, p);
    const uint32_t exact_lds = 64u * 4u * (p.max_stack ? p.max_stack : 1u);
    for (uint32_t b = 0; b < D; ++b) {
        p.bounce = b;
        hipLaunchKernelGGL(pt::k_wisect, dim3(isect_grid), dim3(256), 1024u * p.aux_stack, s, p);
        hipLaunchKernelGGL(pt::k_wexact, dim3(64), dim3(64), exact_lds, s, p);
        hipLaunchKernelGGL(pt::k_wshade, dim3(nt), dim3(256), 0, s, p);
    }
    hipLaunchKernelGGL(pt::k_wfold, dim3(nt), dim3(256), 0, s, p);
    return hipGetLastError();
}
}
