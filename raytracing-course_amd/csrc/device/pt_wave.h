// pt_wave.h -- what the wavefront kernels share (pt_wave.hip, pt_path.hip, pt_wcoop.hip).
//
// A pass advances every owned pixel by `target` samples (src/scene.cpp:
// 189-203) through rounds of launches on one stream:
//
//   k_wcamera   (pass start, pt_wave.hip) the first sample's 2 jitter draws and
//               camera ray (src/scene.cpp:180-199) of every pixel -> fresh queue
//   round r (parity p):
//     k_wpath   (pt_path.hip) the path engine: persistent query waves + a shade
//               wave per workgroup; a pixel's chain (its one ray in flight)
//               keeps going inside the kernel; once the round's work is used
//               up, running queries are suspended (state + LDS stack to the
//               carry queue) and resume next round
//     k_wexact  (pt_wave.hip) the rare rays handed to the exact stack DFS
//     k_wshade  (pt_wave.hip) shades k_wexact's results: the vertex (shade_vertex:
//               material logic and random draws) and its fold record, then either
//               the child ray, or -- path over -- the backward fold into the pixel
//               sum and the next sample's camera ray
//   end of a pass: k_wcoop (pt_wcoop.hip), the cooperative engine -- a team of
//               lanes per remaining chain
//
// Every pixel has at most one ray in flight and consumes its random stream
// in the reference order (jitter, then vertex by vertex), so results are
// bit-identical however the rounds interleave pixels.  The host loops rounds
// until the fresh and carry queues are empty.  Compiled with
// -ffp-contract=off (pt_core.h).
#pragma once
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


#define PT_SUSPENDED 0xfffffffeu   // done.id of a query suspended to the next round

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

}  // namespace pt

// launchers shared between the wavefront units (host side)
hipError_t pt_launch_exact_shade(const pt::WaveParams& p, uint32_t shade_grid, hipStream_t s);
hipError_t pt_preload_kernels_path();
hipError_t pt_preload_kernels_coop();
