// pt_kernels.hip -- gfx950 kernels of the hw5 render loop.
//
//   k_init     seed each owned pixel's RNG stream (global index y*W+x) and zero its sum
//   k_trace    advance every owned pixel by `spp` samples (src/scene.cpp:189-203):
//              one pixel per lane, 16x16-pixel tiles per 256-thread workgroup
//              (a wave = 16x4 pixels: neighbouring rays walk the same nodes);
//              per-lane traversal state (aux stack, candidate list, or the exact
//              DFS stack) lives in LDS ([word][lane], conflict-free),
//              the per-vertex fold records in a lane-strided HBM scratch
//   k_resolve  mean = (1/S)*sum, ACES + saturate (f32) and the exact gamma/8-bit
//              threshold table, packed per tile for the framebuffer gather
//
// Compiled with -ffp-contract=off (see pt_core.h).
#include <hip/hip_runtime.h>

#include "pt_kernels.h"
#include "pt_trace.h"

namespace pt {

// per-lane word memory in LDS, [word][lane] (consecutive lanes -> consecutive banks)
struct LdsMem {
    uint32_t* base;
    __device__ __forceinline__ void set(uint32_t i, uint32_t v) { base[i * 256u] = v; }
    __device__ __forceinline__ uint32_t get(uint32_t i) const { return base[i * 256u]; }
};

struct HbmVStore {
    uint32_t* base;   // + slot
    uint32_t stride;  // n_slots
    __device__ __forceinline__ void put(uint32_t k, uint32_t idm, float s1, float s2) {
        base[(3u * k) * stride] = idm;
        base[(3u * k + 1u) * stride] = f2u(s1);
        base[(3u * k + 2u) * stride] = f2u(s2);
    }
    __device__ __forceinline__ void get(uint32_t k, uint32_t& idm, float& s1, float& s2) const {
        idm = base[(3u * k) * stride];
        s1 = u2f(base[(3u * k + 1u) * stride]);
        s2 = u2f(base[(3u * k + 2u) * stride]);
    }
};

// owned slot -> global pixel (16x16 tiles of the window dealt round-robin to ranks)
__device__ __forceinline__ bool slot_pixel(const TileMap& tm, uint32_t tile_local, uint32_t lane, uint32_t& x,
                                           uint32_t& y) {
    const uint32_t gt = tile_local * tm.world + tm.rank;
    const uint32_t tx = gt % tm.tiles_x, ty = gt / tm.tiles_x;
    const uint32_t wx = tx * 16u + (lane & 15u), wy = ty * 16u + (lane >> 4);
    x = tm.x0 + wx;
    y = tm.y0 + wy;
    return gt < tm.n_tiles && wx < tm.ww && wy < tm.wh;
}

__device__ __forceinline__ void wave_add_u64(unsigned long long* dst, unsigned long long v) {
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63u) == 0u && v != 0ull) atomicAdd(dst, v);
}

__global__ void __launch_bounds__(256) k_init(InitParams P) {
    const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
    uint32_t x, y;
    const bool ok = slot_pixel(P.tm, blockIdx.x, threadIdx.x, x, y);
    const Rng r = rng_seed(ok ? y * P.tm.W + x : 0u);
    P.st.rng_x[slot] = r.x;
    P.st.rng_saved[slot] = r.saved;
    P.st.rng_flag[slot] = r.saved_ok;
    P.st.sum[slot] = 0.f;
    P.st.sum[P.st.n_slots + slot] = 0.f;
    P.st.sum[2u * P.st.n_slots + slot] = 0.f;
}

__global__ void __launch_bounds__(256) k_trace(TraceParams P) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
    uint32_t x, y;
    const bool ok = slot_pixel(P.tm, blockIdx.x, threadIdx.x, x, y);
    Counts C;
    C.rays = C.nodes = C.ptests = C.planes = C.aux = C.fallbacks = 0ull;
    C.errs = 0u;
    if (ok) {
        Rng R;
        R.x = P.st.rng_x[slot];
        R.saved = P.st.rng_saved[slot];
        R.saved_ok = P.st.rng_flag[slot];
        f3 sum = mk3(P.st.sum[slot], P.st.sum[P.st.n_slots + slot], P.st.sum[2u * P.st.n_slots + slot]);
        LdsMem stk{lds_stack + threadIdx.x};
        HbmVStore vs{P.vscratch + slot, P.st.n_slots};
        const float fxb = (float)x, fyb = (float)y;
        for (uint32_t s = 0; s < P.spp; ++s) {
            const float fx = fxb + rng_uniform(R);
            const float fy = fyb + rng_uniform(R);
            const Ray ray = camera_ray(P.cam, fx, fy);
            sum = sum + trace_path(P.S, P.cfg, ray, P.depth, R, stk, vs, C);
        }
        P.st.rng_x[slot] = R.x;
        P.st.rng_saved[slot] = R.saved;
        P.st.rng_flag[slot] = R.saved_ok;
        P.st.sum[slot] = sum.x;
        P.st.sum[P.st.n_slots + slot] = sum.y;
        P.st.sum[2u * P.st.n_slots + slot] = sum.z;
    }
    wave_add_u64(P.counters + 0, C.rays);
    wave_add_u64(P.counters + 1, C.nodes);
    wave_add_u64(P.counters + 2, C.ptests);
    wave_add_u64(P.counters + 3, C.planes);
    wave_add_u64(P.counters + 4, (unsigned long long)C.errs);
    wave_add_u64(P.counters + 5, C.aux);
    wave_add_u64(P.counters + 6, C.fallbacks);
}

__global__ void __launch_bounds__(256) k_resolve(ResolveParams P) {
    __shared__ float thr[256];
    thr[threadIdx.x] = P.thr[threadIdx.x];
    __syncthreads();
    const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
    const float inv = 1.f / (float)P.samples;    // src/scene.cpp:201: (1.f / SAMPLES) * sum
    const float m[3] = {inv * P.st.sum[slot], inv * P.st.sum[P.st.n_slots + slot],
                        inv * P.st.sum[2u * P.st.n_slots + slot]};
    uint8_t* o = P.out + (size_t)slot * 3u;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = (uint8_t)quantize_gamma(aces1(m[c]), thr);
    if (P.rad) {
#pragma unroll
        for (int c = 0; c < 3; ++c) P.rad[(size_t)slot * 3u + c] = m[c];
    }
}

}  // namespace pt

// ---------------------------------------------------------------- launchers
extern "C++" {
hipError_t pt_launch_init(const pt::InitParams& p, uint32_t n_tiles, hipStream_t s) {
    hipLaunchKernelGGL(pt::k_init, dim3(n_tiles), dim3(256), 0, s, p);
    return hipGetLastError();
}
hipError_t pt_launch_trace(const pt::TraceParams& p, uint32_t n_tiles, uint32_t lds_bytes, hipStream_t s) {
    hipLaunchKernelGGL(pt::k_trace, dim3(n_tiles), dim3(256), lds_bytes, s, p);
    return hipGetLastError();
}
hipError_t pt_launch_resolve(const pt::ResolveParams& p, uint32_t n_tiles, hipStream_t s) {
    hipLaunchKernelGGL(pt::k_resolve, dim3(n_tiles), dim3(256), 0, s, p);
    return hipGetLastError();
}
}
