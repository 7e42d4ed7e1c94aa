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

#include "pt_devutil.h"
#include "pt_kernels.h"
#include "pt_trace.h"

namespace pt {

__global__ void __launch_bounds__(256) k_init(InitParams P) {
    const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
    uint32_t x, y;
    const bool ok = slot_pixel(P.tm, blockIdx.x, threadIdx.x, x, y);
    PixelHot h;
    h.R = rng_seed(ok ? y * P.tm.W + x : 0u);
    h.nv = 0u;
    h.done = 0u;
    store_hot(P.st, slot, h);
    store_sum(P.st, slot, mk3(0.f, 0.f, 0.f), ok ? y * P.tm.W + x : 0u);
}

// V bit 0: filtered node tests + flat replay loop (FAST); bit 1: XCD-banded
// tile order -- workgroup b runs on XCD b % 8, so XCD x is given the x-th
// contiguous band of tiles and its 4 MB L2 caches that band's working set.
template <int V>
__global__ void __launch_bounds__(256) k_trace(TraceParams P) {
    extern __shared__ uint32_t lds_stack[];
    uint32_t tile = blockIdx.x;
    if (V & 2) {
        const uint32_t per = (P.n_tiles_local + 7u) / 8u;
        tile = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
        if (tile >= P.n_tiles_local) return;
    }
    uint64_t t_start = 0;
    if (P.wg_prof && threadIdx.x == 0) t_start = __builtin_amdgcn_s_memrealtime();
    const uint32_t slot = tile * 256u + threadIdx.x;
    uint32_t x, y;
    const bool ok = slot_pixel(P.tm, tile, threadIdx.x, x, y);
    Counts C;
    C.rays = C.nodes = C.ptests = C.planes = C.aux = C.fallbacks = 0ull;
    C.errs = 0u;
    if (ok) {
        PixelHot hot = load_hot(P.st, slot);
        Rng R = hot.R;
        f3 sum = load_sum(P.st, slot);
        LdsMem stk{lds_stack + threadIdx.x};
        HbmVStore vs = fold_store(P.st, slot);
        const float fxb = (float)x, fyb = (float)y;
        for (uint32_t s = 0; s < P.spp; ++s) {
            const float fx = fxb + rng_uniform(R);
            const float fy = fyb + rng_uniform(R);
            const Ray ray = camera_ray(P.cam, fx, fy);
            sum = sum + trace_path<(V & 1) != 0>(P.S, P.cfg, ray, P.depth, R, stk, vs, C);
        }
        hot.R = R;
        hot.done += P.spp;
        store_hot(P.st, slot, hot);
        store_sum(P.st, slot, sum, y * P.tm.W + x);
    }
    unsigned long long* ctr = ctr_copy(P.counters);
    wave_add_u64(ctr + 0, C.rays);
    wave_add_u64(ctr + 1, C.nodes);
    wave_add_u64(ctr + 2, C.ptests);
    wave_add_u64(ctr + 3, C.planes);
    wave_add_u64(ctr + 4, (unsigned long long)C.errs);
    wave_add_u64(ctr + 5, C.aux);
    wave_add_u64(ctr + 6, C.fallbacks);
    if (P.wg_prof) {
        __syncthreads();
        if (threadIdx.x == 0) {
            // {start, end (100 MHz), HW_ID, XCC_ID} per workgroup, indexed by tile
            unsigned long long* w = P.wg_prof + 4ull * tile;
            w[0] = t_start;
            w[1] = __builtin_amdgcn_s_memrealtime();
            w[2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            w[3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        }
    }
}

__global__ void __launch_bounds__(256) k_resolve(ResolveParams P) {
    __shared__ float thr[256];
    thr[threadIdx.x] = P.thr[threadIdx.x];
    __syncthreads();
    const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
    // every owned pixel must have taken exactly `samples` samples (src/scene.cpp:192-199,
    // the reference's loop): a chain lost by the engines would leave its pixel short, and
    // an image wrong without any other error -- counted here, an error of the resolve
    uint32_t px, py;
    const bool pix = slot_pixel(P.tm, blockIdx.x, threadIdx.x, px, py);
    wave_add_u64(ctr_copy(P.counters) + CTR_SHORT, pix && load_hot(P.st, slot).done != P.samples ? 1ull : 0ull);
    const float inv = 1.f / (float)P.samples;    // src/scene.cpp:201: (1.f / SAMPLES) * sum
    const f3 s = load_sum(P.st, slot);
    const float m[3] = {inv * s.x, inv * s.y, inv * s.z};
    uint8_t* o = P.out + (size_t)slot * 3u;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = (uint8_t)quantize_gamma(aces1(m[c]), thr);
    if (P.rad) {
#pragma unroll
        for (int c = 0; c < 3; ++c) P.rad[(size_t)slot * 3u + c] = m[c];
    }
}

// The framebuffer from packed 8-bit tiles (src/scene.cpp:243-251's row-major P6
// payload): window tile t (16x16 pixels, row-major inside the tile) is read at byte
// src[t] of `in` (null: t * 768, a one-rank session's own packed buffer), the rest
// of the rows are the window's (ww x wh).  `fb` may be pinned host memory: the
// kernel then writes the image across the link itself (the copy engine's first
// transfer costs ~8 ms on this platform, a kernel's stores ~0.2 ms for 6 MB).
// A tile row is 48 contiguous bytes on both sides: with ww % 16 == 0 every row
// starts 16-B aligned and goes as three 16-B stores (the right edge's partial
// tiles and other widths go byte by byte).  One workgroup per tile.
__global__ void __launch_bounds__(64) k_untile(const uint8_t* in, const uint32_t* src, uint32_t tiles_x, uint32_t ww,
                                               uint32_t wh, uint8_t* fb) {
    const uint32_t t = blockIdx.x;
    const uint32_t x0 = (t % tiles_x) * 16u, y0 = (t / tiles_x) * 16u;
    const uint8_t* tile = in + (src ? (size_t)src[t] : (size_t)t * 768u);
    const uint32_t wpx = ww - x0 < 16u ? ww - x0 : 16u;   // pixels of this tile per row
    if ((ww & 15u) == 0u) {
        // 16 rows x 3 chunks of 16 B (wpx = 16: ww is a multiple of the tile width)
        const uint32_t row = threadIdx.x / 3u, ch = threadIdx.x % 3u;
        if (threadIdx.x >= 48u || y0 + row >= wh) return;
        const uint4 v = *reinterpret_cast<const uint4*>(tile + row * 48u + ch * 16u);
        *reinterpret_cast<uint4*>(fb + ((size_t)(y0 + row) * ww + x0) * 3u + ch * 16u) = v;
        return;
    }
    for (uint32_t i = threadIdx.x; i < 256u * 3u; i += 64u) {
        const uint32_t px = i / 3u, row = px >> 4, col = px & 15u;
        if (col < wpx && y0 + row < wh) fb[((size_t)(y0 + row) * ww + x0 + col) * 3u + i % 3u] = tile[i];
    }
}

// Diagnostics only (PT_TUNE prespin_us, same_device=2): FMA work on every lane for
// `ticks` of the 100-MHz clock, from each wave's own start (the grid is resident at
// once) -- is a GPU that idled through a session's set-up slower at its render's start?
__global__ void __launch_bounds__(256) k_spin(uint32_t ticks, float* sink) {
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    float a = (float)threadIdx.x;
    for (;;) {
#pragma unroll
        for (int k = 0; k < 64; ++k) a = fmaf(a, 1.0001f, 0.5f);
        if ((uint32_t)__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
    }
    if (sink && a == 12345.f) sink[threadIdx.x] = a;   // (a use of the result)
}

}  // namespace pt

// ---------------------------------------------------------------- launchers
extern "C++" {
hipError_t pt_preload_kernels_base() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(pt::k_init));
}
hipError_t pt_launch_init(const pt::InitParams& p, uint32_t n_tiles, hipStream_t s) {
    hipLaunchKernelGGL(pt::k_init, dim3(n_tiles), dim3(256), 0, s, p);
    return hipGetLastError();
}
hipError_t pt_launch_trace(const pt::TraceParams& p, int variant, uint32_t lds_bytes, hipStream_t s) {
    const uint32_t n = p.n_tiles_local, nx = (n + 7u) / 8u * 8u;
    switch (variant) {
        case 0: hipLaunchKernelGGL(pt::k_trace<0>, dim3(n), dim3(256), lds_bytes, s, p); break;
        case 1: hipLaunchKernelGGL(pt::k_trace<1>, dim3(n), dim3(256), lds_bytes, s, p); break;
        case 2: hipLaunchKernelGGL(pt::k_trace<2>, dim3(nx), dim3(256), lds_bytes, s, p); break;
        default: hipLaunchKernelGGL(pt::k_trace<3>, dim3(nx), dim3(256), lds_bytes, s, p); break;
    }
    return hipGetLastError();
}
hipError_t pt_launch_untile(const uint8_t* in, const uint32_t* src, uint32_t tiles_x, uint32_t ww, uint32_t wh,
                            uint8_t* fb, hipStream_t s) {
    const uint32_t n = tiles_x * ((wh + 15u) / 16u);
    if (n) hipLaunchKernelGGL(pt::k_untile, dim3(n), dim3(64), 0, s, in, src, tiles_x, ww, wh, fb);
    return hipGetLastError();
}
hipError_t pt_launch_resolve(const pt::ResolveParams& p, uint32_t n_tiles, hipStream_t s) {
    hipLaunchKernelGGL(pt::k_resolve, dim3(n_tiles), dim3(256), 0, s, p);
    return hipGetLastError();
}
hipError_t pt_launch_spin(uint32_t us, uint32_t blocks, float* sink, hipStream_t s) {
    hipLaunchKernelGGL(pt::k_spin, dim3(blocks), dim3(256), 0, s, us * 100u, sink);
    return hipGetLastError();
}
}
