// pt_kernels.h -- kernel parameter blocks shared by the host driver and the kernels.
#pragma once
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
#include <hip/hip_runtime_api.h>
#endif

#include "pt_trace.h"

namespace pt {

struct TileMap {
    uint32_t W, H;        // full image size (seeds are y*W + x, camera uses W, H)
    uint32_t x0, y0;      // rendered window origin
    uint32_t ww, wh;      // rendered window size (= W, H for a full render)
    uint32_t tiles_x;     // ceil(ww/16)
    uint32_t n_tiles;     // ceil(ww/16)*ceil(wh/16)
    uint32_t rank, world; // window tile t belongs to rank t % world
};

struct PixelState {       // SoA over owned slots (256 per owned tile)
    uint32_t* rng_x;
    float* rng_saved;
    uint32_t* rng_flag;
    float* sum;           // 3 * n_slots (r plane, g plane, b plane)
    uint32_t n_slots;
};

struct InitParams {
    TileMap tm;
    PixelState st;
};

struct TraceParams {
    SceneView S;
    CamView cam;
    TileMap tm;
    PixelState st;
    uint32_t* vscratch;          // 3 * depth * n_slots
    unsigned long long* counters; // rays, nodes, prim tests, plane tests, errors, aux visits, fallbacks
    ReplayCfg cfg;
    uint32_t depth;
    uint32_t spp;
};

struct ResolveParams {
    PixelState st;
    const float* thr;             // 256 gamma thresholds
    uint8_t* out;                 // 3 * n_slots
    float* rad;                   // optional 3 * n_slots
    uint32_t samples;             // samples accumulated so far
};

}  // namespace pt

hipError_t pt_launch_init(const pt::InitParams& p, uint32_t n_tiles, hipStream_t s);
hipError_t pt_launch_trace(const pt::TraceParams& p, uint32_t n_tiles, uint32_t lds_bytes, hipStream_t s);
hipError_t pt_launch_resolve(const pt::ResolveParams& p, uint32_t n_tiles, hipStream_t s);
