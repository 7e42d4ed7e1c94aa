// pt_kernels.h -- kernel parameter blocks shared by the host driver and the kernels.
#pragma once
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
#include <hip/hip_runtime_api.h>
#endif

#include "pt_query.h"

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
    uint32_t n_tiles_local;
    unsigned long long* wg_prof;  // optional per-workgroup {start, end, HW_ID, XCC_ID} (diagnostics)
};

// ---- wavefront renderer (pt_wave.hip) ----------------------------------
struct WaveQueue {                // rays of one bounce, compacted
    F4* ro;                       // {o.xyz, u32 slot}
    F4* rd;                       // {d.xyz, -}
};
struct WaveHits {                 // closest hit per queue entry
    F4* th;                       // {t, n.xyz}
    uint32_t* id;                 // prim | interior << 31, 0xffffffff = miss
};
// per-slot path end state (pstate = nv | end << 8)
enum : uint32_t { PE_LIVE = 0u, PE_MISS = 1u, PE_CUT = 2u, PE_TERM = 3u };

struct WaveParams {
    SceneView S;
    const AuxSL* aux;
    uint32_t n_aux;
    CamView cam;
    TileMap tm;
    PixelState st;
    uint32_t* vscratch;           // 3 * depth * n_slots fold records
    uint32_t* pstate;             // n_slots
    WaveQueue q[2];               // ping-pong: bounce b reads q[b & 1], enqueues into q[(b + 1) & 1]
    WaveHits hits;
    uint32_t* fb;                 // queue indices left to the exact DFS (this bounce)
    uint32_t* ctl;                // [0, D]: queue counts per bounce, [D+1, 2D+1]: fetch heads, [2D+2, 3D+2]: exact counts
    unsigned long long* counters; // rays, nodes, prim tests, plane tests, errors, aux visits, fallbacks
    uint32_t depth;
    uint32_t bounce;
    uint32_t n_tiles_local;
    uint32_t max_stack;           // exact DFS stack words per lane
    uint32_t aux_stack;           // wide aux traversal stack words per lane (LDS)
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
// variant: bit 0 = filtered node tests + flat replay, bit 1 = XCD-banded tile order
hipError_t pt_launch_trace(const pt::TraceParams& p, int variant, uint32_t lds_bytes, hipStream_t s);
// one sample of every owned pixel through the wavefront pipeline (pt_wave.hip)
hipError_t pt_launch_wave_sample(pt::WaveParams p, uint32_t isect_grid, hipStream_t s);
hipError_t pt_launch_resolve(const pt::ResolveParams& p, uint32_t n_tiles, hipStream_t s);
