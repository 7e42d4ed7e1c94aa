/* pt.h -- C ABI of the MI355X-native hw5 path tracer (libpt.so).
 *
 * Drop-in boundary for the reference's render path.  The reference
 * (FeggieBoss/raytracing-course, hw5) has no plugin/FFI seam: its callers are
 * the CLI (hw5/run.sh:1-2 -> hw5/src/main.cpp:6-17) and the in-process trio
 *     Scene::Load(std::istream&)   hw5/include/scene.h:76, src/sceneload.cpp:112-176
 *     Scene::InitScene()           hw5/include/scene.h:78, src/scene.cpp:7-40
 *     Scene::Render(std::ostream&) hw5/include/scene.h:79, src/scene.cpp:205-252
 * Each entry point below names the reference interface it replaces.  Plain
 * pointers and sizes only; no C++/torch types cross this boundary.
 *
 * Conventions: functions return PT_OK (0) or a negative PT_E* code; the
 * message of the last failure on the calling thread is pt_last_error().
 * The caller owns every output buffer; the library owns scenes, sessions and
 * all device memory (released by pt_scene_free / pt_session_free).
 * Rendering requires a gfx950 GPU: there is no CPU fallback (PT_E_NO_GPU).
 */
#ifndef PT_H
#define PT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 6   /* 2: pt_render_opts.gather; 3: pt_stats per-engine (coop_*) fields;
                              4: pt_gather_init, and the session tile deal changed from tile
                              t -> rank t % world to tile (tx, ty) -> rank (tx + ty) % world
                              (local tiles still in ascending tile order): a driver that
                              un-interleaves packed tiles itself must use pt_unpack_tiles
                              (or ptrace.rank_tiles), not its own formula;
                              5: pt_stats.short_pixels / handed_on, and pt_session_resolve fails
                              when an owned pixel's sample count differs from the samples traced;
                              6: pt_stats.gather_allocs (the RCCL gather keeps its buffers per
                              communicator), pt_session_reset */

enum {
    PT_OK = 0,
    PT_E_INVALID = -1,   /* bad argument / state */
    PT_E_IO = -2,        /* file cannot be read / written */
    PT_E_SCENE = -3,     /* scene the reference cannot render either (no non-plane
                            primitive, bad primitive type, zero sizes) */
    PT_E_NO_GPU = -4,    /* no usable gfx950 device */
    PT_E_HIP = -5,       /* HIP runtime error */
    PT_E_RCCL = -6,      /* RCCL error (multi-GPU gather) */
    PT_E_OOM = -7
};

typedef struct pt_scene pt_scene;
typedef struct pt_session pt_session;

/* Scene::Load: parse a hw5 scene text file with the reference's exact grammar
 * and quirks.  Unknown commands produce a warning on stderr like
 * the reference (src/sceneload.cpp:170-172). */
int pt_scene_load(const char* path, pt_scene** out);
/* same, from memory (text, len bytes) */
int pt_scene_load_mem(const char* text, size_t len, pt_scene** out);

/* Scene::InitScene: std::partition of planes to the end, the reference BVH
 * (bit-faithful: same node boxes, preorder and primitive order), the emitter
 * list, and the device-side layouts.  Host-only; no GPU needed. */
int pt_scene_prepare(pt_scene* s);

/* Optional start-up of the HIP runtime on `device`: context creation and the
 * kernels' code objects (no launch).  No reference counterpart: a caller may run
 * it on a second thread while Scene::Load / InitScene parse and build on the
 * CPU, so the runtime's start-up does not add to the wall-clock (cli/main.cpp).
 * pt_render does the same work itself when it has not been done. */
int pt_device_init(int device);

/* Optional creation of the RCCL communicator that pt_render(ngpu = n, gather RCCL)
 * uses over devices device .. device+n-1 (ncclCommInitAll, cached per process).  No
 * reference counterpart (the reference renders on one host): the CLI runs it on its
 * start-up thread beside Scene::Load / InitScene, so the communicator's set-up is not
 * paid between the render and the PPM.  pt_render creates it itself otherwise. */
int pt_gather_init(int device, int ngpu);

typedef struct pt_scene_info {
    uint32_t width, height, samples, ray_depth;
    uint32_t n_prims, n_bvh_prims, n_planes, n_emitters;
    uint32_t n_nodes, tree_depth, max_stack;   /* max_stack = max pending right children */
    uint32_t n_aux_nodes, aux_depth;
    uint32_t n_warnings;
} pt_scene_info;
int pt_scene_get_info(const pt_scene* s, pt_scene_info* info);

/* Override DIMENSIONS / SAMPLES / RAY_DEPTH after loading (0 keeps the value). */
int pt_scene_override(pt_scene* s, uint32_t width, uint32_t height, uint32_t samples, uint32_t ray_depth);

/* BVH fingerprint dump (after prepare), reference layout of SURVEY §8c:
 * nodes: per node 6 f32 (min.xyz, max.xyz) + 4 u32 (left, right, first, count) = 40 B;
 * prims: per primitive u32 type + 9 f32 (a, b, c; b/c zero unless TRIANGLE) + 3 f32 pos = 52 B. */
int pt_scene_dump_bvh(const pt_scene* s, void* nodes_out, size_t nodes_bytes, void* prims_out, size_t prims_bytes);

void pt_scene_free(pt_scene* s);

/* ---------------------------------------------------------------- render */
enum {
    PT_TRAVERSAL_REPLAY = 0, /* default: candidate replay -- auxiliary BVH enumerates the reference
                                leaves the ray can reach, the reference's exact pruning is replayed
                                on their root paths only (bit-identical results) */
    PT_TRAVERSAL_EXACT = 1,  /* full reference-tree stack DFS, exact pruning semantics */
    PT_TRAVERSAL_REPLAY_DIV = 2 /* candidate replay with the reference's IEEE-division slab test at
                                   every node (the unfiltered form; same results, slower) */
};

typedef struct pt_render_opts {
    int32_t device;          /* first HIP device (default 0) */
    int32_t ngpu;            /* GPUs driven by this process (default 1); >1 = pixel tiles
                                dealt round-robin + RCCL gather of the framebuffer */
    uint32_t spp_per_launch; /* samples per kernel launch (0 = auto) */
    uint32_t samples;        /* 0 = the scene's SAMPLES */
    int32_t traversal;       /* PT_TRAVERSAL_* */
    int32_t progress;        /* 1 = print the reference's "Loading: [...]" bar to stdout */
    uint32_t win_x0, win_y0; /* optional window: render only [x0,x0+w) x [y0,y0+h) of the */
    uint32_t win_w, win_h;   /* image, keeping global-index seeds (win_w = 0: full image) */
    int32_t gather;          /* PT_GATHER_*: how the framebuffer tiles reach the caller */
} pt_render_opts;
enum {
    PT_GATHER_AUTO = 0,      /* default: RCCL (ncclGather over xGMI) when ngpu > 1, host copy if RCCL fails */
    PT_GATHER_RCCL = 1,      /* RCCL at any ngpu (also ngpu = 1: a one-rank communicator); failure is an error */
    PT_GATHER_HOST = 2       /* per-device copies through the host, never RCCL */
};
void pt_render_opts_default(pt_render_opts* o);

typedef struct pt_stats {
    uint64_t rays;           /* closest-hit queries (Scene::RayIntersection calls) */
    uint64_t node_visits;    /* BVH node records fetched */
    uint64_t prim_tests;     /* leaf primitive tests */
    uint64_t plane_tests;
    uint64_t samples;        /* pixel samples traced */
    uint64_t errors;         /* exactness guards tripped (must be 0) */
    uint64_t aux_visits;     /* auxiliary BVH node visits (replay traversal) */
    uint64_t fallbacks;      /* queries that took the exact stack DFS under replay */
    double kernel_ms;        /* sum of trace-kernel time (HIP events) */
    double resolve_ms;
    double wall_ms;          /* pt_render: upload + render + gather + tonemap */
    uint64_t node_bytes;     /* bytes of one node record / primitive record / aux node */
    uint64_t prim_bytes;
    uint64_t aux_bytes;
    uint64_t fallbacks_ray;  /* of `fallbacks`: rays with non-finite origin/direction (exact DFS by design) */
    double isect_ms;         /* wavefront engine: time of the closest-hit kernel launches (HIP events) */
    uint64_t isect_launches;
    uint64_t rounds;         /* wavefront rounds run */
    uint64_t gather_rccl;    /* 1: the multi-GPU framebuffer was gathered with RCCL (ncclGather over xGMI) */
    /* the cooperative end-of-pass engine's share of rays / node_visits / prim_tests /
       aux_visits / isect_ms / isect_launches (the rest is the path engine's) */
    uint64_t coop_rays, coop_node_visits, coop_prim_tests, coop_aux_visits;
    double coop_ms;
    uint64_t coop_launches;
    /* ABI 5: pixels found at a resolve with a sample count other than the samples traced
       (a lost chain: pt_session_resolve then fails; must be 0), and work items an early
       cooperative launch's late workgroups handed on to the next round untaken */
    uint64_t short_pixels;
    uint64_t handed_on;
    /* ABI 6: device allocations pt_render's RCCL gather made (its send / receive buffers are
       kept per communicator: 0 on every render after the first of a device set and size) */
    uint64_t gather_allocs;
    /* ABI 6: work items handed on at each place where work changes hands between the
       engines' launches, waves or queues (PT_HO_*; DESIGN.md §4 "Hand-off sites") */
    uint64_t handoff[12];
} pt_stats;
/* pt_stats.handoff sites (each has a PT_TUNE hook that forces it and one, drop=<name>, that
 * drops its items -- the resolve must then fail: INTEGRATION.md) */
enum {
    PT_HO_SUSPEND = 0,      /* path engine, round end: running queries -> the next carry queue */
    PT_HO_FLUSH = 1,        /* path engine, shade wave after the query waves left: next rays -> next fresh queue */
    PT_HO_RINGOUT = 2,      /* path engine, shade wave's exit: ray-ring leftovers -> next fresh queue */
    PT_HO_EXACT = 3,        /* path engine: a query -> the exact-DFS kernels (k_wexact, k_wshade) */
    PT_HO_SIDE_TAKE = 4,    /* early cooperative launch: the heaviest chains taken from the round's work */
    PT_HO_SIDE_YIELD = 5,   /* early launch's stop: its running chains -> the next carry queue */
    PT_HO_SIDE_HANDON = 6,  /* early launch's late workgroups: untaken items -> the next carry queue */
    PT_HO_GROW_YIELD = 7,   /* final launch's grow stop: its running chains -> the bigger teams' launch */
    PT_HO_GROW_HANDON = 8,  /* final launch's late workgroups: untaken items -> the bigger teams' launch */
    PT_HO_N = 9
};

/* Scene::Render minus the stream write: renders W*H*3 u8 (row-major, top row
 * first, exactly the reference's P6 payload) into rgb, and optionally the
 * pre-tonemap fp32 mean radiance (W*H*3) into radiance.  Either may be NULL.
 * With a window, the outputs are win_w*win_h*3 (the same pixels as a full
 * render would give there).  stats may be NULL. */
int pt_render(pt_scene* s, const pt_render_opts* opts, uint8_t* rgb, float* radiance, pt_stats* stats);

/* P6 writer of src/scene.cpp:206-208,243-251 ("P6\n{W} {H}\n255\n" + payload). */
int pt_write_ppm(const char* path, uint32_t width, uint32_t height, const uint8_t* rgb);

/* ------------------------------------------------------- sessions (tiles)
 * Progressive / sharded rendering on ONE device, used by pt_render and by
 * multi-process drivers (one process per GPU): the image is cut into 16x16
 * tiles, tile (tx, ty) belongs to rank (tx + ty) % world (diagonal stripes: every
 * rank gets every row and column of the image); a rank's tiles are kept in
 * ascending tile order (t = ty * tiles_x + tx).  The session keeps every owned
 * pixel's RNG stream and f32 sum resident in HBM, so pt_session_trace(spp)
 * continues each pixel's stream exactly as the reference's sequential spp loop. */
typedef struct pt_session_opts {
    int32_t device;
    uint32_t rank, world;
    int32_t traversal;
    uint32_t win_x0, win_y0, win_w, win_h;   /* optional window (win_w = 0: full image) */
} pt_session_opts;

int pt_session_create(pt_scene* s, const pt_session_opts* o, pt_session** out);
/* number of owned tiles and of packed output bytes (tiles*256*3) */
int pt_session_layout(const pt_session* ss, uint32_t* n_tiles, uint64_t* packed_rgb_bytes);
/* enqueue spp more samples for every owned pixel (asynchronous).  With the
 * wavefront engine consecutive calls are coalesced into ONE pass, run by the
 * next resolve / sync / stats / stream call: a pixel goes on with its next
 * samples as soon as it has finished the current ones, so only the end of the
 * coalesced pass waits for the slowest pixel.  Results are identical either way
 * (each pixel's samples stay in stream order). */
int pt_session_trace(pt_session* ss, uint32_t spp);
/* tonemap the current means (sum / samples so far) into the packed tile
 * buffer: 256*3 u8 per owned tile, pixels of a tile row-major; dev_out is a
 * device pointer on the session's device (NULL = internal buffer).
 * dev_radiance (optional, device) receives 256*3 f32 per tile. */
int pt_session_resolve(pt_session* ss, uint8_t* dev_out, float* dev_radiance);
int pt_session_sync(pt_session* ss);
/* restart every owned pixel at sample 0 (its stream re-seeded, its sum zeroed), the
 * session's buffers and counters kept: the next trace(S) renders exactly what a new
 * session would -- Scene::Render's job again without the set-up (bench.py repeats the
 * metric's 256-spp frame this way).  Runs any trace() not yet run first. */
int pt_session_reset(pt_session* ss);
/* copy the internal packed buffer to host memory (after resolve+sync) */
int pt_session_read_packed(pt_session* ss, uint8_t* host_out, size_t bytes);
/* scatter packed tiles of `rank` (world ranks) into a width*height*3 image
 * (width/height = the rendered window's size) */
int pt_unpack_tiles(uint32_t width, uint32_t height, uint32_t rank, uint32_t world, const uint8_t* packed,
                    uint8_t* rgb);
int pt_unpack_tiles_f32(uint32_t width, uint32_t height, uint32_t rank, uint32_t world, const float* packed,
                        float* rad);
/* counters accumulated by this session (after sync) */
int pt_session_stats(pt_session* ss, pt_stats* st);
/* HIP stream of the session (hipStream_t), for callers that order their own work after it */
void* pt_session_stream(pt_session* ss);
void pt_session_free(pt_session* ss);

const char* pt_last_error(void);
int pt_abi_version(void);

/* ------------------------------------------------------------ test hooks
 * Host execution of the device traversal code (pt_trace.h) for CPU unit
 * tests of the stack-DFS logic.  Never used by pt_render. */
int pt_selftest_ray_intersection(pt_scene* s, int32_t traversal, uint32_t n, const float* rays, int32_t* ids,
                                 float* hits, uint64_t* counters8);
int pt_selftest_render_host(pt_scene* s, int32_t traversal, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                            uint32_t spp, float* radiance);
/* the 256-entry gamma threshold table used by the device tonemap */
int pt_selftest_gamma_table(const pt_scene* s, float* thr256);

#ifdef __cplusplus
}
#endif
#endif /* PT_H */
