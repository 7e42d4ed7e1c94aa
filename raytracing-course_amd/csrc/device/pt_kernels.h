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
    uint32_t rank, world; // window tile t belongs to rank tile_owner(t, tiles_x, world)
    const uint32_t* gtile;   // device: this rank's window tiles in ascending order (local -> window tile)
};

// The deal of a window's 16x16 tiles to the ranks of a multi-GPU render: tile
// (tx, ty) belongs to rank (tx + ty) % world.  Diagonal stripes give every rank
// every column and every row of the image in equal parts; the plain t % world
// deals whole tile columns whenever tiles_x % world == 0 (1080p: 120 tiles per
// row), and the dragon's columns cost more than the walls' (rank-of-8 spread 7 %).
// A rank's local tiles are its window tiles in ascending order.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t tile_owner(uint32_t t, uint32_t tiles_x, uint32_t world) {
    return (t % tiles_x + t / tiles_x) % world;
}

// Per owned slot (256 per owned tile) one 32-B record, read and written as two
// 16-B pieces: a shade touches ONE piece (one vector load + one store instead of
// five scattered dwords), the path end the second one as well.
//   rec[2 slot]     = {rng x, rng saved (f32 bits), rng flag | vertices << 8 (24 bits), samples done}
//   rec[2 slot + 1] = {sum.r, sum.g, sum.b, global pixel index y*W + x (its seed)}
// Fold records (one 16-B record per path vertex: {idm, s1, s2, -}) are slot-major,
// fold[slot * depth + k], so a path's records share lines.
struct PixelState {
    uint4* rec;           // 2 * n_slots
    uint4* fold;          // depth * n_slots
    uint32_t n_slots;
    uint32_t depth;       // fold records per slot (>= 1)
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
    unsigned long long* counters; // rays, nodes, prim tests, plane tests, errors, aux visits, fallbacks
    ReplayCfg cfg;
    uint32_t depth;
    uint32_t spp;
    uint32_t n_tiles_local;
    unsigned long long* wg_prof;  // optional per-workgroup {start, end, HW_ID, XCC_ID} (diagnostics)
};

// ---- wavefront renderer (pt_wave.h: pt_wave.hip, pt_path.hip, pt_wcoop.hip) ----
struct RayQ {                     // rays waiting for a closest-hit query
    F4* ro;                       // {o.xyz, u32 slot}
    F4* rd;                       // {d.xyz, P = closest plane t (computed by the producer)}
    int* pid;                     // the closest plane's prim (-1 none)
    F4* ri;                       // q_prep record {1/d.xyz, dl | par | exact} (computed by the producer)
};
struct DoneQ {                    // finished queries, input of the shade kernel
    F4* ro;                       // {o.xyz, u32 slot}
    F4* rd;                       // {d.xyz, -}
    uint32_t* id;                 // closest prim (the shade kernel recomputes t, n, side from it), 0xffffffff = miss
};
// how a path ended (shade_item)
enum : uint32_t { PE_LIVE = 0u, PE_MISS = 1u, PE_CUT = 2u, PE_TERM = 3u };

// round counters: set p = ctl + PT_CTL_SET * p; the work-batch heads are one per
// XCD, each on its own 128-B line (C_HEADS + 32 x)
enum : uint32_t { C_FRESH = 0u, C_CARRY = 1u, C_DONE = 3u, C_EXACT = 4u, C_FRONT = 5u, C_BACK = 6u, C_WGDONE = 7u,
                  C_DEADLINE = 8u, C_ENDED = 9u, C_HEADS = 32u };
// C_ENDED: k_wcoop chains whose pixel reached the pass target (the final launch stops at
// side_stop_n of them to hand its last chains to whole-wave teams)
// C_WGDONE: k_wpath workgroups that have finished the round; C_DEADLINE: the round's end
// (low 32 bits of the 100-MHz realtime clock, 0 = not set yet; WaveParams::path_ticks)
#define PT_CTL_SET 288u          // words per counter set (C_HEADS + 8 x 32)
// statistics counters: one copy per XCD (PT_CTR_COPIES x PT_CTR_STRIDE u64), summed by the host
#define PT_CTR_COPIES 8u
#define PT_CTR_STRIDE 32u

struct WaveParams {
    SceneView S;
    const AuxSL* top;             // k_wcamera: the wide aux root's entries, then its inner entries' child
                                  // nodes' (entry k's child at top[PT_AUXW (1 + k)]; host form, f32)
    uint32_t n_top;               // entries in top
    uint32_t n_aux;               // wide aux entries in the blob
    CamView cam;
    TileMap tm;
    PixelState st;                // per-slot records (RNG, vertices, samples done, sum) + fold records
    RayQ fq[2];                   // fresh rays: round with parity p reads fq[p], appends to fq[1-p]
    uint32_t* cq[2];              // suspended queries (carry_words each): read cq[p], append to cq[1-p]
    uint32_t carry_cap, carry_words;
    DoneQ done;
    RayQ ex;                      // rays handed to the exact DFS this round
    uint2* endq;                  // per path workgroup PT_CMAX entries: its shade wave's ended paths
                                  // {slot | miss << 31, LDS pixel-table entry}
    uint32_t* ctl;                // 2 x PT_CTL_SET round counters
    unsigned long long* counters; // rays, nodes, prim tests, plane tests, errors, aux visits, fallbacks, ray fallbacks
    uint32_t depth;
    uint32_t parity;
    uint32_t target;              // samples per pixel to reach in this pass
    uint32_t n_tiles_local;
    uint32_t max_stack;           // exact DFS stack words per lane
    uint32_t aux_stack;           // wide aux traversal stack words per lane (LDS)
    unsigned long long* wg_prof;  // optional (diagnostics): per isect workgroup {start, end, HW_ID, XCC_ID, steps}
    // path engine (k_wpath): chains continue inside the kernel
    uint32_t path;                // 1 (k_wshade shades the exact-DFS results only)
    uint32_t path_budget;         // loop trips a query wave keeps its chains going after the round's work ran out
    uint32_t path_ticks;          // ... or, if nonzero, 100-MHz clock ticks after the first wave found it out:
                                  // every wave of the round stops at that one time
    uint32_t path_runend;         // a round with at most this many chains runs them to the end of the pass
    unsigned long long* progress; // optional host-mapped count of finished samples (progress bar), or null
    uint32_t path_cap;            // chains a workgroup may hold (<= PT_CMAX)
    uint32_t lstack;              // aux stack words a query lane may use (<= PT_LSTACK; deeper: exact DFS)
    const uint32_t* tile_order;   // k_wcamera: block b seeds local tile tile_order[b] (null: tile b)
    uint32_t sparse_steps;        // steps per loop trip of the end-of-pass (sparse) kernel
    uint32_t coop_reserve;        // k_wcoop: aux stack words kept free for a depth-first descent (3 (aux depth + 2))
    // k_wpath's per-trip step mix (the host may change it per round, from the chains left)
    uint32_t probe_every;         // candidate probes every n-th trip (>= 1) ...
    uint32_t probe_min;           // ... or whenever this many lanes wait for one
    uint32_t aux_extra;           // extra aux-node steps per trip for the lanes whose next step is one
    uint32_t batch;               // k_wpath: round-queue entries a wave takes per pull (at most)
    uint32_t end_min;             // k_wpath: ended paths the shade wave folds in a batch of their own (1..64;
                                  // fewer when nothing else waits: PT_END_MIN)
    // k_wcoop's intake order (null: queue order): the round's work items by the pixels'
    // remaining samples, most first (k_coop_order); `order_cur` = its 256 bucket cursors
    uint32_t* order;
    uint32_t* order_cur;
    // k_wpath's intake through an index list (null: the queues in order): work item i of
    // the round is queue item pin[i], i < pin_n (the round after an early cooperative
    // launch took the first entries of the intake order)
    const uint32_t* pin;
    uint32_t pin_n;
    // a cooperative launch beside a path round (the early launch): it stops at a chain
    // cycle's end once side_stop counts side_stop_n finished path workgroups, and yields its
    // chains as suspended queries at their start (q_init_pre: the ray was counted when it was
    // first taken) to yield_cq (counter yield_ctr: the path round's next carry queue).  The
    // pass's final launch uses the same stop with side_stop = its own C_ENDED: once all but
    // its last chains have ended, those go to a launch of whole-wave teams
    const uint32_t* side_stop;
    uint32_t side_stop_n;
    uint32_t* yield_cq;
    uint32_t* yield_ctr;
    uint32_t side_flags;          // PT_SIDE_* test hooks of that launch (0 in every render)
    // test hook (PT_TUNE drop=<site>): 1 + the hand-off site (PT_HO_*, include/pt.h) whose
    // items are dropped instead of handed on -- their chains are lost, which the resolve
    // must report (0 in every render)
    uint32_t drop;
};
// k_wcoop beside a path round, test hooks (PT_TUNE side_late / handon): every workgroup
// behaves as one that started after the round's end (takes nothing, hands every item on);
// the untaken items are dropped instead of handed on (a lost chain: the resolve's check)
#define PT_SIDE_LATE 1u
#define PT_SIDE_NO_HANDON 2u
// the final launch's stop: side_stop (its C_ENDED) against n_total - side_stop_n
#define PT_STOP_GROW 4u
// ... test hook (PT_TUNE grow_late): that launch's odd workgroups behave as late ones
// (stop at once and hand their untaken items on, through the intake order)
#define PT_GROW_LATE 8u
// ... test hook (PT_TUNE side_stop_now): the early launch stops after its first chain cycle
// (every team then yields its chain to the next round's carry queue)
#define PT_SIDE_STOP_NOW 16u
// path rounds, test hook (PT_TUNE shade_hold): the shade wave shades nothing until every
// query wave has left (in rounds with a budget), so all it shades goes through its flush
#define PT_SHADE_HOLD 32u
#define PT_ORDER_BUCKETS 256u

// path engine geometry: PT_NQ query waves + 1 shade wave per workgroup; at most
// PT_CMAX chains resident per workgroup (= the capacity of its ray ring).
// Two query waves per shade wave since the hit-region query made the queries
// cheaper than their shading (3 -> 2 at 4 workgroups per CU: +13 % at rank-of-1,
// +20 % at rank-of-8; 1 query wave: -8 %)
#ifndef PT_NQ
#define PT_NQ 2u
#endif
#define PT_PATH_WG (64u * (PT_NQ + 1u))
#ifndef PT_PATH_WAVES_PER_EU
#define PT_PATH_WAVES_PER_EU 3u        // k_wpath occupancy (waves per SIMD) the compiler is held to
#endif
// k_wpath's default step mix (WaveParams probe_every / probe_min / aux_extra)
#define PT_PROBE_EVERY 3u              // candidate probes every n-th trip (1: every trip; 2 / 4 / 8 measured
                                       // within 1 % of 3, all +8-10 % over 1)
#define PT_AUX2 1u                     // extra aux-node steps per trip for the lanes whose next step is one
                                       // (+4.5 % at rank-of-1; 167 VGPRs)
#ifndef PT_END_MIN
#define PT_END_MIN 64u                 // k_wpath: the shade wave folds ended paths in batches of their own, once
                                       // this many wait (or nothing else is there to shade); 32 / 48 measured
                                       // +3.7 % / +5.6 %, 64 +6.2 % over folding in every shade batch
#endif
#ifndef PT_END_MIN_LOW
#define PT_END_MIN_LOW 48u             // ... in the low-chain rounds (WaveParams::end_min; round 5, three
                                       // interleaved repeats against 64: rank of 8 -3 %, of 4 -1 %, of 1 +-0;
                                       // 16 / 32 no better)
#endif
#define PT_PROBE_MIN 32u               // ... or whenever this many lanes wait for one (round 5: 32 against 16,
                                       // three interleaved repeats: rank of 1 -1.2 %, of 4 -1 %, of 8 -4 %;
                                       // 24 / 40 / 48 / 64 between or worse)
#ifndef PT_CMAX
#define PT_CMAX 384u                   // (512 until round 3; the LDS pixel table took the room)
#endif
// The rings, the query lanes' aux stacks and the resident chains' pixel records
// live in LDS (4 workgroups per CU; pt_path.hip static_asserts the fit):
//   pixel table PT_CMAX entries (16 B: RNG, vertex count, samples done -- rec[2 slot]
//              while the chain stays in the workgroup) and their free ring
//   ray ring   PT_CMAX entries (54 B: ray, slot, plane t and prim, q_prep record, table entry)
//   done rings PT_DQN entries per query wave (34 B: ray, slot, closest prim, table entry),
//              flow-controlled (a finished query waits in its lane while its ring is full)
//   aux stack  PT_LSTACK words per query lane; a query that would need more takes the
//              exact DFS (none of 10^6 measured queries needed more than 11)
#define PT_DQN 48u                     // (64 until round 3; the LDS pixel table took the room)
#define PT_LSTACK 16u                  // (+1 word per lane: the stack's trash word)

// cooperative engine (k_wcoop, the end of a pass): one wave per chain, QC_WAVES
// independent waves per workgroup, per-team and per-wave LDS for the query (pt_wcoop.hip QcTeamLds, QcPoolLds)
#ifndef QC_WAVES
#define QC_WAVES 4u
#endif
#define QC_SCAP_MIN 128u           // aux stack words per team (the smallest; also the exact DFS stack)
#ifndef QC_EPL
#define QC_EPL 1u                  // aux entries a team lane tests per expansion round (nodes per round:
                                   // QC_EPL x team / 4)
#endif
#define QC_FOLD 6u                 // fold records held in LDS per chain (deeper vertices: HBM fold records)
#define QC_NPL 8u                  // plane records copied to LDS per workgroup (further planes: from HBM)
#define QC_NEM 8u                  // emitter records copied to LDS per workgroup (further emitters: from HBM)
#define QC_TOPN 21u                // aux BVH nodes 0..20 (BFS order: the top three levels) copied to LDS

struct ResolveParams {
    PixelState st;
    TileMap tm;                   // which slots are pixels (the rest of a partial edge tile are not)
    const float* thr;             // 256 gamma thresholds
    uint8_t* out;                 // 3 * n_slots
    float* rad;                   // optional 3 * n_slots
    uint32_t samples;             // samples accumulated so far
    unsigned long long* counters; // statistics counters: C_SHORT counts the owned pixels whose
                                  // samples done differ from `samples` (a lost chain; must be 0)
};
// statistics counter slots (per copy, PT_CTR_STRIDE u64) besides rays .. fallbacks_ray (0-7)
// and the cooperative engine's share (8-10, 13); CTR_HO + PT_HO_*: the items handed on at
// each hand-off site (include/pt.h PT_HO_*; DESIGN.md §4 "Hand-off sites")
enum : uint32_t { CTR_SHORT = 11u, CTR_HANDON = 12u, CTR_HO = 16u };
// the hand-off sites (include/pt.h PT_HO_*, which the host checks these against)
enum : uint32_t { HO_SUSPEND = 0u, HO_FLUSH, HO_RINGOUT, HO_EXACT, HO_SIDE_TAKE, HO_SIDE_YIELD, HO_SIDE_HANDON,
                  HO_GROW_YIELD, HO_GROW_HANDON, HO_N };

}  // namespace pt

hipError_t pt_preload_kernels_base();
hipError_t pt_preload_kernels_wave();
hipError_t pt_launch_init(const pt::InitParams& p, uint32_t n_tiles, hipStream_t s);
// diagnostics (PT_TUNE prespin_us): every lane busy for `us` microseconds
hipError_t pt_launch_spin(uint32_t us, uint32_t blocks, float* sink, hipStream_t s);
// variant: bit 0 = filtered node tests + flat replay, bit 1 = XCD-banded tile order
hipError_t pt_launch_trace(const pt::TraceParams& p, int variant, uint32_t lds_bytes, hipStream_t s);
// wavefront pipeline (pt_wave.hip, pt_path.hip, pt_wcoop.hip): start a pass (first camera ray of every
// owned pixel), then path-engine rounds
hipError_t pt_launch_wave_start(pt::WaveParams p, hipStream_t s);
// path engine round: {k_wpath, k_wexact, k_wshade (exact results)}
// sparse: the end-of-pass kernel (few chains: every step kind and several steps per trip)
hipError_t pt_launch_path_round(pt::WaveParams p, uint32_t path_grid, uint32_t shade_grid, hipStream_t s, bool sparse,
                                hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
// the cooperative engine's intake order (WaveParams::order): the round's n work items
// counting-sorted by their pixels' remaining samples, most first
hipError_t pt_launch_coop_order(pt::WaveParams p, uint32_t n, hipStream_t s);
// the early cooperative launch's queue: the first k items of p.order (the pixels with the
// most samples left) copied into `side` -- fresh rays as they are, suspended queries as
// restart records (their ray and slot) -- whose round counters side_ctl[C_CARRY / C_FRESH]
// count them (zeroed by the caller)
hipError_t pt_launch_side_take(pt::WaveParams p, uint32_t k, pt::RayQ side, uint32_t* side_carry, uint32_t* side_ctl,
                               hipStream_t s);
// cooperative engine: one launch runs every remaining chain of the pass to its end
// team = lanes per chain (8 -- the default --, 16, 32 or 64)
// big: the scene exceeds the LDS tables (QC_FOLD / QC_NPL / QC_NEM; team 8 or 64 then)
hipError_t pt_launch_coop(pt::WaveParams p, uint32_t grid, uint32_t team, bool big, hipStream_t s,
                          hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t pt_launch_resolve(const pt::ResolveParams& p, uint32_t n_tiles, hipStream_t s);
// the row-major ww x wh x 3 framebuffer from packed tiles: window tile t at byte src[t] of `in`
// (src null: t * 768, the packed buffer of a session that owns every tile)
hipError_t pt_launch_untile(const uint8_t* in, const uint32_t* src, uint32_t tiles_x, uint32_t ww, uint32_t wh,
                            uint8_t* fb, hipStream_t s);
