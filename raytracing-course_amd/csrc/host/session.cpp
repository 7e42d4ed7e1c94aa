// session.cpp -- tile sessions (pt_session_*): one rank's pixels on one device, their
// buffers in one allocation, the megakernel pass (exact / division-form traversals),
// the device tonemap with its lost-chain check, statistics, and the tile un-interleave.
// The wavefront pass itself is rounds.cpp.
#include <stdio.h>
#include <string.h>

#include <map>
#include "api_internal.h"

namespace pti {

double wall_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int finish_pending(pt_session* ss) {
    for (auto& e : ss->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) ss->kernel_ms += ms;
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    ss->pending.clear();
    // diagnostics (PT_TUNE roundlog=1): per-launch ms of the rounds, one line per sync
    const bool log = tune_int("roundlog", 0) == 1 && !ss->pending_isect.empty();
    if (log) fprintf(stderr, "rounds_ms");
    for (size_t i = 0; i < ss->pending_isect.size(); ++i) {
        const auto& e = ss->pending_isect[i];
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) {
            ss->isect_ms += ms;
            if (i < ss->pending_isect_coop.size() && ss->pending_isect_coop[i]) ss->coop_ms += ms;
        }
        if (log) fprintf(stderr, " %.3f", ms);
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    if (log) fprintf(stderr, "\n");
    ss->pending_isect.clear();
    ss->pending_isect_coop.clear();
    return PT_OK;
}

// the window tiles dealt to `rank` (pt_kernels.h tile_owner), ascending
std::vector<uint32_t> rank_tiles(uint32_t n_tiles, uint32_t tiles_x, uint32_t rank, uint32_t world) {
    std::vector<uint32_t> v;
    v.reserve(n_tiles / world + 1);
    for (uint32_t t = 0; t < n_tiles; ++t)
        if (pt::tile_owner(t, tiles_x, world) == rank) v.push_back(t);
    return v;
}

uint64_t owned_pixels(const pt_session* ss) {
    uint64_t px = 0;
    for (uint32_t t = 0; t < ss->n_tiles_local; ++t) {
        const uint32_t gt = ss->gtiles[t];
        const uint32_t tx = gt % ss->tm.tiles_x, ty = gt / ss->tm.tiles_x;
        const uint32_t w = std::min(16u, ss->tm.ww - tx * 16u), h = std::min(16u, ss->tm.wh - ty * 16u);
        px += (uint64_t)w * h;
    }
    return px;
}

// the statistics counters, summed over their per-XCD copies (after the stream's work)
hipError_t read_counters(pt_session* ss, unsigned long long c[PT_CTR_STRIDE]) {
    unsigned long long cc[PT_CTR_COPIES * PT_CTR_STRIDE];
    // (on the session's stream: the null stream would also wait for other sessions' work)
    hipError_t e = hipMemcpyAsync(cc, ss->counters, sizeof(cc), hipMemcpyDeviceToHost, ss->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ss->stream);
    for (uint32_t k = 0; k < PT_CTR_STRIDE; ++k) c[k] = 0ull;
    if (e != hipSuccess) return e;
    for (uint32_t x = 0; x < PT_CTR_COPIES; ++x)
        for (uint32_t k = 0; k < PT_CTR_STRIDE; ++k) c[k] += cc[PT_CTR_STRIDE * x + k];
    return hipSuccess;
}

// run the coalesced trace() calls of the wavefront engine as one pass
int flush_trace(pt_session* ss) {
    if (!ss->deferred_spp) return PT_OK;
    const uint32_t spp = ss->deferred_spp;
    ss->deferred_spp = 0;
    HIP_TRY(hipSetDevice(ss->dev));
    return trace_wave(ss, spp);
}

bool coop_big(const pt_session* ss) {
    const pt_scene* s = ss->sc;
    return ss->depth > QC_FOLD || s->planes.size() > QC_NPL || s->emitters.size() > QC_NEM;
}

}  // namespace pti

using namespace pti;

extern "C" {

// ------------------------------------------------------------- sessions ---
int pt_session_create(pt_scene* s, const pt_session_opts* o, pt_session** out) {
    if (!s || !o || !out) return fail(PT_E_INVALID, "null argument");
    if (!s->prepared) return fail(PT_E_INVALID, "scene not prepared (call pt_scene_prepare)");
    if (o->world == 0 || o->rank >= o->world) return fail(PT_E_INVALID, "bad rank/world");
    if (s->hs.W == 0 || s->hs.H == 0) return fail(PT_E_SCENE, "zero image size");
    if ((uint64_t)s->hs.W * s->hs.H >= 2147483647ull) return fail(PT_E_SCENE, "image too large for per-pixel seeds");
    // the slot record keeps the current path's vertex count in 24 bits (pt_devutil.h PixelHot)
    if (s->hs.depth >= (1u << 24)) return fail(PT_E_SCENE, "RAY_DEPTH too large (at most 16777215)");
    int rc = check_device(o->device);
    if (rc) return rc;
    // the megakernel (exact / division-form traversal, PT_TUNE engine=mega) also reads the BVH2 aux
    const bool mega = o->traversal != PT_TRAVERSAL_REPLAY || tune_str("engine") == "mega";
    DevScene* ds = nullptr;
    double up_ms = 0.0;
    if ((rc = ensure_device_scene(s, o->device, mega, &ds, &up_ms))) return rc;
    auto* ss = new pt_session();
    ss->sc = s;
    ss->dev = o->device;
    ss->ds = ds;
    ss->upload_ms = up_ms;
    ss->traversal = o->traversal;
    ss->depth = s->hs.depth;
    ss->tm.W = s->hs.W;
    ss->tm.H = s->hs.H;
    ss->tm.x0 = o->win_w ? o->win_x0 : 0u;
    ss->tm.y0 = o->win_w ? o->win_y0 : 0u;
    ss->tm.ww = o->win_w ? o->win_w : s->hs.W;
    ss->tm.wh = o->win_w ? o->win_h : s->hs.H;
    if (ss->tm.ww == 0 || ss->tm.wh == 0 || (uint64_t)ss->tm.x0 + ss->tm.ww > s->hs.W ||
        (uint64_t)ss->tm.y0 + ss->tm.wh > s->hs.H) {
        delete ss;
        return fail(PT_E_INVALID, "window outside the image");
    }
    ss->tm.tiles_x = (ss->tm.ww + 15u) / 16u;
    ss->tm.n_tiles = ss->tm.tiles_x * ((ss->tm.wh + 15u) / 16u);
    ss->tm.rank = o->rank;
    ss->tm.world = o->world;
    ss->gtiles = rank_tiles(ss->tm.n_tiles, ss->tm.tiles_x, o->rank, o->world);
    ss->n_tiles_local = (uint32_t)ss->gtiles.size();
    ss->n_slots = ss->n_tiles_local * 256u;
    ss->cam = make_cam(s);
    auto cleanup = [&](int code) {
        pt_session_free(ss);
        return code;
    };
    if (hipSetDevice(ss->dev) != hipSuccess) return cleanup(fail(PT_E_HIP, "hipSetDevice failed"));
    DevProps props;
    if ((rc = device_props(ss->dev, &props))) return cleanup(rc);
    const uint32_t cus = (uint32_t)props.cus;
    const size_t n = std::max<size_t>(ss->n_slots, 1);
    ss->st.depth = std::max<uint32_t>(ss->depth, 1u);
    ss->st.n_slots = ss->n_slots;
    // engine: the wavefront pipeline for the (filtered) replay traversal; the
    // megakernel for the exact DFS and the division-form replay (PT_TUNE engine=mega forces it)
    ss->wave = o->traversal == PT_TRAVERSAL_REPLAY;
    if (tune_str("engine") == "mega") ss->wave = false;
    std::vector<uint32_t> ord;   // wavefront: the local tiles' seeding order
    if (ss->wave) {
        ss->shade_grid = std::min<uint32_t>(cus * 8u, std::max(1u, ss->n_tiles_local));
        // path engine: PT_NQ query waves + 1 shade wave per workgroup, as many workgroups
        // per CU as its waves-per-SIMD occupancy holds (4 SIMDs per CU)
        ss->path_budget = (uint32_t)std::max(1, tune_int("budget", (int)ss->path_budget));
        // rounds end at one time for every wave (budget_us after the work ran out; 0: each
        // wave after `budget` trips of its own, also the mode of an explicit budget=N alone)
        // (at most 10 s: the device compares 32-bit clock differences as signed)
        ss->path_ticks = (uint32_t)std::min(10000000, std::max(0, tune_int("budget_us", tune_has("budget") ? 0 : 2500))) * 100u;
        // ... and the low-chain rounds' deadline: 5 ms (fewer rounds, each of which re-sorts and
        // re-takes the early launch's heaviest chains; with coop_grow 16 per CU, one GPU call,
        // 3 repeats of every rank (tools/gpu_r5_ab.sh, profiles/r05_ab): rank of 8 mean 83.5 ->
        // 80.2 ms per 256-spp pass, rank of 4 139.9 -> 137.6, of 2 259.2 -> 255.6, one GPU
        // 488.8 -> 486.3); with budget_us=0 (trip budgets) the path rounds' mode
        // (lowq_budget_us=0: trip budgets in those rounds, as budget_us=0 for every round)
        ss->low_ticks = tune_has("lowq_budget_us")
                            ? (uint32_t)std::min(10000000, std::max(0, tune_int("lowq_budget_us", 5000))) * 100u
                            : ss->path_ticks == 0 ? 0u : 500000u;
        const int wg_cu = std::max(1, (int)(PT_PATH_WAVES_PER_EU * 4u / (PT_NQ + 1u)));
        ss->path_grid = cus * (uint32_t)std::max(1, tune_int("wg_per_cu", wg_cu));
        // suspended-query records: Query | slot | aux stack, rounded to 16 B.  Only a
        // query lane suspends (one query at round end), and a pixel has at most one ray
        // in flight, so a round appends at most min(pixels, query lanes) of them: the
        // carry queue can never overflow.  The exact-DFS hand-over queues (ex, done, hid)
        // do NOT have that bound: a lane that hands its ray over goes on with another
        // chain of the round's supply, so a round can hand over a ray of every chain --
        // at most one per pixel (a chain that leaves for k_wexact leaves the round).
        // They hold n entries.
        ss->carry_words = ((uint32_t)(sizeof(pt::Query) / 4) + 1u + std::max<uint32_t>(s->auxw_stack, 1u) + 3u) & ~3u;
        ss->lane_cap = (uint32_t)std::min<uint64_t>(n, (uint64_t)ss->path_grid * PT_NQ * 64u);
        ss->carry_cap = ss->lane_cap;
        // a round whose chains are this few runs them to the end of the pass (a few
        // per query wave: rebalancing them costs more rounds than it saves)
        ss->path_runend = ss->path_grid * PT_NQ * 4u;
        ss->path_runend = (uint32_t)std::max(0, tune_int("runend", (int)ss->path_runend));
        // rounds with fewer chains than this run the end-of-pass (sparse) kernel
        ss->path_sparse = ss->path_grid * PT_NQ * 32u;
        ss->path_sparse = (uint32_t)std::max(0, tune_int("sparse", (int)ss->path_sparse));
        ss->sparse_steps = (uint32_t)std::max(1, tune_int("sparse_steps", (int)ss->sparse_steps));
        // a round whose chains are at most this many runs the cooperative engine (one
        // wave per chain) to the end of the pass; it needs a wave's aux stack to hold
        // a depth-first descent below its expansion limit, and lane 0's exact DFS stack
        // 49,152 on the 256-CU part (2 query waves per shade wave, hit-region query; rank-of-4 /
        // rank-of-8 per GPU, teams of 8, two runs each: 32 k 2,758-2,782 / 2,348-2,396, 49 k
        // 2,754-2,774 / 2,377-2,421, 65 k 2,731-2,763 / 2,318-2,338, 98 k 2,695-2,699 / 2,220-2,324,
        // 131 k 2,599-2,603 / 2,358-2,430 Mray/s)
        ss->coop_max = cus * 192u;
        ss->coop_max = (uint32_t)std::max(0, tune_int("coop", (int)ss->coop_max));
        ss->coop_grid = cus * 8u;
        // (a depth-first descent below the expansion limit adds at most 3 entries per level)
        const uint32_t reserve = 3u * (s->auxsl_depth + 2u);
        // a team size's stacks hold this tree: the expansion (its own stack, or for teams of 4
        // the wave's pool of 1,024 words) a depth-first descent below the reserve, and the
        // leader's exact DFS (its stack, or its 64-word slice of the pool) the whole tree
        // (and for teams below 64 the pool's items, chain << 29 | node -- teams of 4: << 28 -- hold
        // every aux entry index)
        auto team_ok = [&](uint32_t t) {
            if (t < 64u && s->auxsl.size() >= (1ull << (t == 4u ? 28 : 29))) return false;
            if (t == 4u) return 1024u >= reserve + 64u && s->max_stack <= 64u;
            const uint32_t scap = t == 64u ? 448u : t == 32u ? 192u : QC_SCAP_MIN;
            return scap >= reserve + 64u && s->max_stack <= scap;
        };
        ss->coop_team = (uint32_t)tune_int("coop_team", (int)ss->coop_team);
        if (ss->coop_team != 4u && ss->coop_team != 8u && ss->coop_team != 16u && ss->coop_team != 32u)
            ss->coop_team = 64u;
        if (!team_ok(ss->coop_team)) ss->coop_team = 64u;   // deep trees: whole-wave teams
        // (paths deeper than QC_FOLD keep their further fold records in HBM, planes and
        // emitters beyond QC_NPL / QC_NEM come from HBM: no scene limit besides the stacks)
        if (448u < reserve + 64u || s->max_stack > 448u)
            ss->coop_max = 0;
        else ss->coop_reserve = reserve;
        // with the cooperative engine the path engine never runs a round to the end:
        // its rounds stay budget-limited, so the host sees the chains fall below coop_max
        if (ss->coop_max && !tune_has("runend")) ss->path_runend = 0;
        // ... and the end-of-pass (sparse) path kernel, whose rounds are long, never runs
        // above the hand-over
        if (ss->coop_max && !tune_has("sparse")) ss->path_sparse = std::min(ss->path_sparse, ss->coop_max);
        ss->round_batch = (uint32_t)std::max(1, tune_int("round_batch", (int)ss->round_batch));
        ss->coop_order = tune_int("coop_order", 1) != 0;
        // the final launch's last chains to whole-wave teams: 16 per CU (4 per CU measured within
        // the spread of 0; 16 with the 5-ms low-round deadline above: see low_ticks)
        ss->coop_grow = (uint32_t)std::max(0, tune_int("coop_grow", (int)(cus * 16u)));
        // ... and, before that, its last coop_grow_mid chains to teams of 32 (0: no such stage; a
        // tree too deep for the teams-of-32 stack skips it)
        ss->coop_grow_mid = (uint32_t)std::max(0, tune_int("coop_grow_mid", 0));
        if (192u < reserve + 64u || s->max_stack > 192u) ss->coop_grow_mid = 0u;
        // Early cooperative launch (teams of side_team lanes, QC_WAVES waves per workgroup):
        // the low-chain rounds leave each CU room for one more workgroup, which the heaviest
        // chains use from then on instead of waiting for the final hand-over
        ss->early_wg = (uint32_t)std::max(1, tune_int("early_wg", 1));
        ss->early_at = (uint32_t)std::max(0, tune_int("early_at", (int)(cus * 768u)));
        ss->early_k = (uint32_t)std::max(0, tune_int("early", 1));
        // lanes per chain of that launch: 4 (default: 16 chains per wave, its pooled query keeps
        // a wave's lanes busy with half as many lanes per chain; rank 0 of 8 73.5-75.2 ms against
        // 76.4-83.1 with teams of 8, of 4 130.4-132.0 against 131.1-133.7, of 1 472-476 against
        // 476-480: profiles/r06_coop/team4), 8, 16, 32 or 64
        // (a scene beyond the LDS tables has only the teams-of-8 BIG instantiation)
        const bool big = coop_big(ss);
        {
            const int st = tune_int("side_team", 4);
            ss->side_team = !big && (st == 4 || st == 16 || st == 32 || st == 64) ? (uint32_t)st : 8u;
            if (!team_ok(ss->side_team)) ss->side_team = team_ok(8u) ? 8u : 64u;
        }
        if (ss->early_k == 1u) ss->early_k = cus * ss->early_wg * QC_WAVES * (64u / ss->side_team);   // early=1: what it holds
        if (!ss->coop_max || (ss->coop_team != 8u && ss->coop_team != 4u) || ss->side_team == 64u) ss->early_k = 0;
        // a round's carry output also takes the early launch's yielded chains
        ss->carry_cap = (uint32_t)std::min<uint64_t>(n, (uint64_t)ss->lane_cap + ss->early_k);
        {
            static const char* keys[4] = {"probe_every", "probe_min", "aux_extra", "end_min"};
            static const char* lkeys[4] = {"lowq_probe_every", "lowq_probe_min", "lowq_aux_extra", "lowq_end_min"};
            for (int i = 0; i < 4; ++i) {
                const int lo = i == 0 || i == 3 ? 1 : 0;
                ss->mix[i] = (uint32_t)std::max(lo, tune_int(keys[i], (int)ss->mix[i]));
                // (the low rounds' end_min has a default of its own; the others follow the full rounds')
                ss->mix_low[i] = (uint32_t)std::max(lo, tune_int(lkeys[i], (int)(i == 3 ? ss->mix_low[i] : ss->mix[i])));
            }
            ss->mix[3] = std::min<uint32_t>(ss->mix[3], 64u);
            ss->mix_low[3] = std::min<uint32_t>(ss->mix_low[3], 64u);
            // Rounds that start with fewer than 768 chains per CU run on 2 path workgroups
            // per CU (PT_CMAX chains each) instead of 4: with that few chains the rounds are
            // bound by each chain's latency, and a query trip's instruction stream shares its
            // SIMD with fewer waves.  Rank-of-1 / 2 / 4 / 8 (rank 0, three interleaved
            // repeats, profiles/r03_lowq): +2.3 / +2 / +4 / +3-10 %; 150 k / 250 k chains
            // within 1 % at ranks of 1-4, and 300 k (every round of a rank of 8, the first
            // included) -25 % at rank-of-8.
            ss->lowq = (uint32_t)std::max(0, tune_int("lowq", (int)(cus * 768u)));
            ss->low_grid = std::min(ss->path_grid, cus * (uint32_t)std::max(1, tune_int("lowq_wg", 2)));
        }
        if (ss->n_tiles_local) {
            // seeding order of the pass: the local tiles sorted by the Z-order (Morton)
            // code of their tile coordinates
            std::vector<std::pair<uint64_t, uint32_t>> key(ss->n_tiles_local);
            for (uint32_t t = 0; t < ss->n_tiles_local; ++t) {
                const uint32_t gt = ss->gtiles[t];
                const uint32_t tx = gt % ss->tm.tiles_x, ty = gt / ss->tm.tiles_x;
                uint64_t m = 0;
                for (int b = 0; b < 16; ++b)
                    m |= (uint64_t)((tx >> b) & 1u) << (2 * b) | (uint64_t)((ty >> b) & 1u) << (2 * b + 1);
                key[t] = {m, t};
            }
            std::sort(key.begin(), key.end());
            ord.resize(ss->n_tiles_local);
            for (uint32_t t = 0; t < ss->n_tiles_local; ++t) ord[t] = key[t].second;
        }
    }
    // Every device buffer of the session in ONE allocation (sections at 256-B
    // offsets), and the two small host-made tables with one copy: session set-up is
    // a handful of runtime calls, whatever the pixel count.
    {
        size_t at = 0;
        auto sec = [&at](size_t bytes) {
            const size_t o = at;
            at = (at + std::max<size_t>(bytes, 16) + 255) & ~(size_t)255;
            return o;
        };
        const size_t tables = sec((ss->gtiles.size() + ord.size()) * 4);
        const size_t a_rec = sec(2 * n * sizeof(uint4)), a_fold = sec((size_t)ss->st.depth * n * sizeof(uint4));
        const size_t a_ctr = sec(8 * PT_CTR_COPIES * PT_CTR_STRIDE), a_out = sec(3 * n);
        // the window's framebuffer (pt_render's device-side gather; rank 0's session)
        const size_t a_fb = o->rank == 0 ? sec(3ull * ss->tm.ww * ss->tm.wh) : 0;
        size_t a_fq[2][3] = {{0, 0, 0}, {0, 0, 0}}, a_pid = 0, a_dq[2] = {0, 0}, a_ex[2] = {0, 0}, a_hid = 0;
        size_t a_carry = 0, a_ctl = 0, a_endq = 0, a_order = 0, a_side[6] = {0, 0, 0, 0, 0, 0};
        if (ss->wave) {
            for (int q = 0; q < 2; ++q)
                for (int k = 0; k < 3; ++k) a_fq[q][k] = sec(n * 16);
            a_pid = sec(2 * n * 4);
            for (int k = 0; k < 2; ++k) { a_dq[k] = sec(n * 16); a_ex[k] = sec(n * 16); }
            a_hid = sec(n * 4);
            a_carry = sec(2ull * ss->carry_cap * ss->carry_words * 4);
            a_ctl = sec(8 * PT_CTL_SET);
            a_endq = sec((size_t)ss->path_grid * PT_CMAX * sizeof(uint2));
            a_order = sec((n + 2 * PT_ORDER_BUCKETS) * 4);
            if (ss->early_k) {
                for (int k = 0; k < 3; ++k) a_side[k] = sec((size_t)ss->early_k * 16);
                a_side[3] = sec((size_t)ss->early_k * 4);
                a_side[4] = sec((size_t)ss->early_k * ss->carry_words * 4);
                a_side[5] = sec(8 * PT_CTL_SET);
            }
        }
        if (take_stream(ss->dev, &ss->stream) != hipSuccess) return cleanup(fail(PT_E_HIP, "stream creation failed"));
        // the early launch's stream and events: made on a helper thread beside the set-up and
        // the pass's first rounds (a stream's creation costs ~10 ms: neither on the set-up's
        // path nor in the pass), joined where the first early launch needs them
        if (ss->early_k) {
            const int dev = ss->dev;
            auto make = [ss, dev] {
                ss->side_rc = hipSetDevice(dev);
                if (ss->side_rc == hipSuccess) ss->side_rc = take_stream(dev, &ss->side_stream, true);
                if (ss->side_rc == hipSuccess) ss->side_rc = hipEventCreateWithFlags(&ss->side_taken, hipEventDisableTiming);
                if (ss->side_rc == hipSuccess) ss->side_rc = hipEventCreateWithFlags(&ss->side_end, hipEventDisableTiming);
            };
            try {
                ss->side_th = std::thread(make);
            } catch (const std::system_error&) {
                // (no helper thread: made here, and the current device set back)
                make();
                if (hipSetDevice(ss->dev) != hipSuccess) return cleanup(fail(PT_E_HIP, "hipSetDevice failed"));
            }
        }
        void* p = nullptr;
        if (hipMalloc(&p, at) != hipSuccess) return cleanup(fail(PT_E_OOM, "device allocation failed (session buffers)"));
        ss->arena = static_cast<unsigned char*>(p);
        unsigned char* A = ss->arena;
        if (!ss->gtiles.empty()) {
            std::vector<uint32_t> t(ss->gtiles);
            t.insert(t.end(), ord.begin(), ord.end());
            if (hipMemcpy(A + tables, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
                return cleanup(fail(PT_E_HIP, "tile tables upload failed"));
            ss->tm.gtile = reinterpret_cast<const uint32_t*>(A + tables);
            if (!ord.empty()) ss->tile_order = reinterpret_cast<uint32_t*>(A + tables) + ss->gtiles.size();
        }
        ss->st.rec = reinterpret_cast<uint4*>(A + a_rec);
        ss->st.fold = reinterpret_cast<uint4*>(A + a_fold);
        ss->counters = reinterpret_cast<unsigned long long*>(A + a_ctr);
        ss->out = A + a_out;
        if (o->rank == 0) ss->fb = A + a_fb;
        if (ss->wave) {
            for (int q = 0; q < 2; ++q) {
                ss->fq[q].ro = reinterpret_cast<pt::F4*>(A + a_fq[q][0]);
                ss->fq[q].rd = reinterpret_cast<pt::F4*>(A + a_fq[q][1]);
                ss->fq[q].ri = reinterpret_cast<pt::F4*>(A + a_fq[q][2]);
                ss->fq[q].pid = reinterpret_cast<int*>(A + a_pid) + q * n;
            }
            ss->done = pt::DoneQ{reinterpret_cast<pt::F4*>(A + a_dq[0]), reinterpret_cast<pt::F4*>(A + a_dq[1]),
                                 reinterpret_cast<uint32_t*>(A + a_hid)};
            ss->ex = pt::RayQ{reinterpret_cast<pt::F4*>(A + a_ex[0]), reinterpret_cast<pt::F4*>(A + a_ex[1]), nullptr,
                              nullptr};
            ss->carry = reinterpret_cast<uint32_t*>(A + a_carry);
            ss->ctl = reinterpret_cast<uint32_t*>(A + a_ctl);
            ss->endq = reinterpret_cast<uint2*>(A + a_endq);
            ss->order = reinterpret_cast<uint32_t*>(A + a_order);
            if (ss->early_k) {
                ss->side.ro = reinterpret_cast<pt::F4*>(A + a_side[0]);
                ss->side.rd = reinterpret_cast<pt::F4*>(A + a_side[1]);
                ss->side.ri = reinterpret_cast<pt::F4*>(A + a_side[2]);
                ss->side.pid = reinterpret_cast<int*>(A + a_side[3]);
                ss->side_carry = reinterpret_cast<uint32_t*>(A + a_side[4]);
                ss->side_ctl = reinterpret_cast<uint32_t*>(A + a_side[5]);
            }
            if (hipHostMalloc(&ss->ctl_host, 64) != hipSuccess)
                return cleanup(fail(PT_E_OOM, "host allocation failed (round counters)"));
        }
        ss->arena_bytes = at;
    }
    if (hipMemsetAsync(ss->counters, 0, 8 * PT_CTR_COPIES * PT_CTR_STRIDE, ss->stream) != hipSuccess) return cleanup(fail(PT_E_HIP, "memset failed"));
    if (ss->n_tiles_local) {
        pt::InitParams ip;
        ip.tm = ss->tm;
        ip.st = ss->st;
        if (pt_launch_init(ip, ss->n_tiles_local, ss->stream) != hipSuccess)
            return cleanup(fail(PT_E_HIP, "k_init launch failed"));
    }
    *out = ss;
    return PT_OK;
}

int pt_session_layout(const pt_session* ss, uint32_t* n_tiles, uint64_t* packed_rgb_bytes) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (n_tiles) *n_tiles = ss->n_tiles_local;
    if (packed_rgb_bytes) *packed_rgb_bytes = 3ull * ss->n_slots;
    return PT_OK;
}

int pt_session_trace(pt_session* ss, uint32_t spp) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (spp == 0 || ss->n_tiles_local == 0) { ss->samples_done += spp; return PT_OK; }
    if (ss->wave) {
        // Consecutive calls are one pass: a pixel goes on with its next samples as soon
        // as it is done with the current ones, so only the last call waits for the
        // slowest pixel.  The pass runs at the next resolve / sync / stats.
        if (ss->deferred_spp > 0xffffffffu - spp) {
            const int rc = flush_trace(ss);
            if (rc) return rc;
        }
        ss->deferred_spp += spp;
        return PT_OK;
    }
    HIP_TRY(hipSetDevice(ss->dev));
    const DevScene& ds = *ss->ds;
    pt::TraceParams tp;
    const pt_scene* s = ss->sc;
    tp.S.aux = ss->traversal == PT_TRAVERSAL_EXACT ? nullptr : ds.aux;
    tp.cfg = replay_cfg(s);
    tp.S.nodes = ds.nodes;
    tp.S.prims = ds.prims;
    tp.S.shade = ds.shade;
    tp.S.planes = ds.planes;
    tp.S.emitters = ds.emitters;
    tp.S.n_planes = (uint32_t)s->planes.size();
    tp.S.n_emitters = (uint32_t)s->emitters.size();
    tp.S.inv_emitters = s->emitters.empty() ? 0.f : 1.f / (float)s->emitters.size();
    tp.S.bg = pt::mk3(s->hs.bg[0], s->hs.bg[1], s->hs.bg[2]);
    tp.S.box_extent = s->box_extent;
    tp.S.anc_info = ds.anc_info;
    tp.S.anc = ds.anc;
    tp.cam = ss->cam;
    tp.tm = ss->tm;
    tp.st = ss->st;
    tp.counters = ss->counters;
    tp.depth = ss->depth;
    tp.spp = spp;
    tp.n_tiles_local = ss->n_tiles_local;
    tp.wg_prof = nullptr;
    // kernel variant: filtered tests unless the division form was asked for; XCD-banded tile order
    const int variant = (ss->traversal == PT_TRAVERSAL_REPLAY ? 1 : 0) | 2;
    const std::string wgps = tune_str("wgprof");
    const char* wgp = wgps.c_str();
    if (*wgp) {
        if (!ss->wg_prof) HIP_TRY(hipMalloc(&ss->wg_prof, 32ull * std::max(ss->n_tiles_local, 1u)));
        HIP_TRY(hipMemsetAsync(ss->wg_prof, 0, 32ull * std::max(ss->n_tiles_local, 1u), ss->stream));
        tp.wg_prof = ss->wg_prof;
    }
    const uint32_t lds = 256u * 4u * lane_words(s, ss->traversal);
    if (lds > 160u * 1024u) return fail(PT_E_SCENE, "BVH too deep for the LDS traversal stack");
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, ss->stream));
    HIP_TRY(pt_launch_trace(tp, variant, lds, ss->stream));
    HIP_TRY(hipEventRecord(e1, ss->stream));
    if (tp.wg_prof) {
        // diagnostics: append this launch's per-workgroup timeline to the wgprof file
        std::vector<unsigned long long> h(4ull * ss->n_tiles_local);
        HIP_TRY(hipMemcpyAsync(h.data(), tp.wg_prof, h.size() * 8, hipMemcpyDeviceToHost, ss->stream));
        HIP_TRY(hipStreamSynchronize(ss->stream));
        if (FILE* f = fopen(wgp, "ab")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
    ss->pending.emplace_back(e0, e1);
    ss->samples_done += spp;
    return PT_OK;
}

int pt_session_resolve(pt_session* ss, uint8_t* dev_out, float* dev_radiance) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (ss->n_tiles_local == 0) return PT_OK;
    if (const int rc = flush_trace(ss)) return rc;
    HIP_TRY(hipSetDevice(ss->dev));
    pt::ResolveParams rp;
    rp.st = ss->st;
    rp.tm = ss->tm;
    rp.counters = ss->counters;
    rp.thr = ss->ds->thr;
    rp.out = dev_out ? dev_out : ss->out;
    rp.rad = dev_radiance;
    rp.samples = (uint32_t)ss->samples_done;
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, ss->stream));
    HIP_TRY(pt_launch_resolve(rp, ss->n_tiles_local, ss->stream));
    HIP_TRY(hipEventRecord(e1, ss->stream));
    HIP_TRY(hipStreamSynchronize(ss->stream));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess) ss->resolve_ms += ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    // pixels short of (or past) the samples so far: a chain was lost -- an error, not an image
    unsigned long long c[PT_CTR_STRIDE];
    HIP_TRY(read_counters(ss, c));
    if (c[pt::CTR_SHORT] != ss->short_seen) {
        const unsigned long long k = c[pt::CTR_SHORT] - ss->short_seen;
        ss->short_seen = c[pt::CTR_SHORT];
        if (tune_int("shortlog", 0)) {
            // diagnostics: how far the short pixels are from the target, and where they are
            std::vector<uint4> rec(2ull * ss->n_slots);
            if (hipMemcpy(rec.data(), ss->st.rec, rec.size() * sizeof(uint4), hipMemcpyDeviceToHost) == hipSuccess) {
                std::map<int, uint32_t> hist;
                uint32_t shown = 0;
                for (uint32_t i = 0; i < ss->n_slots; ++i) {
                    const uint32_t done = rec[2 * i].w, nv = rec[2 * i].z >> 8;
                    if (done == rp.samples || rec[2 * i + 1].w == 0xFFFFFFFFu) continue;
                    hist[(int)done - (int)rp.samples]++;
                    if (shown++ < 8)
                        fprintf(stderr, "short: slot %u pixel %u done %u nv %u\n", i, rec[2 * i + 1].w, done, nv);
                }
                for (auto& h : hist) fprintf(stderr, "short: done - samples = %d: %u pixels\n", h.first, h.second);
            }
        }
        return fail(PT_E_HIP, std::to_string(k) + " pixel(s) did not take exactly " + std::to_string(rp.samples) +
                                  " samples (a chain was lost)");
    }
    return PT_OK;
}

int pt_session_sync(pt_session* ss) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (const int rc = flush_trace(ss)) return rc;
    HIP_TRY(hipSetDevice(ss->dev));
    HIP_TRY(hipStreamSynchronize(ss->stream));
    return finish_pending(ss);
}

int pt_session_reset(pt_session* ss) {
    if (!ss) return fail(PT_E_INVALID, "null session");
    if (const int rc = flush_trace(ss)) return rc;
    HIP_TRY(hipSetDevice(ss->dev));
    if (ss->n_tiles_local) {
        pt::InitParams ip;
        ip.tm = ss->tm;
        ip.st = ss->st;
        HIP_TRY(pt_launch_init(ip, ss->n_tiles_local, ss->stream));
    }
    ss->samples_done = 0;
    return PT_OK;
}

int pt_session_read_packed(pt_session* ss, uint8_t* host_out, size_t bytes) {
    if (!ss || !host_out) return fail(PT_E_INVALID, "null argument");
    if (bytes < 3ull * ss->n_slots) return fail(PT_E_INVALID, "buffer too small");
    if (ss->n_slots == 0) return PT_OK;
    HIP_TRY(hipSetDevice(ss->dev));
    HIP_TRY(hipMemcpyAsync(host_out, ss->out, 3ull * ss->n_slots, hipMemcpyDeviceToHost, ss->stream));
    HIP_TRY(hipStreamSynchronize(ss->stream));
    return PT_OK;
}

int pt_session_stats(pt_session* ss, pt_stats* st) {
    if (!ss || !st) return fail(PT_E_INVALID, "null argument");
    int rc = pt_session_sync(ss);
    if (rc) return rc;
    unsigned long long c[PT_CTR_STRIDE];
    HIP_TRY(read_counters(ss, c));
    memset(st, 0, sizeof(*st));
    st->rays = c[0];
    st->node_visits = c[1];
    st->prim_tests = c[2];
    st->plane_tests = c[3];
    st->errors = c[4];
    st->aux_visits = c[5];
    st->fallbacks = c[6];
    st->fallbacks_ray = c[7];
    st->samples = owned_pixels(ss) * ss->samples_done;
    st->kernel_ms = ss->kernel_ms;
    st->resolve_ms = ss->resolve_ms;
    st->node_bytes = sizeof(pt::Node);
    st->prim_bytes = sizeof(pt::Prim);
    // algorithmic bytes per counted unit: wavefront query = 4-wide aux node (128 B),
    // reference node record (32 B), primitive geometry (48 B: the 64-B compact record
    // adds the precomputed triangle normal, a layout choice, not counted)
    st->aux_bytes = ss->wave ? PT_AUXW * sizeof(pt::AuxSL) : sizeof(pt::AuxNode);
    if (ss->wave) st->prim_bytes = 48;
    st->isect_ms = ss->isect_ms;
    st->isect_launches = ss->isect_launches;
    st->rounds = ss->rounds;
    st->coop_rays = c[8];
    st->coop_node_visits = c[9];
    st->coop_prim_tests = c[10];
    st->coop_aux_visits = c[13];
    st->coop_ms = ss->coop_ms;
    st->coop_launches = ss->coop_launches;
    st->short_pixels = c[pt::CTR_SHORT];
    st->handed_on = c[pt::CTR_HANDON];
    for (uint32_t k = 0; k < PT_HO_N; ++k) st->handoff[k] = c[pt::CTR_HO + k];
    return PT_OK;
}

void* pt_session_stream(pt_session* ss) {
    if (!ss) return nullptr;
    (void)flush_trace(ss);   // work ordered after the stream sees every trace() so far (errors: pt_last_error)
    return (void*)ss->stream;
}

void pt_session_free(pt_session* ss) {
    if (!ss) return;
    if (ss->side_th.joinable()) ss->side_th.join();
    (void)hipSetDevice(ss->dev);
    // both streams drained before any buffer goes (a side launch may still run after a
    // failed pass)
    if (ss->stream) (void)hipStreamSynchronize(ss->stream);
    if (ss->side_stream) (void)hipStreamSynchronize(ss->side_stream);
    finish_pending(ss);
    (void)hipFree(ss->arena);
    (void)hipFree(ss->rad); (void)hipFree(ss->wg_prof);
    if (ss->ctl_host) (void)hipHostFree(ss->ctl_host);
    if (ss->prog_host) (void)hipHostFree(ss->prog_host);
    if (ss->side_taken) (void)hipEventDestroy(ss->side_taken);
    if (ss->side_end) (void)hipEventDestroy(ss->side_end);
    // back to the device's pools for the next session (no destroy/create per render)
    give_stream(ss->dev, ss->stream, false);
    give_stream(ss->dev, ss->side_stream, true);
    delete ss;
}

int pt_unpack_tiles(uint32_t W, uint32_t H, uint32_t rank, uint32_t world, const uint8_t* packed, uint8_t* rgb) {
    if (!packed || !rgb || world == 0) return fail(PT_E_INVALID, "bad argument");
    const uint32_t tiles_x = (W + 15u) / 16u, n_tiles = tiles_x * ((H + 15u) / 16u);
    uint32_t lt = 0;
    for (uint32_t gt = 0; gt < n_tiles; ++gt) {
        if (pt::tile_owner(gt, tiles_x, world) != rank) continue;
        const uint32_t tx = gt % tiles_x, ty = gt / tiles_x;
        for (uint32_t j = 0; j < 16u; ++j) {
            const uint32_t y = ty * 16u + j;
            if (y >= H) break;
            const uint32_t x0 = tx * 16u, w = std::min(16u, W - x0);
            memcpy(rgb + ((size_t)y * W + x0) * 3, packed + ((size_t)lt * 256u + j * 16u) * 3, (size_t)w * 3);
        }
        ++lt;
    }
    return PT_OK;
}

int pt_unpack_tiles_f32(uint32_t W, uint32_t H, uint32_t rank, uint32_t world, const float* packed, float* rad) {
    if (!packed || !rad || world == 0) return fail(PT_E_INVALID, "bad argument");
    const uint32_t tiles_x = (W + 15u) / 16u, n_tiles = tiles_x * ((H + 15u) / 16u);
    uint32_t lt = 0;
    for (uint32_t gt = 0; gt < n_tiles; ++gt) {
        if (pt::tile_owner(gt, tiles_x, world) != rank) continue;
        const uint32_t tx = gt % tiles_x, ty = gt / tiles_x;
        for (uint32_t j = 0; j < 16u; ++j) {
            const uint32_t y = ty * 16u + j;
            if (y >= H) break;
            const uint32_t x0 = tx * 16u, w = std::min(16u, W - x0);
            memcpy(rad + ((size_t)y * W + x0) * 3, packed + ((size_t)lt * 256u + j * 16u) * 3, (size_t)w * 12);
        }
        ++lt;
    }
    return PT_OK;
}

}  // extern "C"
