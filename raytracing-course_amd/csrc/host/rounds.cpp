// rounds.cpp -- the wavefront pass of a session (trace_wave): k_wcamera seeds it,
// path rounds (k_wpath -> k_wexact -> k_wshade) run until the chains are few, the
// early cooperative launch runs beside the low-chain rounds on the side stream, and
// the final cooperative launch (teams of 4, then whole-wave teams) runs the rest to
// the end of the pass.  DESIGN.md §4 describes each step.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include "api_internal.h"

namespace pti {

int trace_wave(pt_session* ss, uint32_t spp) {
    const DevScene& ds = *ss->ds;
    const pt_scene* s = ss->sc;
    pt::WaveParams wp;
    memset(&wp, 0, sizeof(wp));
    wp.S.aux = nullptr;
    wp.S.nodes = ds.nodes;
    wp.S.prims = ds.prims;
    wp.S.shade = ds.shade;
    wp.S.planes = ds.planes;
    wp.S.emitters = ds.emitters;
    wp.S.n_planes = (uint32_t)s->planes.size();
    wp.S.n_emitters = (uint32_t)s->emitters.size();
    wp.S.inv_emitters = s->emitters.empty() ? 0.f : 1.f / (float)s->emitters.size();
    wp.S.bg = pt::mk3(s->hs.bg[0], s->hs.bg[1], s->hs.bg[2]);
    wp.S.box_extent = s->box_extent;
    wp.S.anc_info = ds.anc_info;
    wp.S.anc = ds.anc;
    set_blob(wp.S, s, ds.blob);
    wp.top = ds.top;
    wp.n_top = ds.n_top;
    wp.n_aux = (uint32_t)s->auxsl.size();
    wp.cam = ss->cam;
    wp.tm = ss->tm;
    wp.st = ss->st;
    wp.fq[0] = ss->fq[0];
    wp.fq[1] = ss->fq[1];
    wp.done = ss->done;
    wp.ex = ss->ex;
    wp.endq = ss->endq;
    wp.cq[0] = ss->carry;
    wp.cq[1] = ss->carry + (size_t)ss->carry_cap * ss->carry_words;
    wp.carry_cap = ss->carry_cap;
    wp.carry_words = ss->carry_words;
    wp.ctl = ss->ctl;
    wp.counters = ss->counters;
    wp.depth = ss->depth;
    wp.target = (uint32_t)(ss->samples_done + spp);
    wp.n_tiles_local = ss->n_tiles_local;
    wp.max_stack = std::max<uint32_t>(s->max_stack, 1u);
    wp.aux_stack = std::max<uint32_t>(s->auxw_stack, 1u);
    wp.path = 1u;
    wp.path_budget = ss->path_budget;
    wp.path_ticks = ss->path_ticks;
    wp.path_runend = ss->path_runend;
    // Chains a workgroup may hold: 5/8 of the pixels' fair share, within
    // [256, PT_CMAX].  Below the share, about a third of the chains wait in the
    // queue and go to whichever workgroup drains first, instead of every
    // workgroup filling to its share and the costly ones finishing last
    // (1920x1080 on 1,024 workgroups: rank of 4 -> 319 instead of 478, +1 % over
    // three alternating pairs; ranks of 1 and 2 stay at 512, a rank of 8 at 256).
    {
        const uint64_t share = ((uint64_t)ss->n_slots + ss->path_grid - 1) / std::max(1u, ss->path_grid);
        wp.path_cap = (uint32_t)std::min<uint64_t>(PT_CMAX, std::max<uint64_t>(256u, share * 5u / 8u));
    }
    if (tune_has("cap")) wp.path_cap = std::min<uint32_t>(PT_CMAX, (uint32_t)std::max(64, tune_int("cap", 0)));
    wp.tile_order = ss->tile_order;
    wp.sparse_steps = ss->sparse_steps;
    wp.coop_reserve = ss->coop_reserve;
    // aux stack words per query lane (PT_TUNE lstack=N < PT_LSTACK: tests of the exact-DFS
    // hand-over of queries that outgrow it)
    // round-queue entries a query wave takes per pull: 32 (64 before round 3's low-chain
    // rounds): a workgroup fills closer to its chain cap in finer pulls; rank-of-1 / 2 / 4 / 8,
    // two calls: +0.5 / +0.5 / +3.5 / +3 % (8 and 16 the same at ranks of 1-4; profiles/r03_lowq)
    wp.batch = (uint32_t)std::min(64, std::max(1, tune_int("batch", 32)));
    wp.end_min = ss->mix[3];
    wp.lstack = std::min<uint32_t>(PT_LSTACK, (uint32_t)std::max(1, tune_int("lstack", (int)PT_LSTACK)));
    // test hooks: PT_TUNE shade_hold=1 (path rounds: the shade wave waits for the query waves to
    // leave), drop=<site> (the items of one hand-off site are lost: the resolve must fail)
    wp.side_flags = tune_int("shade_hold", 0) ? PT_SHADE_HOLD : 0u;
    wp.drop = 0u;
    if (const std::string d = tune_str("drop"); !d.empty()) {
        const int site = handoff_site(d.c_str());
        if (site < 0) return fail(PT_E_INVALID, "PT_TUNE drop=" + d + ": no such hand-off site");
        wp.drop = 1u + (uint32_t)site;
    }
    if (ss->on_progress && !ss->prog_host) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ss->prog_host), 8, hipHostMallocMapped | hipHostMallocCoherent));
        *ss->prog_host = 0ull;
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&ss->prog_dev), ss->prog_host, 0));
    }
    wp.progress = ss->on_progress ? ss->prog_dev : nullptr;
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, ss->stream));
    HIP_TRY(pt_launch_wave_start(wp, ss->stream));
    if (tune_int("roundlog", 0) >= 2) {
        HIP_TRY(hipStreamSynchronize(ss->stream));
        ss->roundlog_t = wall_ms();
        unsigned long long cc[PT_CTR_COPIES * PT_CTR_STRIDE];
        HIP_TRY(hipMemcpy(cc, ss->counters, sizeof(cc), hipMemcpyDeviceToHost));
        ss->roundlog_rays = 0;
        for (uint32_t x = 0; x < PT_CTR_COPIES; ++x) ss->roundlog_rays += cc[PT_CTR_STRIDE * x];
    }
    // rounds until no fresh ray and no suspended query is left; counts are
    // checked every few rounds (empty rounds are cheap, syncs are not free)
    // (the first round is counted alone: it ends once the pass's work is handed out, and
    // the cooperative engine may take over right after it)
    uint32_t p = 0, batch = ss->coop_max ? 1u : 4u;
    // end-of-pass kernel when the chains of the last counted round are few; before
    // the first count, the pass's pixels (at most one chain each) decide
    bool sparse = ss->n_slots < ss->path_sparse;
    // the cooperative engine once the chains are few (before the first count: the pixels)
    uint32_t chains = ss->n_slots;
    bool counted = false;
    for (uint32_t guard = 0;; ++guard) {
        if (chains <= ss->coop_max) {
            // The cooperative engine runs every remaining chain to the end of the pass.  A
            // launch of teams of 4 (the default) stops once all but ss->coop_grow of its chains
            // have ended and hands those -- the pass's slowest, whose chain cycle sets the
            // launch's end -- to a launch of whole-wave teams (the shortest cycle).
            // (a scene beyond the engine's LDS tables runs the BIG instantiation: teams of 8 or 64)
            const bool big = coop_big(ss);
            uint32_t team = big && ss->coop_team != 64u ? 8u : ss->coop_team;
            for (;;) {
                // the next stage: teams of 4 or 8 -> (coop_grow_mid, from 8) teams of 32 -> (coop_grow) whole waves
                uint32_t keep = 0u, next_team = 64u;
                if (team == 8u && !big && ss->coop_grow_mid > ss->coop_grow && chains > ss->coop_grow_mid) {
                    keep = ss->coop_grow_mid;
                    next_team = 32u;
                } else if (team != 64u && ss->coop_grow && chains > ss->coop_grow) {
                    keep = ss->coop_grow;
                }
                // (the chains still running at the stop, at most `keep`, go to the next carry
                // queue: never more than it holds)
                keep = std::min(keep, ss->carry_cap);
                const bool grow = keep != 0u;
                // (test hook grow_late: its late workgroups hand on every item they find
                // untaken, up to all of the launch's -- within the carry queue only)
                const bool grow_late = grow && tune_int("grow_late", 0) != 0;
                if (grow_late && chains > ss->carry_cap)
                    return fail(PT_E_INVALID, "PT_TUNE grow_late: more chains than the carry queue holds");
                wp.parity = p;
                hipEvent_t i0, i1;
                HIP_TRY(hipEventCreate(&i0));
                HIP_TRY(hipEventCreate(&i1));
                ss->pending_isect.emplace_back(i0, i1);
                ss->pending_isect_coop.resize(ss->pending_isect.size(), false);
                ss->pending_isect_coop.back() = true;
                ss->isect_launches++;
                ss->coop_launches++;
                const uint32_t per_wg = QC_WAVES * (64u / team);   // chains per workgroup
                const uint32_t grid = std::max(1u, std::min(ss->coop_grid, (chains + per_wg - 1u) / per_wg));
                const bool cprof = tune_has("cprof");   // -DPT_CPROF builds: per-phase cycles on stderr
                if (cprof) {
                    if (!ss->wg_prof) HIP_TRY(hipMalloc(&ss->wg_prof, 512ull * ss->path_grid));
                    HIP_TRY(hipMemsetAsync(ss->wg_prof, 0, 512, ss->stream));
                    wp.wg_prof = ss->wg_prof;
                }
                if (ss->coop_order) {
                    const size_t cap = std::min<size_t>(std::max<size_t>(ss->n_slots, 1),
                                                        std::max<uint32_t>(ss->coop_max, 1u));
                    if (chains > cap) return fail(PT_E_HIP, "cooperative intake order: more chains than entries");
                    wp.order_cur = ss->order;
                    wp.order = ss->order + 2 * PT_ORDER_BUCKETS;
                    HIP_TRY(pt_launch_coop_order(wp, chains, ss->stream));
                }
                pt::WaveParams cp_ = wp;
                if (grow) {
                    // stop at the chain cycle after all but coop_grow chains have ended (its own
                    // C_ENDED); the rest go to the next launch's input as suspended queries
                    uint32_t* out = ss->ctl + PT_CTL_SET * (1u - p);
                    cp_.side_stop = out + pt::C_ENDED;
                    cp_.side_stop_n = keep;            // (against the launch's own item count: before
                    cp_.side_flags = PT_STOP_GROW |     //  the first count, `chains` is the slot count)
                                     (grow_late ? PT_GROW_LATE : 0u);
                    cp_.yield_cq = wp.cq[1u - p];
                    cp_.yield_ctr = out + pt::C_CARRY;
                }
                HIP_TRY(pt_launch_coop(cp_, grid, team, big, ss->stream, i0, i1));
                wp.order = wp.order_cur = nullptr;
                if (cprof) {
                    unsigned long long cp[64];
                    HIP_TRY(hipMemcpyAsync(cp, wp.wg_prof, 512, hipMemcpyDeviceToHost, ss->stream));
                    HIP_TRY(hipStreamSynchronize(ss->stream));
                    float ms = 0.f;
                    HIP_TRY(hipEventElapsedTime(&ms, i0, i1));
                    const double cyc = (double)std::max(1ull, cp[5] + cp[6]) / (64.0 / team);
                    fprintf(stderr, "coop T=%u chains %u grid %u: %.2f ms, chain cycles %llu, chains %llu; cycles per chain "
                            "cycle: expand %.0f cand %.0f decide %.0f shade %.0f nextray %.0f; wave lifetime %.0f\n",
                            team, chains, grid, ms, cp[5], cp[6], cp[0] / cyc, cp[1] / cyc, cp[2] / cyc, cp[3] / cyc,
                            cp[4] / cyc, (double)cp[7] / (grid * (double)QC_WAVES));
                    // chains ending per 2^20-cycle bucket of their wave's lifetime
                    fprintf(stderr, "coop chain ends per 2^20 cycles:");
                    for (int i = 16; i < 64; ++i) fprintf(stderr, " %llu", cp[i]);
                    fprintf(stderr, "\n");
                    wp.wg_prof = nullptr;
                }
                ss->rounds++;
                p ^= 1u;
                HIP_TRY(hipMemcpyAsync(ss->ctl_host, ss->ctl + PT_CTL_SET * p, 8, hipMemcpyDeviceToHost, ss->stream));
                if (wp.progress) {
                    hipError_t e;
                    while ((e = hipStreamQuery(ss->stream)) == hipErrorNotReady) {
                        ss->on_progress(__atomic_load_n(ss->prog_host, __ATOMIC_RELAXED));
                        std::this_thread::sleep_for(std::chrono::microseconds(500));
                    }
                    HIP_TRY(e);
                }
                HIP_TRY(hipStreamSynchronize(ss->stream));
                if (ss->ctl_host[pt::C_CARRY] > ss->carry_cap)
                    return fail(PT_E_HIP, "carry queue overflow (a lost chain)");
                const uint32_t left = ss->ctl_host[pt::C_CARRY] + ss->ctl_host[pt::C_FRESH];
                if (left == 0u) break;
                if (!grow) return fail(PT_E_HIP, "cooperative engine left chains behind");
                // the last chains: bigger teams
                chains = left;
                team = next_team;
                if (tune_int("roundlog", 0) >= 2) fprintf(stderr, "coop grow: %u chains to teams of %u\n", left, team);
            }
            break;
        }
        // The early cooperative launch, beside every low-chain round: the round's heaviest
        // chains (most samples left) run in a cooperative launch on the second stream while
        // the path round runs the others (through wp.pin); the launch stops at a chain cycle's
        // end once the round's path workgroups have all finished, its chains yielded to the
        // next round's carry queue, and the next round starts when both are done.
        // (only after a count: before the first one `chains` is the slot count, not the
        // queue's, and every pixel has the same samples left)
        bool side = false;
        // (test hook side_late: the side launch runs after the path round, on its stream --
        // every workgroup one that started after the round's end)
        pt::WaveParams late_sp;
        bool late = false;
        uint32_t late_grid = 0;
        if (ss->early_k && counted && chains < ss->early_at && chains > ss->coop_max) {
            const uint32_t k = std::min(ss->early_k, chains / 4u);
            const uint32_t grid = chains < ss->lowq && ss->low_grid ? ss->low_grid : ss->path_grid;
            if (k) {
                side = true;
                if (ss->side_th.joinable()) {
                    ss->side_th.join();
                    if (ss->side_rc != hipSuccess) return fail(PT_E_HIP, "side stream creation failed");
                }
                if (!ss->side_stream && take_stream(ss->dev, &ss->side_stream, true) != hipSuccess)
                    return fail(PT_E_HIP, "stream creation failed");
                wp.parity = p;
                wp.order_cur = ss->order;
                wp.order = ss->order + 2 * PT_ORDER_BUCKETS;
                HIP_TRY(pt_launch_coop_order(wp, chains, ss->stream));
                HIP_TRY(hipMemsetAsync(ss->side_ctl, 0, 8 * PT_CTL_SET, ss->stream));
                HIP_TRY(pt_launch_side_take(wp, k, ss->side, ss->side_carry, ss->side_ctl, ss->stream));
                // the round's output counters (its finished-workgroup count among them) are zero
                // before the side launch can look at them
                uint32_t* out = ss->ctl + PT_CTL_SET * (1u - p);
                HIP_TRY(hipMemsetAsync(out, 0, 4u * PT_CTL_SET, ss->stream));
                if (!ss->side_taken) HIP_TRY(hipEventCreateWithFlags(&ss->side_taken, hipEventDisableTiming));
                if (!ss->side_end) HIP_TRY(hipEventCreateWithFlags(&ss->side_end, hipEventDisableTiming));
                HIP_TRY(hipEventRecord(ss->side_taken, ss->stream));
                HIP_TRY(hipStreamWaitEvent(ss->side_stream, ss->side_taken, 0));
                pt::WaveParams sp = wp;
                sp.fq[0] = ss->side;
                sp.cq[0] = ss->side_carry;
                sp.ctl = ss->side_ctl;
                sp.parity = 0u;
                sp.order = sp.order_cur = nullptr;
                sp.pin = nullptr;
                sp.side_stop = out + pt::C_WGDONE;
                sp.side_stop_n = grid;
                sp.yield_cq = wp.cq[1u - p];
                sp.yield_ctr = out + pt::C_CARRY;
                sp.side_flags = (tune_int("side_late", 0) ? PT_SIDE_LATE : 0u) |
                                (tune_int("side_stop_now", 0) ? PT_SIDE_STOP_NOW : 0u) |
                                (tune_int("handon", 1) ? 0u : PT_SIDE_NO_HANDON);
                hipEvent_t i0, i1;
                HIP_TRY(hipEventCreate(&i0));
                HIP_TRY(hipEventCreate(&i1));
                ss->pending_isect.emplace_back(i0, i1);
                ss->pending_isect_coop.resize(ss->pending_isect.size(), false);
                ss->pending_isect_coop.back() = true;
                ss->isect_launches++;
                ss->coop_launches++;
                const bool big = coop_big(ss);
                if (sp.side_flags & PT_SIDE_LATE) {
                    late = true;
                    late_sp = sp;
                    late_grid = ss->early_wg * (ss->coop_grid / 8u);
                    HIP_TRY(hipEventRecord(i0, ss->stream));   // (timed with the round)
                    HIP_TRY(hipEventRecord(i1, ss->stream));
                } else {
                    HIP_TRY(pt_launch_coop(sp, ss->early_wg * (ss->coop_grid / 8u), ss->side_team, big, ss->side_stream, i0, i1));
                    HIP_TRY(hipEventRecord(ss->side_end, ss->side_stream));
                }
                // the path round takes the other chains: items k .. chains of the order
                wp.pin = wp.order + k;
                wp.pin_n = chains - k;
                wp.order = wp.order_cur = nullptr;
                batch = 1u;   // (the next round reads what the side launch yields)
            }
        }
        for (uint32_t r = 0; r < batch; ++r) {
            wp.parity = p;
            const std::string wgps = tune_str("wgprof");
            const char* wgp = wgps.c_str();
            if (*wgp) {
                // diagnostics: per-round path workgroup timelines (32 u64 each) appended to the file
                const size_t wgb = 512ull * ss->path_grid;
                if (!ss->wg_prof) HIP_TRY(hipMalloc(&ss->wg_prof, wgb));
                HIP_TRY(hipMemsetAsync(ss->wg_prof, 0, wgb, ss->stream));
                wp.wg_prof = ss->wg_prof;
            }
            hipEvent_t i0, i1;
            HIP_TRY(hipEventCreate(&i0));
            HIP_TRY(hipEventCreate(&i1));
            ss->pending_isect.emplace_back(i0, i1);
            ss->isect_launches++;
            uint32_t grid = ss->path_grid;
            {
                const bool low = chains < ss->lowq;
                wp.path_ticks = low ? ss->low_ticks : ss->path_ticks;
                const uint32_t* m = low ? ss->mix_low : ss->mix;
                wp.probe_every = m[0];
                wp.probe_min = m[1];
                wp.aux_extra = m[2];
                wp.end_min = m[3];
                if (low && ss->low_grid) {
                    grid = ss->low_grid;
                    if (!tune_has("cap")) wp.path_cap = PT_CMAX;   // (an explicit cap=N stays)
                }
            }
            HIP_TRY(pt_launch_path_round(wp, grid, 64u, ss->stream, sparse, i0, i1));
            wp.pin = nullptr;   // (only the round beside the early launch skips its chains)
            if (late) {
                // (it yields into the round's output counters, which the round's own launch
                // zeroed: a side launch that could yield before that zeroing would lose items)
                const bool big = coop_big(ss);
                HIP_TRY(pt_launch_coop(late_sp, late_grid, ss->side_team, big, ss->stream));
                HIP_TRY(hipEventRecord(ss->side_end, ss->stream));
                late = false;
            }
            if (wp.wg_prof) {
                uint32_t cnt[2][8];
                HIP_TRY(hipMemcpyAsync(cnt[0], ss->ctl + PT_CTL_SET * p, 32, hipMemcpyDeviceToHost, ss->stream));
                HIP_TRY(hipMemcpyAsync(cnt[1], ss->ctl + PT_CTL_SET * (1u - p), 32, hipMemcpyDeviceToHost, ss->stream));
                HIP_TRY(hipStreamSynchronize(ss->stream));
                fprintf(stderr, "round %u: in fresh %u carry %u -> out fresh %u carry %u exact %u\n", ss->rounds,
                        cnt[0][pt::C_FRESH], cnt[0][pt::C_CARRY], cnt[1][pt::C_FRESH], cnt[1][pt::C_CARRY],
                        cnt[1][pt::C_EXACT]);
                std::vector<unsigned long long> h(64ull * ss->path_grid);
                HIP_TRY(hipMemcpyAsync(h.data(), wp.wg_prof, h.size() * 8, hipMemcpyDeviceToHost, ss->stream));
                HIP_TRY(hipStreamSynchronize(ss->stream));
                if (FILE* f = fopen(wgp, "ab")) {
                    fwrite(h.data(), 8, h.size(), f);
                    fclose(f);
                }
            }
            ss->rounds++;
            p ^= 1u;
        }
        // (a side launch yields into this round's output: the count waits for it)
        if (side) HIP_TRY(hipStreamWaitEvent(ss->stream, ss->side_end, 0));
        HIP_TRY(hipMemcpyAsync(ss->ctl_host, ss->ctl + PT_CTL_SET * p, 8, hipMemcpyDeviceToHost, ss->stream));
        if (wp.progress) {
            // report the finished samples while the rounds run
            hipError_t e;
            while ((e = hipStreamQuery(ss->stream)) == hipErrorNotReady) {
                ss->on_progress(__atomic_load_n(ss->prog_host, __ATOMIC_RELAXED));
                std::this_thread::sleep_for(std::chrono::microseconds(500));
            }
            HIP_TRY(e);
        }
        HIP_TRY(hipStreamSynchronize(ss->stream));
        if (tune_int("roundlog", 0) >= 2) {
            // diagnostics: each round's chains, kind, wall time and rays (roundlog=3: also how
            // far behind the pass target the unfinished pixels are)
            const double now = wall_ms();
            unsigned long long cc[PT_CTR_COPIES * PT_CTR_STRIDE], rays = 0;
            HIP_TRY(hipMemcpy(cc, ss->counters, sizeof(cc), hipMemcpyDeviceToHost));
            for (uint32_t x = 0; x < PT_CTR_COPIES; ++x) rays += cc[PT_CTR_STRIDE * x];
            const double ms = now - ss->roundlog_t;
            fprintf(stderr, "round %u chains %u -> %u+%u (%s%s) %.2f ms rays %llu %.0f Mray/s", ss->rounds, chains,
                    ss->ctl_host[pt::C_FRESH], ss->ctl_host[pt::C_CARRY], chains < ss->lowq ? "low" : "full",
                    side ? "+side" : "", ms, rays - ss->roundlog_rays, (rays - ss->roundlog_rays) / ms / 1e3);
            ss->roundlog_rays = rays;
            if (tune_int("roundlog", 0) == 3) {
                std::vector<uint4> rec(2ull * ss->n_slots);
                HIP_TRY(hipMemcpy(rec.data(), ss->st.rec, rec.size() * sizeof(uint4), hipMemcpyDeviceToHost));
                std::vector<uint32_t> lag;
                for (uint32_t i = 0; i < ss->n_slots; ++i)
                    if (rec[2 * i].w < wp.target) lag.push_back(wp.target - rec[2 * i].w);
                std::sort(lag.begin(), lag.end());
                const size_t m = lag.size();
                fprintf(stderr, "; unfinished %zu lag p50 %u p90 %u p99 %u max %u", m, m ? lag[m / 2] : 0u,
                        m ? lag[m * 9 / 10] : 0u, m ? lag[m * 99 / 100] : 0u, m ? lag[m - 1] : 0u);
            }
            fprintf(stderr, "\n");
            ss->roundlog_t = wall_ms();
        }
        if (tune_int("dupcheck", 0)) {
            // diagnostics: every slot at most once in the next round's work (fresh rays + carry)
            const uint32_t nf = ss->ctl_host[pt::C_FRESH], nc = ss->ctl_host[pt::C_CARRY];
            std::vector<pt::F4> ro(nf);
            std::vector<uint32_t> cw((size_t)nc * ss->carry_words);
            if (nf) HIP_TRY(hipMemcpy(ro.data(), wp.fq[p].ro, nf * sizeof(pt::F4), hipMemcpyDeviceToHost));
            if (nc) HIP_TRY(hipMemcpy(cw.data(), wp.cq[p], cw.size() * 4, hipMemcpyDeviceToHost));
            std::vector<uint8_t> seen(ss->n_slots, 0);
            uint32_t dup = 0, bad = 0;
            auto see = [&](uint32_t slot) {
                if (slot >= ss->n_slots) { ++bad; return; }
                if (seen[slot]++) ++dup;
            };
            for (uint32_t i = 0; i < nf; ++i) see(pt::f2u(ro[i].w));
            for (uint32_t i = 0; i < nc; ++i) see(cw[(size_t)i * ss->carry_words + sizeof(pt::Query) / 4]);
            if (dup || bad)
                fprintf(stderr, "dupcheck: round %u (%s%s) fresh %u carry %u: %u duplicate slot(s), %u out of range\n",
                        ss->rounds, chains < ss->lowq ? "low" : "full", side ? "+side" : "", nf, nc, dup, bad);
        }
        if (ss->ctl_host[pt::C_CARRY] > ss->carry_cap) return fail(PT_E_HIP, "carry queue overflow (a lost chain)");
        if (ss->ctl_host[pt::C_FRESH] == 0u && ss->ctl_host[pt::C_CARRY] == 0u) break;
        if (guard > 100000u) return fail(PT_E_HIP, "wavefront rounds did not drain");
        chains = ss->ctl_host[pt::C_FRESH] + ss->ctl_host[pt::C_CARRY];
        counted = true;
        // near the cooperative hand-over every round is counted (the tail's rounds take ms)
        batch = chains > 4096u && chains > 4u * ss->coop_max ? ss->round_batch : (chains > 4096u ? 1u : 2u);
        sparse = chains < ss->path_sparse;
    }
    HIP_TRY(hipEventRecord(e1, ss->stream));
    ss->pending.emplace_back(e0, e1);
    ss->samples_done += spp;
    return PT_OK;
}

}  // namespace pti
