// pt_wprof.h -- per-workgroup timelines of the path engine (k_wpath), for
// diagnostics builds only (-DPT_WPROF; PT_TUNE wgprof=FILE; tools/wg_path.py).
// Each wave keeps its counters in a QProf (query waves) or SProf (shade wave);
// in product builds both are empty and every hook compiles to nothing, so the
// kernel's loop carries no instrumentation.  Record layout: 64 u64 per
// workgroup per round (indices as tools/wg_path.py reads them).
#pragma once
#include "pt_devutil.h"

namespace pt {

#ifdef PT_WPROF
struct QProf {
    uint64_t trips = 0, act = 0, sleep_ = 0, ring_ = 0, pulled_ = 0, exit_budget_ = 0, res = 0, dq = 0, rq = 0;
    uint64_t tripcyc = 0, refillcyc = 0, stepcyc = 0, auxtrips = 0, picktrips = 0, stepped = 0, donecyc = 0;
    uint64_t t0, s0 = 0, s1 = 0;
    uint64_t qlat = 0, qn = 0, qsteps = 0, qstart = 0;   // per lane
    uint32_t qs = 0;
    // per step kind (0 aux node, 1 probe, 2 leaf check, 3 walk entries, 4 walk nodes): times its
    // code was issued for the wave, and the lanes that used it
    uint64_t kiss[5] = {0, 0, 0, 0, 0}, klanes[5] = {0, 0, 0, 0, 0};
    __device__ QProf() : t0(__builtin_amdgcn_s_memtime()) {}
    // (LL = PathLds; read through volatile generic pointers, diagnostics only)
    template <class LL>
    __device__ void trip(uint32_t nidle, const LL& L, uint32_t wq) {
        auto rd = [](const uint32_t& v) { return *(const volatile uint32_t*)&v; };
        const uint64_t t = __builtin_amdgcn_s_memtime();
        tripcyc += t - t0;
        t0 = t;
        trips++;
        act += 64u - nidle;
        res += rd(L.resident);
        dq += rd(L.dq_tail[wq]) - rd(L.dq_head[wq]);
        rq += rd(L.rq_tail) - rd(L.rq_head);
    }
    __device__ void exit_budget() { exit_budget_ = 1; }
    __device__ void ring(uint32_t n) { ring_ += n; }
    __device__ void pulled(uint32_t n) { pulled_ += n; }
    __device__ void query_start() { qstart = __builtin_amdgcn_s_memtime(); qs = 0; }
    __device__ void sleep() { sleep_++; }
    __device__ void refill_end(bool active) {
        refillcyc += __builtin_amdgcn_s_memtime() - t0;
        if (active) qs++;
        s0 = __builtin_amdgcn_s_memtime();
    }
    __device__ void kinds(bool aux_lane, bool pick, bool stepped_lane) {
        if (__ballot(aux_lane) != 0ull) auxtrips++;
        if (pick) picktrips++;
        stepped += (uint64_t)__popcll(__ballot(stepped_lane));
    }
    // cat: this lane's step kind in the trip's step (> 4: none)
    __device__ void kind_mix(uint32_t cat) {
        for (uint32_t k = 0; k < 5u; ++k) {
            const unsigned long long m = __ballot(cat == k);
            if (m) {
                kiss[k]++;
                klanes[k] += (uint64_t)__popcll(m);
            }
        }
    }
    // an extra aux-node step of the same trip, for n lanes
    __device__ void extra_aux(uint32_t n) {
        kiss[0]++;
        klanes[0] += n;
    }
    __device__ void step_end() {
        s1 = __builtin_amdgcn_s_memtime();
        stepcyc += s1 - s0;
    }
    __device__ void query_done() {
        if (qstart) {
            qlat += __builtin_amdgcn_s_memtime() - qstart;
            qn++;
            qsteps += qs;
        }
    }
    __device__ void done_end() { donecyc += __builtin_amdgcn_s_memtime() - s1; }
    __device__ void store(unsigned long long* prof, uint64_t rays) const {
        if (!prof) return;
        unsigned long long* w = prof + 64ull * blockIdx.x;
        if (lane_id() == 0u) {
            atomicAdd(w + 2, trips);
            atomicAdd(w + 3, act);
            atomicAdd(w + 4, sleep_);
            atomicAdd(w + 5, ring_);
            atomicAdd(w + 6, (unsigned long long)rays);
            atomicAdd(w + 11, pulled_);
            atomicAdd(w + 12, exit_budget_);
            atomicAdd(w + 13, res);
            atomicAdd(w + 14, dq);
            atomicAdd(w + 15, rq);
            atomicAdd(w + 16, tripcyc);
            atomicAdd(w + 21, refillcyc);
            atomicAdd(w + 22, stepcyc);
            atomicAdd(w + 23, auxtrips);
            atomicAdd(w + 24, picktrips);
            atomicAdd(w + 25, stepped);
            atomicAdd(w + 26, donecyc);
            const uint32_t ki[5] = {37u, 38u, 39u, 44u, 45u};
            for (uint32_t k = 0; k < 5u; ++k) {
                atomicAdd(w + ki[k], kiss[k]);
                atomicAdd(w + 59u + k, klanes[k]);
            }
        }
        wave_add_u64(w + 17, qlat);
        wave_add_u64(w + 18, qn);
        wave_add_u64(w + 19, qsteps);
    }
};
struct SProf {
    uint64_t batches = 0, items = 0, spin_ = 0, cyc = 0, shc = 0, pushc = 0, c0 = 0, c1 = 0, c2 = 0;
    __device__ void begin() { c0 = c2 = __builtin_amdgcn_s_memtime(); }
    __device__ void spin() { spin_++; }
    __device__ void batch(uint32_t n) {
        c0 = __builtin_amdgcn_s_memtime();
        batches++;
        items += n;
    }
    __device__ void read_done() { c1 = __builtin_amdgcn_s_memtime(); }
    __device__ void shaded() {
        c2 = __builtin_amdgcn_s_memtime();
        shc += c2 - c1;
    }
    __device__ void end() {
        const uint64_t c3 = __builtin_amdgcn_s_memtime();
        pushc += c3 - c2;
        cyc += c3 - c0;
    }
    __device__ void store(unsigned long long* prof) const {
        if (!prof || lane_id() != 0u) return;
        unsigned long long* w = prof + 64ull * blockIdx.x;
        w[7] = batches;
        w[8] = items;
        w[9] = spin_;
        w[10] = cyc;
        w[27] = shc;
        w[28] = pushc;
        w[1] = __builtin_amdgcn_s_memrealtime();
    }
};
__device__ __forceinline__ void wprof_start(unsigned long long* prof) {
    if (prof && threadIdx.x == 0u) prof[64ull * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}
#else
struct QProf {
    template <class LL>
    __device__ void trip(uint32_t, const LL&, uint32_t) {}
    __device__ void exit_budget() {}
    __device__ void ring(uint32_t) {}
    __device__ void pulled(uint32_t) {}
    __device__ void query_start() {}
    __device__ void sleep() {}
    __device__ void refill_end(bool) {}
    __device__ void kinds(bool, bool, uint32_t) {}
    __device__ void kind_mix(uint32_t) {}
    __device__ void extra_aux(uint32_t) {}
    __device__ void step_end() {}
    __device__ void query_done() {}
    __device__ void done_end() {}
    __device__ void store(unsigned long long*, uint64_t) const {}
};
struct SProf {
    __device__ void begin() {}
    __device__ void spin() {}
    __device__ void batch(uint32_t) {}
    __device__ void read_done() {}
    __device__ void shaded() {}
    __device__ void end() {}
    __device__ void store(unsigned long long*) const {}
};
__device__ __forceinline__ void wprof_start(unsigned long long*) {}
#endif

}  // namespace pt
