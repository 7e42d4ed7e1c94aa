// pt_wave.hip -- the wavefront pass's small kernels: the pass's seeding (k_wcamera,
// k_wcamera_merge), the cooperative engine's intake order (k_coop_hist /
// k_coop_scatter) and the early launch's queue (k_side_take), the exact-DFS
// hand-over (k_wexact) and its shading (k_wshade).  The path engine is pt_path.hip,
// the cooperative engine pt_wcoop.hip; pt_wave.h has the pass's outline.
#include "pt_wave.h"

namespace pt {

__global__ void __launch_bounds__(256) k_wcamera(WaveParams P) {
    // blocks append in about block order: the queue follows tile_order (Z-order of
    // the tiles, so the pixels resident together form compact image regions)
    const uint32_t t = P.tile_order ? P.tile_order[blockIdx.x] : blockIdx.x;
    const uint32_t slot = t * 256u + threadIdx.x;
    uint32_t x, y;
    const bool ok = slot_pixel(P.tm, t, threadIdx.x, x, y);
    bool want = false;
    Ray ray;
    if (ok) {
        PixelHot hot = load_hot(P.st, slot);
        Rng R = hot.R;
        uint32_t done = hot.done;
        if (P.depth == 0u) {
            // RayTrace(.., 0) = 0: only the jitter draws and sum += 0 per sample
            f3 sum = load_sum(P.st, slot);
            for (; done < P.target; ++done) {
                (void)camera_sample(P.cam, R, x, y);
                sum = sum + mk3(0.f, 0.f, 0.f);
            }
            store_sum(P.st, slot, sum, y * P.tm.W + x);
        } else if (done < P.target) {
            ray = camera_sample(P.cam, R, x, y);
            want = true;
        }
        hot.R = R;
        hot.done = done;
        hot.nv = 0u;
        store_hot(P.st, slot, hot);
    }
    // Pull order of the pass: pixels whose camera ray enters the BVH's boxes first
    // (the costly ones -- a pass ends with its slowest pixel, and pixels are pulled
    // as capacity frees up), the others after them (k_wcamera_merge).
    bool front = false;
    if (want) {
        // the (conservative) boxes of the aux BVH's top two levels: tighter than the
        // reference root box (root entries +2.6 % over it, two levels +2.5 % more)
        const f3 rinv = mk3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
        const f3 oinv = mk3(ray.o.x * rinv.x, ray.o.y * rinv.y, ray.o.z * rinv.z);
        for (uint32_t k = 0; k < PT_AUXW && k < P.n_top; ++k) {
            const AuxSL e = P.top[k];
            const uint32_t code = f2u(e.b.w);
            if (code == 0xffffffffu || !aux_box(e.a.x, e.a.y, e.a.z, e.a.w, e.b.x, e.b.y, rinv, oinv)) continue;
            if (code & 0x80000000u) {
                front = true;
                continue;
            }
            for (uint32_t j = 0; j < PT_AUXW; ++j) {   // one level down
                const AuxSL c = P.top[code * PT_AUXW + j];   // (code = 1 + k in the host's top copy)
                front = front || (f2u(c.b.w) != 0xffffffffu && aux_box(c.a.x, c.a.y, c.a.z, c.a.w, c.b.x, c.b.y, rinv, oinv));
            }
        }
    }
    __shared__ uint32_t agg[5];
    uint32_t* ctl = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t qf = block_append<4u>(ctl + C_FRONT, want && front, agg);
    const uint32_t qb = block_append<4u>(ctl + C_BACK, want && !front, agg);
    if (want) push_ray(P, front ? P.fq[P.parity] : P.fq[1u - P.parity], front ? qf : qb, ray, slot);
}

// the back class after the front one: fq[1-p][0, n_back) -> fq[p][n_front + i]
__global__ void __launch_bounds__(256) k_wcamera_merge(WaveParams P) {
    uint32_t* ctl = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t nf = ctl[C_FRONT], nb = ctl[C_BACK];
    const RayQ A = P.fq[P.parity], B = P.fq[1u - P.parity];
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nb; i += gridDim.x * 256u) {
        A.ro[nf + i] = B.ro[i];
        A.rd[nf + i] = B.rd[i];
        A.pid[nf + i] = B.pid[i];
        A.ri[nf + i] = B.ri[i];
    }
    if (blockIdx.x == 0u && threadIdx.x == 0u) ctl[C_FRESH] = nf + nb;
}

// The cooperative engine's intake order.  Its launch runs until the pixel with the
// most work left reaches the pass target, and a chain keeps its team to the end, so
// with more chains than teams (a hand-over at 49 k chains, 24.6 k resident teams
// of 8) the chains that wait for a team must be the ones with the least left.  A
// counting sort of the round's work items (suspended queries, then fresh rays) by
// their pixels' remaining samples, in PT_ORDER_BUCKETS buckets, most first.
__device__ __forceinline__ uint32_t coop_order_bucket(const WaveParams& P, uint32_t gi, uint32_t n_carry) {
    const uint32_t slot = gi < n_carry ? P.cq[P.parity][(size_t)gi * P.carry_words + sizeof(Query) / 4u]
                                       : f2u(P.fq[P.parity].ro[gi - n_carry].w);
    const uint32_t done = P.st.rec[2u * slot].w;
    const uint32_t rem = done < P.target ? P.target - done : 0u;
    const uint64_t b = (uint64_t)rem * PT_ORDER_BUCKETS / ((uint64_t)P.target + 1u);
    return PT_ORDER_BUCKETS - 1u - (uint32_t)b;   // bucket 0 = the most samples left
}
__global__ void __launch_bounds__(256) k_coop_hist(WaveParams P) {
    __shared__ uint32_t h[PT_ORDER_BUCKETS];
    const uint32_t* in = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t n_carry = in[C_CARRY], n = in[C_FRESH] + n_carry;
    h[threadIdx.x] = 0u;
    __syncthreads();
    for (uint32_t gi = blockIdx.x * 256u + threadIdx.x; gi < n; gi += gridDim.x * 256u)
        atomicAdd(&h[coop_order_bucket(P, gi, n_carry)], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(P.order_cur + PT_ORDER_BUCKETS + threadIdx.x, h[threadIdx.x]);
}
__global__ void __launch_bounds__(256) k_coop_scatter(WaveParams P) {
    __shared__ uint32_t base[PT_ORDER_BUCKETS];
    const uint32_t* in = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t n_carry = in[C_CARRY], n = in[C_FRESH] + n_carry;
    if (threadIdx.x == 0u) {
        // (every block scans the 256 counts itself)
        uint32_t t = 0u;
        for (uint32_t b = 0; b < PT_ORDER_BUCKETS; ++b) {
            base[b] = t;
            t += P.order_cur[PT_ORDER_BUCKETS + b];
        }
    }
    __syncthreads();
    for (uint32_t gi = blockIdx.x * 256u + threadIdx.x; gi < n; gi += gridDim.x * 256u) {
        const uint32_t b = coop_order_bucket(P, gi, n_carry);
        P.order[base[b] + atomicAdd(P.order_cur + b, 1u)] = gi;
    }
}

// The early cooperative launch's queue (pt_launch_side_take): item j < k of the
// intake order, a fresh ray copied as it is, a suspended query as a restart record
// (the cooperative engine restarts a query from its ray and slot alone).  side_ctl's
// C_CARRY / C_FRESH count the two kinds as they are appended (the launch's round
// counters: carry records first in its work numbering, as in every round).
__global__ void __launch_bounds__(256) k_side_take(WaveParams P, uint32_t k, RayQ side, uint32_t* side_carry,
                                                   uint32_t* side_ctl) {
    const uint32_t* in = P.ctl + PT_CTL_SET * P.parity;
    const uint32_t n_carry = in[C_CARRY];
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    const bool on = j < k;
    const uint32_t gi = on ? P.order[j] : 0u;
    // (hand-off site HO_SIDE_TAKE; PT_TUNE drop=side_take loses the items instead: the path
    // round skips them all the same)
    const bool keep = on && P.drop != 1u + HO_SIDE_TAKE;
    wave_add_u64(ctr_copy(P.counters) + CTR_HO + HO_SIDE_TAKE, on ? 1ull : 0ull);
    const bool carry = keep && gi < n_carry;
    const uint32_t kc = wave_append(side_ctl + C_CARRY, carry);
    const uint32_t kf = wave_append(side_ctl + C_FRESH, keep && !carry);
    if (carry) {
        const uint32_t* w = P.cq[P.parity] + (size_t)gi * P.carry_words;
        uint32_t* d = side_carry + (size_t)kc * P.carry_words;
        *reinterpret_cast<Ray*>(d) = reinterpret_cast<const Query*>(w)->ray;
        d[sizeof(Query) / 4u] = w[sizeof(Query) / 4u];
    } else if (keep) {
        const RayQ& F = P.fq[P.parity];
        const uint32_t fi = gi - n_carry;
        side.ro[kf] = F.ro[fi];
        side.rd[kf] = F.rd[fi];
        side.pid[kf] = F.pid[fi];
        side.ri[kf] = F.ri[fi];
    }
}

// The rays the path engine hands back (Q_EXACT: an aux stack deeper than the
// engine's LDS stack, a hitting-leaf list full of entered hits, non-finite
// components); 64-lane workgroups, one ray per lane, stack in LDS.  The replay
// first, with a stack as deep as the wide aux tree needs (a ray that only
// overflowed the engine's 16 words -- the common case -- costs its ~100 aux
// steps, not a whole reference DFS of ~10^4 node visits, tens of ms on one lane),
// then the exact stack DFS for what the replay cannot take (q_run).
__global__ void __launch_bounds__(64) k_wexact(WaveParams P) {
    extern __shared__ uint32_t lds_stack[];
    uint32_t* out = P.ctl + PT_CTL_SET * (1u - P.parity);
    const uint32_t n = out[C_EXACT];
    const uint32_t words = P.max_stack > P.aux_stack ? P.max_stack : P.aux_stack;
    LdsMemN<64u> stk{lds_stack + threadIdx.x, words, words};   // (+ a trash word)
    QCounts C{0u, 0u, 0u, 0u};
    uint32_t err = 0u;
    for (uint32_t k = blockIdx.x * 64u + threadIdx.x; k < n; k += gridDim.x * 64u) {
        const F4 o = P.ex.ro[k], d = P.ex.rd[k];
        Ray ray;
        ray.o = mk3(o.x, o.y, o.z);
        ray.d = mk3(d.x, d.y, d.z);
        Hit h;
        uint32_t used = 0u;
        const int id = q_run(P.S, ray, stk, h, C, used);
        // q_run flags a recomputed hit that differs from the query's in the plane count's
        // top bit (must never happen): an exactness error, not plane tests
        err += C.planes >> 31;
        C.planes = 0u;   // (the path engine counted this ray's plane tests when it took it)
        const uint32_t j = f2u(d.w);   // the ray's work index
        P.done.ro[j] = o;
        P.done.rd[j] = F4{d.x, d.y, d.z, 0.f};
        P.done.id[j] = id < 0 ? 0xffffffffu : (uint32_t)id;
    }
    unsigned long long* ctr = ctr_copy(P.counters);
    wave_add_u64(ctr + 1, C.nodes);
    wave_add_u64(ctr + 2, C.ptests);
    wave_add_u64(ctr + 4, err);
}

__global__ void __launch_bounds__(256) k_wshade(WaveParams P) {
    __shared__ uint32_t agg[5];
    uint32_t* out = P.ctl + PT_CTL_SET * (1u - P.parity);
    // the exact-DFS results of this round (the path engine shades everything else itself)
    const uint32_t n = out[C_EXACT];
    const RayQ N = P.fq[1u - P.parity];
    const uint32_t stride = gridDim.x * 256u;
    // grid-stride with a block-uniform trip count (the block-aggregated append needs every thread)
    for (uint32_t base = blockIdx.x * 256u; base < n; base += stride) {
        const uint32_t i = base + threadIdx.x;
        bool emit = false, sdone = false;
        Ray ray;
        uint32_t slot = 0u;
        const uint32_t hid = i < n ? P.done.id[i] : PT_SUSPENDED;
        if (hid != PT_SUSPENDED) {
            const F4 o = P.done.ro[i], d = P.done.rd[i];
            slot = f2u(o.w);
            ray.o = mk3(o.x, o.y, o.z);
            ray.d = mk3(d.x, d.y, d.z);
            emit = shade_item(P, EmitGlobal{P.S}, slot, ray, hid, sdone);
        }
        if (P.progress) {
            const uint32_t nd = (uint32_t)__popcll(__ballot(sdone));
            if (nd && (threadIdx.x & 63u) == 0u)
                __hip_atomic_fetch_add(P.progress, (unsigned long long)nd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const uint32_t qn = block_append<4u>(out + C_FRESH, emit, agg);
        if (emit) push_ray(P, N, qn, ray, slot);
    }
}

}  // namespace pt

extern "C++" {
// load the wavefront code objects onto the current device (no launch): this unit's,
// the path engine's and the cooperative engine's
hipError_t pt_preload_kernels_wave() {
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(pt::k_wcamera));
    if (e == hipSuccess) e = pt_preload_kernels_path();
    if (e == hipSuccess) e = pt_preload_kernels_coop();
    return e;
}

hipError_t pt_launch_wave_start(pt::WaveParams p, hipStream_t s) {
    hipError_t e = hipMemsetAsync(p.ctl, 0, 4u * 2u * PT_CTL_SET, s);
    if (e != hipSuccess) return e;
    p.parity = 0u;
    hipLaunchKernelGGL(pt::k_wcamera, dim3(p.n_tiles_local), dim3(256), 0, s, p);
    hipLaunchKernelGGL(pt::k_wcamera_merge, dim3(p.n_tiles_local < 1024u ? p.n_tiles_local : 1024u), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t pt_launch_coop_order(pt::WaveParams p, uint32_t n, hipStream_t s) {
    hipError_t e = hipMemsetAsync(p.order_cur, 0, 2u * PT_ORDER_BUCKETS * 4u, s);
    if (e != hipSuccess) return e;
    const uint32_t grid = n / 256u + 1u < 1024u ? n / 256u + 1u : 1024u;
    hipLaunchKernelGGL(pt::k_coop_hist, dim3(grid), dim3(256), 0, s, p);
    hipLaunchKernelGGL(pt::k_coop_scatter, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t pt_launch_side_take(pt::WaveParams p, uint32_t k, pt::RayQ side, uint32_t* side_carry, uint32_t* side_ctl,
                               hipStream_t s) {
    if (k == 0u) return hipSuccess;
    hipLaunchKernelGGL(pt::k_side_take, dim3((k + 255u) / 256u), dim3(256), 0, s, p, k, side, side_carry, side_ctl);
    return hipGetLastError();
}

// the round's exact-DFS hand-over and its shading, after the path engine's launch
hipError_t pt_launch_exact_shade(const pt::WaveParams& p, uint32_t shade_grid, hipStream_t s) {
    const uint32_t xw = p.max_stack > p.aux_stack ? p.max_stack : p.aux_stack;
    const uint32_t exact_lds = 64u * 4u * ((xw ? xw : 1u) + 1u);
    hipLaunchKernelGGL(pt::k_wexact, dim3(64), dim3(64), exact_lds, s, p);
    hipLaunchKernelGGL(pt::k_wshade, dim3(shade_grid), dim3(256), 0, s, p);
    return hipGetLastError();
}

}
