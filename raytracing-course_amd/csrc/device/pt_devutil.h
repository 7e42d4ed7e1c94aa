// pt_devutil.h -- small device helpers shared by the gfx950 kernel files.
#pragma once
#include <hip/hip_runtime.h>

#include "pt_kernels.h"

namespace pt {

// per-lane word memory in LDS, [word][lane] (consecutive lanes -> consecutive banks)
template <uint32_t STRIDE>
struct LdsMemN {
    uint32_t* base;
    __device__ __forceinline__ void set(uint32_t i, uint32_t v) { base[i * STRIDE] = v; }
    __device__ __forceinline__ uint32_t get(uint32_t i) const { return base[i * STRIDE]; }
};
using LdsMem = LdsMemN<256u>;

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(0xffffffffu, __builtin_amdgcn_mbcnt_lo(0xffffffffu, 0u));
}
// number of set bits of m below this lane
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// wave-aggregated append: one atomic per wave; returns this lane's position (want lanes only)
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool want) {
    const unsigned long long m = __ballot(want);
    if (m == 0ull) return 0u;
    const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1u;
    uint32_t base = 0u;
    if (lane_id() == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader, 64);
    return base + lanes_below(m);
}

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

// The XCD (of 8) this wave runs on (HW_REG_XCC_ID).  Same-address atomics from
// the whole chip serialise at ~11.5 ns each on MI355X (tools/micro/atomics.hip);
// one copy of a hot counter per XCD, each on its own 128-B line, cuts that 8x.
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u; }

// this XCD's copy of the statistics counters (PT_CTR_COPIES x PT_CTR_STRIDE u64; the host sums them)
__device__ __forceinline__ unsigned long long* ctr_copy(unsigned long long* counters) {
    return counters + PT_CTR_STRIDE * xcc_id();
}

// block-aggregated append: ONE atomic per workgroup (every thread of the block
// must call it, NW = waves per block); returns this lane's position (want lanes only)
template <uint32_t NW>
__device__ __forceinline__ uint32_t block_append(uint32_t* counter, bool want, uint32_t* lds) {
    const unsigned long long m = __ballot(want);
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 0u) lds[w] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0u) {
        uint32_t tot = 0u;
#pragma unroll
        for (uint32_t k = 0; k < NW; ++k) {
            const uint32_t c = lds[k];
            lds[k] = tot;
            tot += c;
        }
        lds[NW] = tot ? atomicAdd(counter, tot) : 0u;
    }
    __syncthreads();
    const uint32_t r = lds[NW] + lds[w] + lanes_below(m);
    __syncthreads();   // lds is reused by the next call
    return r;
}

}  // namespace pt
