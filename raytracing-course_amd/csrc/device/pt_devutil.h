// pt_devutil.h -- small device helpers shared by the gfx950 kernel files.
#pragma once
#include <hip/hip_runtime.h>

#include "pt_kernels.h"

namespace pt {

// per-lane word memory in LDS, [word][lane] (consecutive lanes -> consecutive banks)
template <uint32_t STRIDE>
struct LdsMemN {
    uint32_t* base;
    uint32_t cap = 0xffffffffu;   // words available (a query needing more takes the exact DFS)
    uint32_t trash = 0u;          // a word setc may write when its condition is false (0: none)
    __device__ __forceinline__ void set(uint32_t i, uint32_t v) { base[i * STRIDE] = v; }
    __device__ __forceinline__ uint32_t get(uint32_t i) const { return base[i * STRIDE]; }
    // set(i, v) if c; with a trash word the store is unconditional (no exec-mask branch)
    __device__ __forceinline__ void setc(uint32_t i, uint32_t v, bool c) {
        if (trash) base[(c ? i : trash) * STRIDE] = v;
        else if (c) base[i * STRIDE] = v;
    }
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

// a slot's fold records: one 16-B store per vertex, contiguous per slot
struct HbmVStore {
    uint4* base;      // fold + slot * depth
    __device__ __forceinline__ void put(uint32_t k, uint32_t idm, float s1, float s2) {
        base[k] = make_uint4(idm, f2u(s1), f2u(s2), 0u);
    }
    __device__ __forceinline__ void get(uint32_t k, uint32_t& idm, float& s1, float& s2) const {
        const uint4 v = base[k];
        idm = v.x;
        s1 = u2f(v.y);
        s2 = u2f(v.z);
    }
};
__device__ __forceinline__ HbmVStore fold_store(const PixelState& st, uint32_t slot) {
    return HbmVStore{st.fold + (size_t)slot * st.depth};
}

// the RNG / progress piece of a slot's record
struct PixelHot {
    Rng R;
    uint32_t nv;      // vertices of the current path (fold records written; 24 bits: RAY_DEPTH < 2^24)
    uint32_t done;    // samples completed in this session
};
// its 16-B form (rec[2 slot], and k_wpath's LDS pixel table)
__device__ __forceinline__ PixelHot hot_unpack(uint4 v) {
    PixelHot h;
    h.R.x = v.x;
    h.R.saved = u2f(v.y);
    h.R.saved_ok = v.z & 1u;
    h.nv = v.z >> 8;
    h.done = v.w;
    return h;
}
__device__ __forceinline__ uint4 hot_pack(const PixelHot& h) {
    return make_uint4(h.R.x, f2u(h.R.saved), (h.R.saved_ok & 1u) | (h.nv << 8), h.done);
}
__device__ __forceinline__ PixelHot load_hot(const PixelState& st, uint32_t slot) { return hot_unpack(st.rec[2u * slot]); }
__device__ __forceinline__ void store_hot(const PixelState& st, uint32_t slot, const PixelHot& h) {
    st.rec[2u * slot] = hot_pack(h);
}
__device__ __forceinline__ f3 load_sum(const PixelState& st, uint32_t slot) {
    const uint4 v = st.rec[2u * slot + 1u];
    return mk3(u2f(v.x), u2f(v.y), u2f(v.z));
}
// the sum and the slot's global pixel index (one 16-B load)
__device__ __forceinline__ f3 load_sum_pix(const PixelState& st, uint32_t slot, uint32_t& pix) {
    const uint4 v = st.rec[2u * slot + 1u];
    pix = v.w;
    return mk3(u2f(v.x), u2f(v.y), u2f(v.z));
}
__device__ __forceinline__ void store_sum(const PixelState& st, uint32_t slot, f3 s, uint32_t pix) {
    st.rec[2u * slot + 1u] = make_uint4(f2u(s.x), f2u(s.y), f2u(s.z), pix);
}

// owned slot -> global pixel (16x16 tiles of the window, dealt to ranks by tile_owner)
__device__ __forceinline__ bool slot_pixel(const TileMap& tm, uint32_t tile_local, uint32_t lane, uint32_t& x,
                                           uint32_t& y) {
    const uint32_t gt = tm.gtile[tile_local];
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
