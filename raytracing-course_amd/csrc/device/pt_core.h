// pt_core.h -- exact-arithmetic building blocks of the hw5 hot path, written
// once for the gfx950 kernels (and compiled for the host only by the
// pt_selftest_* hooks that unit-test the traversal logic without a GPU).
//
// Every float op follows the reference's evaluation order so that, compiled
// with -ffp-contract=off (no FMA contraction; IEEE div/sqrt, denormals kept --
// hipcc's defaults on gfx950), results are bit-identical to the reference's
// x86-64 -O3 build.  Citations are into /root/reference/hw5.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PT_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define PT_HD inline
#endif

namespace pt {

// true if the predicate holds on any active lane of the wave (host: that thread)
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ bool pt_any(bool p) { return __ballot(p) != 0ull; }
#else
inline bool pt_any(bool p) { return p; }
#endif

// ------------------------------------------------------------ vectors -----
struct f3 { float x, y, z; };
struct alignas(16) F4 { float x, y, z, w; };

PT_HD f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
PT_HD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD f3 operator/(f3 a, f3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
PT_HD f3 operator*(float k, f3 a) { return mk3(k * a.x, k * a.y, k * a.z); }  // src/point.cpp:20-22
PT_HD f3 operator*(f3 a, float k) { return mk3(a.x * k, a.y * k, a.z * k); }  // glm vec*scalar
PT_HD f3 operator/(f3 a, float k) { return mk3(a.x / k, a.y / k, a.z / k); }
// glm/detail/func_geometric.inl:48-54: tmp = a*b; (tmp.x + tmp.y) + tmp.z
PT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// glm/detail/func_geometric.inl:68-78
PT_HD f3 cross(f3 a, f3 b) { return mk3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
PT_HD float fsqrt(float x) { return sqrtf(x); }
// glm normalize = v * inversesqrt(dot(v,v)), inversesqrt = 1 / sqrt
PT_HD f3 normalize(f3 v) { return v * (1.f / fsqrt(dot(v, v))); }
PT_HD float length(f3 v) { return fsqrt(dot(v, v)); }
// libstdc++ std::min / std::max (NaN-order semantics matter in the slab test)
PT_HD float smin(float a, float b) { return (b < a) ? b : a; }
PT_HD float smax(float a, float b) { return (a < b) ? b : a; }
PT_HD float fabs_(float a) { return fabsf(a); }

struct q4 { float x, y, z, w; };
// glm/ext/quaternion_common.inl:113-116
PT_HD q4 conj(q4 q) { q4 r; r.x = -q.x; r.y = -q.y; r.z = -q.z; r.w = q.w; return r; }
// glm/detail/type_quat.inl:359-366: v + ((uv*w) + uuv) * 2
PT_HD f3 qrot(q4 q, f3 v) {
    const f3 qv = mk3(q.x, q.y, q.z);
    const f3 uv = cross(qv, v);
    const f3 uuv = cross(qv, uv);
    return v + ((uv * q.w) + uuv) * 2.f;
}

#define PT_INF 1e18f          // include/bvh.h:9
#define PT_PI_F 3.14159274101257324f  // (float)acos(-1), include/distributions.h:14

PT_HD uint32_t f2u(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
PT_HD float u2f(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }

// ------------------------------------------------------------- libm -------
// glibc 2.35 logf (sysdeps/ieee754/flt-32/e_logf.c, table e_logf_data.c) --
// the function libstdc++'s std::log(float) calls in the reference's
// normal_distribution.  Restated so the device matches it exactly; pinned by
// an exhaustive comparison against the host libm over every float in (0, 1]
// (the only range the polar method feeds it).
struct LogfEntry { double invc, logc; };
// table in constant memory on the device (a dynamically indexed local array
// would be materialised in 32 VGPRs)
#if defined(__HIP_DEVICE_COMPILE__)
#define PT_TABLE __constant__
#else
#define PT_TABLE
#endif
PT_TABLE static const LogfEntry kLogfT[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
PT_HD float logf_glibc(float x) {
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = f2u(x);
    if (ix == 0x3f800000u) return 0.f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        // only (0,1] reaches here from the polar method: subnormal inputs
        ix = f2u(x * 0x1p23f);
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16u);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & (0x1ffu << 23));
    const double invc = kLogfT[i].invc, logc = kLogfT[i].logc;
    const double z = (double)u2f(iz);
    const double r = z * invc - 1.0;
    const double y0 = logc + (double)k * Ln2;
    const double r2 = r * r;
    double y = A1 * r + A2;
    y = A0 * r2 + y;
    y = y * r2 + (y0 + r);
    return (float)y;
}

// correctly rounded (double)x^5 for float-valued x (double-double products);
// stands in for glibc pow(x, 5.) at src/scene.cpp:151 -- the result is then
// rounded to float, where the two agree.
PT_HD double pow5_cr(double x) {
    const double x2 = x * x;                  // exact: 48 significant bits
    const double h4 = x2 * x2;
    const double l4 = fma(x2, x2, -h4);       // exact low part
    const double h5 = h4 * x;
    const double e5 = fma(h4, x, -h5);        // exact low part of h4*x
    return h5 + (e5 + l4 * x);
}

// ------------------------------------------------------------- RNG --------
// libstdc++ GCC 11: minstd_rand (random.tcc:116-124), generate_canonical<float,24>
// (random.tcc:3348-3378), normal_distribution<float> (random.tcc:1802-1835).
// One stream per pixel, seeded with the global pixel index (src/scene.cpp:216).
struct Rng {
    uint32_t x;
    float saved;
    uint32_t saved_ok;
};
PT_HD Rng rng_seed(uint32_t seed) {
    Rng r;
    const uint32_t s = seed % 2147483647u;
    r.x = (s == 0u) ? 1u : s;
    r.saved = 0.f;
    r.saved_ok = 0u;
    return r;
}
PT_HD uint32_t rng_next(Rng& r) {
    // 48271 * x mod (2^31 - 1) without a 64-bit modulo (Schrage-free Mersenne fold)
    const uint64_t p = (uint64_t)r.x * 48271u;
    uint32_t v = (uint32_t)(p & 0x7fffffffu) + (uint32_t)(p >> 31);
    v = (v & 0x7fffffffu) + (v >> 31);
    if (v == 0x7fffffffu) v = 0u;
    r.x = v;
    return v;
}
PT_HD float rng_uniform(Rng& r) {
    const float sum = (float)(rng_next(r) - 1u);
    float u = sum / 2147483648.0f;
    if (u >= 1.0f) u = 0x1.fffffep-1f;   // nextafter(1, 0)
    return u * 1.0f + 0.0f;
}
PT_HD float rng_normal(Rng& r) {
    if (r.saved_ok) { r.saved_ok = 0u; return r.saved * 1.0f + 0.0f; }
    float a, b, r2;
    do {
        a = (float)((double)(2.0f * rng_uniform(r)) - 1.0);
        b = (float)((double)(2.0f * rng_uniform(r)) - 1.0);
        r2 = a * a + b * b;
    } while (r2 > 1.0f || r2 == 0.0f);
    const float m = fsqrt(-2.0f * logf_glibc(r2) / r2);
    r.saved = a * m;
    r.saved_ok = 1u;
    return b * m * 1.0f + 0.0f;
}

// -------------------------------------------------------- scene layout ----
// Device records (built by host/bvh_build.cpp, uploaded once per device):
//  Node  (32 B, reference preorder; left child of an interior node = index+1)
//    a = {center.x, center.y, center.z, s.x}   center = 0.5f*(max+min), s = 0.5f*(max-min)
//    b = {s.y, s.z, u32 ref, u32 info}         interior: ref = right child, info = 0x80000000 | end
//                                                        (end = one past the subtree in preorder)
//                                              leaf:     ref = first prim, info = count (>= 1)
//  AuxNode (64 B): auxiliary BVH2 over the reference leaf boxes (host/aux_bvh.cpp)
//    a = {c0.lo.xyz, c0.hi.x}, b = {c0.hi.yz, c1.lo.xy}, c = {c1.lo.z, c1.hi.xyz},
//    d = {code0, code1, -, -}: code = aux node index, or 0x80000000 | reference leaf node, or ~0 (none)
//  Prim  (80 B): p0 = {pos.xyz, type}, p1 = {rot.xyzw}, p2 = {a.xyz, -}, p3 = {b.xyz, c.x}, p4 = {c.y, c.z, -, -}
//  Shade (32 B): s0 = {col.xyz, ior}, s1 = {emission.xyz, material}
enum : uint32_t { T_PLANE = 1, T_BOX = 2, T_ELLIPSOID = 4, T_TRIANGLE = 8 };  // include/primitives.h:13-18
enum : uint32_t { M_DIFFUSE = 0, M_METALLIC = 1, M_DIELECTRIC = 2 };         // include/materials.h:4-6

struct Node { F4 a, b; };
struct AuxNode { F4 a, b, c, d; };
#define PT_NODE_INTERIOR 0x80000000u
struct Prim { F4 p0, p1, p2, p3, p4; };
struct Shade { F4 s0, s1; };

struct SceneView {
    const Node* nodes;
    const AuxNode* aux;         // auxiliary BVH (may be null: exact stack DFS only)
    const Prim* prims;
    const Shade* shade;
    const uint32_t* planes;     // prim indices of planes (tested first, in order)
    const uint32_t* emitters;   // prim indices of BOX/ELLIPSOID emitters
    uint32_t n_planes, n_emitters;
    f3 bg;
    float box_extent;           // max |coordinate| over the reference node boxes (replay certification)
    const uint32_t* anc_info;   // per reference node: offset | length << 26 of its ancestor list (leaves)
    const uint32_t* anc;        // ancestor lists: root .. parent, the leaf, padding to 4 (ascending)
    // the query's single fetch space: every array above that the wavefront query
    // reads lives in one 16-B-aligned blob, addressed by 32-bit byte offsets
    const F4* blob;
    uint32_t o_nodes, o_aux, o_ainfo, o_anc, o_qprim, o_prim, o_bundle;
    uint32_t aux_rshift;        // wide aux entries: leaf range packed >> aux_rshift (pt_query.h)
    float inv_emitters;         // 1.f / (float)n_emitters (pdf_mix_e), divided once on the host: the
                                // kernels would hoist the uniform division into a VGPR for their lifetime
};

struct Ray { f3 o, d; };
struct Hit { float t; f3 n; uint32_t interior; };

// ---------------------------------------------------- primitive tests -----
// src/primitives.cpp:55-66
PT_HD bool isect_plane(const Ray& r, f3 n, Hit& h) {
    const float dn = dot(r.d, n);
    const float t = -dot(r.o, n) / dn;
    if (t > 1e5f) return false;     // (double)t > 1e5 <=> t > 1e5f: 1e5 is exact in float
    if (t > 0.f) {
        if (dn >= 0.f) { h.t = t; h.n = -1.f * n; h.interior = 1u; return true; }
        h.t = t; h.n = n; h.interior = 0u;
        return true;
    }
    return false;
}

// slab test of src/primitives.cpp:70-94 (t and interior only)
PT_HD bool slab(f3 o, f3 d, f3 s, float& t, uint32_t& interior) {
    const f3 t1xyz = (-1.f * s - o) / d;
    const f3 t2xyz = (s - o) / d;
    const float t1x = smin(t1xyz.x, t2xyz.x), t2x = smax(t1xyz.x, t2xyz.x);
    const float t1y = smin(t1xyz.y, t2xyz.y), t2y = smax(t1xyz.y, t2xyz.y);
    const float t1z = smin(t1xyz.z, t2xyz.z), t2z = smax(t1xyz.z, t2xyz.z);
    const float t1 = smax(smax(t1x, t1y), t1z);
    const float t2 = smin(smin(t2x, t2y), t2z);
    if (t1 > t2) return false;
    if (t2 < 0.f) return false;
    interior = (t1 < 0.f) ? 1u : 0u;
    t = interior ? t2 : t1;
    return true;
}

// src/primitives.cpp:70-117
PT_HD bool isect_box(const Ray& r, f3 s, Hit& h) {
    float t;
    uint32_t in;
    if (!slab(r.o, r.d, s, t, in)) return false;
    const f3 p = r.o + t * r.d;
    f3 n = p / s;
    if (in) n = -1.f * n;
    // std::max({fabs..}) = max_element (first largest); exact in float or double
    const float ax = fabs_(n.x), ay = fabs_(n.y), az = fabs_(n.z);
    float mx = ax;
    if (mx < ay) mx = ay;
    if (mx < az) mx = az;
    if (ax != mx) n.x = 0.f;
    if (ay != mx) n.y = 0.f;
    if (az != mx) n.z = 0.f;
    h.t = t; h.n = normalize(n); h.interior = in;
    return true;
}

// src/primitives.cpp:120-146: the ellipsoid's t and side (roots in f64: ::sqrt(double) at :130-131)
PT_HD bool ellipsoid_root(const Ray& r, f3 rad, float& t, uint32_t& in) {
    const float a = dot(r.d / rad, r.d / rad);
    const float b = 2.f * dot(r.o / rad, r.d / rad);
    const float c = dot(r.o / rad, r.o / rad) - 1.f;
    const float d = b * b - 4.f * a * c;
    if (d <= 0.f) return false;
    const double sd = sqrt((double)d);
    float x1 = (float)(((double)-b - sd) / (double)(2.f * a));
    float x2 = (float)(((double)-b + sd) / (double)(2.f * a));
    if (x1 > x2) { const float tt = x1; x1 = x2; x2 = tt; }
    if (x2 < 0.f) return false;
    in = (x1 < 0.f) ? 1u : 0u;
    t = in ? x2 : x1;
    return true;
}
// src/primitives.cpp:120-152
PT_HD bool isect_ellipsoid(const Ray& r, f3 rad, Hit& h) {
    float t;
    uint32_t in;
    if (!ellipsoid_root(r, rad, t, in)) return false;
    const f3 p = r.o + t * r.d;
    f3 n = normalize(p / (rad * rad));
    if (in) n = -1.f * n;
    h.t = t; h.n = n; h.interior = in;
    return true;
}

// src/primitives.cpp:155-174 -- plane through the LOCAL ORIGIN;
// n = normalize(cross(b - a, c - a)) given (the query's records store it, computed
// by the host with these same operations: bit-identical)
PT_HD bool isect_triangle_n(const Ray& r, f3 a, f3 b, f3 c, f3 n, Hit& h) {
    Hit ph;
    if (!isect_plane(r, n, ph)) return false;
    const f3 p = r.o + ph.t * r.d;
    if (!(dot(cross(b - a, p - a), n) > 0.f)) return false;
    if (!(dot(cross(p - a, c - a), n) > 0.f)) return false;
    if (!(dot(cross(c - b, p - b), n) > 0.f)) return false;
    h = ph;
    return true;
}
PT_HD bool isect_triangle(const Ray& r, f3 a, f3 b, f3 c, Hit& h) {
    return isect_triangle_n(r, a, b, c, normalize(cross(b - a, c - a)), h);
}

// src/primitives.cpp:14-52: world -> local by conj(q), test, normal back + renormalise
PT_HD bool prim_intersect(const Prim& P, const Ray& ray, Hit& h) {
    const f3 pos = mk3(P.p0.x, P.p0.y, P.p0.z);
    const uint32_t type = f2u(P.p0.w);
    q4 q; q.x = P.p1.x; q.y = P.p1.y; q.z = P.p1.z; q.w = P.p1.w;
    const q4 cq = conj(q);
    Ray lr;
    lr.o = qrot(cq, ray.o + -1.f * pos);
    lr.d = qrot(cq, ray.d);
    const f3 a = mk3(P.p2.x, P.p2.y, P.p2.z);
    bool ok;
    if (type == T_TRIANGLE) {
        ok = isect_triangle(lr, a, mk3(P.p3.x, P.p3.y, P.p3.z), mk3(P.p3.w, P.p4.x, P.p4.y), h);
    } else if (type == T_PLANE) {
        ok = isect_plane(lr, a, h);
    } else if (type == T_BOX) {
        ok = isect_box(lr, a, h);
    } else {
        ok = isect_ellipsoid(lr, a, h);
    }
    if (ok) h.n = normalize(qrot(q, h.n));
    return ok;
}

// prim_intersect for BVH primitives (std::partition keeps planes out of the
// BVH, src/scene.cpp:16-21): same operations without the plane branch
PT_HD bool bvh_prim_intersect(const Prim& P, const Ray& ray, Hit& h) {
    const f3 pos = mk3(P.p0.x, P.p0.y, P.p0.z);
    const uint32_t type = f2u(P.p0.w);
    q4 q; q.x = P.p1.x; q.y = P.p1.y; q.z = P.p1.z; q.w = P.p1.w;
    const q4 cq = conj(q);
    Ray lr;
    lr.o = qrot(cq, ray.o + -1.f * pos);
    lr.d = qrot(cq, ray.d);
    const f3 a = mk3(P.p2.x, P.p2.y, P.p2.z);
    bool ok;
    if (type == T_TRIANGLE) {
        ok = isect_triangle(lr, a, mk3(P.p3.x, P.p3.y, P.p3.z), mk3(P.p3.w, P.p4.x, P.p4.y), h);
    } else if (type == T_BOX) {
        ok = isect_box(lr, a, h);
    } else {
        ok = isect_ellipsoid(lr, a, h);
    }
    if (ok) h.n = normalize(qrot(q, h.n));
    return ok;
}

// plane-only form of prim_intersect (the scene's plane list): same operations
PT_HD bool plane_intersect(const Prim& P, const Ray& ray, Hit& h) {
    const f3 pos = mk3(P.p0.x, P.p0.y, P.p0.z);
    q4 q; q.x = P.p1.x; q.y = P.p1.y; q.z = P.p1.z; q.w = P.p1.w;
    const q4 cq = conj(q);
    Ray lr;
    lr.o = qrot(cq, ray.o + -1.f * pos);
    lr.d = qrot(cq, ray.d);
    if (!isect_plane(lr, mk3(P.p2.x, P.p2.y, P.p2.z), h)) return false;
    h.n = normalize(qrot(q, h.n));
    return true;
}

// ------------------------------------------------- light distributions -----
// src/distributions.cpp:102-110
PT_HD f3 normal01_vec(Rng& R) {
    const float f1 = rng_normal(R);
    const float f2 = rng_normal(R);
    const float f3_ = rng_normal(R);
    return normalize(mk3(f1, f2, f3_));
}
// src/distributions.cpp:144-159
PT_HD f3 sample_cosine(Rng& R, f3 n) {
    f3 dir = normal01_vec(R);
    dir = dir + n;
    if (dot(dir, n) <= 1e-8f) return n;
    if ((double)length(dir) <= 1e-4) return n;
    return normalize(dir);
}
// src/distributions.cpp:161-164
PT_HD float pdf_cosine(f3 n, f3 d) { return smax(0.f, 1.f / PT_PI_F * dot(d, n)); }

// src/distributions.cpp:170-198
PT_HD int points_for_pdf(const Prim& P, f3 x, f3 d, Hit& h1, Hit& h2) {
    Ray r; r.o = x; r.d = d;
    if (!prim_intersect(P, r, h1)) return 0;
    const float t = h1.t;
    if ((double)t <= 1e-8) return 0;   // reference also prints a stderr diagnostic here
    const float eps = 1e-4f;
    Ray r2; r2.o = x + (t + eps) * d; r2.d = d;
    if (!prim_intersect(P, r2, h2)) return 1;
    h2.t += t + eps;
    return 2;
}

// src/distributions.cpp:227-269
PT_HD f3 sample_box(Rng& R, const Prim& B, f3 x) {
    const f3 s = mk3(B.p2.x, B.p2.y, B.p2.z);
    const float wx = s.x * s.x, wy = s.y * s.y, wz = s.z * s.z;
    const f3 pos = mk3(B.p0.x, B.p0.y, B.p0.z);
    q4 q; q.x = B.p1.x; q.y = B.p1.y; q.z = B.p1.z; q.w = B.p1.w;
    for (;;) {
        float u = rng_uniform(R);
        const float side = (rng_uniform(R) <= 0.5f) ? 1.f : -1.f;
        u *= wx + wy + wz;
        float c1 = rng_uniform(R);
        float c2 = rng_uniform(R);
        float c3 = rng_uniform(R);
        c1 = 2.f * c1 - 1.f;
        c2 = 2.f * c2 - 1.f;
        c3 = 2.f * c3 - 1.f;
        f3 pnt = mk3(c1 * s.x, c2 * s.y, c3 * s.z);
        if (u < wx) pnt.x = side * s.x;
        else if (u < wx + wy) pnt.y = side * s.y;
        else pnt.z = side * s.z;
        const f3 on_box = qrot(q, pnt) + pos;
        const f3 smp = normalize(on_box - x);
        Hit h;
        Ray r; r.o = x; r.d = smp;
        if (prim_intersect(B, r, h)) return smp;
    }
}
// src/distributions.cpp:271-287 (1./(8W) and the final quotient are f64 ops
// rounded to float: identical to the f32 ops, double rounding is innocuous)
PT_HD float pdf_point_box(const Prim& B, float dist2, f3 n, f3 d) {
    const float wx = B.p2.x * B.p2.x, wy = B.p2.y * B.p2.y, wz = B.p2.z * B.p2.z;
    const float p_y = 1.f / (8.f * (wx + wy + wz));
    return (p_y * dist2) / fabs_(dot(d, n));
}
// src/distributions.cpp:289-312
PT_HD float pdf_box(const Prim& B, f3 x, f3 d) {
    Hit h1, h2;
    const int k = points_for_pdf(B, x, d, h1, h2);
    if (k == 0) return 1e-9f;
    const f3 cp = x + h1.t * d;
    float sum = pdf_point_box(B, dot(x - cp, x - cp), h1.n, d);
    if (k == 2) {
        const f3 op = x + h2.t * d;
        sum += pdf_point_box(B, dot(x - op, x - op), h2.n, d);
    }
    return sum;
}
// src/distributions.cpp:318-338
PT_HD f3 sample_ellipsoid(Rng& R, const Prim& E, f3 x) {
    const f3 rr = mk3(E.p2.x, E.p2.y, E.p2.z);
    const f3 pos = mk3(E.p0.x, E.p0.y, E.p0.z);
    q4 q; q.x = E.p1.x; q.y = E.p1.y; q.z = E.p1.z; q.w = E.p1.w;
    for (;;) {
        const f3 k = normal01_vec(R);
        const f3 on = qrot(q, rr * k) + pos;
        const f3 smp = normalize(on - x);
        Hit h;
        Ray r; r.o = x; r.d = smp;
        if (prim_intersect(E, r, h)) return smp;
    }
}
// src/distributions.cpp:340-347
PT_HD float pdf_point_ellipsoid(const Prim& E, float dist2, f3 y, f3 n_, f3 d) {
    const f3 rr = mk3(E.p2.x, E.p2.y, E.p2.z);
    const f3 pos = mk3(E.p0.x, E.p0.y, E.p0.z);
    q4 q; q.x = E.p1.x; q.y = E.p1.y; q.z = E.p1.z; q.w = E.p1.w;
    const f3 n = qrot(conj(q), y - pos) / rr;
    const float p_y = 1.f / (4.f * PT_PI_F * length(mk3(n.x * rr.y * rr.z, rr.x * n.y * rr.z, rr.x * rr.y * n.z)));
    return (p_y * dist2) / fabs_(dot(d, n_));
}
// src/distributions.cpp:349-372
PT_HD float pdf_ellipsoid(const Prim& E, f3 x, f3 d) {
    Hit h1, h2;
    const int k = points_for_pdf(E, x, d, h1, h2);
    if (k == 0) return 1e-9f;
    const f3 cp = x + h1.t * d;
    float sum = pdf_point_ellipsoid(E, dot(x - cp, x - cp), cp, h1.n, d);
    if (k == 2) {
        const f3 op = x + h2.t * d;
        sum += pdf_point_ellipsoid(E, dot(x - op, x - op), op, h2.n, d);
    }
    return sum;
}
// The emitter records the mixture reads: EmitGlobal = the scene's arrays; the
// cooperative engine passes a workgroup copy in LDS (same bits).
struct EmitGlobal {
    const SceneView& S;
    PT_HD Prim operator()(uint32_t k) const { return S.prims[S.emitters[k]]; }
};
// src/distributions.cpp:385-399
template <class EM>
PT_HD f3 sample_mix_e(const SceneView& S, const EM& em, Rng& R, f3 x, f3 n) {
    const float flip = rng_uniform(R);
    if (S.n_emitters == 0u || flip <= 0.5f) return sample_cosine(R, n);
    const float fid = rng_uniform(R);
    const uint32_t id = (uint32_t)floorf(fid * (float)S.n_emitters);
    const Prim E = em(id);
    return f2u(E.p0.w) == T_BOX ? sample_box(R, E, x) : sample_ellipsoid(R, E, x);
}
PT_HD f3 sample_mix(const SceneView& S, Rng& R, f3 x, f3 n) { return sample_mix_e(S, EmitGlobal{S}, R, x, n); }
// src/distributions.cpp:401-416
template <class EM>
PT_HD float pdf_mix_e(const SceneView& S, const EM& em, f3 x, f3 n, f3 d) {
    float sum = pdf_cosine(n, d);
    if (S.n_emitters != 0u) {
        float ps = 0.f;
        for (uint32_t k = 0; k < S.n_emitters; ++k) {
            const Prim E = em(k);
            ps += f2u(E.p0.w) == T_BOX ? pdf_box(E, x, d) : pdf_ellipsoid(E, x, d);
        }
        ps *= S.inv_emitters;   // = 1.f / (float)S.n_emitters (IEEE division on the host)
        sum = 0.5f * sum + 0.5f * ps;
    }
    return sum;
}
PT_HD float pdf_mix(const SceneView& S, f3 x, f3 n, f3 d) { return pdf_mix_e(S, EmitGlobal{S}, x, n, d); }

// src/scene.cpp:79-81
PT_HD f3 reflect(f3 n, f3 dir) { return dir - (2.0f * n) * dot(n, dir); }

// ------------------------------------------------------------ tonemap -----
// src/color.cpp:19-35 (ACES + saturate, f32); the gamma pow + round is done
// by the threshold table built on the host from the host's own powf
// (see host: build_gamma_thresholds) so the device matches glibc exactly.
PT_HD float saturate1(float v) { return smax(smin(1.f, v), 0.f); }
PT_HD float aces1(float x) {
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    return saturate1((x * (a * x + b)) / (x * (c * x + d) + e));
}
// thr[k] (k = 0..255) = smallest float v in [0,1] with round(255*powf(v, 1/2.2)) >= k+1
// (thr[255] = +inf); the 8-bit value is the number of thresholds <= v.
PT_HD uint32_t quantize_gamma(float v, const float* thr) {
    uint32_t lo = 0;
    // binary search over 256 entries (branch-free steps)
    for (uint32_t step = 128; step >= 1; step >>= 1)
        if (thr[lo + step - 1] <= v) lo += step;
    return lo;
}

}  // namespace pt
