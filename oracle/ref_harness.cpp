// ref_harness.cpp -- fixture dumper linked against the UNMODIFIED reference
// hw5 sources (see oracle/build_ref.sh; the reference headers are included
// under a private->public define so that private members can be read; the
// reference TUs themselves are compiled untouched).  Test infrastructure only: it
// generates the golden vectors under tests/golden/ that pin oracle/pt_oracle.cpp
// and, through it, the HIP renderer.  Nothing here is shipped or timed.
//
// Modes (all outputs little-endian binary, written to the given path):
//   bvh    <scene> <nodes.bin> <prims.bin>
//          node array after Scene::InitScene (hw5/src/scene.cpp:7-21,
//          hw5/src/bvh.cpp:99-179): per node 6 f32 (min.xyz,max.xyz) +
//          4 u32 (left,right,first,count); primitive order: per primitive
//          u32 type + 9 f32 (dop_data, dop_data1, dop_data2 -- the latter two
//          zero unless TRIANGLE) + 3 f32 pos.
//   render <scene> <out.ppm> <radiance.f32> [x0 y0 w h [ystride]]
//          restates Scene::Render's per-pixel loop (hw5/src/scene.cpp:205-252)
//          around the reference's own Scene::Sample, additionally saving the
//          pre-tonemap fp32 mean radiance.  With a window, only those pixels
//          are rendered (seeds stay the global index y*W+x), the PPM is the
//          window crop; with ystride, the window's h rows are y0, y0+ystride, ...
//          Load+InitScene and render times go to stderr (bench.py cpu_baseline).
//   rng    <seed> <n> <out.bin>
//          libstdc++ minstd_rand + uniform_real<float> + normal<float> streams
//          exactly as hw5/src/scene.cpp:216-223 builds them: n uniforms, then
//          n normals from a fresh engine, then a mixed u/n pattern.
//   trav   <scene> <nrays> <seed> <out.bin>
//          random rays -> reference Scene::RayIntersection (scene.cpp:46-77)
//          and BVH_t::Intersect with INF bound (bvh.cpp:181-225).
// Standard and glm headers first, so that only the reference's own classes
// see the access override below.
#include <algorithm>
#include <cassert>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <istream>
#include <memory>
#include <optional>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <variant>
#include <vector>
#include <omp.h>
#define GLM_ENABLE_EXPERIMENTAL
#include <glm/vec3.hpp>
#include <glm/gtc/quaternion.hpp>
#include <glm/gtx/norm.hpp>
#define private public
#include "scene.h"
#undef private

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

static void put_u32(std::ofstream& o, uint32_t v) { o.write(reinterpret_cast<const char*>(&v), 4); }
static void put_f32(std::ofstream& o, float v) { o.write(reinterpret_cast<const char*>(&v), 4); }
static void put_i32(std::ofstream& o, int32_t v) { o.write(reinterpret_cast<const char*>(&v), 4); }

static void load(Scene& s, const char* path) {
    std::ifstream in(path);
    if (!in) { std::fprintf(stderr, "cannot open %s\n", path); std::exit(2); }
    s.Load(in);
    s.InitScene();
}

static int mode_bvh(int argc, char** argv) {
    if (argc < 5) return 2;
    Scene s;
    load(s, argv[2]);
    std::ofstream on(argv[3], std::ios::binary), op(argv[4], std::ios::binary);
    for (const NODE_t& n : s.scene_bvh.nodes) {
        put_f32(on, n.aabb.aabb_min.x); put_f32(on, n.aabb.aabb_min.y); put_f32(on, n.aabb.aabb_min.z);
        put_f32(on, n.aabb.aabb_max.x); put_f32(on, n.aabb.aabb_max.y); put_f32(on, n.aabb.aabb_max.z);
        put_u32(on, n.left_child); put_u32(on, n.right_child);
        put_u32(on, n.first_primitive_id); put_u32(on, n.primitive_count);
    }
    for (const Primitive& p : s.primitives) {
        put_u32(op, (uint32_t)p.primitive_type);
        const bool tri = p.primitive_type == PRIMITIVE_TYPE::TRIANGLE;
        put_f32(op, p.dop_data.x); put_f32(op, p.dop_data.y); put_f32(op, p.dop_data.z);
        put_f32(op, tri ? p.dop_data1.x : 0.f); put_f32(op, tri ? p.dop_data1.y : 0.f); put_f32(op, tri ? p.dop_data1.z : 0.f);
        put_f32(op, tri ? p.dop_data2.x : 0.f); put_f32(op, tri ? p.dop_data2.y : 0.f); put_f32(op, tri ? p.dop_data2.z : 0.f);
        put_f32(op, p.pos.x); put_f32(op, p.pos.y); put_f32(op, p.pos.z);
    }
    return 0;
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int mode_render(int argc, char** argv) {
    if (argc < 5) return 2;
    Scene s;
    const double t0 = now_s();
    load(s, argv[2]);
    const double t1 = now_s();
    // threads as the reference sets them (hw5/src/scene.cpp:212), unless REF_THREADS
    // names the host's usable CPU share (bench.py cpu_baseline)
    const char* rt = std::getenv("REF_THREADS");
    const int threads = rt && *rt ? std::atoi(rt) : (int)std::thread::hardware_concurrency();
    omp_set_num_threads(threads);
    const unsigned W = s.cam.width, H = s.cam.height;
    unsigned x0 = 0, y0 = 0, w = W, h = H, ystride = 1;
    if (argc >= 9) {
        x0 = (unsigned)std::atoi(argv[5]); y0 = (unsigned)std::atoi(argv[6]);
        w = (unsigned)std::atoi(argv[7]); h = (unsigned)std::atoi(argv[8]);
    }
    if (argc >= 10) ystride = (unsigned)std::max(1, std::atoi(argv[9]));   // rows y0, y0+ystride, ...
    std::vector<float> rad((size_t)w * h * 3);
    std::vector<unsigned char> rgb((size_t)w * h * 3);
    #pragma omp parallel for schedule(dynamic)
    for (long long k = 0; k < (long long)w * h; ++k) {
        const unsigned x = x0 + (unsigned)(k % w), y = y0 + (unsigned)(k / w) * ystride;
        const unsigned i = y * W + x;
        std::minstd_rand rnd(i);
        std::uniform_real_distribution<float> uniform01{0.f, 1.f};
        std::normal_distribution<float> normal01{0.f, 1.f};
        RANDOM_t random{rnd, uniform01, normal01};
        Color c = s.Sample(random, x, y);
        rad[k * 3 + 0] = c.r(); rad[k * 3 + 1] = c.g(); rad[k * 3 + 2] = c.b();
        Color t = GammaCorrected(AcesTonemap(c));
        unsigned char* u = t.toUInts();
        rgb[k * 3 + 0] = u[0]; rgb[k * 3 + 1] = u[1]; rgb[k * 3 + 2] = u[2];
        delete[] u;
    }
    const double t2 = now_s();
    std::fprintf(stderr, "ref_harness: load_init_s=%.6f render_s=%.6f threads=%d hardware_concurrency=%u\n", t1 - t0,
                 t2 - t1, threads, std::thread::hardware_concurrency());
    std::ofstream out(argv[3], std::ios::binary);
    out << "P6\n" << w << " " << h << "\n" << 255 << "\n";
    out.write(reinterpret_cast<const char*>(rgb.data()), (std::streamsize)rgb.size());
    std::ofstream orad(argv[4], std::ios::binary);
    orad.write(reinterpret_cast<const char*>(rad.data()), (std::streamsize)(rad.size() * 4));
    return 0;
}

static int mode_rng(int argc, char** argv) {
    if (argc < 5) return 2;
    const unsigned seed = (unsigned)std::strtoul(argv[2], nullptr, 10);
    const int n = std::atoi(argv[3]);
    std::ofstream o(argv[4], std::ios::binary);
    {
        std::minstd_rand rnd(seed);
        std::uniform_real_distribution<float> u{0.f, 1.f};
        for (int k = 0; k < n; ++k) put_f32(o, u(rnd));
    }
    {
        std::minstd_rand rnd(seed);
        std::normal_distribution<float> g{0.f, 1.f};
        for (int k = 0; k < n; ++k) put_f32(o, g(rnd));
    }
    {
        // mixed pattern: draw kind decided by a fixed bit pattern
        std::minstd_rand rnd(seed);
        std::uniform_real_distribution<float> u{0.f, 1.f};
        std::normal_distribution<float> g{0.f, 1.f};
        for (int k = 0; k < n; ++k) {
            const bool use_u = ((k * 2654435761u) >> 7) & 1u;
            put_f32(o, use_u ? u(rnd) : g(rnd));
        }
    }
    return 0;
}

static int mode_trav(int argc, char** argv) {
    if (argc < 6) return 2;
    Scene s;
    load(s, argv[2]);
    const int nrays = std::atoi(argv[3]);
    std::mt19937 gen((unsigned)std::strtoul(argv[4], nullptr, 10));
    std::uniform_real_distribution<float> U(0.f, 1.f);
    std::normal_distribution<float> N(0.f, 1.f);
    std::ofstream o(argv[5], std::ios::binary);
    // scene extent from the root box (planes excluded from the BVH)
    const AABB_t& root = s.scene_bvh.nodes[0].aabb;
    for (int k = 0; k < nrays; ++k) {
        Ray r;
        if (k & 1) {
            // from the camera through a random pixel (unnormalised, as GetToRay)
            r = s.cam.GetToRay(U(gen) * s.cam.width, U(gen) * s.cam.height);
        } else {
            // from a random point of the (slightly grown) root box, random direction
            glm::vec3 p;
            for (int a = 0; a < 3; ++a) {
                const float lo = root.aabb_min[a], hi = root.aabb_max[a];
                const float ext = hi - lo;
                p[a] = lo - 0.25f * ext + 1.5f * ext * U(gen);
            }
            glm::vec3 d{N(gen), N(gen), N(gen)};
            if (k % 7 == 2) d.x = 0.f;  // exercise zero direction components
            if (k % 11 == 4) d.y = -0.f;
            r = Ray(p, glm::normalize(d));
        }
        ray_intersection_t a = s.RayIntersection(r);
        ray_intersection_t b = s.scene_bvh.Intersect(s.primitives, r, INF);
        put_f32(o, r.o.x); put_f32(o, r.o.y); put_f32(o, r.o.z);
        put_f32(o, r.d.x); put_f32(o, r.d.y); put_f32(o, r.d.z);
        for (const ray_intersection_t* q : {&a, &b}) {
            put_i32(o, q->id);
            const bool h = q->id != -1;
            put_f32(o, h ? q->isec.t : 0.f);
            put_f32(o, h ? q->isec.normal.x : 0.f); put_f32(o, h ? q->isec.normal.y : 0.f);
            put_f32(o, h ? q->isec.normal.z : 0.f);
            put_u32(o, h ? (uint32_t)q->isec.interior : 0u);
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: ref_harness bvh|render|rng|trav ...\n"); return 2; }
    const std::string m = argv[1];
    int rc = 2;
    if (m == "bvh") rc = mode_bvh(argc, argv);
    else if (m == "render") rc = mode_render(argc, argv);
    else if (m == "rng") rc = mode_rng(argc, argv);
    else if (m == "trav") rc = mode_trav(argc, argv);
    if (rc == 2) std::fprintf(stderr, "bad arguments for mode %s\n", m.c_str());
    return rc;
}
