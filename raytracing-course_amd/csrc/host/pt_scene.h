// pt_scene.h -- host-side scene model of libpt (internal).
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "../device/pt_query.h"

namespace pth {

// include/primitives.h:31-64 (hw5)
struct HPrim {
    uint32_t type = 0;  // 0 = never set (the reference leaves it uninitialised)
    uint32_t mat = pt::M_DIFFUSE;
    float col[3] = {0.f, 0.f, 0.f};
    float emis[3] = {0.f, 0.f, 0.f};
    float pos[3] = {0.f, 0.f, 0.f};
    float rot[4] = {0.f, 0.f, 0.f, 1.f};  // x y z w; default (w=1) = include/primitives.h:44
    float ior = 0.f;
    float a[3] = {0.f, 0.f, 0.f};  // dop_data   (plane n, box s, ellipsoid r, triangle a)
    float b[3] = {0.f, 0.f, 0.f};  // dop_data1  (triangle b)
    float c[3] = {0.f, 0.f, 0.f};  // dop_data2  (triangle c)
};

// include/bvh.h:28-34
struct HNode {
    float mn[3], mx[3];
    uint32_t left, right, first, count;
};

struct HScene {
    uint32_t W = 0, H = 0, depth = 0, samples = 0;
    float bg[3] = {0.f, 0.f, 0.f};
    float cam_pos[3] = {0, 0, 0}, cam_right[3] = {0, 0, 0}, cam_up[3] = {0, 0, 0}, cam_fwd[3] = {0, 0, 0};
    float fov_x = 0.f;
    std::vector<HPrim> prims;
    std::vector<std::string> warnings;
};

// Parse the hw5 grammar (scene_load.cpp).  Throws std::runtime_error on I/O failure only.
void parse_scene(const char* text, size_t len, HScene& S);

// Faithful reference BVH (bvh_build.cpp): reorders prims[0, n) like
// BVH_t::InitTree and appends nodes in preorder.
void build_reference_bvh(std::vector<HPrim>& prims, uint32_t n, std::vector<HNode>& nodes);

// Auxiliary BVH2 over the reference leaf boxes (aux_bvh.cpp)
// (regions: 6 floats per reference node, the leaf's hit region {lo, hi}, or lo > hi: none)
void build_aux_bvh(const std::vector<HNode>& nodes, const std::vector<float>& regions, std::vector<pt::AuxNode>& out,
                   uint32_t& max_depth);

// Stackless preorder form of the auxiliary BVH for the wavefront query (aux_bvh.cpp)
void build_aux_stackless(const std::vector<pt::AuxNode>& pairs, const std::vector<pt::Node>& dnodes,
                         std::vector<pt::AuxSL>& out, uint32_t& max_depth);

// W-ary form of the auxiliary BVH (aux_bvh.cpp)
// (regions: as for build_aux_bvh, or empty: the collapse weighs the own boxes alone)
void build_aux_wide(const std::vector<pt::AuxNode>& pairs, const std::vector<pt::Node>& dnodes, uint32_t W,
                    std::vector<pt::AuxSL>& out, uint32_t& max_depth, uint32_t& max_stack,
                    const std::vector<float>& regions = {});

// per-entry reference-leaf ranges of the wide aux BVH (aux_bvh.cpp)
void annotate_aux_ranges(std::vector<pt::AuxSL>& out, uint32_t W, uint32_t n_ref_nodes, uint32_t& shift);

// Gamma/quantise threshold table (tonemap.cpp)
void build_gamma_thresholds(float thr[256]);

}  // namespace pth
