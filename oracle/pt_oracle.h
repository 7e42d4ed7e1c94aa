/* pt_oracle.h -- C API of the CPU restatement (TEST INFRASTRUCTURE ONLY).
 * See pt_oracle.cpp.  Loaded by tests/ (ctypes), __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg; never by the product library. */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef struct oracle_scene oracle_scene;
oracle_scene* oracle_load(const char* path);
void oracle_free(oracle_scene* o);
int oracle_info(const oracle_scene* o, uint32_t* out8);
int oracle_dump_bvh(const oracle_scene* o, void* nodes_out, void* prims_out);
int oracle_render(oracle_scene* o, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t spp,
                  int nthreads, uint8_t* rgb, float* rad, uint64_t* counters);
int oracle_ray_intersection(const oracle_scene* o, uint32_t n, const float* rays, int32_t* ids, float* hit);
int oracle_rng(uint32_t seed, uint32_t n, float* out);
void oracle_tonemap(uint32_t n, const float* rad, uint8_t* rgb);
void oracle_gamma_u8(uint32_t n, const float* v, uint8_t* out);
uint64_t oracle_check_gamma_table(const float* thr);
#ifdef __cplusplus
}
#endif
#endif
