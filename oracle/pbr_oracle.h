/*
 * pbr_oracle.h — TEST INFRASTRUCTURE ONLY (checker, never product).
 *
 * CPU restatement of the reference renderer's hot path (G0T-cha/PysicalBasedRaytracer,
 * read-only at /root/reference during development).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so; the product path (pysicalbasedraytracer_amd)
 * never links or calls it.
 *
 * Parity pinning: this restatement is checked against outputs of the reference
 * itself — oracle/_ref/libpbr_ref.so, compiled from the reference's unmodified sources by
 * oracle/ref/Makefile — recorded in tests/golden/ref_fixtures.json (renders, whole frames, BVH
 * node-array hashes, hit records, camera rays), plus the Halton / Li captures of SURVEY.md §4 and
 * analytic known-answer tests where the reference cannot speak (its sphere is a stub).
 *
 * Deliberate, documented deviations from the reference (all listed in DESIGN.md):
 *   F1  the Render loop iterates x∈[0,W), y∈[0,H) (the reference swaps its axes)
 *   F2  Sphere is a working pbrt-v3-style sphere (the reference's is a stub)
 *   F6/F11  no double-destroy, no racy counters
 *   F7  the float frame buffer is written
 *   transcendentals (sin/cos/atan2/asin/exp/log/pow/tan) are evaluated as
 *   (float)f((double)x), i.e. correctly rounded — the reference's bits here depend on the libm.
 */
#ifndef PBR_ORACLE_H
#define PBR_ORACLE_H
#include "../include/pbr_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Render the tiles of desc (same packing as pbr_hip_render). threads<=0: OpenMP default. */
int oracle_render(const pbr_scene_desc* scene, const pbr_render_desc* desc,
                  float* rgb_out, uint8_t* rgba_out, int threads, double* seconds);
/* Instrumented render: counts per sample (node visits, prim tests, rays, shading events). */
int oracle_render_stats(const pbr_scene_desc* scene, const pbr_render_desc* desc, int threads,
                        uint64_t* counters /* [4]: rays, node_visits, prim_tests, shading */);
/* Halton SampleDimension for (px, py, sample, dim) quadruples, image bounds (0,0)-(w,h). */
int oracle_halton(int width, int height, int spp, int n, const int32_t* px_py_s_dim, float* out);
/* pbrt-v3 SobolSampler: index (SobolIntervalToIndex) and SampleDimension for (px, py, sample, dim)
 * quadruples at raster (width, height); matrices in SobolMatrices32 layout, NULL → built-in. */
int oracle_sobol(int width, int height, int n, const int32_t* px_py_s_dim, const uint32_t* matrices, int dims,
                 float* out, int64_t* index_out);
/* The built-in Sobol' generator matrices (dims × 52 uint32). */
int oracle_sobol_matrices(int dims, uint32_t* out);
/* Radical inverse permutation table for the first n_primes primes (RNG default seed). */
int oracle_halton_perms(int n_primes, uint16_t* out, int* n_out);
/* Camera rays (o.xyz, d.xyz) for raster positions pfilm (x,y). */
int oracle_camera_rays(const pbr_camera_desc* cam, int n, const float* pfilm, float* out);
/* Flattened BVH: 32-B nodes + ordered primitive ids. NULL buffers → counts only. */
int oracle_build_bvh(const pbr_scene_desc* scene, void* nodes_out, int* n_nodes,
                     int32_t* prim_ids_out, int* n_prims);
/* Closest / any hit: rays = o.xyz d.xyz tmax (7 floats), out = {hit, t, prim, b1, b2}. */
int oracle_intersect(const pbr_scene_desc* scene, int n, const float* rays, float* out, int any_hit);
/* Li for one camera sample of one pixel (returns linear RGB), integrator from desc. */
int oracle_li_pixel(const pbr_scene_desc* scene, const pbr_render_desc* desc, int px, int py,
                    int sample, float* rgb);
/* Watertight triangle test on explicit data: tri = 9 floats, ray = 7 floats,
 * out = {hit, t, b0, b1, b2}. */
int oracle_triangle_test(const float* tri, const float* ray, float* out);
int oracle_sizeof_linear_bvh_node(void);

#ifdef __cplusplus
}
#endif
#endif
