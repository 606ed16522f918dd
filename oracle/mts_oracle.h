/*
 * mts_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of Mitsuba 0.6's `path` integrator hot path, used as the
 * parity checker for the HIP product (libmtsgpu.so) and as the timed CPU
 * baseline ("port") in bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product never does.
 *
 * Parity pinning: see oracle/mts_oracle.c header and DESIGN.md section 3.
 */
#ifndef MTS_ORACLE_H
#define MTS_ORACLE_H

#include "../include/mtsgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* libm mode: 0 = glibc float functions exactly as the reference calls them;
 * 1 = correctly-rounded-by-double evaluation (the product's device libm). */
int oracle_render(const mtsgpu_scene_desc *scene, const mtsgpu_render_params *params,
                  float *film, float *samples, mtsgpu_stats *stats,
                  int libm_mode, int threads);

/* Unit-level entry points (tests/) */
int oracle_sobol_init(const char *joe_kuo_path);
/* SFMT19937 (random.cpp): the first n outputs of Random(seed), or of its clone-th clone */
int oracle_sfmt_u64(uint64_t seed, uint64_t *out, int n, int clone);
/* the reference's render order over a width x height crop: blocks in
   BlockedImageProcess's spiral, pixels on each block's Hilbert curve;
   out: 2 ints per pixel, block_start: num_blocks + 1 entries */
int oracle_render_order(int width, int height, int blockSize, int *out, int *block_start, int *num_blocks);
float oracle_sobol_sample(uint64_t index, uint32_t dim, uint32_t scramble);
uint64_t oracle_sobol_lookup(uint32_t m, uint32_t frame, uint32_t px, uint32_t py, uint64_t scramble);
uint32_t oracle_sobol_matrix(uint32_t dim, uint32_t col);
/* TriAccel load + test (triaccel.h:58-160); out = {k,n_u,n_v,n_d,a_u,a_v,b_nu,b_nv,c_nu,c_nv} */
int oracle_triaccel_load(const float *A, const float *B, const float *C, float *out10);
int oracle_triaccel_intersect(const float *ta10, const float *o, const float *d,
                              float mint, float maxt, float *uvt);
/* Camera: returns sampleToCamera (16) and near-plane differentials dx,dy (3+3) */
/* environment emitter tables of `scene` (same layout as mtsgpu_debug_env_tables,
 * texels with 4 halves per texel) */
int oracle_env_tables(const mtsgpu_scene_desc *scene, float *params, uint16_t *texels, size_t texel_cap,
                      float *rows, float *cols, float *weights);
/* configure() only: the status the reference's plugin constructors/configure() raise */
int oracle_configure(const mtsgpu_scene_desc *scene);
int oracle_trace_rays(const mtsgpu_scene_desc *scene, const float *rays, uint32_t n, int shadow, float *hits);
float oracle_rdiel_trans_weight(int type, float alpha, float eta, const float *wi3, float sx, float sy, int walter);
void oracle_set_kdtree(const uint32_t *nodes, const uint32_t *indices);
int oracle_trace_rays_kd(const mtsgpu_scene_desc *scene, const uint32_t *nodes, const uint32_t *indices,
                         const float *rays, uint32_t n, int shadow, float *hits);
int oracle_intersect(const mtsgpu_scene_desc *scene, const float *o, const float *d, float *out16);
int oracle_camera(const mtsgpu_sensor_desc *s, float *sample_to_camera16, float *dxdy6);
/* Microfacet / BSDF probes for consistency tests: see mts_oracle.c */
int oracle_bsdf_sample(const mtsgpu_bsdf_desc *b, const float *wi3, const float *u3,
                       float *wo3, float *weight3, float *pdf, float *eta, int libm_mode);
/* fresnelDiffuseReflectance(eta, false) (util.cpp:814-860): plastic's m_fdrInt/m_fdrExt */
float oracle_fresnel_diffuse_reflectance(float eta);
int oracle_bsdf_eval(const mtsgpu_bsdf_desc *b, const float *wi3, const float *wo3,
                     float *value3, float *pdf, int libm_mode);

#ifdef __cplusplus
}
#endif
#endif
