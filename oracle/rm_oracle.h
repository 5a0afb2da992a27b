/*
 * rm_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path shaders/computeShader.glsl:68-344
 * (Qirias/OpenGL-RayMarching-in-Compute-Shader), used as the parity checker
 * for librm's HIP kernels and as the CPU baseline in bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (librm) never links, calls or falls back to it.
 *
 * Parity status: the GLSL itself cannot run here (no GL context, no GLSL
 * compiler) and the reference ships no tests, golden vectors or
 * fixtures.  The restatement is pinned by (1) analytic known-answer tests
 * derived from the shader text and (2) camera goldens produced from the
 * reference's vendored GLM 0.9.8.5 (oracle/gen_camera_goldens.cpp).  At the
 * GLSL built-in boundary (precision of normalize/pow/sin inside the vendor's
 * GL driver) parity is UNPINNED: the built-in semantics contract in DESIGN.md
 * defines "the reference" there.
 */
#ifndef RM_ORACLE_H
#define RM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/rm_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Render rows of a W x H frame exactly as computeShader.glsl:main (291-344)
 * would for pixel_coords = (px, py).
 *   rows      : list of global row indices py to render (NULL = all H rows)
 *   nrows     : number of entries in rows (ignored when rows == NULL)
 *   rgba32f   : [nrows][W][4] float, the texture's storage format (may be NULL)
 *   rgba8     : [nrows][W][4] uint8, round(clamp(c,0,1)*255) (may be NULL)
 *   sdf_counts: [nrows][W] per-pixel sdf() calls over all samples (may be NULL)
 *   counters  : frame totals of LIVE work (may be NULL) — what librm's kernels
 *               execute: the reference's work minus the provably dead tail of
 *               bounce() after a MATTE hit and the unused last-bounce-miss normal
 *   full_counters: frame totals of ALL work the GLSL executes (may be NULL)
 *   nthreads  : OpenMP threads (<= 0: library default)
 * Output row i corresponds to rows[i].  Returns 0, or -1 on bad arguments. */
int rmo_render(const rm_uniforms *u, int32_t W, int32_t H, const int32_t *rows, int32_t nrows,
               float *rgba32f, uint8_t *rgba8, uint32_t *sdf_counts, rm_counters *counters,
               rm_counters *full_counters, int32_t nthreads);

/* rmo_render with the runtime scene table prims[0..nprims) in place of the
 * GLSL's own sdf(): the same primitives and opU rule,
 * in table order.  Returns -1 on bad arguments. */
int rmo_render_scene(const rm_uniforms *u, const rm_primitive *prims, int32_t nprims, int32_t W,
                     int32_t H, const int32_t *rows, int32_t nrows, float *rgba32f,
                     uint8_t *rgba8, uint32_t *sdf_counts, rm_counters *counters,
                     rm_counters *full_counters, int32_t nthreads);

/* Single-function entry points for known-answer tests (all follow the GLSL
 * line-for-line; see rm_oracle.c for the per-function citations). */
typedef struct rmo_hit {
  float hitpoint;
  float color[3];
  int32_t id;
  float material;
} rmo_hit;

void rmo_sdf(const rm_uniforms *u, const float pos[3], rmo_hit *out);
void rmo_raymarch(const rm_uniforms *u, const float ro[3], const float rd[3], int32_t reflected,
                  rmo_hit *out, uint32_t *steps);
void rmo_get_normal(const rm_uniforms *u, const float pos[3], float out[3]);
float rmo_softshadow(const rm_uniforms *u, const float ro[3], const float rd[3], float k,
                     uint32_t *steps);
void rmo_point_light(const rm_uniforms *u, const float color[3], const float normal[3],
                     const float pos[3], float out[3]);
void rmo_cast_ray(const rm_uniforms *u, float uvx, float uvy, float ro[3], float rd[3]);
void rmo_render_ray(const rm_uniforms *u, const float ro[3], const float rd[3], float out[3]);
void rmo_pixel(const rm_uniforms *u, int32_t W, int32_t H, int32_t px, int32_t py, float out[4]);
uint8_t rmo_quantize(float c);
int rmo_max_threads(void);

#ifdef __cplusplus
}
#endif

#endif
