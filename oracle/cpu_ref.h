/*
 * cpu_ref.h — CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of render::CPUPathTracer
 *   (/root/reference libs/render/src/engines/pathtracer/backends/cpu/CPUPathTracer.cpp:43-326,
 *    libs/render/include/render/Color.h:7-10)
 * used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
 * and the CPU baseline. The product (libspt_hip.so) never links, loads or calls it.
 *
 * Pinning: the reference cannot be built here (Embree 4.4.0, glm and <format> are absent and
 * building it against stand-ins is not allowed), so this restatement is pinned by the reference's
 * only known-answer case — the Embree demo rays of src/main.cpp:38-75 (analytic answers in
 * SURVEY.md §4) — and by the closed forms of sphere.md:145-188. The integrator logic (RNG, seeds,
 * sampling, Russian roulette, accumulation, resolve) follows the source line by line; beyond the
 * KATs its parity with the reference binary is UNPINNED.
 */
#ifndef SPT_CPU_REF_H
#define SPT_CPU_REF_H

#include <stdint.h>

#include "spt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ref_config {
    uint32_t width, height;
    uint32_t max_bounces; /* reference: 4 (CPUPathTracer.cpp:199) */
    uint32_t rr_depth;    /* reference: 2 (CPUPathTracer.cpp:264) */
    uint32_t flags;       /* SPT_FLAG_ABS_FLOAT selects fabs for CPUPathTracer.cpp:320 */
} ref_config;

typedef struct ref_scene ref_scene;

/* pieces of the integrator (unit-testable) */
uint32_t ref_rng_seed(uint32_t x, uint32_t y, uint32_t width, uint32_t frame1); /* :192-195 */
float ref_random_float(uint32_t* state);                                         /* :294-301 */
void ref_primary_dir(uint32_t x, uint32_t y, uint32_t width, uint32_t height, float out[3]); /* :53-73 */
void ref_sample_sky(const spt_env* env, const float dir[3], float out[3]);      /* :286-292 */
void ref_bounce_dir(const float n[3], uint32_t* state, uint32_t flags, float out[3]); /* :303-326 */

/* scene: the same per-primitive constants as libspt_hip (formulas restated in cpu_ref.c) */
ref_scene* ref_scene_create(const spt_prim* prims, uint32_t n_prims, const spt_material* mats, uint32_t n_mats,
                            const spt_env* env);
void ref_scene_destroy(ref_scene* s);
/* environment map (octahedral RGBA, as spt_set_env_map; NULL: the gradient sky) */
void ref_set_env_map(ref_scene* s, const float* rgba, uint32_t w, uint32_t h);
uint32_t ref_octa_texel(float dx, float dy, float dz, uint32_t w, uint32_t h);
/* closest hit with t >= tmin; returns 1 on hit (prim = input index, ng = unnormalized normal) */
int ref_intersect(const ref_scene* s, const float o[3], const float d[3], float tmin, float* t, uint32_t* prim,
                  float ng[3]);

/* next-event estimation (SPT_FLAG_NEE, superset): the light sample at a hit (three draws: emitter,
 * u, v; returns 1 with the shadow ray and the estimate T * (Le * g), 0 if the sampled point is behind
 * either surface), and the shadow ray's test (nothing with 0.001 <= t < tmax) */
int ref_light_sample(const ref_scene* s, const float x[3], const float n[3], const float T[3], uint32_t* rng,
                     float w[3], float* tmax, float add[3]);
int ref_visible(const ref_scene* s, const float o[3], const float w[3], float tmax);
uint32_t ref_emitter_count(const ref_scene* s);

/* trace_ray (:197-284): returns (L, 1) */
void ref_trace_ray(const ref_scene* s, const ref_config* cfg, const float o[3], const float d[3], uint32_t* rng,
                   float out[4]);

/* render() (:43-85) over frames [first_frame, first_frame + n_frames) for the pixel rectangle
 * [x0,x1) x [y0,y1) of the full image (row stride x1-x0 in accum, RGBA floats, added to).
 * `row_step`/`row_offset` select rows y = y0 + row_offset + k*row_step (row shards; 1/0 = all rows).
 * threads <= 0: OpenMP default. Pixels are independent, so the result is thread-count invariant. */
int ref_render(const ref_scene* s, const ref_config* cfg, uint32_t first_frame, uint32_t n_frames, uint32_t x0,
               uint32_t y0, uint32_t x1, uint32_t y1, uint32_t row_step, uint32_t row_offset, float* accum,
               int threads);

/* get_render_result (:87-117) + rgba_to_uint32 (Color.h:7-10) */
void ref_resolve_rgba8(const float* accum, uint64_t n_pixels, uint32_t frame_count, uint32_t* out);
/* the same with RenderSettings exposure applied to r, g, b after the division (the reference's
 * commented-out :101-104) */
void ref_resolve_rgba8_exposure(const float* accum, uint64_t n_pixels, uint32_t frame_count, float exposure,
                                uint32_t* out);

/* segments (rays) traced per bounce by the last ref_render on this thread set (for bench bytes) */
uint64_t ref_last_segments(void);
/* NEE light samples (shadow rays considered) drawn by the last ref_render */
uint64_t ref_last_light_samples(void);

#ifdef __cplusplus
}
#endif
#endif
