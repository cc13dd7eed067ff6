/*
 * spt.h — C-ABI of libspt_hip.so, the MI355X (gfx950) path-tracing integrator.
 *
 * This is the drop-in boundary for the one hot path of imisumi/software-path-tracer:
 * the per-pixel integrator of render::CPUPathTracer
 *   (reference: libs/render/src/engines/pathtracer/backends/cpu/CPUPathTracer.cpp:43-326).
 * The C++ backend render::HIPPathTracer (software-path-tracer_amd/csrc/HIPPathTracer.cpp)
 * implements the reference's render::PathTracer interface (libs/render/include/render/PathTracer.h:13-51)
 * on top of these entry points; Python (ctypes) and any other FFI bind the same symbols.
 *
 * Conventions:
 *   - every int-returning call returns SPT_OK (0) on success and a negative spt_status otherwise;
 *     spt_last_error(ctx) gives the message. No call aborts: the C++ wrapper turns failures into
 *     the reference's fail-stop verify() (render_assert.h:15-25).
 *   - all arrays are plain POD owned by the caller; the ctx copies what it keeps.
 *   - a ctx is single-threaded (the reference calls its backend from App's main thread only,
 *     App.cpp:231-232) and bound to one HIP device. Multi-GPU = one ctx per process/GPU, each
 *     rendering an interleaved row shard (spt_config.shard_rank / shard_count); the shards are
 *     gathered to rank 0 over RCCL by spt_gather_image.
 *   - no torch / HIP types in signatures; a HIP stream is passed as an opaque void*.
 */
#ifndef SPT_H
#define SPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPT_ABI_VERSION 3  /* 3: SPT_FLAG_NEE, spt_stats.shadow_rays / emitters */

typedef enum spt_status {
    SPT_OK = 0,
    SPT_ERR_INVALID = -1,     /* bad argument / call order                                   */
    SPT_ERR_HIP = -2,         /* HIP runtime error (message in spt_last_error)              */
    SPT_ERR_NO_DEVICE = -3,   /* no gfx950 device / HIP runtime unusable                    */
    SPT_ERR_NO_SCENE = -4,    /* render before spt_set_scene (CPUPathTracer.cpp:46 verify)   */
    SPT_ERR_NOT_CONFIGURED = -5,
    SPT_ERR_CAPACITY = -6     /* caller buffer too small                                    */
} spt_status;

/* ---- scene input (replaces the Embree geometry of CPUPathTracer.cpp:328-404) ---------------- */

typedef enum spt_prim_type {
    SPT_PRIM_SPHERE = 0,   /* reference type: RTC_GEOMETRY_TYPE_SPHERE_POINT (CPUPathTracer.cpp:374) */
    SPT_PRIM_QUAD = 1,     /* superset: parallelogram Q + a*u + b*v, a,b in [0,1]                     */
    SPT_PRIM_TRIANGLE = 2  /* superset: (v0, v1, v2)                                                  */
} spt_prim_type;

/* 64-byte input record. Sphere: p0 = (cx, cy, cz, r) exactly the Embree FLOAT4 vertex
 * (CPUPathTracer.cpp:377-384). Quad: p0.xyz = Q, p1.xyz = u, p2.xyz = v.
 * Triangle: p0.xyz, p1.xyz, p2.xyz = v0, v1, v2. Unused lanes must be 0. */
typedef struct spt_prim {
    uint32_t type;       /* spt_prim_type                           */
    uint32_t material;   /* index into the material array           */
    uint32_t reserved[2];
    float p0[4];
    float p1[4];
    float p2[4];
} spt_prim;

/* Reference mode: every surface has albedo 0.7 (CPUPathTracer.cpp:260) and no emission. */
typedef struct spt_material {
    float albedo[3];
    float emission[3];
} spt_material;

/* Sky on miss: L += T * mix(horizon, zenith, 0.5*(d.y+1))  (CPUPathTracer.cpp:231-235, 286-292).
 * Reference values: horizon (1,1,1), zenith (0.5,0.7,1.0). */
typedef struct spt_env {
    uint32_t sky_enabled;
    float horizon[3];
    float zenith[3];
} spt_env;

/* ---- render configuration (RenderSettings, Types.h:43-95, as CPUPathTracer actually uses it) -- */

enum spt_flags {
    /* get_random_bounche's `abs(normal.z)` (CPUPathTracer.cpp:320) binds to ::abs(int) under
     * libstdc++ (the reference's Linux build); set this flag for the intended float fabs. */
    SPT_FLAG_ABS_FLOAT = 1u << 0,
    /* Schedule: trace each bounce as a separate closest-hit (k_extend) and shading (k_shade) launch
     * instead of the default fused bounce kernel. Same results; exposes the traversal kernel alone. */
    SPT_FLAG_SPLIT_KERNELS = 1u << 1,
    /* Schedule: keep the wavefront (queue) schedule instead of the persistent launches
     * (k_paths for calls of >= SPT_PERSISTENT_MIN_FRAMES frames, k_frame per frame below). */
    SPT_FLAG_WAVEFRONT = 1u << 2,
    /* Schedule (BVH scenes): the split wavefront with sorted ray queues — before every bounce >= 1
     * closest-hit launch the queued rays are binned by (direction octant, cell of the origin in an
     * 8x8x8 grid over the scene bounds) with a device counting sort and traced in bin order, so
     * neighbouring lanes and waves walk the same subtrees. Same results. Implies SPT_FLAG_WAVEFRONT
     * and SPT_FLAG_SPLIT_KERNELS. */
    SPT_FLAG_SORTED_RAYS = 1u << 3,
    /* Integrator (superset, SURVEY.md §8a.6, north_star "BRDF + light sampling"; the reference's bounce
     * loop, CPUPathTracer.cpp:229-281, has none): next-event estimation. At every hit that continues
     * (bounce_count < max_bounces, before Russian roulette) one point is sampled on the scene's emitters
     * — the quads, triangles and spheres whose material emits, in primitive order, chosen uniformly; a
     * point uniform over the chosen one's area — and a shadow ray from the offset hit point tests it; if
     * nothing lies in [0.001, 0.999 * distance) the Lambertian estimate T * Le * cos_s * cos_l * area *
     * n_emitters / (pi * distance^2) is added (a sphere's cos_l counts its side facing the hit point
     * only; quads and triangles emit from both sides). Emission reached by a BSDF ray then counts on
     * the camera segment only.
     * RNG draw order per hit: emitter, u, v (NEE), then Russian roulette, then the direction.
     * oracle/cpu_ref.c restates it (ref_light_sample); every schedule gives identical results. */
    SPT_FLAG_NEE = 1u << 4
};

/* Which schedule spt_render used (spt_stats.schedule); every schedule gives identical results. */
enum spt_schedule {
    SPT_SCHEDULE_SPLIT = 0,      /* per bounce: k_extend + k_shade launches (BVH scenes)          */
    SPT_SCHEDULE_FUSED = 1,      /* per bounce: one k_shade<fused> launch, then k_trace_tail      */
    SPT_SCHEDULE_PERSISTENT = 2, /* one k_paths launch per call (per 1024 frames)                 */
    SPT_SCHEDULE_FRAME = 3       /* one k_frame launch per frame (calls of < 4 frames)            */
};
#define SPT_PERSISTENT_MIN_FRAMES 4

typedef struct spt_config {
    uint32_t width;             /* image width  (RenderSettings::getWidth,  CPUPathTracer.cpp:140) */
    uint32_t height;            /* image height                                                     */
    uint32_t max_bounces;       /* reference: hard-coded 4 (CPUPathTracer.cpp:199)                  */
    uint32_t rr_depth;          /* RR when bounce_count > rr_depth; reference: 2 (:264)             */
    uint32_t flags;             /* spt_flags                                                         */
    uint32_t shard_rank;        /* this ctx renders rows y with y % shard_count == shard_rank        */
    uint32_t shard_count;       /* 1 = whole image                                                   */
    uint32_t frames_in_flight;  /* frames traced concurrently per wavefront pass; 0 = auto           */
} spt_config;

/* Counters since the last spt_stats_clear. Per-kernel times are only collected while profiling
 * events are enabled (spt_set_profiling, SPT_PROFILE_EVENTS); they are HIP-event times on the ctx
 * stream. segments / radiance_updates / lane_* of the persistent schedules (k_paths, k_frame; their
 * time and launches are persistent_ms / persistent_launches) are only counted with
 * SPT_PROFILE_COUNTERS (the wavefront schedules count them always: their queues need the lengths). */
#define SPT_MAX_BOUNCES 32
typedef struct spt_stats {
    uint64_t frames;                          /* frames accumulated                          */
    uint64_t paths;                           /* camera paths traced (= samples)             */
    uint64_t segments[SPT_MAX_BOUNCES];       /* rays traced at each bounce depth            */
    uint64_t segments_total;
    uint64_t passes;                          /* wavefront passes launched                   */
    /* profiling (0 when disabled) */
    uint64_t extend_launches;                 /* k_extend launches timed                     */
    double extend_ms;                         /* summed k_extend duration                    */
    uint64_t extend_segments;                 /* rays processed by the timed k_extend launches */
    uint64_t shade_launches;
    double shade_ms;
    double other_ms;                          /* generate + accumulate                       */
    double extend_ms_bounce[SPT_MAX_BOUNCES]; /* k_extend time per bounce depth              */
    double shade_ms_bounce[SPT_MAX_BOUNCES];  /* k_shade time per bounce depth               */
    uint64_t bvh_nodes;                       /* nodes in the uploaded BVH (0 = flat scene)  */
    uint64_t scene_bytes;                     /* device bytes of node + primitive arrays     */
    uint64_t radiance_updates[SPT_MAX_BOUNCES]; /* per bounce >= 1: misses/emitter hits that
                                                   read-modify-wrote a path's radiance          */
    double tail_ms;                           /* k_trace_tail time (profiling)                */
    uint64_t tail_launches;
    uint64_t tail_bounce;                     /* bounces >= this run in k_trace_tail          */
    uint64_t fused;                           /* 1: extend+shade fused per bounce (shade_ms)  */
    double persistent_ms;                     /* k_paths time (profiling)                     */
    uint64_t persistent_launches;
    uint64_t schedule;                        /* SPT_SCHEDULE_* the last spt_render used      */
    uint64_t lane_slots;                      /* k_paths: 64 x wave tracing steps              */
    uint64_t lane_busy;                       /* k_paths: lanes that traced a segment in them  */
    uint64_t bvh_node_visits;                 /* k_paths, BVH scenes: interior nodes visited   */
    uint64_t prim_tests;                      /* k_paths, BVH scenes: primitives tested        */
    uint64_t flat_fast_path;                  /* 1: the scene is in the range of the flat loop's
                                                 unscaled-division fast path (same results)     */
    uint64_t specialized;                     /* 1: the last k_paths / k_frame launch ran the kernel
                                                 compiled for the flat scene's shape (same results) */
    uint64_t shadow_rays;                     /* SPT_FLAG_NEE: shadow rays traced by k_paths / k_frame
                                                 (counted with SPT_PROFILE_COUNTERS)              */
    uint64_t emitters;                        /* emitters SPT_FLAG_NEE samples in the current scene */
    uint64_t stack_bytes;                     /* BVH scenes: device bytes of the persistent kernels'
                                                 traversal stacks (not in scene_bytes)            */
    uint64_t stack_need;                      /* BVH scenes: the most entries a traversal stack of the
                                                 tree holds; spt_set_scene refuses a tree needing
                                                 more than 96 (SPT_ERR_CAPACITY)                   */
    uint64_t stalled_waves;                   /* k_paths waves that stopped at their step loop's safety
                                                 bound (a logic error; spt_get_stats then fails with
                                                 SPT_ERR_HIP after filling *out)                   */
} spt_stats;

typedef struct spt_ctx spt_ctx;

/* ---- library / device ---------------------------------------------------------------------- */
int spt_abi_version(void);
/* Number of HIP devices visible (0 when the runtime has none). */
int spt_device_count(int* count);

/* ---- lifecycle (CPUPathTracer ctor/dtor, CPUPathTracer.cpp:25-41) -------------------------- */
int spt_create(spt_ctx** out, int device_id);
void spt_destroy(spt_ctx* ctx);
const char* spt_last_error(const spt_ctx* ctx);
/* Launch on a caller-owned hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the ctx's own stream. */
int spt_set_stream(spt_ctx* ctx, void* hip_stream);

/* ---- scene (rebuild_scene, CPUPathTracer.cpp:328-404) ------------------------------------- */
/* Copies the primitives, builds the acceleration structure on the host (flat list for small
 * scenes, SAH BVH otherwise), uploads it, and resets accumulation (frameCount = 0, :122-131). */
int spt_set_scene(spt_ctx* ctx, const spt_prim* prims, uint32_t n_prims,
                  const spt_material* mats, uint32_t n_mats, const spt_env* env);

/* Incremental edit (the reference re-runs rebuild_scene on any change,
 * CPUPathTracer.cpp:119-161, 328-404): replace primitives indices[0..n) of the current scene with
 * prims[0..n) (indices into the array spt_set_scene was given; materials index its material array).
 * A BVH scene keeps its tree: the changed records are uploaded in place, the bounds refitted bottom-up
 * and the node array re-uploaded — no rebuild; a flat scene re-uploads its few records. Results are
 * those of spt_set_scene with the edited array (the traversal is exact for any valid tree). Resets
 * the progressive accumulation like spt_set_scene. */
int spt_update_prims(spt_ctx* ctx, const uint32_t* indices, const spt_prim* prims, uint32_t n);

/* ---- settings / progressive state (invalidate, CPUPathTracer.cpp:119-161) ----------------- */
/* (Re)allocates device buffers when the size or shard changes, and always resets accumulation. */
int spt_configure(spt_ctx* ctx, const spt_config* cfg);
/* Zero the accumulation buffer and the frame counter (:151-154). */
int spt_reset(spt_ctx* ctx);
int spt_get_frame_count(const spt_ctx* ctx, uint32_t* frame_count);

/* ---- the hot path (render, CPUPathTracer.cpp:43-85) ---------------------------------------- */
/* Traces frames [first_frame, first_frame + n_frames): frame k is seeded with k + 1 exactly as
 * get_rng_state(.., m_frameCount + 1) (:61, :192-195), and adds each frame's radiance to the
 * accumulation buffer in frame order (:77-80). Asynchronous on the ctx stream, with one exception:
 * the first one-frame call after spt_set_scene / spt_update_prims / spt_configure stores the pixels'
 * camera hits and, for scenes that use the compacted live-pixel lists, waits for that frame to read
 * the live-pixel count back (once per change). The progressive renderer calls
 * spt_render(ctx, frame_count, 1) once per App frame. */
int spt_render(spt_ctx* ctx, uint32_t first_frame, uint32_t n_frames);
int spt_synchronize(spt_ctx* ctx);

/* ---- results (get_render_result, CPUPathTracer.cpp:87-117) ------------------------------- */
/* Number of pixels this ctx owns (width*height for shard_count 1). */
int spt_shard_pixels(const spt_ctx* ctx, uint64_t* n_pixels);
/* Copy the shard's float RGBA accumulation (n_pixels * 4 floats, row-major over the shard's rows). */
int spt_read_accum(spt_ctx* ctx, float* host_rgba);
/* Device pointer / byte size of the accumulation buffer (valid until the next spt_configure). */
int spt_accum_device_ptr(spt_ctx* ctx, void** dptr, size_t* bytes);
/* Stream-ordered device-to-device copy of the accumulation buffer (n_pixels * 16 bytes) to `dst`,
 * e.g. into a caller-owned tensor that a collective then gathers. */
int spt_copy_accum_device(spt_ctx* ctx, void* dst);
/* Resolve on the device: c = accum / frame_count, clamp [0,1], (uint8)(c*255) truncation,
 * r<<24 | g<<16 | b<<8 | a (Color.h:7-10), then copy n_pixels u32 to the host. */
int spt_resolve_rgba8(spt_ctx* ctx, uint32_t frame_count, uint32_t* host_out);
/* The same with RenderSettings::getExposure (Types.h:56,66) applied as the reference's commented-out
 * code would (CPUPathTracer.cpp:101-104): c = (accum / frame_count) * exposure on r, g, b (not a),
 * before the clamp. exposure = 1 is exactly spt_resolve_rgba8. */
int spt_resolve_rgba8_exposure(spt_ctx* ctx, uint32_t frame_count, float exposure, uint32_t* host_out);
/* Register the caller's host image buffer [host_out, host_out + bytes) for the two resolves above:
 * the buffer is page-locked and mapped into the GPU's address space, and a resolve into exactly
 * `host_out` (while bytes >= 4 * n_pixels) has the resolve kernel store the pixels straight into it
 * over PCIe — no device staging buffer, no DMA copy — then waits as before. Any other pointer takes
 * the staging-and-copy path. The caller keeps the memory allocated until it registers another
 * buffer, passes (NULL, 0) to unregister, or destroys the ctx (the backend's RenderResult buffer:
 * HIPPathTracer re-registers it whenever it resizes). One buffer per ctx. */
int spt_register_host_output(spt_ctx* ctx, void* host_out, size_t bytes);
/* spt_render(first_frame, n_frames) followed by spt_resolve_rgba8_exposure(frame_count, exposure,
 * host_out), with the resolve fused into the call's last frame when that frame runs the one-frame
 * kernel and host_out is the registered buffer: each pixel's RGBA8 is stored over PCIe as its path
 * ends, so the image's transfer overlaps the frame (the App's render() + get_render_result(),
 * App.cpp:230-240). frame_count is the divisor: the frames accumulated after this call. Same pixels
 * as the two calls; waits for the stream. */
int spt_render_resolve_rgba8(spt_ctx* ctx, uint32_t first_frame, uint32_t n_frames, uint32_t frame_count,
                             float exposure, uint32_t* host_out);
/* Multi-GPU assembly on the root: `gathered` (device) holds shard_count row-shards, each padded to
 * ceil(height/shard_count)*width RGBA pixels, in rank order (the layout of an all-gather /
 * gather into one tensor). Writes the full width*height RGBA image to `out` (device). */
int spt_assemble_rows(spt_ctx* ctx, const void* gathered, void* out);

/* ---- environment map (superset — the reference's SkyBox, Scene.h:268-278,
 * is loaded by dead code and never sampled) -------------------------------------------------- */
/* Miss radiance from an octahedral environment map instead of sample_sky's gradient (only while
 * the scene's env.sky_enabled is set): `rgba` holds width*height texels of 4 floats, texel
 * (ix, iy) at iy*width + ix; a direction d maps to the octahedron |x|+|y|+|z| = 1 (y up, lower
 * hemisphere folded over the diagonals) and takes the nearest texel (octa_texel in
 * csrc/spt_device.h). rgba = NULL restores the gradient sky. Resets the progressive accumulation. */
int spt_set_env_map(spt_ctx* ctx, const float* rgba, uint32_t width, uint32_t height);
/* Host utility: resample an equirectangular RGB image (src_width x src_height x 3 floats, row 0 at
 * +y, column 0 at phi = -pi with phi = atan2(x, -z)) into an octahedral RGBA map (dst_width x
 * dst_height x 4 floats, alpha 1), nearest source texel per destination texel centre. */
int spt_env_octa_from_equirect(const float* src_rgb, uint32_t src_width, uint32_t src_height, float* dst_rgba,
                               uint32_t dst_width, uint32_t dst_height);

/* ---- measurement --------------------------------------------------------------------------- */
enum spt_profile {
    SPT_PROFILE_EVENTS = 1,   /* HIP events around every launch (per-kernel times in spt_stats)     */
    SPT_PROFILE_COUNTERS = 2, /* k_paths counts segments per bounce (a slower kernel variant)       */
    SPT_PROFILE_SPAN = 4      /* k_paths / k_frame: ONE event pair around all their launches until
                               * profiling is switched off — from before the first launch to after
                               * the last — instead of one per launch (per-launch events cost a
                               * one-frame call ~15 %); persistent_ms is that span, persistent_launches
                               * the launches inside it. Other kernels are not timed in this mode. */
};
int spt_set_profiling(spt_ctx* ctx, int mode);  /* mode: OR of spt_profile, 0 = off */
int spt_get_stats(spt_ctx* ctx, spt_stats* out);   /* synchronizes the ctx stream */
int spt_stats_clear(spt_ctx* ctx);

/* ---- multi-GPU: row shards gathered over RCCL ------------------------------
 * One process and one ctx per GPU; ctx r is configured with shard_rank = r, shard_count = N. The
 * ranks share one RCCL communicator, created from an id that rank 0 makes and the host passes to
 * the others out of band (a TCP store, MPI, a file). RCCL is resolved at run time: the copy already
 * loaded in the process (e.g. PyTorch's) is used, else librccl.so.1 from the ROCm install. */
#define SPT_COMM_ID_BYTES 128
/* SPT_OK if this process can reach RCCL (the library and the symbols spt_comm_* bind resolve; no
 * communicator and no bootstrap socket are created), SPT_ERR_NO_DEVICE otherwise. Every rank can ask
 * before the collective spt_comm_init, so that all agree on the gather path first. */
int spt_comm_available(void);
/* Rank 0: a new communicator id (ncclGetUniqueId). */
int spt_comm_unique_id(uint8_t id[SPT_COMM_ID_BYTES]);
/* Join the communicator as `rank` of `n_ranks` (ncclCommInitRank; collective: every rank calls it,
 * each on its own ctx/GPU). rank / n_ranks must equal the ctx's shard_rank / shard_count. */
int spt_comm_init(spt_ctx* ctx, const uint8_t id[SPT_COMM_ID_BYTES], int n_ranks, int rank);
/* Collective: every rank's accumulation shard, padded to ceil(height / N) rows, is gathered to rank 0
 * (one ncclGather on the ctx stream, 16 B per padded shard pixel per rank), and rank 0 de-interleaves
 * the shards into the full width*height float RGBA image at `root_image` (device memory, rank 0;
 * ignored on the others). Asynchronous on the ctx stream, like spt_render. */
int spt_gather_image(spt_ctx* ctx, void* root_image);
/* The same collective overlapped with rendering (a progressive renderer showing every step's image on
 * rank 0 while the GPUs render on): the shard is snapshot on the ctx stream (a device copy, 16 B per
 * shard pixel), and the gather and rank 0's assembly run on a stream of the ctx's own, so the next
 * spt_render calls start at once. `root_image` holds the image of the frames rendered before this
 * call once spt_gather_wait has ordered the ctx stream after it (or the device is synchronized).
 * A later gather first waits for this one to have read the snapshot. */
int spt_gather_image_overlapped(spt_ctx* ctx, void* root_image);
/* Orders the ctx stream after the last overlapped gather (no host wait); a no-op without one. */
int spt_gather_wait(spt_ctx* ctx);
/* Leave the communicator (also done by spt_destroy). */
int spt_comm_destroy(spt_ctx* ctx);

/* ---- schedule tuning (measurement and tests; results never depend on it) ----------------------
 * Every field 0 (or -1 where noted) = the library's automatic choice, which is what production uses.
 * Replaces per-process environment overrides: a tuned ctx is explicit in the caller's code. */
typedef struct spt_tuning {
    int32_t fused;             /* flat wavefront schedule: -1 auto, 0 split extend/shade, 1 fused     */
    uint32_t tail_bounce;      /* wavefront: bounces >= this run in k_trace_tail (0 auto)            */
    int32_t persistent;        /* -1 auto, 0 never k_paths, 1 k_paths for every call                  */
    int32_t frame_kernel;      /* calls of < SPT_PERSISTENT_MIN_FRAMES: -1 auto, 0 wavefront, 1 k_frame */
    uint32_t chunks_per_wave;  /* k_paths: chunks per resident wave in each small tail tier (0 = auto:
                                  4 for BVH scenes of <= 256 K primitives, 2 otherwise)                */
    uint32_t px_shift;         /* k_paths: force chunks of 1 << px_shift pixels, 2..5 (0 auto)         */
    uint32_t subqueues;        /* wavefront: block-private sub-queues (0 = 12 per CU)                  */
    uint32_t bvh_max_leaf;     /* BVH build: primitives per leaf, 1..15 (0 auto), next spt_set_scene   */
    uint32_t bvh_bins;         /* BVH build: SAH bins per axis, 2..64 (0 = 64), next spt_set_scene     */
    int32_t specialize;        /* flat scenes: the persistent kernels compiled at run time for the scene's
                                  shape (hiprtc; the generic ones if that fails). 0: compiled on a
                                  background thread started by spt_set_scene, the generic kernels run
                                  until it is ready (a render call never waits on the compiler);
                                  1: compiled inside the first launch that needs it; -1: never          */
} spt_tuning;
/* Applies to later calls; subqueues re-sizes at the next spt_configure. */
int spt_set_tuning(spt_ctx* ctx, const spt_tuning* tuning);

/* ---- run-time specialization (flat scenes) ---------------------------------------------------
 * Flat scenes (<= 32 primitives) run k_paths / k_frame compiled for their shape — the number of
 * primitives of each kind — and the launch configuration their step loop reads (max bounces, RR
 * depth, the sky switch, SPT_FLAG_ABS_FLOAT) with hiprtc (~2 s per key and kernel, cached per process);
 * positions and materials are not baked in, so editing them re-uses the kernels. spt_set_scene and
 * spt_configure start a new key's compiles on a background thread and spt_render runs the generic
 * kernels (same results) until they are ready, so no render call stalls on the compiler.
 * spt_specialize_scene (call it after spt_configure) waits for (or runs) the current scene's
 * compiles and loads the kernels now, so the next frame runs them; a BVH scene is a no-op. */
int spt_specialize_scene(spt_ctx* ctx);
/* Host only, no device needed: compile the specialized k_paths and k_frame for the flat scene
 * `prims` (env_map: the environment-map variant; the shape alone, on run-time configuration values)
 * into the process cache. 0 on success; otherwise
 * SPT_ERR_INVALID (not a flat scene) or SPT_ERR_HIP with the compiler log in `log`. */
int spt_compile_flat_kernels(const spt_prim* prims, uint32_t n_prims, int env_map, char* log, size_t log_bytes);

/* ---- host-only scene builders (no device needed) ------------------------------------------- */
/* Capacity protocol: pass NULL arrays to query the counts, then call again with room for them.
 * Scenes are deterministic (fixed seeds). SPT_SCENE_* ids: */
typedef enum spt_scene_id {
    SPT_SCENE_C1_SPHERE_GROUND = 0, /* App.cpp:101-111: r=1 @ (0,-1,5), r=100 @ (0,-102,5)          */
    SPT_SCENE_APP_DEFAULT = 1,      /* App.cpp:98-122: the above + 6x6 grid of r=0.5 at z=10          */
    SPT_SCENE_CORNELL = 2,          /* C2/C3: 5 walls + ceiling emitter quad + 2 spheres */
    SPT_SCENE_BUNNYLIKE = 3,        /* C4: displaced icosphere (81,920 tris) in the Cornell box      */
    SPT_SCENE_INTERIOR_1M = 4       /* C5: room + 64 displaced meshes, 1,000,000 triangles            */
} spt_scene_id;
int spt_build_scene(uint32_t scene_id, spt_prim* prims, uint32_t* n_prims,
                    spt_material* mats, uint32_t* n_mats, spt_env* env);

#ifdef __cplusplus
}
#endif
#endif /* SPT_H */
