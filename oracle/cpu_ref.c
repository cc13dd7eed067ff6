/*
 * cpu_ref.c — CPU ORACLE. TEST INFRASTRUCTURE ONLY (see cpu_ref.h).
 *
 * Line-by-line restatement of render::CPUPathTracer
 * (/root/reference/libs/render/src/engines/pathtracer/backends/cpu/CPUPathTracer.cpp) in C, with
 * the evaluation order of the reference's Linux build:
 *   - compiled -ffp-contract=off on x86-64 SSE (no FMA, no x87 excess precision), like the
 *     reference's default-flag Debug build (build.sh:14);
 *   - glm formulas restated (glm is an empty submodule in the reference, .gitmodules:5-7):
 *     dot = (x*x'+y*y')+z*z', cross, normalize = v*(1/sqrt(dot)), mix = x*(1-a)+y*a;
 *   - get_random_bounche's unqualified sqrt/cos/sin bind to the C double functions under
 *     libstdc++ (CPUPathTracer.cpp:310-316), and abs(normal.z) to ::abs(int) (:320).
 * Embree's rtcIntersect1 (:227) is replaced by the analytic tests of sphere.md:145-188 (spheres)
 * and, for the superset scenes, parallelogram and Moller-Trumbore tests.
 */
#include "cpu_ref.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ glm restatement */
static inline float dot3(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
static inline void cross3(const float a[3], const float b[3], float out[3]) {
    const float x = a[1] * b[2] - b[1] * a[2];
    const float y = a[2] * b[0] - b[2] * a[0];
    const float z = a[0] * b[1] - b[0] * a[1];
    out[0] = x; out[1] = y; out[2] = z;
}
static inline void normalize3(const float v[3], float out[3]) {
    const float inv = 1.0f / sqrtf(dot3(v, v)); /* glm::inversesqrt = 1/sqrt */
    out[0] = v[0] * inv; out[1] = v[1] * inv; out[2] = v[2] * inv;
}
#define SPT_INV_PI_F 0.318309886183790671538f /* 1 / pi (libspt_hip: scene.cpp kInvPiF) */
#define SPT_PI_F 3.14159265358979323846f     /* pi (libspt_hip: spt_device.h kPiF, glm::pi<float>()) */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* ------------------------------------------------------------------ integrator pieces */

/* CPUPathTracer::get_rng_state, :192-195 */
uint32_t ref_rng_seed(uint32_t x, uint32_t y, uint32_t width, uint32_t frame1) {
    return x + y * width + frame1 * 982451653U;
}

/* CPUPathTracer::random_float, :294-301 */
float ref_random_float(uint32_t* state) {
    uint32_t result;
    *state = (uint32_t)((uint64_t)(*state * 747796405u) + 2891336453ull); /* int * + long literal, mod 2^32 */
    result = ((*state >> ((*state >> 28) + 4)) ^ *state) * 277803737u;
    result = (result >> 22) ^ result;
    return ((float)result / 4294967295.0f);
}

/* CPUPathTracer::render, :53-73 */
void ref_primary_dir(uint32_t x, uint32_t y, uint32_t width, uint32_t height, float out[3]) {
    const float inv_height = 1.0f / height;
    const float inv_width = 1.0f / width;
    const float aspect_ratio = (float)width / (float)height;
    float u = x * inv_width;
    float v = 1.0f - y * inv_height;
    float uv_x = (u * 2.0f - 1.0f) * aspect_ratio;
    float uv_y = v * 2.0f - 1.0f;
    float len = sqrtf(uv_x * uv_x + uv_y * uv_y + 1.0f);
    out[0] = uv_x / len;
    out[1] = uv_y / len;
    out[2] = 1.0f / len;
}

/* CPUPathTracer::sample_sky, :286-292 (glm::mix(horizon, sky, t)) */
void ref_sample_sky(const spt_env* env, const float dir[3], float out[3]) {
    float t = 0.5f * (dir[1] + 1.0f);
    for (int k = 0; k < 3; ++k) out[k] = env->horizon[k] * (1.0f - t) + env->zenith[k] * t;
}

/* Environment map lookup (libspt_hip's octa_texel, csrc/spt_device.h; superset, SURVEY.md §8f
 * row 4): nearest texel of an octahedral map, +, -, *, / and fabs only. */
uint32_t ref_octa_texel(float dx, float dy, float dz, uint32_t w, uint32_t h) {
    const float s = (fabsf(dx) + fabsf(dy)) + fabsf(dz);
    float px = dx / s, pz = dz / s;
    if (dy < 0.0f) {
        const float fx = (1.0f - fabsf(pz)) * (px >= 0.0f ? 1.0f : -1.0f);
        const float fz = (1.0f - fabsf(px)) * (pz >= 0.0f ? 1.0f : -1.0f);
        px = fx;
        pz = fz;
    }
    const float u = fminf(fmaxf(px * 0.5f + 0.5f, 0.0f), 1.0f);
    const float v = fminf(fmaxf(pz * 0.5f + 0.5f, 0.0f), 1.0f);
    uint32_t ix = (uint32_t)(u * (float)w), iy = (uint32_t)(v * (float)h);
    if (ix >= w) ix = w - 1;
    if (iy >= h) iy = h - 1;
    return iy * w + ix;
}

/* CPUPathTracer::get_random_bounche, :303-326 */
void ref_bounce_dir(const float normal[3], uint32_t* state, uint32_t flags, float out[3]) {
    float u1 = ref_random_float(state);
    float u2 = ref_random_float(state);
    /* sqrt/cos/sin are the C double functions here (libstdc++ overload resolution) */
    float cosTheta = (float)sqrt((double)u1);
    float sinTheta = (float)sqrt((double)(1.0f - u1));
    float phi = 2.0f * 3.14159265358979323846f * u2;
    float x = (float)((double)sinTheta * cos((double)phi));
    float y = (float)((double)sinTheta * sin((double)phi));
    float z = cosTheta;
    int not_pole;
    if (flags & SPT_FLAG_ABS_FLOAT) not_pole = fabsf(normal[2]) < 0.999f;
    else not_pole = (float)abs((int)normal[2]) < 0.999f; /* ::abs(int) */
    const float up[3] = {not_pole ? 0.0f : 1.0f, 0.0f, not_pole ? 1.0f : 0.0f};
    float c[3], tangent[3], bitangent[3];
    cross3(up, normal, c);
    normalize3(c, tangent);
    cross3(normal, tangent, bitangent);
    for (int k = 0; k < 3; ++k) out[k] = (x * tangent[k] + y * bitangent[k]) + z * normal[k];
}

/* ------------------------------------------------------------------ scene */
typedef struct rprim {
    uint32_t type, material;
    uint32_t axis;                /* quads: 1 + the axis of an axis-aligned normal (scene.cpp), else 0 */
    float a[4], b[4], c[4], d[4]; /* same constants as libspt_hip's DevPrim */
    float lo[3], hi[3];           /* padded bounds (oracle BVH) */
} rprim;

typedef struct rnode {
    float lo[3], hi[3];
    uint32_t left, first, count; /* count > 0: leaf over order[first, first+count) */
} rnode;

/* next-event estimation (SPT_FLAG_NEE; libspt_hip's build_emitters, csrc/scene.cpp): one sampled
 * emitter, a parallelogram (base + a*e1 + b*e2, a, b in [0,1]), a triangle (base + a*e1 + b*e2,
 * a + b <= 1) or a sphere (center base, radius r) */
typedef struct remit {
    float base[3], e1[3], e2[3];
    float nl[3];  /* unit normal: cross(e1, e2) * (1 / sqrt(dot)) */
    float le[3];  /* the material's emission */
    float wgt;    /* area * n_emitters / pi */
    uint32_t tri;
    uint32_t sphere;
    float r;
} remit;

struct ref_scene {
    rprim* prims;
    uint32_t n;
    remit* emit;
    uint32_t n_emit;
    spt_material* mats;
    uint32_t n_mats;
    spt_env env;
    float* env_map; /* octahedral RGBA texels (spt_set_env_map) or NULL */
    uint32_t env_w, env_h;
    rnode* nodes;
    uint32_t n_nodes;
    uint32_t* order;
};

/* Restates libspt_hip's prepare_prims (software-path-tracer_amd/csrc/scene.cpp). */
static void prepare(const spt_prim* p, rprim* r) {
    memset(r, 0, sizeof(*r));
    r->type = p->type;
    r->material = p->material;
    if (p->type == SPT_PRIM_SPHERE) {
        for (int k = 0; k < 4; ++k) r->a[k] = p->p0[k];
        for (int k = 0; k < 3; ++k) { r->lo[k] = p->p0[k] - p->p0[3]; r->hi[k] = p->p0[k] + p->p0[3]; }
    } else if (p->type == SPT_PRIM_QUAD) {
        float n[3], w[3], A[3], B[3];
        cross3(p->p1, p->p2, n);
        const float nn = dot3(n, n);
        w[0] = n[0] / nn; w[1] = n[1] / nn; w[2] = n[2] / nn;
        cross3(p->p2, w, A);
        cross3(w, p->p1, B);
        for (int k = 0; k < 3; ++k) { r->a[k] = p->p0[k]; r->b[k] = n[k]; r->c[k] = A[k]; r->d[k] = B[k]; }
        r->a[3] = dot3(n, p->p0);
        for (int ax = 0; ax < 3; ++ax) {  /* scene.cpp prepare_prims: the axis-aligned short form */
            const int u1 = (ax + 1) % 3, u2 = (ax + 2) % 3;
            if (n[u1] == 0.0f && n[u2] == 0.0f && A[ax] == 0.0f && B[ax] == 0.0f && n[ax] != 0.0f) r->axis = (uint32_t)ax + 1u;
        }
        for (int k = 0; k < 3; ++k) {
            float c0 = p->p0[k], c1 = p->p0[k] + p->p1[k], c2 = p->p0[k] + p->p2[k], c3 = p->p0[k] + p->p1[k] + p->p2[k];
            r->lo[k] = fminf(fminf(c0, c1), fminf(c2, c3));
            r->hi[k] = fmaxf(fmaxf(c0, c1), fmaxf(c2, c3));
        }
    } else {
        for (int k = 0; k < 3; ++k) {
            r->a[k] = p->p0[k];
            r->b[k] = p->p1[k] - p->p0[k];
            r->c[k] = p->p2[k] - p->p0[k];
        }
        cross3(r->b, r->c, r->d);
        for (int k = 0; k < 3; ++k) {
            r->lo[k] = fminf(fminf(p->p0[k], p->p1[k]), p->p2[k]);
            r->hi[k] = fmaxf(fmaxf(p->p0[k], p->p1[k]), p->p2[k]);
        }
    }
}

/* ---- primitive tests: sphere.md:145-188 and the superset shapes (same formulas as the GPU) ---- */
static float isect_sphere(const rprim* s, const float o[3], const float d[3], float tmin) {
    const float lx = o[0] - s->a[0], ly = o[1] - s->a[1], lz = o[2] - s->a[2];
    const float a = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    const float b = 2.0f * ((lx * d[0] + ly * d[1]) + lz * d[2]);
    const float c = ((lx * lx + ly * ly) + lz * lz) - s->a[3] * s->a[3];
    const float disc = b * b - 4.0f * a * c;
    if (!(disc >= 0.0f)) return INFINITY;
    const float sq = sqrtf(disc);
    const float t1 = (-b - sq) / (2.0f * a);
    if (t1 >= tmin) return t1;
    const float t2 = (-b + sq) / (2.0f * a);
    if (t2 >= tmin) return t2;
    return INFINITY;
}

static float isect_quad(const rprim* q, const float o[3], const float d[3], float tmin) {
    float t;
    if (q->axis) {  /* axis-aligned: the plane x[ax] = Q[ax] */
        const int ax = (int)q->axis - 1;
        t = (q->a[ax] - o[ax]) / d[ax];
    } else {
        const float denom = (q->b[0] * d[0] + q->b[1] * d[1]) + q->b[2] * d[2];
        t = (q->a[3] - ((q->b[0] * o[0] + q->b[1] * o[1]) + q->b[2] * o[2])) / denom;
    }
    if (!(t >= tmin) || t == INFINITY) return INFINITY;
    const float hx = (o[0] + t * d[0]) - q->a[0];
    const float hy = (o[1] + t * d[1]) - q->a[1];
    const float hz = (o[2] + t * d[2]) - q->a[2];
    const float al = (hx * q->c[0] + hy * q->c[1]) + hz * q->c[2];
    const float be = (hx * q->d[0] + hy * q->d[1]) + hz * q->d[2];
    if (!(al >= 0.0f && al <= 1.0f && be >= 0.0f && be <= 1.0f)) return INFINITY;
    return t;
}

static float isect_tri(const rprim* r, const float o[3], const float d[3], float tmin) {
    const float* e1 = r->b;
    const float* e2 = r->c;
    const float px = d[1] * e2[2] - e2[1] * d[2];
    const float py = d[2] * e2[0] - e2[2] * d[0];
    const float pz = d[0] * e2[1] - e2[0] * d[1];
    const float det = (e1[0] * px + e1[1] * py) + e1[2] * pz;
    const float inv = 1.0f / det;
    const float tx = o[0] - r->a[0], ty = o[1] - r->a[1], tz = o[2] - r->a[2];
    const float u = ((tx * px + ty * py) + tz * pz) * inv;
    if (!(u >= 0.0f && u <= 1.0f)) return INFINITY;
    const float qx = ty * e1[2] - e1[1] * tz;
    const float qy = tz * e1[0] - e1[2] * tx;
    const float qz = tx * e1[1] - e1[0] * ty;
    const float v = ((d[0] * qx + d[1] * qy) + d[2] * qz) * inv;
    if (!(v >= 0.0f && u + v <= 1.0f)) return INFINITY;
    const float t = ((e2[0] * qx + e2[1] * qy) + e2[2] * qz) * inv;
    if (!(t >= tmin) || t == INFINITY) return INFINITY;
    return t;
}

static float isect_prim(const rprim* p, const float o[3], const float d[3], float tmin) {
    if (p->type == SPT_PRIM_SPHERE) return isect_sphere(p, o, d, tmin);
    if (p->type == SPT_PRIM_QUAD) return isect_quad(p, o, d, tmin);
    return isect_tri(p, o, d, tmin);
}

/* ---- oracle BVH (independent of the product's: median split, its own layout) ---- */
static int g_axis;
static const rprim* g_sort_prims;
static int cmp_centroid(const void* a, const void* b) {
    const rprim* pa = &g_sort_prims[*(const uint32_t*)a];
    const rprim* pb = &g_sort_prims[*(const uint32_t*)b];
    const float ca = pa->lo[g_axis] + pa->hi[g_axis], cb = pb->lo[g_axis] + pb->hi[g_axis];
    if (ca < cb) return -1;
    if (ca > cb) return 1;
    const uint32_t ia = *(const uint32_t*)a, ib = *(const uint32_t*)b;
    return ia < ib ? -1 : (ia > ib ? 1 : 0);
}

static uint32_t build(ref_scene* s, uint32_t first, uint32_t count) {
    const uint32_t ni = s->n_nodes++;
    rnode* n = &s->nodes[ni];
    for (int k = 0; k < 3; ++k) { n->lo[k] = INFINITY; n->hi[k] = -INFINITY; }
    for (uint32_t i = first; i < first + count; ++i) {
        const rprim* p = &s->prims[s->order[i]];
        for (int k = 0; k < 3; ++k) {
            if (p->lo[k] < n->lo[k]) n->lo[k] = p->lo[k];
            if (p->hi[k] > n->hi[k]) n->hi[k] = p->hi[k];
        }
    }
    if (count <= 4) {
        n->first = first;
        n->count = count;
        n->left = 0;
        return ni;
    }
    int axis = 0;
    float ext = n->hi[0] - n->lo[0];
    for (int k = 1; k < 3; ++k)
        if (n->hi[k] - n->lo[k] > ext) { ext = n->hi[k] - n->lo[k]; axis = k; }
    g_axis = axis;
    g_sort_prims = s->prims;
    qsort(s->order + first, count, sizeof(uint32_t), cmp_centroid);
    const uint32_t half = count / 2;
    n->count = 0;
    const uint32_t l = build(s, first, half);
    const uint32_t r = build(s, first + half, count - half);
    (void)r;
    s->nodes[ni].left = l; /* right = the node built next after the whole left subtree: store both */
    s->nodes[ni].first = r;
    return ni;
}

ref_scene* ref_scene_create(const spt_prim* prims, uint32_t n_prims, const spt_material* mats, uint32_t n_mats,
                            const spt_env* env) {
    ref_scene* s = (ref_scene*)calloc(1, sizeof(ref_scene));
    s->n = n_prims;
    s->prims = (rprim*)calloc(n_prims ? n_prims : 1, sizeof(rprim));
    for (uint32_t i = 0; i < n_prims; ++i) prepare(&prims[i], &s->prims[i]);
    /* conservative padding for the oracle's own slab test: 1e-5 of the scene's coordinate magnitude */
    float mag = 1.0f;
    for (uint32_t i = 0; i < n_prims; ++i)
        for (int k = 0; k < 3; ++k) mag = fmaxf(mag, fmaxf(fabsf(s->prims[i].lo[k]), fabsf(s->prims[i].hi[k])));
    for (uint32_t i = 0; i < n_prims; ++i)
        for (int k = 0; k < 3; ++k) {
            s->prims[i].lo[k] -= mag * 1e-5f;
            s->prims[i].hi[k] += mag * 1e-5f;
        }
    s->mats = (spt_material*)calloc(n_mats ? n_mats : 1, sizeof(spt_material));
    memcpy(s->mats, mats, sizeof(spt_material) * n_mats);
    /* emitters for SPT_FLAG_NEE: quads and triangles of an emitting material with nonzero area and
     * every sphere of an emitting material, in primitive order (restates libspt_hip's build_emitters,
     * csrc/scene.cpp) */
    s->emit = (remit*)calloc(n_prims ? n_prims : 1, sizeof(remit));
    for (int pass = 0; pass < 2; ++pass) {
        uint32_t k = 0;
        for (uint32_t i = 0; i < n_prims; ++i) {
            const spt_prim* p = &prims[i];
            const float* em = mats[p->material].emission;
            if (!(em[0] != 0.0f || em[1] != 0.0f || em[2] != 0.0f)) continue;
            remit e;
            memset(&e, 0, sizeof e);
            if (p->type == SPT_PRIM_SPHERE) {
                e.sphere = 1;
                e.r = p->p0[3];
                for (int c = 0; c < 3; ++c) {
                    e.base[c] = p->p0[c];
                    e.le[c] = em[c];
                }
                const float area = ((4.0f * SPT_PI_F) * e.r) * e.r;
                if (pass == 1) {
                    e.wgt = (area * (float)s->n_emit) * SPT_INV_PI_F;
                    s->emit[k] = e;
                }
                ++k;
                continue;
            }
            for (int c = 0; c < 3; ++c) {
                e.base[c] = p->p0[c];
                e.e1[c] = p->type == SPT_PRIM_QUAD ? p->p1[c] : p->p1[c] - p->p0[c];
                e.e2[c] = p->type == SPT_PRIM_QUAD ? p->p2[c] : p->p2[c] - p->p0[c];
                e.le[c] = em[c];
            }
            float n[3];
            cross3(e.e1, e.e2, n);
            const float nn = dot3(n, n);
            if (!(nn > 0.0f)) continue;
            const float len = sqrtf(nn);
            const float inv = 1.0f / len;
            for (int c = 0; c < 3; ++c) e.nl[c] = n[c] * inv;
            e.tri = p->type == SPT_PRIM_TRIANGLE;
            const float area = e.tri ? 0.5f * len : len;
            if (pass == 1) {
                e.wgt = (area * (float)s->n_emit) * SPT_INV_PI_F;
                s->emit[k] = e;
            }
            ++k;
        }
        if (pass == 0) s->n_emit = k;
    }
    s->n_mats = n_mats;
    s->env = *env;
    if (n_prims > 64) {
        s->order = (uint32_t*)malloc(sizeof(uint32_t) * n_prims);
        for (uint32_t i = 0; i < n_prims; ++i) s->order[i] = i;
        s->nodes = (rnode*)calloc(2 * (size_t)n_prims, sizeof(rnode));
        build(s, 0, n_prims);
    }
    return s;
}

void ref_set_env_map(ref_scene* s, const float* rgba, uint32_t w, uint32_t h) {
    free(s->env_map);
    s->env_map = NULL;
    s->env_w = s->env_h = 0;
    if (!rgba || !w || !h) return;
    s->env_map = (float*)malloc(sizeof(float) * 4 * (size_t)w * h);
    memcpy(s->env_map, rgba, sizeof(float) * 4 * (size_t)w * h);
    s->env_w = w;
    s->env_h = h;
}

void ref_scene_destroy(ref_scene* s) {
    if (!s) return;
    free(s->env_map);
    free(s->prims);
    free(s->emit);
    free(s->mats);
    free(s->nodes);
    free(s->order);
    free(s);
}

static int box_hit(const rnode* n, const float o[3], const float inv[3], float tmin, float tmax) {
    float t0 = tmin, t1 = tmax;
    for (int k = 0; k < 3; ++k) {
        float a = (n->lo[k] - o[k]) * inv[k], b = (n->hi[k] - o[k]) * inv[k];
        float lo = fminf(a, b), hi = fmaxf(a, b); /* fminf/fmaxf skip the NaN of 0*inf */
        t0 = fmaxf(t0, lo);
        t1 = fminf(t1, hi);
    }
    return t0 <= t1;
}

/* the closest hit with tmin <= t < tmax (tmax = INFINITY: rtcIntersect1's tfar, :221-224) */
static void closest(const ref_scene* s, const float o[3], const float d[3], float tmin, float tmax, float* best_t,
                    uint32_t* best_k) {
    float best = tmax;
    uint32_t best_i = 0xffffffffu;
    if (!s->nodes) {
        /* every primitive in index order; strict '<' keeps the lowest index on equal t */
        for (uint32_t i = 0; i < s->n; ++i) {
            const float t = isect_prim(&s->prims[i], o, d, tmin);
            if (t < best) { best = t; best_i = i; }
        }
    } else {
        const float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
        uint32_t stack[128];
        int sp = 0;
        stack[sp++] = 0;
        while (sp > 0) {
            const rnode* n = &s->nodes[stack[--sp]];
            if (!box_hit(n, o, inv, tmin, best)) continue;
            if (n->count) {
                for (uint32_t k = n->first; k < n->first + n->count; ++k) {
                    const uint32_t i = s->order[k];
                    const float t = isect_prim(&s->prims[i], o, d, tmin);
                    if (t < best || (t == best && t != INFINITY && i < best_i)) { best = t; best_i = i; }
                }
            } else {
                stack[sp++] = n->first; /* right */
                stack[sp++] = n->left;
            }
        }
    }
    *best_t = best;
    *best_k = best_i;
}

int ref_intersect(const ref_scene* s, const float o[3], const float d[3], float tmin, float* t_out, uint32_t* prim,
                  float ng[3]) {
    float best;
    uint32_t best_i;
    closest(s, o, d, tmin, INFINITY, &best, &best_i);
    if (best_i == 0xffffffffu) return 0;
    *t_out = best;
    *prim = best_i;
    if (ng) {
        const rprim* p = &s->prims[best_i];
        if (p->type == SPT_PRIM_SPHERE) {
            /* Ng = hit - center with hit = o + t*d, the integrator's own origin update (:239-241) */
            for (int k = 0; k < 3; ++k) ng[k] = (o[k] + best * d[k]) - p->a[k];
        } else {
            const float* nv = p->type == SPT_PRIM_QUAD ? p->b : p->d;
            float sgn = dot3(nv, d) > 0.0f ? -1.0f : 1.0f; /* two-sided superset primitives */
            for (int k = 0; k < 3; ++k) ng[k] = sgn < 0.0f ? -nv[k] : nv[k];
        }
    }
    return 1;
}

/* ------------------------------------------------------------------ next-event estimation (SPT_FLAG_NEE) */
/* A point on a uniformly chosen emitter, seen from the offset hit point x with shading normal n:
 * three draws (emitter, u, v). Returns 1 with the shadow ray (x, w, tmax) and the estimate
 * add = T * (Le * g), g = cos_s * cos_l * area * n_emit / (pi * dist^2); 0 if the point is not
 * in front of both surfaces. Restated by libspt_hip's light_sample (csrc/spt_device.h). */
int ref_light_sample(const ref_scene* s, const float x[3], const float n[3], const float T[3], uint32_t* rng,
                     float w[3], float* tmax, float add[3]) {
    const float u0 = ref_random_float(rng);
    const float u1 = ref_random_float(rng);
    const float u2 = ref_random_float(rng);
    uint32_t j = (uint32_t)(u0 * (float)s->n_emit);
    if (j >= s->n_emit) j = s->n_emit - 1u;
    const remit* e = &s->emit[j];
    float v[3], nl[3];
    if (e->sphere) { /* uniform over the sphere's area: normal (s cos phi, s sin phi, z), z = 1 - 2 u1 */
        const float z = 1.0f - 2.0f * u1;
        const float sn = sqrtf(1.0f - z * z);
        const float phi = 2.0f * SPT_PI_F * u2;
        nl[0] = (float)((double)sn * cos((double)phi)); /* the C double functions, as ref_bounce_dir */
        nl[1] = (float)((double)sn * sin((double)phi));
        nl[2] = z;
        for (int k = 0; k < 3; ++k) v[k] = (e->base[k] + e->r * nl[k]) - x[k];
    } else {
        float a = u1, b = u2;
        if (e->tri) { /* uniform on the triangle: sqrt(u1) * (1 - u2), sqrt(u1) * u2 */
            const float su = sqrtf(u1);
            a = su * (1.0f - u2);
            b = su * u2;
        }
        for (int k = 0; k < 3; ++k) v[k] = ((e->base[k] + a * e->e1[k]) + b * e->e2[k]) - x[k];
        for (int k = 0; k < 3; ++k) nl[k] = e->nl[k];
    }
    const float d2 = dot3(v, v);
    const float dist = sqrtf(d2);
    const float inv = 1.0f / dist;
    for (int k = 0; k < 3; ++k) w[k] = v[k] * inv;
    const float cs = dot3(n, w);
    /* a sphere emits towards x from the side x sees: outside (its far side is occluded by the sphere
     * itself) or, for x inside the sphere (a dome), inside */
    const float dl = dot3(nl, w);
    float cl = fabsf(dl);
    if (e->sphere) {
        const float xc[3] = {x[0] - e->base[0], x[1] - e->base[1], x[2] - e->base[2]};
        cl = dot3(xc, xc) < e->r * e->r ? dl : -dl;
    }
    if (!(cs > 0.0f) || !(cl > 0.0f)) return 0;
    const float g = ((cs * cl) * e->wgt) / d2;
    *tmax = dist * 0.999f;
    for (int k = 0; k < 3; ++k) add[k] = T[k] * (e->le[k] * g);
    return 1;
}

/* the shadow ray: nothing with 0.001 <= t < tmax */
int ref_visible(const ref_scene* s, const float o[3], const float w[3], float tmax) {
    float best;
    uint32_t best_i;
    closest(s, o, w, 0.001f, tmax, &best, &best_i);
    return !(best < tmax);
}

uint32_t ref_emitter_count(const ref_scene* s) { return s->n_emit; }

/* ------------------------------------------------------------------ trace_ray, :197-284 */
static __thread uint64_t tl_segments;
static __thread uint64_t tl_shadow; /* NEE light samples drawn */

void ref_trace_ray(const ref_scene* s, const ref_config* cfg, const float ray_origin[3], const float ray_direction[3],
                   uint32_t* rng_state, float out[4]) {
    const int max_bounces = (int)cfg->max_bounces;
    const int nee = (cfg->flags & SPT_FLAG_NEE) && s->n_emit > 0;
    float accumulated_color[3] = {0.0f, 0.0f, 0.0f};
    float ray_throughput[3] = {1.0f, 1.0f, 1.0f};
    float current_origin[3] = {ray_origin[0], ray_origin[1], ray_origin[2]};
    float current_direction[3] = {ray_direction[0], ray_direction[1], ray_direction[2]};
    int bounce_count = 0;
    while (bounce_count < max_bounces) {
        float hit_t, ng[3];
        uint32_t prim;
        tl_segments++;
        /* rtcIntersect1 with tnear = 0.001f, tfar = INFINITY (:214-227) */
        if (!ref_intersect(s, current_origin, current_direction, 0.001f, &hit_t, &prim, ng)) {
            if (s->env.sky_enabled) {
                float sky[3];
                if (s->env_map) {
                    const float* e = s->env_map + 4 * (size_t)ref_octa_texel(current_direction[0], current_direction[1],
                                                                             current_direction[2], s->env_w, s->env_h);
                    sky[0] = e[0];
                    sky[1] = e[1];
                    sky[2] = e[2];
                } else {
                    ref_sample_sky(&s->env, current_direction, sky);
                }
                for (int k = 0; k < 3; ++k) accumulated_color[k] += ray_throughput[k] * sky[k];
            }
            break;
        }
        current_origin[0] += hit_t * current_direction[0];
        current_origin[1] += hit_t * current_direction[1];
        current_origin[2] += hit_t * current_direction[2];
        const float nx = ng[0], ny = ng[1], nz = ng[2];
        const float inv_len = 1.0f / sqrtf(nx * nx + ny * ny + nz * nz);
        const float normal[3] = {nx * inv_len, ny * inv_len, nz * inv_len};
        const spt_material* m = &s->mats[s->prims[prim].material];
        /* with NEE every emitter is sampled (quad, triangle, sphere): its emission counts on the camera
         * segment only */
        const int counted = !nee || bounce_count == 0;
        if ((m->emission[0] != 0.0f || m->emission[1] != 0.0f || m->emission[2] != 0.0f) && counted) {
            for (int k = 0; k < 3; ++k) accumulated_color[k] += ray_throughput[k] * m->emission[k];
        }
        /* ray_throughput *= 0.7f in reference mode (:260) */
        for (int k = 0; k < 3; ++k) ray_throughput[k] *= m->albedo[k];
        bounce_count++;
        if (nee && bounce_count < max_bounces) { /* next-event estimation, before Russian roulette */
            const float x[3] = {current_origin[0] + normal[0] * 1e-4f, current_origin[1] + normal[1] * 1e-4f,
                                current_origin[2] + normal[2] * 1e-4f};
            float w[3], tmax, add[3];
            tl_shadow++;
            if (ref_light_sample(s, x, normal, ray_throughput, rng_state, w, &tmax, add) &&
                ref_visible(s, x, w, tmax)) {
                for (int k = 0; k < 3; ++k) accumulated_color[k] += add[k];
            }
        }
        if (bounce_count > (int)cfg->rr_depth) {
            float p = ray_throughput[0];
            if (ray_throughput[1] > p) p = ray_throughput[1];
            if (ray_throughput[2] > p) p = ray_throughput[2];
            if (ref_random_float(rng_state) > p) break;
            for (int k = 0; k < 3; ++k) ray_throughput[k] /= p;
        }
        ref_bounce_dir(normal, rng_state, cfg->flags, current_direction);
        const float EPSILON = 1e-4f;
        current_origin[0] += normal[0] * EPSILON;
        current_origin[1] += normal[1] * EPSILON;
        current_origin[2] += normal[2] * EPSILON;
    }
    out[0] = accumulated_color[0];
    out[1] = accumulated_color[1];
    out[2] = accumulated_color[2];
    out[3] = 1.0f;
}

/* ------------------------------------------------------------------ render, :43-85 */
static uint64_t g_last_segments;
static uint64_t g_last_shadow;

int ref_render(const ref_scene* s, const ref_config* cfg, uint32_t first_frame, uint32_t n_frames, uint32_t x0,
               uint32_t y0, uint32_t x1, uint32_t y1, uint32_t row_step, uint32_t row_offset, float* accum,
               int threads) {
    if (!s || !cfg || !accum || x1 < x0 || y1 < y0 || x1 > cfg->width || y1 > cfg->height) return -1;
    if (row_step == 0) row_step = 1;
    const uint32_t cw = x1 - x0;
    const int64_t n_rows = (y1 > y0 + row_offset) ? (int64_t)((y1 - y0 - row_offset + row_step - 1) / row_step) : 0;
    uint64_t segs = 0, shadow = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel reduction(+ : segs, shadow)
    {
        tl_segments = 0;
        tl_shadow = 0;
#pragma omp for schedule(dynamic, 1)
        for (int64_t r = 0; r < n_rows; ++r) {
            const uint32_t y = y0 + row_offset + (uint32_t)r * row_step;
            for (uint32_t x = x0; x < x1; ++x) {
                float* acc = &accum[4 * ((size_t)r * cw + (x - x0))];
                for (uint32_t f = 0; f < n_frames; ++f) {
                    /* frame k is seeded with k + 1 (m_frameCount + 1, :61) */
                    uint32_t rng_state = ref_rng_seed(x, y, cfg->width, first_frame + f + 1u);
                    const float ray_origin[3] = {0.0f, 0.0f, 0.0f};
                    float ray_direction[3];
                    ref_primary_dir(x, y, cfg->width, cfg->height, ray_direction);
                    float color[4];
                    ref_trace_ray(s, cfg, ray_origin, ray_direction, &rng_state, color);
                    acc[0] += color[0];
                    acc[1] += color[1];
                    acc[2] += color[2];
                    acc[3] += color[3];
                }
            }
        }
        segs += tl_segments;
        shadow += tl_shadow;
    }
    g_last_segments = segs;
    g_last_shadow = shadow;
    return 0;
}

uint64_t ref_last_segments(void) { return g_last_segments; }
uint64_t ref_last_light_samples(void) { return g_last_shadow; }

/* ------------------------------------------------------------------ get_render_result, :87-117 */
static inline uint8_t to_u8(float v, float fc, float exposure) {
    float c = v / fc;
    c = c * exposure; /* the commented-out "r *= getExposure()" (:101-104); 1.0f: identity (alpha) */
    c = c < 0.0f ? 0.0f : (1.0f < c ? 1.0f : c); /* std::clamp */
    if (c != c) c = 0.0f;                         /* NaN: UB in the reference, 0 here and on the GPU */
    return (uint8_t)(c * 255.0f);
}

void ref_resolve_rgba8_exposure(const float* accum, uint64_t n, uint32_t frame_count, float exposure, uint32_t* out) {
    const float fc = (float)frame_count;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = to_u8(accum[4 * i + 0], fc, exposure), g = to_u8(accum[4 * i + 1], fc, exposure);
        const uint32_t b = to_u8(accum[4 * i + 2], fc, exposure), a = to_u8(accum[4 * i + 3], fc, 1.0f);
        out[i] = (r << 24) | (g << 16) | (b << 8) | (a << 0); /* rgba_to_uint32, Color.h:7-10 */
    }
}

void ref_resolve_rgba8(const float* accum, uint64_t n, uint32_t frame_count, uint32_t* out) {
    ref_resolve_rgba8_exposure(accum, n, frame_count, 1.0f, out);
}
