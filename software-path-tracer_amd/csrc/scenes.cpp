// scenes.cpp — deterministic synthetic scenes for the BASELINE.json configs.
//
// The reference ships no assets: its only scene is the sphere set built in
// App::App (src/App.cpp:98-122). Everything else is generated procedurally here, with fixed seeds,
// so every host (this container, the GPU box) builds bit-identical primitive arrays.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "spt.h"

namespace {

struct SceneOut {
    std::vector<spt_prim> prims;
    std::vector<spt_material> mats;
    spt_env env{};
};

spt_prim sphere(float cx, float cy, float cz, float r, uint32_t mat) {
    spt_prim p{};
    p.type = SPT_PRIM_SPHERE;
    p.material = mat;
    p.p0[0] = cx; p.p0[1] = cy; p.p0[2] = cz; p.p0[3] = r;
    return p;
}

spt_prim quad(const float Q[3], const float u[3], const float v[3], uint32_t mat) {
    spt_prim p{};
    p.type = SPT_PRIM_QUAD;
    p.material = mat;
    for (int k = 0; k < 3; ++k) {
        p.p0[k] = Q[k];
        p.p1[k] = u[k];
        p.p2[k] = v[k];
    }
    return p;
}

spt_prim tri(const float a[3], const float b[3], const float c[3], uint32_t mat) {
    spt_prim p{};
    p.type = SPT_PRIM_TRIANGLE;
    p.material = mat;
    for (int k = 0; k < 3; ++k) {
        p.p0[k] = a[k];
        p.p1[k] = b[k];
        p.p2[k] = c[k];
    }
    return p;
}

spt_material mat(float r, float g, float b, float er = 0.f, float eg = 0.f, float eb = 0.f) {
    spt_material m{};
    m.albedo[0] = r; m.albedo[1] = g; m.albedo[2] = b;
    m.emission[0] = er; m.emission[1] = eg; m.emission[2] = eb;
    return m;
}

// Reference sky (CPUPathTracer.cpp:286-292): mix(white, (0.5, 0.7, 1.0), 0.5*(d.y+1)).
spt_env reference_sky(bool enabled) {
    spt_env e{};
    e.sky_enabled = enabled ? 1u : 0u;
    e.horizon[0] = 1.0f; e.horizon[1] = 1.0f; e.horizon[2] = 1.0f;
    e.zenith[0] = 0.5f; e.zenith[1] = 0.7f; e.zenith[2] = 1.0f;
    return e;
}

// C1: the two-sphere part of App::App (src/App.cpp:101-111). Reference mode: albedo 0.7
// (CPUPathTracer.cpp:260), no emission, sky on.
void scene_c1(SceneOut& s) {
    s.mats.push_back(mat(0.7f, 0.7f, 0.7f));
    s.prims.push_back(sphere(0.0f, -1.0f, 5.0f, 1.0f, 0));
    s.prims.push_back(sphere(0.0f, -102.0f, 5.0f, 100.0f, 0));
    s.env = reference_sky(true);
}

// App default scene (src/App.cpp:98-122): C1 plus a 6x6 grid of r=0.5 spheres at z=10,
// x,y in {-5,-3,-1,1,3,5}, in node-creation order (x outer, y inner).
void scene_app_default(SceneOut& s) {
    scene_c1(s);
    const int dims = 5;
    for (int x = -dims; x <= dims; x += 2)
        for (int y = -dims; y <= dims; y += 2) s.prims.push_back(sphere((float)x, (float)y, 10.0f, 0.5f, 0));
}

// Cornell box walls: x,y in [-2.5, 2.5], z in [3, 8], open at z=3 (facing the camera at the
// origin), normals (u x v) pointing inward. Materials 0 white, 1 red, 2 green, 3 light.
void cornell_walls(SceneOut& s, bool light) {
    const uint32_t base = (uint32_t)s.mats.size();
    s.mats.push_back(mat(0.73f, 0.73f, 0.73f));
    s.mats.push_back(mat(0.65f, 0.05f, 0.05f));
    s.mats.push_back(mat(0.12f, 0.45f, 0.15f));
    s.mats.push_back(mat(0.78f, 0.78f, 0.78f, 15.0f, 15.0f, 15.0f));
    {  // floor y=-2.5, normal +y
        const float Q[3] = {-2.5f, -2.5f, 3.0f}, u[3] = {0, 0, 5}, v[3] = {5, 0, 0};
        s.prims.push_back(quad(Q, u, v, base + 0));
    }
    {  // ceiling y=+2.5, normal -y
        const float Q[3] = {-2.5f, 2.5f, 3.0f}, u[3] = {5, 0, 0}, v[3] = {0, 0, 5};
        s.prims.push_back(quad(Q, u, v, base + 0));
    }
    {  // back wall z=8, normal -z
        const float Q[3] = {-2.5f, -2.5f, 8.0f}, u[3] = {0, 5, 0}, v[3] = {5, 0, 0};
        s.prims.push_back(quad(Q, u, v, base + 0));
    }
    {  // left wall x=-2.5, red, normal +x
        const float Q[3] = {-2.5f, -2.5f, 3.0f}, u[3] = {0, 5, 0}, v[3] = {0, 0, 5};
        s.prims.push_back(quad(Q, u, v, base + 1));
    }
    {  // right wall x=+2.5, green, normal -x
        const float Q[3] = {2.5f, -2.5f, 3.0f}, u[3] = {0, 0, 5}, v[3] = {0, 5, 0};
        s.prims.push_back(quad(Q, u, v, base + 2));
    }
    if (light) {  // 1x1 emitter just below the ceiling, normal -y, emission 15
        const float Q[3] = {-0.5f, 2.495f, 5.0f}, u[3] = {1, 0, 0}, v[3] = {0, 0, 1};
        s.prims.push_back(quad(Q, u, v, base + 3));
    }
}

// C2/C3 Cornell box: 6 quads + 2 spheres r=0.8 at (-1,-1.7,6) and (1,-1.7,5).
void scene_cornell(SceneOut& s) {
    cornell_walls(s, true);
    s.prims.push_back(sphere(-1.0f, -1.7f, 6.0f, 0.8f, 0));
    s.prims.push_back(sphere(1.0f, -1.7f, 5.0f, 0.8f, 0));
    s.env = reference_sky(true);
}

// ---- procedural meshes ------------------------------------------------------------------------
uint32_t pcg_hash(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}

double lattice(int x, int y, int z, uint32_t seed) {
    uint32_t h = pcg_hash((uint32_t)x * 73856093u ^ pcg_hash((uint32_t)y * 19349663u ^
                                                             pcg_hash((uint32_t)z * 83492791u ^ seed)));
    return (double)h / 4294967296.0 * 2.0 - 1.0;
}

double smooth(double t) { return t * t * (3.0 - 2.0 * t); }

// Trilinear value noise in [-1, 1].
double value_noise(double x, double y, double z, uint32_t seed) {
    const double fx = std::floor(x), fy = std::floor(y), fz = std::floor(z);
    const int ix = (int)fx, iy = (int)fy, iz = (int)fz;
    const double tx = smooth(x - fx), ty = smooth(y - fy), tz = smooth(z - fz);
    double c[2][2][2];
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int d = 0; d < 2; ++d) c[a][b][d] = lattice(ix + a, iy + b, iz + d, seed);
    double x00 = c[0][0][0] + (c[1][0][0] - c[0][0][0]) * tx;
    double x10 = c[0][1][0] + (c[1][1][0] - c[0][1][0]) * tx;
    double x01 = c[0][0][1] + (c[1][0][1] - c[0][0][1]) * tx;
    double x11 = c[0][1][1] + (c[1][1][1] - c[0][1][1]) * tx;
    double y0 = x00 + (x10 - x00) * ty;
    double y1 = x01 + (x11 - x01) * ty;
    return y0 + (y1 - y0) * tz;
}

double fbm(double x, double y, double z, uint32_t seed) {
    double sum = 0.0, amp = 0.5, f = 1.0;
    for (int o = 0; o < 4; ++o) {
        sum += amp * value_noise(x * f, y * f, z * f, seed + (uint32_t)o * 1013u);
        amp *= 0.5;
        f *= 2.0;
    }
    return sum;  // in about [-0.94, 0.94]
}

struct V3 {
    double x, y, z;
};

V3 normalized(V3 v) {
    const double l = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    return {v.x / l, v.y / l, v.z / l};
}

// Icosphere with `sub` subdivisions: 20 * 4^sub triangles on the unit sphere.
void icosphere(int sub, std::vector<V3>& verts, std::vector<uint32_t>& idx) {
    const double t = (1.0 + std::sqrt(5.0)) / 2.0;
    verts = {{-1, t, 0}, {1, t, 0}, {-1, -t, 0}, {1, -t, 0}, {0, -1, t}, {0, 1, t},
             {0, -1, -t}, {0, 1, -t}, {t, 0, -1}, {t, 0, 1}, {-t, 0, -1}, {-t, 0, 1}};
    for (auto& v : verts) v = normalized(v);
    idx = {0, 11, 5, 0, 5, 1, 0, 1, 7, 0, 7, 10, 0, 10, 11, 1, 5, 9, 5, 11, 4, 11, 10, 2, 10, 7, 6, 7, 1, 8,
           3, 9, 4, 3, 4, 2, 3, 2, 6, 3, 6, 8, 3, 8, 9, 4, 9, 5, 2, 4, 11, 6, 2, 10, 8, 6, 7, 9, 8, 1};
    for (int s = 0; s < sub; ++s) {
        std::vector<uint32_t> next;
        next.reserve(idx.size() * 4);
        // midpoint cache keyed by sorted edge
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> cache(verts.size());
        auto mid = [&](uint32_t a, uint32_t b) -> uint32_t {
            if (a > b) std::swap(a, b);
            for (auto& e : cache[a])
                if (e.first == b) return e.second;
            const V3 m = normalized({(verts[a].x + verts[b].x) * 0.5, (verts[a].y + verts[b].y) * 0.5,
                                     (verts[a].z + verts[b].z) * 0.5});
            const uint32_t id = (uint32_t)verts.size();
            verts.push_back(m);
            cache[a].push_back({b, id});
            return id;
        };
        for (size_t f = 0; f < idx.size(); f += 3) {
            const uint32_t a = idx[f], b = idx[f + 1], c = idx[f + 2];
            const uint32_t ab = mid(a, b), bc = mid(b, c), ca = mid(c, a);
            const uint32_t tris[12] = {a, ab, ca, b, bc, ab, c, ca, bc, ab, bc, ca};
            next.insert(next.end(), tris, tris + 12);
        }
        idx.swap(next);
    }
}

// Emit a mesh as triangles: v -> center + radius * (1 + amp * fbm(3 v)) * v.
void emit_displaced(SceneOut& s, const std::vector<V3>& verts, const std::vector<uint32_t>& idx, V3 c,
                    double radius, double amp, uint32_t seed, uint32_t m) {
    std::vector<float> P(verts.size() * 3);
    for (size_t i = 0; i < verts.size(); ++i) {
        const V3& v = verts[i];
        const double d = 1.0 + amp * fbm(3.0 * v.x + 11.0, 3.0 * v.y + 7.0, 3.0 * v.z + 5.0, seed);
        P[3 * i + 0] = (float)(c.x + radius * d * v.x);
        P[3 * i + 1] = (float)(c.y + radius * d * v.y);
        P[3 * i + 2] = (float)(c.z + radius * d * v.z);
    }
    for (size_t f = 0; f < idx.size(); f += 3)
        s.prims.push_back(tri(&P[3 * idx[f]], &P[3 * idx[f + 1]], &P[3 * idx[f + 2]], m));
}

// UV sphere with `slices` x `stacks`, pole-aware: 2 * slices * (stacks - 1) triangles.
void uvsphere(int slices, int stacks, std::vector<V3>& verts, std::vector<uint32_t>& idx) {
    verts.clear();
    idx.clear();
    const double pi = 3.14159265358979323846;
    verts.push_back({0, 1, 0});  // north pole
    for (int i = 1; i < stacks; ++i) {
        const double th = pi * i / stacks;
        for (int j = 0; j < slices; ++j) {
            const double ph = 2.0 * pi * j / slices;
            verts.push_back({std::sin(th) * std::cos(ph), std::cos(th), std::sin(th) * std::sin(ph)});
        }
    }
    verts.push_back({0, -1, 0});  // south pole
    const uint32_t south = (uint32_t)verts.size() - 1;
    auto ring = [&](int i, int j) { return (uint32_t)(1 + (i - 1) * slices + (j % slices)); };
    for (int j = 0; j < slices; ++j) {
        idx.insert(idx.end(), {0u, ring(1, j + 1), ring(1, j)});
    }
    for (int i = 1; i < stacks - 1; ++i)
        for (int j = 0; j < slices; ++j) {
            const uint32_t a = ring(i, j), b = ring(i, j + 1), c = ring(i + 1, j), d = ring(i + 1, j + 1);
            idx.insert(idx.end(), {a, b, c, b, d, c});
        }
    for (int j = 0; j < slices; ++j) idx.insert(idx.end(), {south, ring(stacks - 1, j), ring(stacks - 1, j + 1)});
}

// C4: "bunny-like" displaced icosphere, subdivision 6 = 81,920 triangles, amplitude 0.15, seed
// 0x5eed, sitting on the floor of the C2 Cornell box (the Stanford bunny is not available offline).
void scene_bunnylike(SceneOut& s) {
    cornell_walls(s, true);
    const uint32_t m = (uint32_t)s.mats.size();
    s.mats.push_back(mat(0.73f, 0.73f, 0.73f));
    std::vector<V3> v;
    std::vector<uint32_t> idx;
    icosphere(6, v, idx);
    emit_displaced(s, v, idx, {0.0, -1.25, 5.5}, 1.1, 0.15, 0x5eedu, m);
    s.env = reference_sky(true);
}

// Split a rectangle (Q, u, v) into an nu x nv grid of quads, each as two triangles.
void grid_tris(SceneOut& s, const float Q[3], const float u[3], const float v[3], int nu, int nv, uint32_t m) {
    for (int i = 0; i < nu; ++i)
        for (int j = 0; j < nv; ++j) {
            float p[4][3];
            for (int c = 0; c < 4; ++c) {
                const float a = (float)(i + (c & 1)) / nu, b = (float)(j + ((c >> 1) & 1)) / nv;
                for (int k = 0; k < 3; ++k) p[c][k] = Q[k] + a * u[k] + b * v[k];
            }
            s.prims.push_back(tri(p[0], p[1], p[3], m));
            s.prims.push_back(tri(p[0], p[3], p[2], m));
        }
}

// C5: closed room around the camera (x in [-10,10], y in [-3,5], z in [-2,30]; sky off) lit by
// 8 ceiling emitters, with 64 displaced UV spheres (124 slices x 64 stacks = 15,624 triangles
// each) on an 8x8 grid. Walls: 6 x 8 triangles, lights: 8 x 2 -> exactly 1,000,000 triangles.
void scene_interior_1m(SceneOut& s) {
    const uint32_t wall = 0, light = 1;
    s.mats.push_back(mat(0.7f, 0.7f, 0.7f));
    s.mats.push_back(mat(0.78f, 0.78f, 0.78f, 8.0f, 8.0f, 8.0f));
    const float x0 = -10, x1 = 10, y0 = -3, y1 = 5, z0 = -2, z1 = 30;
    {  // floor, normal +y
        const float Q[3] = {x0, y0, z0}, u[3] = {0, 0, z1 - z0}, v[3] = {x1 - x0, 0, 0};
        grid_tris(s, Q, u, v, 2, 2, wall);
    }
    {  // ceiling, normal -y
        const float Q[3] = {x0, y1, z0}, u[3] = {x1 - x0, 0, 0}, v[3] = {0, 0, z1 - z0};
        grid_tris(s, Q, u, v, 2, 2, wall);
    }
    {  // far wall z1
        const float Q[3] = {x0, y0, z1}, u[3] = {0, y1 - y0, 0}, v[3] = {x1 - x0, 0, 0};
        grid_tris(s, Q, u, v, 2, 2, wall);
    }
    {  // near wall z0 (behind the camera)
        const float Q[3] = {x0, y0, z0}, u[3] = {x1 - x0, 0, 0}, v[3] = {0, y1 - y0, 0};
        grid_tris(s, Q, u, v, 2, 2, wall);
    }
    {  // left wall x0
        const float Q[3] = {x0, y0, z0}, u[3] = {0, y1 - y0, 0}, v[3] = {0, 0, z1 - z0};
        grid_tris(s, Q, u, v, 2, 2, wall);
    }
    {  // right wall x1
        const float Q[3] = {x1, y0, z0}, u[3] = {0, 0, z1 - z0}, v[3] = {0, y1 - y0, 0};
        grid_tris(s, Q, u, v, 2, 2, wall);
    }
    for (int l = 0; l < 8; ++l) {  // 2x2 emitters at y = 4.99
        const float lx = -7.0f + 4.0f * (float)(l % 4), lz = 6.0f + 10.0f * (float)(l / 4);
        const float Q[3] = {lx, 4.99f, lz}, u[3] = {2, 0, 0}, v[3] = {0, 0, 2};
        grid_tris(s, Q, u, v, 1, 1, light);
    }
    std::vector<V3> v;
    std::vector<uint32_t> idx;
    uvsphere(124, 64, v, idx);
    for (int m = 0; m < 64; ++m) {
        const uint32_t mi = (uint32_t)s.mats.size();
        const uint32_t h = pcg_hash(0x5eedu + (uint32_t)m);
        const float r = 0.3f + 0.6f * (float)(h & 0xff) / 255.0f;
        const float g = 0.3f + 0.6f * (float)((h >> 8) & 0xff) / 255.0f;
        const float b = 0.3f + 0.6f * (float)((h >> 16) & 0xff) / 255.0f;
        s.mats.push_back(mat(r, g, b));
        const double cx = -8.75 + 2.5 * (m % 8);
        const double cz = 4.0 + 3.0 * (m / 8);
        emit_displaced(s, v, idx, {cx, -2.0, cz}, 0.95, 0.2, 0x5eedu + 977u * (uint32_t)m, mi);
    }
    s.env = reference_sky(false);
}

}  // namespace

extern "C" int spt_build_scene(uint32_t scene_id, spt_prim* prims, uint32_t* n_prims, spt_material* mats,
                               uint32_t* n_mats, spt_env* env) {
    if (!n_prims || !n_mats) return SPT_ERR_INVALID;
    SceneOut s;
    switch (scene_id) {
        case SPT_SCENE_C1_SPHERE_GROUND: scene_c1(s); break;
        case SPT_SCENE_APP_DEFAULT: scene_app_default(s); break;
        case SPT_SCENE_CORNELL: scene_cornell(s); break;
        case SPT_SCENE_BUNNYLIKE: scene_bunnylike(s); break;
        case SPT_SCENE_INTERIOR_1M: scene_interior_1m(s); break;
        default: return SPT_ERR_INVALID;
    }
    const uint32_t np = (uint32_t)s.prims.size(), nm = (uint32_t)s.mats.size();
    if (!prims || !mats) {
        *n_prims = np;
        *n_mats = nm;
        if (env) *env = s.env;
        return SPT_OK;
    }
    if (*n_prims < np || *n_mats < nm) {
        *n_prims = np;
        *n_mats = nm;
        return SPT_ERR_CAPACITY;
    }
    std::memcpy(prims, s.prims.data(), sizeof(spt_prim) * np);
    std::memcpy(mats, s.mats.data(), sizeof(spt_material) * nm);
    *n_prims = np;
    *n_mats = nm;
    if (env) *env = s.env;
    return SPT_OK;
}
