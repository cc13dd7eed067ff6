// scene.cpp — host-side scene preparation and the deterministic scene builders of libspt_hip.so.
//
// Stands in for the Embree scene path of the reference:
//   rtcNewGeometry / rtcSetNewGeometryBuffer / rtcCommitScene
//   (libs/render/src/engines/pathtracer/backends/cpu/CPUPathTracer.cpp:362-403).
// Compiled with -ffp-contract=off: the precomputed constants must equal the oracle's bit for bit
// (oracle/cpu_ref.c restates prepare_prims' formulas).
#include "scene.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>

namespace spt {

namespace {

inline void cross3(const float a[3], const float b[3], float out[3]) {
    // glm::cross formula
    out[0] = a[1] * b[2] - b[1] * a[2];
    out[1] = a[2] * b[0] - b[2] * a[0];
    out[2] = a[0] * b[1] - b[0] * a[1];
}
inline float dot3(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
inline uint32_t f2u(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}
inline float u2f(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

}  // namespace

bool prepare_prims(const spt_prim* prims, uint32_t n, uint32_t n_mats, std::vector<DevPrim>& out,
                   const char** msg) {
    out.assign(n, DevPrim{});
    for (uint32_t i = 0; i < n; ++i) {
        const spt_prim& p = prims[i];
        DevPrim& d = out[i];
        if (p.material >= n_mats) {
            *msg = "primitive material index out of range";
            return false;
        }
        if (p.material >= (1u << 28)) {
            *msg = "too many materials";
            return false;
        }
        switch (p.type) {
            case SPT_PRIM_SPHERE: {
                if (!(p.p0[3] > 0.0f)) {
                    *msg = "sphere radius must be > 0";
                    return false;
                }
                for (int k = 0; k < 4; ++k) d.a[k] = p.p0[k];
                d.b[0] = p.p0[3] * p.p0[3];  // r * r, the same correctly rounded product the device's
                                             // isect_sphere forms (the flat fast path reads it from here)
                break;
            }
            case SPT_PRIM_QUAD: {
                const float* Q = p.p0;
                const float* u = p.p1;
                const float* v = p.p2;
                float nrm[3], w[3], A[3], B[3];
                cross3(u, v, nrm);
                const float nn = dot3(nrm, nrm);
                if (!(nn > 0.0f)) {
                    *msg = "degenerate quad";
                    return false;
                }
                w[0] = nrm[0] / nn;
                w[1] = nrm[1] / nn;
                w[2] = nrm[2] / nn;
                cross3(v, w, A);
                cross3(w, u, B);
                d.a[0] = Q[0]; d.a[1] = Q[1]; d.a[2] = Q[2]; d.a[3] = dot3(nrm, Q);
                d.b[0] = nrm[0]; d.b[1] = nrm[1]; d.b[2] = nrm[2];
                d.c[0] = A[0]; d.c[1] = A[1]; d.c[2] = A[2];
                d.d[0] = B[0]; d.d[1] = B[1]; d.d[2] = B[2];
                // axis-aligned quad (normal along one axis, both edges in the plane): axis + 1 in
                // c.w's bits 2.. selects isect_quad's short form, which drops the zero terms (same
                // results); c.w's bits 0-1 hold the type (set below)
                for (int ax = 0; ax < 3; ++ax) {
                    const int u1 = (ax + 1) % 3, u2 = (ax + 2) % 3;
                    if (nrm[u1] == 0.0f && nrm[u2] == 0.0f && A[ax] == 0.0f && B[ax] == 0.0f && nrm[ax] != 0.0f) {
                        d.c[3] = u2f(((uint32_t)ax + 1u) << kMetaTypeBits);
                        // A rectangle whose dual basis runs (0, a), (b, 0) in the in-plane axes (U, V) of the
                        // device's axis test (the right, floor and back walls of the Cornell box): A and B
                        // swapped, so every such wall has the (a, 0), (0, b) form the device's short form
                        // tests (spt_device.h isect_quad_axis_fast). The in-plane test `0 <= alpha, beta <= 1`
                        // is symmetric in the two, t and the normal do not involve them: same hits.
                        const int U = ax == 0 ? 1 : 0, V = ax == 2 ? 1 : 2;
                        if (!(A[V] == 0.0f && B[U] == 0.0f) && A[U] == 0.0f && B[V] == 0.0f)
                            for (int k = 0; k < 3; ++k) std::swap(d.c[k], d.d[k]);
                    }
                }
                break;
            }
            case SPT_PRIM_TRIANGLE: {
                const float* v0 = p.p0;
                float e1[3] = {p.p1[0] - v0[0], p.p1[1] - v0[1], p.p1[2] - v0[2]};
                float e2[3] = {p.p2[0] - v0[0], p.p2[1] - v0[1], p.p2[2] - v0[2]};
                float ng[3];
                cross3(e1, e2, ng);
                d.a[0] = v0[0]; d.a[1] = v0[1]; d.a[2] = v0[2];
                d.b[0] = e1[0]; d.b[1] = e1[1]; d.b[2] = e1[2];
                d.c[0] = e2[0]; d.c[1] = e2[1]; d.c[2] = e2[2];
                d.d[0] = ng[0]; d.d[1] = ng[1]; d.d[2] = ng[2];
                break;
            }
            default:
                *msg = "unknown primitive type";
                return false;
        }
        d.d[3] = u2f(meta_pack(p.type, p.material));
        d.c[3] = u2f(f2u(d.c[3]) | p.type);  // the type again, so a BVH primitive test loads a, b, c only
        d.b[3] = u2f(i);  // original index: the closest-hit tie-break key (lowest index wins)
    }
    return true;
}

bool fast_division_ok(const spt_prim* prims, uint32_t n, const std::vector<DevPrim>& dp) {
    const double lim = 268435456.0;  // 2^28
    for (uint32_t i = 0; i < n; ++i) {
        const spt_prim& p = prims[i];
        for (int k = 0; k < 3; ++k) {
            double m = 0.0;
            if (p.type == SPT_PRIM_SPHERE) {
                m = std::fabs((double)p.p0[k]) + (double)p.p0[3];
            } else if (p.type == SPT_PRIM_QUAD) {
                m = std::fabs((double)p.p0[k]) + std::fabs((double)p.p1[k]) + std::fabs((double)p.p2[k]);
            } else {
                m = std::max(std::fabs((double)p.p0[k]), std::max(std::fabs((double)p.p1[k]), std::fabs((double)p.p2[k])));
            }
            if (!(m < lim)) return false;  // NaN too
        }
    }
    (void)dp;
    return true;
}

uint32_t flat_kind(const DevPrim& p) {
    const uint32_t type = f2u(p.d[3]) & ((1u << kMetaTypeBits) - 1u);
    if (type == SPT_PRIM_SPHERE) return 0;
    if (type == SPT_PRIM_QUAD) {
        const uint32_t axis = f2u(p.c[3]) >> kMetaTypeBits;  // 1 + the normal's axis, 0: general
        return axis ? axis : 4u;
    }
    return 5;
}

void sort_flat_by_kind(const std::vector<DevPrim>& dp, std::vector<DevPrim>& sorted, uint32_t ends[kFlatKinds - 1]) {
    sorted.clear();
    sorted.reserve(dp.size());
    for (uint32_t g = 0; g < kFlatKinds; ++g) {
        for (const DevPrim& p : dp)
            if (flat_kind(p) == g) sorted.push_back(p);
        if (g + 1 < kFlatKinds) ends[g] = (uint32_t)sorted.size();
    }
}

uint32_t flat_rect_bits(const std::vector<DevPrim>& sorted, const uint32_t ends[kFlatKinds - 1]) {
    uint32_t bits = 0;
    for (int ax = 0; ax < 3; ++ax) {
        const int u = ax == 0 ? 1 : 0, v = ax == 2 ? 1 : 2;  // spt_device.h isect_quad_axis_fast's U, V
        const uint32_t b = ends[ax], e = ends[ax + 1];        // group ax + 1: [ends[ax], ends[ax + 1])
        bool all = e > b;
        for (uint32_t k = b; k < e && all; ++k)
            all = ((f2u(sorted[k].c[v]) | f2u(sorted[k].d[u])) & 0x7fffffffu) == 0u;
        if (all) bits |= 1u << ax;
    }
    return bits;
}

void prepare_materials(const spt_material* mats, uint32_t n, std::vector<DevMaterial>& out) {
    out.assign(n, DevMaterial{});
    for (uint32_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k) {
            out[i].albedo[k] = mats[i].albedo[k];
            out[i].emission[k] = mats[i].emission[k];
        }
        const bool emissive = mats[i].emission[0] != 0.0f || mats[i].emission[1] != 0.0f ||
                              mats[i].emission[2] != 0.0f;
        out[i].emission[3] = emissive ? 1.0f : 0.0f;
    }
}

void build_emitters(const spt_prim* prims, uint32_t n, const spt_material* mats, std::vector<DevEmitter>& out) {
    out.clear();
    for (uint32_t i = 0; i < n; ++i) {
        const spt_prim& p = prims[i];
        const float* em = mats[p.material].emission;
        if (!(em[0] != 0.0f || em[1] != 0.0f || em[2] != 0.0f)) continue;
        DevEmitter e{};
        if (p.type == SPT_PRIM_SPHERE) {  // (center, 2), (r, 0, 0, area): every emissive sphere (r = 0: area 0)
            const float r = p.p0[3];
            for (int c = 0; c < 3; ++c) {
                e.base[c] = p.p0[c];
                e.le[c] = em[c];
            }
            e.base[3] = u2f(2u);
            e.e1[0] = r;
            e.e1[3] = ((4.0f * 3.14159265358979323846f) * r) * r;  // 4 pi r^2 (oracle: the same expression)
            out.push_back(e);
            continue;
        }
        for (int c = 0; c < 3; ++c) {
            e.base[c] = p.p0[c];
            e.e1[c] = p.type == SPT_PRIM_QUAD ? p.p1[c] : p.p1[c] - p.p0[c];
            e.e2[c] = p.type == SPT_PRIM_QUAD ? p.p2[c] : p.p2[c] - p.p0[c];
            e.le[c] = em[c];
        }
        float nv[3];
        cross3(e.e1, e.e2, nv);
        const float nn = dot3(nv, nv);
        if (!(nn > 0.0f)) continue;  // degenerate: never hit, never sampled
        const float len = std::sqrt(nn);
        const float inv = 1.0f / len;
        for (int c = 0; c < 3; ++c) e.nl[c] = nv[c] * inv;
        const bool tri = p.type == SPT_PRIM_TRIANGLE;
        e.base[3] = u2f(tri ? 1u : 0u);
        e.e1[3] = tri ? 0.5f * len : len;  // the area until the count is known
        out.push_back(e);
    }
    const float count = (float)out.size();
    for (DevEmitter& e : out) e.e1[3] = (e.e1[3] * count) * kInvPiF;  // area * n_emitters / pi
}

// ------------------------------------------------------------------------------------------------
// BVH: binned SAH, 64 bins, over primitive centroids.
// ------------------------------------------------------------------------------------------------
namespace {

struct Aabb {
    float lo[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                   std::numeric_limits<float>::infinity()};
    float hi[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                   -std::numeric_limits<float>::infinity()};
    void grow(const float p[3]) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    void grow(const Aabb& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    double area() const {
        if (!(hi[0] >= lo[0])) return 0.0;
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

Aabb prim_bounds(const spt_prim& p) {
    Aabb b;
    if (p.type == SPT_PRIM_SPHERE) {
        const float r = p.p0[3];
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = p.p0[k] - r;
            b.hi[k] = p.p0[k] + r;
        }
    } else if (p.type == SPT_PRIM_QUAD) {
        // corners Q, Q+u, Q+v, Q+u+v
        for (int c = 0; c < 4; ++c) {
            float q[3];
            for (int k = 0; k < 3; ++k)
                q[k] = p.p0[k] + ((c & 1) ? p.p1[k] : 0.0f) + ((c & 2) ? p.p2[k] : 0.0f);
            b.grow(q);
        }
    } else {
        b.grow(p.p0);
        b.grow(p.p1);
        b.grow(p.p2);
    }
    return b;
}

// Pad a box outward by an absolute epsilon = 1e-5 x the scene's coordinate magnitude, so the
// few-ulp rounding of the slab test ((lo - o) * inv, error ~1e-7 of the ray-box distance, itself
// bounded by the scene extent) and of the primitive tests can never cull a box whose primitives
// the exact test would hit. A box-local epsilon is not enough: the error scales with the distance
// from the ray origin, not with the box.
void pad(Aabb& b, float eps) {
    for (int k = 0; k < 3; ++k) {
        b.lo[k] -= eps;
        b.hi[k] += eps;
    }
}

struct Builder {
    std::vector<DevPrim>& prims;
    std::vector<Aabb> pb;        // per-prim bounds
    std::vector<float> cent;     // 3 per prim
    std::vector<uint32_t> idx;   // permutation
    std::vector<BvhNode>& nodes;
    uint32_t max_leaf;
    float eps = 0.0f;
    int bins = 64;  // SAH bins per axis (<= 64; C4: 16 -> 64 bins +9 %, C5 unchanged)

    void set_node(uint32_t ni, const Aabb& b, uint32_t first_or_left, uint32_t count) {
        Aabb p = b;
        pad(p, eps);
        BvhNode& n = nodes[ni];
        for (int k = 0; k < 3; ++k) {
            n.lo[k] = p.lo[k];
            n.hi[k] = p.hi[k];
        }
        n.lo[3] = u2f(first_or_left);
        n.hi[3] = u2f(count);
    }

    void build(uint32_t ni, uint32_t begin, uint32_t end, uint32_t depth) {
        Aabb bounds, cb;
        for (uint32_t i = begin; i < end; ++i) {
            bounds.grow(pb[idx[i]]);
            cb.grow(&cent[3 * idx[i]]);
        }
        const uint32_t count = end - begin;
        if (count <= max_leaf) {
            set_node(ni, bounds, begin, count);
            return;
        }
        if (depth >= kBvhMaxDepth) {
            // past the SAH depth cap: a leaf if it fits the traversal's 4-bit count, else halve the
            // index range (depth <= kBvhMaxDepth + log2(n / kBvhMaxLeaf) + 1 < 64 = the stack)
            if (count <= kBvhMaxLeaf) {
                set_node(ni, bounds, begin, count);
                return;
            }
            const uint32_t mid = begin + count / 2;
            const uint32_t left = uint32_t(nodes.size());
            nodes.emplace_back();
            nodes.emplace_back();
            set_node(ni, bounds, left, 0);
            build(left, begin, mid, depth + 1);
            build(left + 1, mid, end, depth + 1);
            return;
        }
        // binned SAH
        constexpr int kMaxBins = 64;
        const int kBins = bins;
        int best_axis = -1;
        int best_split = -1;
        double best_cost = std::numeric_limits<double>::infinity();
        for (int axis = 0; axis < 3; ++axis) {
            const float lo = cb.lo[axis], hi = cb.hi[axis];
            if (!(hi > lo)) continue;
            const double scale = kBins / (double(hi) - double(lo));
            Aabb bin_box[kMaxBins];
            uint32_t bin_cnt[kMaxBins] = {};
            for (uint32_t i = begin; i < end; ++i) {
                int bi = int((double(cent[3 * idx[i] + axis]) - lo) * scale);
                bi = std::min(std::max(bi, 0), kBins - 1);
                bin_cnt[bi]++;
                bin_box[bi].grow(pb[idx[i]]);
            }
            double left_area[kMaxBins];
            uint32_t left_cnt[kMaxBins];
            Aabb acc;
            uint32_t c = 0;
            for (int b = 0; b < kBins; ++b) {
                acc.grow(bin_box[b]);
                c += bin_cnt[b];
                left_area[b] = acc.area();
                left_cnt[b] = c;
            }
            Aabb racc;
            uint32_t rc = 0;
            for (int b = kBins - 1; b >= 1; --b) {
                racc.grow(bin_box[b]);
                rc += bin_cnt[b];
                const uint32_t lc = left_cnt[b - 1];
                if (lc == 0 || rc == 0) continue;
                const double cost = left_area[b - 1] * lc + racc.area() * rc;
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_split = b;
                }
            }
        }
        uint32_t mid;
        if (best_axis < 0) {
            // all centroids coincide: split in the middle of the index range
            mid = begin + count / 2;
        } else {
            const float lo = cb.lo[best_axis], hi = cb.hi[best_axis];
            const double scale = kBins / (double(hi) - double(lo));
            auto it = std::partition(idx.begin() + begin, idx.begin() + end, [&](uint32_t p) {
                int bi = int((double(cent[3 * p + best_axis]) - lo) * scale);
                bi = std::min(std::max(bi, 0), kBins - 1);
                return bi < best_split;
            });
            mid = uint32_t(it - idx.begin());
            if (mid == begin || mid == end) mid = begin + count / 2;
        }
        const uint32_t left = uint32_t(nodes.size());
        nodes.emplace_back();
        nodes.emplace_back();
        set_node(ni, bounds, left, 0);
        build(left, begin, mid, depth + 1);
        build(left + 1, mid, end, depth + 1);
    }
};

}  // namespace

void build_bvh(const spt_prim* in, std::vector<DevPrim>& prims, std::vector<BvhNode>& nodes,
               uint32_t max_leaf, uint32_t bins) {
    const uint32_t n = uint32_t(prims.size());
    nodes.clear();
    nodes.reserve(2 * size_t(n) + 1);
    Builder b{prims, {}, {}, {}, nodes, max_leaf};
    if (bins >= 2 && bins <= 64) b.bins = (int)bins;  // spt_tuning (measurement runs)
    b.pb.resize(n);
    b.cent.resize(3 * size_t(n));
    b.idx.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        b.pb[i] = prim_bounds(in[i]);
        for (int k = 0; k < 3; ++k) b.cent[3 * i + k] = 0.5f * (b.pb[i].lo[k] + b.pb[i].hi[k]);
        b.idx[i] = i;
    }
    float mag = 1.0f;
    for (uint32_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) mag = std::max({mag, std::fabs(b.pb[i].lo[k]), std::fabs(b.pb[i].hi[k])});
    b.eps = mag * 1e-5f;
    nodes.emplace_back();
    nodes.emplace_back();  // pad: child pairs start at even indices (64-B aligned)
    if (n == 0) {
        nodes[0] = BvhNode{};
        nodes[0].lo[3] = u2f(0);
        nodes[0].hi[3] = u2f(0);
        for (int k = 0; k < 3; ++k) {
            nodes[0].lo[k] = 1.0f;
            nodes[0].hi[k] = -1.0f;
        }
        return;
    }
    b.build(0, 0, n, 0);
    std::vector<DevPrim> reordered(n);
    for (uint32_t i = 0; i < n; ++i) reordered[i] = prims[b.idx[i]];
    prims.swap(reordered);
}

void refit_bvh(const spt_prim* in, uint32_t n, const std::vector<DevPrim>& prims, std::vector<BvhNode>& nodes) {
    if (n == 0 || nodes.empty()) return;
    float mag = 1.0f;  // the padding of build_bvh, from the edited scene's coordinate magnitude
    for (uint32_t i = 0; i < n; ++i) {
        const Aabb b = prim_bounds(in[i]);
        for (int k = 0; k < 3; ++k) mag = std::max({mag, std::fabs(b.lo[k]), std::fabs(b.hi[k])});
    }
    const float eps = mag * 1e-5f;
    // children are allocated after their parent (build_bvh), so one reverse pass is bottom-up; node 1
    // is the alignment pad, never referenced
    for (size_t i = nodes.size(); i-- > 0;) {
        if (i == 1) continue;
        BvhNode& nd = nodes[i];
        const uint32_t first = f2u(nd.lo[3]), count = f2u(nd.hi[3]);
        Aabb b;
        if (count > 0) {
            for (uint32_t j = first; j < first + count; ++j) b.grow(prim_bounds(in[f2u(prims[j].b[3])]));
            pad(b, eps);
        } else {  // union of the padded children = the padded union (the same eps on every side)
            for (uint32_t c = first; c < first + 2u; ++c) {
                b.grow(nodes[c].lo);
                b.grow(nodes[c].hi);
            }
        }
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = b.lo[k];
            nd.hi[k] = b.hi[k];
        }
    }
}

}  // namespace spt

namespace spt {

// ------------------------------------------------------------------------------------------------
// W-wide collapse of the binary BVH (W = 4 or 8)
// ------------------------------------------------------------------------------------------------
namespace {

float node_area(const BvhNode& n) {
    const float dx = n.hi[0] - n.lo[0], dy = n.hi[1] - n.lo[1], dz = n.hi[2] - n.lo[2];
    return dx * dy + dy * dz + dz * dx;
}

uint32_t node_count(const BvhNode& n) { return f2u(n.hi[3]); }
uint32_t node_first(const BvhNode& n) { return f2u(n.lo[3]); }

template <int W>
uint32_t collapse(const std::vector<BvhNode>& bin, uint32_t b, std::vector<BvhNodeW<W>>& out) {
    // children of binary interior node b, opened up to W (largest interior child first)
    uint32_t kids[W] = {node_first(bin[b]), node_first(bin[b]) + 1};
    uint32_t nk = 2;
    while (nk < (uint32_t)W) {
        int best = -1;
        float best_area = -1.0f;
        for (uint32_t i = 0; i < nk; ++i)
            if (node_count(bin[kids[i]]) == 0 && node_area(bin[kids[i]]) > best_area) {
                best_area = node_area(bin[kids[i]]);
                best = int(i);
            }
        if (best < 0) break;
        const uint32_t c = kids[best];
        kids[best] = node_first(bin[c]);
        kids[nk++] = node_first(bin[c]) + 1;
    }
    const uint32_t me = uint32_t(out.size());
    out.emplace_back();
    for (uint32_t i = 0; i < (uint32_t)W; ++i) {
        BvhNodeW<W>& n = out[me];
        if (i >= nk) {
            n.ref[i] = kRefEmpty;
            n.lo_x[i] = n.lo_y[i] = n.lo_z[i] = 0.0f;
            n.hi_x[i] = n.hi_y[i] = n.hi_z[i] = 0.0f;
            continue;
        }
        const BvhNode& c = bin[kids[i]];
        n.lo_x[i] = c.lo[0];
        n.lo_y[i] = c.lo[1];
        n.lo_z[i] = c.lo[2];
        n.hi_x[i] = c.hi[0];
        n.hi_y[i] = c.hi[1];
        n.hi_z[i] = c.hi[2];
        n.ref[i] = node_count(c) > 0 ? (node_first(c) << 4 | node_count(c)) : 0u;  // interior: set below
    }
    for (uint32_t i = 0; i < nk; ++i) {
        const BvhNode& c = bin[kids[i]];
        if (node_count(c) == 0) {
            const uint32_t child = collapse<W>(bin, kids[i], out);  // may reallocate `out`
            out[me].ref[i] = child << 4;
        }
    }
    return me;
}

// Exponent e (2^e normal) of an axis with child bounds in [mn, mx]: the smallest e for which
// the span fits 8 bits and the origin's multiple of 2^e stays below 2^24 - 255.
int quant_exponent(float mn, float mx) {
    int e = -126;  // start a little below the answer: the span and magnitude bound it from below
    const double span = (double)mx - (double)mn;
    if (span > 0.0) e = std::max(e, (int)std::floor(std::log2(span / 255.0)) - 1);
    const double mag = std::max(std::fabs((double)mn), std::fabs((double)mx));
    if (mag > 0.0) e = std::max(e, (int)std::floor(std::log2(mag)) - 25);
    for (; e <= 127; ++e) {
        const double s = std::ldexp(1.0, -e);
        const double o = std::floor((double)mn * s);
        const double top = std::ceil((double)mx * s);
        if (top - o <= 255.0 && std::fabs(o) + 255.0 < 16777216.0) return e;
    }
    return 127;
}

// One axis of a W-wide node quantized: the origin and biased exponent, and each valid child's 8-bit
// lower (rounded down) and upper (rounded up) bound through put(j, ql, qh).
template <int W, class Put>
void quantize_axis(const BvhNodeW<W>& n, const float* lo, const float* hi, float& origin, uint32_t& ebias, Put put) {
    float mn = 0.0f, mx = 0.0f;
    bool any = false;
    for (int j = 0; j < W; ++j) {
        if (n.ref[j] == kRefEmpty) continue;
        mn = any ? std::min(mn, lo[j]) : lo[j];
        mx = any ? std::max(mx, hi[j]) : hi[j];
        any = true;
    }
    const int e = quant_exponent(mn, mx);
    const double s = std::ldexp(1.0, -e);
    const double o = std::floor((double)mn * s);
    origin = (float)std::ldexp(o, e);  // exact: |o| < 2^24
    ebias = (uint32_t)(e + 127);
    for (int j = 0; j < W; ++j) {
        if (n.ref[j] == kRefEmpty) continue;
        put(j, (uint32_t)(std::floor((double)lo[j] * s) - o), (uint32_t)(std::ceil((double)hi[j] * s) - o));
    }
}

float decode_q(uint32_t q, uint32_t ebias, float origin) {
    const uint32_t sbits = ebias << 23;
    float scale;
    std::memcpy(&scale, &sbits, 4);
    return std::fmaf((float)q, scale, origin);  // q * 2^e exact, the sum exact: fma == mul + add
}

}  // namespace

void quantize_bvh4(const std::vector<BvhNode4>& in, std::vector<BvhNodeQ>& out) {
    out.assign(in.size(), BvhNodeQ{});
    for (size_t k = 0; k < in.size(); ++k) {
        const BvhNode4& n = in[k];
        BvhNodeQ& q = out[k];
        const float* lo[3] = {n.lo_x, n.lo_y, n.lo_z};
        const float* hi[3] = {n.hi_x, n.hi_y, n.hi_z};
        q.exps = 0;
        for (int a = 0; a < 3; ++a) {
            uint32_t eb = 0;
            q.qlo[a] = q.qhi[a] = 0;
            quantize_axis<4>(n, lo[a], hi[a], q.origin[a], eb, [&](int j, uint32_t ql, uint32_t qh) {
                q.qlo[a] |= ql << (8 * j);
                q.qhi[a] |= qh << (8 * j);
            });
            q.exps |= eb << (8 * a);
        }
        for (int j = 0; j < 4; ++j) q.ref[j] = n.ref[j];
    }
}

void dequantize_child(const BvhNodeQ& n, int j, float lo[3], float hi[3]) {
    for (int a = 0; a < 3; ++a) {
        const uint32_t eb = (n.exps >> (8 * a)) & 0xffu;
        lo[a] = decode_q((n.qlo[a] >> (8 * j)) & 0xffu, eb, n.origin[a]);
        hi[a] = decode_q((n.qhi[a] >> (8 * j)) & 0xffu, eb, n.origin[a]);
    }
}

template <int W>
uint32_t bvh_w_stack_need(const std::vector<BvhNodeW<W>>& nodes, uint32_t i) {
    uint32_t valid = 0, below = 0;
    for (uint32_t r : nodes[i].ref) {
        if (r == kRefEmpty) continue;
        ++valid;
        if ((r & 15u) == 0u) below = std::max(below, bvh_w_stack_need<W>(nodes, r >> 4));
    }
    return (valid ? valid - 1u : 0u) + below;
}

template <int W>
uint32_t bvh_w_max_ref(const std::vector<BvhNodeW<W>>& nodes) {
    uint32_t m = 0;
    for (const BvhNodeW<W>& n : nodes)
        for (uint32_t r : n.ref)
            if (r != kRefEmpty) m = std::max(m, r);
    return m;
}

template <int W>
void collapse_bvh_w(const std::vector<BvhNode>& bin, std::vector<BvhNodeW<W>>& out) {
    out.clear();
    if (bin.empty()) return;
    out.reserve(bin.size() / (W / 2) + 1);
    if (node_count(bin[0]) > 0 || bin.size() < 4) {  // root is a leaf: one node holding it
        out.emplace_back();
        BvhNodeW<W>& n = out[0];
        for (uint32_t i = 0; i < (uint32_t)W; ++i) {
            n.ref[i] = kRefEmpty;
            n.lo_x[i] = n.lo_y[i] = n.lo_z[i] = 0.0f;
            n.hi_x[i] = n.hi_y[i] = n.hi_z[i] = 0.0f;
        }
        n.lo_x[0] = bin[0].lo[0]; n.lo_y[0] = bin[0].lo[1]; n.lo_z[0] = bin[0].lo[2];
        n.hi_x[0] = bin[0].hi[0]; n.hi_y[0] = bin[0].hi[1]; n.hi_z[0] = bin[0].hi[2];
        n.ref[0] = node_first(bin[0]) << 4 | node_count(bin[0]);
        return;
    }
    collapse<W>(bin, 0, out);
    // Breadth-first numbering: the root and the levels below it come first, so a kernel can keep
    // the top nodes in LDS by index range (k_paths); children still follow their parent (refit_bvh's
    // reverse pass relies on that), and every node's interior children stay contiguous.
    std::vector<uint32_t> order;
    order.reserve(out.size());
    order.push_back(0);
    for (size_t h = 0; h < order.size(); ++h)
        for (uint32_t r : out[order[h]].ref)
            if (r != kRefEmpty && (r & 15u) == 0u) order.push_back(r >> 4);
    std::vector<uint32_t> renum(out.size());
    for (uint32_t i = 0; i < (uint32_t)order.size(); ++i) renum[order[i]] = i;
    std::vector<BvhNodeW<W>> bfs(out.size());
    for (uint32_t i = 0; i < (uint32_t)order.size(); ++i) {
        bfs[i] = out[order[i]];
        for (uint32_t& r : bfs[i].ref)
            if (r != kRefEmpty && (r & 15u) == 0u) r = renum[r >> 4] << 4;
    }
    out.swap(bfs);
}

template void collapse_bvh_w<4>(const std::vector<BvhNode>&, std::vector<BvhNode4>&);
template uint32_t bvh_w_stack_need<4>(const std::vector<BvhNode4>&, uint32_t);
template uint32_t bvh_w_max_ref<4>(const std::vector<BvhNode4>&);

}  // namespace spt
