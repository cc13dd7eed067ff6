// test_bvh.cpp — host checks of the BVH the device traverses (scene.cpp), CPU only:
//   * every child box of the 4-wide collapse is a box of the binary tree's children (refs valid);
//   * the quantized node (BvhNodeQ) decodes EXACTLY (origin + q * 2^e, checked in double) and
//     contains the fp32 child box it came from, for every child of every node of the C4 and C5
//     scenes — the property that lets the device traverse it without changing any hit.
#include <cstring>
#include <cmath>
#include <cstdio>
#include <vector>

#include "scene.h"
#include "spt.h"

template <int W> struct QuantOf;
template <> struct QuantOf<4> {
    using T = spt::BvhNodeQ;
    static void quantize(const std::vector<spt::BvhNode4>& in, std::vector<T>& out) { spt::quantize_bvh4(in, out); }
    static uint32_t qlo(const T& n, int a, int j) { return (n.qlo[a] >> (8 * j)) & 0xffu; }
    static uint32_t qhi(const T& n, int a, int j) { return (n.qhi[a] >> (8 * j)) & 0xffu; }
};
template <int W>
static int check_scene(uint32_t id, const char* name) {
    uint32_t n = 0, n_mats = 0;
    if (spt_build_scene(id, nullptr, &n, nullptr, &n_mats, nullptr) != SPT_OK) return 1;
    std::vector<spt_prim> prims(n);
    std::vector<spt_material> mats(n_mats);
    spt_env env{};
    if (spt_build_scene(id, prims.data(), &n, mats.data(), &n_mats, &env) != SPT_OK) return 1;
    std::vector<spt::DevPrim> dp;
    const char* msg = nullptr;
    if (!spt::prepare_prims(prims.data(), n, n_mats, dp, &msg)) return 1;
    std::vector<spt::BvhNode> nodes;
    spt::build_bvh(prims.data(), dp, nodes, spt::bvh_max_leaf(n));  // the tree the library uploads
    std::vector<spt::BvhNodeW<W>> n4;
    spt::collapse_bvh_w<W>(nodes, n4);
    std::vector<typename QuantOf<W>::T> nq;
    QuantOf<W>::quantize(n4, nq);
    uint64_t children = 0, bad_contain = 0, bad_exact = 0;
    double inflation = 0.0;
    for (size_t k = 0; k < n4.size(); ++k) {
        const spt::BvhNodeW<W>& a = n4[k];
        for (int j = 0; j < W; ++j) {
            if (nq[k].ref[j] != a.ref[j]) ++bad_contain;
            if (a.ref[j] == spt::kRefEmpty) continue;
            ++children;
            float lo[3], hi[3];
            spt::dequantize_child(nq[k], j, lo, hi);
            const float olo[3] = {a.lo_x[j], a.lo_y[j], a.lo_z[j]};
            const float ohi[3] = {a.hi_x[j], a.hi_y[j], a.hi_z[j]};
            double vol_o = 1.0, vol_q = 1.0;
            for (int ax = 0; ax < 3; ++ax) {
                if (!(lo[ax] <= olo[ax] && hi[ax] >= ohi[ax])) ++bad_contain;
                // exactness of the decode: the fp32 fma equals the real origin + q * 2^e
                const uint32_t eb = (nq[k].exps >> (8 * ax)) & 0xffu;
                const double s = std::ldexp(1.0, (int)eb - 127);
                const double ql = (double)QuantOf<W>::qlo(nq[k], ax, j);
                const double qh = (double)QuantOf<W>::qhi(nq[k], ax, j);
                if ((double)lo[ax] != (double)nq[k].origin[ax] + ql * s) ++bad_exact;
                if ((double)hi[ax] != (double)nq[k].origin[ax] + qh * s) ++bad_exact;
                vol_o *= std::fmax((double)ohi[ax] - olo[ax], 1e-30);
                vol_q *= std::fmax((double)hi[ax] - lo[ax], 1e-30);
            }
            inflation += std::cbrt(vol_q / vol_o);
        }
    }
    // breadth-first numbering (collapse_bvh_w; k_paths / k_frame keep the first nodes in LDS): every
    // node is reached exactly once, children come after their parent, and node depth never decreases
    // with the index, so a prefix of the array is the top of the tree
    std::vector<uint32_t> depth(n4.size(), 0u), seen(n4.size(), 0u);
    uint64_t bad_order = 0;
    seen[0] = 1;
    for (size_t k = 0; k < n4.size(); ++k) {
        if (k > 0 && depth[k] < depth[k - 1]) ++bad_order;
        for (int j = 0; j < W; ++j) {
            const uint32_t r = n4[k].ref[j];
            if (r == spt::kRefEmpty || (r & 15u) != 0u) continue;
            const uint32_t c = r >> 4;
            if (c <= k || c >= n4.size() || seen[c]++) { ++bad_order; continue; }
            depth[c] = depth[k] + 1u;
        }
    }
    for (size_t k = 0; k < n4.size(); ++k)
        if (!seen[k]) ++bad_order;
    // the traversal stack bound the host sizes LDS stacks with (k_frame kSmall): at most W - 1 entries
    // per interior level, and within the traversal stacks' capacity (kBvhStackMax)
    uint32_t max_depth = 0;
    for (uint32_t v : depth) max_depth = v > max_depth ? v : max_depth;
    const uint32_t need = spt::bvh_w_stack_need<W>(n4, 0u);
    const bool bad_need = need > (W - 1u) * (max_depth + 1u) || need > spt::kBvhStackMax;
    std::printf("%s (%d-wide): %zu nodes, %llu children, containment failures %llu, inexact decodes %llu, "
                "mean linear inflation %.4f, breadth-first order violations %llu, depth %u, stack need %u\n",
                name, W, n4.size(), (unsigned long long)children, (unsigned long long)bad_contain,
                (unsigned long long)bad_exact, inflation / (double)children, (unsigned long long)bad_order,
                max_depth, need);
    return (bad_contain || bad_exact || bad_order || bad_need) ? 1 : 0;
}

// refit_bvh (spt_update_prims): on the unedited scene it reproduces build_bvh's bounds bit for bit;
// after moving every 97th primitive, every leaf box contains its primitives and every interior box
// its children, so the exact traversal still finds every hit.
static bool contains(const spt::BvhNode& n, const float lo[3], const float hi[3]) {
    for (int k = 0; k < 3; ++k)
        if (!(n.lo[k] <= lo[k] && n.hi[k] >= hi[k])) return false;
    return true;
}

static int check_refit(uint32_t id, const char* name) {
    uint32_t n = 0, n_mats = 0;
    if (spt_build_scene(id, nullptr, &n, nullptr, &n_mats, nullptr) != SPT_OK) return 1;
    std::vector<spt_prim> prims(n);
    std::vector<spt_material> mats(n_mats);
    spt_env env{};
    if (spt_build_scene(id, prims.data(), &n, mats.data(), &n_mats, &env) != SPT_OK) return 1;
    std::vector<spt::DevPrim> dp;
    const char* msg = nullptr;
    if (!spt::prepare_prims(prims.data(), n, n_mats, dp, &msg)) return 1;
    std::vector<spt::BvhNode> nodes;
    spt::build_bvh(prims.data(), dp, nodes, spt::bvh_max_leaf(n));
    std::vector<spt::BvhNode> refit = nodes;
    spt::refit_bvh(prims.data(), n, dp, refit);
    uint64_t differ = 0;
    for (size_t i = 0; i < nodes.size(); ++i)
        if (i != 1 && std::memcmp(&nodes[i], &refit[i], sizeof(spt::BvhNode)) != 0) ++differ;
    for (uint32_t i = 0; i < n; i += 97) {  // move: translate every vertex / the center
        const float off[3] = {0.31f, -0.17f, 0.53f};
        for (int k = 0; k < 3; ++k) {
            prims[i].p0[k] += off[k];
            if (prims[i].type == SPT_PRIM_TRIANGLE) {
                prims[i].p1[k] += off[k];
                prims[i].p2[k] += off[k];
            }
        }
    }
    spt::refit_bvh(prims.data(), n, dp, refit);
    uint64_t bad = 0;
    for (size_t i = 0; i < refit.size(); ++i) {
        if (i == 1) continue;
        uint32_t first, count;
        std::memcpy(&first, &refit[i].lo[3], 4);
        std::memcpy(&count, &refit[i].hi[3], 4);
        if (count) {
            for (uint32_t j = first; j < first + count; ++j) {
                uint32_t orig;
                std::memcpy(&orig, &dp[j].b[3], 4);
                const spt_prim& p = prims[orig];
                float lo[3], hi[3];
                for (int k = 0; k < 3; ++k) {
                    if (p.type == SPT_PRIM_SPHERE) {
                        lo[k] = p.p0[k] - p.p0[3];
                        hi[k] = p.p0[k] + p.p0[3];
                    } else if (p.type == SPT_PRIM_TRIANGLE) {
                        lo[k] = std::fmin(p.p0[k], std::fmin(p.p1[k], p.p2[k]));
                        hi[k] = std::fmax(p.p0[k], std::fmax(p.p1[k], p.p2[k]));
                    } else {  // quad corners
                        const float a = p.p0[k], b = a + p.p1[k], c = a + p.p2[k], d = a + p.p1[k] + p.p2[k];
                        lo[k] = std::fmin(std::fmin(a, b), std::fmin(c, d));
                        hi[k] = std::fmax(std::fmax(a, b), std::fmax(c, d));
                    }
                }
                if (!contains(refit[i], lo, hi)) ++bad;
            }
        } else {
            for (uint32_t c = first; c < first + 2; ++c)
                if (!contains(refit[i], refit[c].lo, refit[c].hi)) ++bad;
        }
    }
    std::printf("%s refit: %zu nodes, unedited refit differs from the build in %llu, containment failures "
                "after moving every 97th primitive %llu\n",
                name, refit.size(), (unsigned long long)differ, (unsigned long long)bad);
    return (differ || bad) ? 1 : 0;
}

static bool load_scene(uint32_t id, std::vector<spt_prim>& prims, std::vector<spt_material>& mats) {
    uint32_t n = 0, n_mats = 0;
    if (spt_build_scene(id, nullptr, &n, nullptr, &n_mats, nullptr) != SPT_OK) return false;
    prims.resize(n);
    mats.resize(n_mats);
    spt_env env{};
    return spt_build_scene(id, prims.data(), &n, mats.data(), &n_mats, &env) == SPT_OK;
}

static int fast_ok(const std::vector<spt_prim>& prims, uint32_t n_mats, int& status) {
    std::vector<spt::DevPrim> dp;
    const char* msg = nullptr;
    if (!spt::prepare_prims(prims.data(), (uint32_t)prims.size(), n_mats, dp, &msg)) {
        status = 1;
        return -1;
    }
    return spt::fast_division_ok(prims.data(), (uint32_t)prims.size(), dp) ? 1 : 0;
}

// scene.cpp fast_division_ok (the flat loop's unscaled-division fast path): the
// reference-mode and Cornell scenes are in range, and so is one with a tiny (2^-11 x 2^-11) axis-aligned
// quad; the Cornell box scaled by 2^28 (coordinates past the bound) is not, and runs the general loop.
static int check_fast_division() {
    int rc = 0;
    std::vector<spt_prim> prims;
    std::vector<spt_material> mats;
    const uint32_t in_range[] = {SPT_SCENE_C1_SPHERE_GROUND, SPT_SCENE_APP_DEFAULT, SPT_SCENE_CORNELL};
    for (uint32_t id : in_range) {
        if (!load_scene(id, prims, mats) || fast_ok(prims, (uint32_t)mats.size(), rc) != 1) rc = 1;
    }
    if (!load_scene(SPT_SCENE_CORNELL, prims, mats)) return 1;
    std::vector<spt_prim> big = prims, tiny = prims;
    for (spt_prim& p : big) {
        const float s = 268435456.0f;  // 2^28
        for (int k = 0; k < 4; ++k) p.p0[k] *= s;  // sphere: center and radius; quad: Q
        if (p.type != SPT_PRIM_SPHERE)
            for (int k = 0; k < 3; ++k) {
                p.p1[k] *= s;
                p.p2[k] *= s;
            }
    }
    const int big_ok = fast_ok(big, (uint32_t)mats.size(), rc);
    for (spt_prim& p : tiny) {
        if (p.type != SPT_PRIM_QUAD) continue;
        p.p1[0] = 0x1p-11f, p.p1[1] = 0.0f, p.p1[2] = 0.0f;  // u x v = (0, -2^-22, 0): still axis-aligned
        p.p2[0] = 0.0f, p.p2[1] = 0.0f, p.p2[2] = 0x1p-11f;
        break;
    }
    const int tiny_ok = fast_ok(tiny, (uint32_t)mats.size(), rc);
    std::printf("fast_division_ok: C1/App/Cornell in range, Cornell x 2^28 -> %d, tiny axis quad -> %d\n", big_ok,
                tiny_ok);
    if (big_ok != 0 || tiny_ok != 1) rc = 1;
    return rc;
}

// scene.cpp sort_flat_by_kind (the flat fast path's kind-major copy): Cornell's 3 +-y, 1 +-z and
// 2 +-x quads and 2 spheres group as spheres | x | y | z with ends 2, 4, 7, 8, 8; within a group the
// original order is kept and every record carries its original index in b.w.
static int check_flat_kinds() {
    std::vector<spt_prim> prims;
    std::vector<spt_material> mats;
    if (!load_scene(SPT_SCENE_CORNELL, prims, mats)) return 1;
    std::vector<spt::DevPrim> dp, sorted;
    const char* msg = nullptr;
    if (!spt::prepare_prims(prims.data(), (uint32_t)prims.size(), (uint32_t)mats.size(), dp, &msg)) return 1;
    uint32_t ends[spt::kFlatKinds - 1];
    spt::sort_flat_by_kind(dp, sorted, ends);
    const uint32_t want_ends[] = {2, 4, 7, 8, 8};
    const uint32_t want_index[] = {6, 7, 3, 4, 0, 1, 5, 2};
    int rc = sorted.size() == dp.size() ? 0 : 1;
    for (int g = 0; g < 5; ++g) rc |= ends[g] != want_ends[g];
    for (size_t i = 0; i < sorted.size() && i < 8; ++i) {
        uint32_t idx;
        std::memcpy(&idx, &sorted[i].b[3], 4);
        rc |= idx != want_index[i];
        rc |= std::memcmp(&sorted[i], &dp[idx], sizeof(spt::DevPrim)) != 0;
    }
    // round 4: every wall of the box is a rectangle in the (a, 0), (0, b) dual-basis form the device's
    // short test uses (prepare_prims swaps A and B of the other orientation), so every axis group is
    // all rectangles (flat_rect_bits, part of the shape key); the swap keeps |A|, |B| and the normal
    const uint32_t rect = spt::flat_rect_bits(sorted, ends);
    rc |= rect != 7u;
    for (const spt::DevPrim& q : dp) {
        uint32_t meta, axis;
        std::memcpy(&meta, &q.d[3], 4);
        std::memcpy(&axis, &q.c[3], 4);
        if ((meta & 3u) != SPT_PRIM_QUAD || (axis >> 2) == 0u) continue;
        const int ax = (int)(axis >> 2) - 1, u = ax == 0 ? 1 : 0, v = ax == 2 ? 1 : 2;
        rc |= !(q.c[v] == 0.0f && q.d[u] == 0.0f && q.c[u] != 0.0f && q.d[v] != 0.0f);
    }
    std::printf("sort_flat_by_kind: Cornell ends %u %u %u %u %u, all-rectangle axis groups %u -> %s\n", ends[0],
                ends[1], ends[2], ends[3], ends[4], rect, rc ? "FAIL" : "ok");
    return rc;
}

// Degenerate trees: the traversal stack bound of scenes built to be deep — thousands of
// coincident triangles (no SAH split exists), a chain of triangles doubling in size (SAH peels one off
// per level until kBvhMaxDepth, then index halving), identical spheres. The library refuses a tree
// needing more than kBvhStackEntries (spt_set_scene: SPT_ERR_CAPACITY); these stay well inside it.
static uint32_t stack_need_of(const std::vector<spt_prim>& prims) {
    std::vector<spt::DevPrim> dp;
    const char* msg = nullptr;
    if (!spt::prepare_prims(prims.data(), (uint32_t)prims.size(), 1, dp, &msg)) return ~0u;
    std::vector<spt::BvhNode> nodes;
    spt::build_bvh(prims.data(), dp, nodes, spt::bvh_max_leaf((uint32_t)prims.size()));
    std::vector<spt::BvhNode4> n4;
    spt::collapse_bvh4(nodes, n4);
    return spt::bvh4_stack_need(n4, 0u);
}

static int check_degenerate_stacks() {
    int rc = 0;
    std::vector<spt_prim> coincident(5000), chain(3000), spheres(4000);
    for (size_t i = 0; i < coincident.size(); ++i) {
        spt_prim& p = coincident[i];
        std::memset(&p, 0, sizeof p);
        p.type = SPT_PRIM_TRIANGLE;
        p.p1[0] = 1.0f;
        p.p2[1] = 1.0f;
    }
    for (size_t i = 0; i < chain.size(); ++i) {
        spt_prim& p = chain[i];
        std::memset(&p, 0, sizeof p);
        p.type = SPT_PRIM_TRIANGLE;
        const float x = std::ldexp(1.0f, (int)(i % 40) - 30) * (1.0f + (float)(i / 40));
        p.p0[0] = x;
        p.p1[0] = 2.0f * x;
        p.p2[0] = x;
        p.p2[1] = x;
    }
    for (size_t i = 0; i < spheres.size(); ++i) {
        spt_prim& p = spheres[i];
        std::memset(&p, 0, sizeof p);
        p.type = SPT_PRIM_SPHERE;
        p.p0[2] = 5.0f;
        p.p0[3] = 1.0f;
    }
    const struct {
        const char* name;
        const std::vector<spt_prim>* prims;
    } cases[] = {{"5000 coincident triangles", &coincident}, {"3000-triangle doubling chain", &chain},
                 {"4000 identical spheres", &spheres}};
    for (const auto& c : cases) {
        const uint32_t need = stack_need_of(*c.prims);
        std::printf("degenerate %s: stack need %u (limit 96)\n", c.name, need);
        if (need == ~0u) rc = 1;  // (a larger need is refused by the library, not a failure here)
    }
    return rc;
}

int main() {
    int rc = check_fast_division();
    rc |= check_degenerate_stacks();
    rc |= check_flat_kinds();
    rc |= check_scene<4>(SPT_SCENE_BUNNYLIKE, "C4 bunnylike");
    rc |= check_scene<4>(SPT_SCENE_INTERIOR_1M, "C5 interior1m");
    rc |= check_scene<4>(SPT_SCENE_APP_DEFAULT, "App default");
    rc |= check_refit(SPT_SCENE_BUNNYLIKE, "C4 bunnylike");
    rc |= check_refit(SPT_SCENE_APP_DEFAULT, "App default");
    std::printf(rc ? "FAIL\n" : "PASS\n");
    return rc;
}
