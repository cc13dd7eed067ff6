// scene.h — host-side scene preparation for libspt_hip.so (internal, not part of the C-ABI).
//
// Replaces the Embree scene build of CPUPathTracer::rebuild_scene
// (libs/render/src/engines/pathtracer/backends/cpu/CPUPathTracer.cpp:328-404): the caller's
// spt_prim records are turned into 64-byte device records with the per-primitive constants the
// intersectors need precomputed once, and (for large scenes) a binned-SAH BVH is built.
// All float arithmetic here is compiled with -ffp-contract=off; the oracle restates the same
// formulas (oracle/cpu_ref.c) so both sides intersect against bit-identical constants.
#pragma once

#include <cstdint>
#include <vector>

#include "spt.h"

namespace spt {

// Device primitive record: 4 x float4 = 64 B, loaded with scalar (uniform) or 16-B vector loads.
//   sphere  : a = (c.xyz, r)            b = c = 0           d = (0,0,0, meta)
//   quad    : a = (Q.xyz, D = n.Q)      b = (n = u x v, 0)  c = (A = v x w, axis)  d = (B = w x u, meta)
//             with w = n / (n.n); for hit point h: alpha = (h-Q).A, beta = (h-Q).B
//   triangle: a = (v0.xyz, 0)           b = (e1, 0)         c = (e2, 0)         d = (Ng = e1 x e2, meta)
// meta = type | material << 2 stored as raw bits in d.w; b.w = original index (tie-break key);
// c.w = type | (1 + the axis of an axis-aligned quad's normal, 0: general) << 2, as raw bits.
struct DevPrim {
    float a[4], b[4], c[4], d[4];
};
static_assert(sizeof(DevPrim) == 64, "DevPrim must be 64 bytes");

struct DevMaterial {
    float albedo[4];    // rgb, 0
    float emission[4];  // rgb, flag(1 if any emission component != 0)
};
static_assert(sizeof(DevMaterial) == 32, "DevMaterial must be 32 bytes");

// BVH node, 32 B: bounds + (first child | first prim, count). Leaves have count > 0.
//   lo = (min.xyz, left_or_first as bits), hi = (max.xyz, count as bits)
// Interior node: children are nodes[left] and nodes[left+1].
struct BvhNode {
    float lo[4];
    float hi[4];
};
static_assert(sizeof(BvhNode) == 32, "BvhNode must be 32 bytes");

constexpr uint32_t kMetaTypeBits = 2;

inline uint32_t meta_pack(uint32_t type, uint32_t material) { return type | (material << kMetaTypeBits); }

// Next-event estimation (SPT_FLAG_NEE): one record per sampled emitter, 80 B (spt_device.h
// light_sample): the quads and triangles whose material emits and whose area is nonzero, and every
// sphere whose material emits, in primitive order (oracle/cpu_ref.c restates the same formulas).
//   base = (Q | v0, 1 if triangle else 0 as bits)  e1 = (u | v1 - v0, area * n_emitters / pi)
//   e2 = (v | v2 - v0, 0)  nl = (cross(e1, e2) * (1 / sqrt(dot)), 0)  le = (emission, 0)
//   a sphere: base = (center, 2 as bits)  e1 = (r, 0, 0, 4 pi r^2 * n_emitters / pi)  e2 = nl = 0
struct DevEmitter {
    float base[4], e1[4], e2[4], nl[4], le[4];
};
static_assert(sizeof(DevEmitter) == 80, "DevEmitter must be 80 bytes");
constexpr float kInvPiF = 0.318309886183790671538f;  // 1 / pi (oracle: SPT_INV_PI_F)
void build_emitters(const spt_prim* prims, uint32_t n, const spt_material* mats, std::vector<DevEmitter>& out);

// Validates and precomputes device records. Returns false (with msg) on invalid input.
bool prepare_prims(const spt_prim* prims, uint32_t n, uint32_t n_mats, std::vector<DevPrim>& out,
                   const char** msg);
void prepare_materials(const spt_material* mats, uint32_t n, std::vector<DevMaterial>& out);

// Whether the flat closest-hit loop may use its unscaled-division fast path (spt_device.h div_ref,
// isect_sphere_fast, isect_quad_axis_fast): every primitive's points within 2^28 of the origin in
// each coordinate (sphere: |center| + radius; quad: |Q| + |u| + |v|; triangle: its vertices).
// `dp` are the prims prepared from them.
bool fast_division_ok(const spt_prim* prims, uint32_t n, const std::vector<DevPrim>& dp);

// The flat fast path's kind-major copy (spt_kernels.hip closest_flat): the prepared primitives
// stably grouped as spheres | quads with normal +-x | +-y | +-z | other quads | triangles, so the
// device tests each group in a loop of its own with no per-primitive type dispatch. ends[g] is the
// end offset of group g (the triangles end at n). Each record keeps its original index in b.w, the
// tie-break key, which makes the closest hit independent of the order the groups are tested in.
constexpr uint32_t kFlatKinds = 6;
uint32_t flat_kind(const DevPrim& p);
void sort_flat_by_kind(const std::vector<DevPrim>& dp, std::vector<DevPrim>& sorted, uint32_t ends[kFlatKinds - 1]);
// Bit AX (0..2) set when the axis-AX group of the kind-major copy is non-empty and every quad in it is a
// rectangle along the in-plane axes (the wall of a box: the two edge-basis products the device's short
// form drops are exactly zero). Part of the flat shape key (spt_kernels.h flat_shape_key).
uint32_t flat_rect_bits(const std::vector<DevPrim>& sorted, const uint32_t ends[kFlatKinds - 1]);

// Binned-SAH BVH over the prepared primitives. Reorders `prims` into leaf order.
// Boxes are padded outward by 1e-5 of the scene's coordinate magnitude, so the (rounded) slab test
// never culls a primitive whose exact intersection test would accept the ray.
// `in` are the caller's records that `prims` was prepared from (bounds come from them).
// SAH splits stop at depth kBvhMaxDepth; deeper subtrees are halved by index until their leaves hold
// at most kBvhMaxLeaf primitives (the traversal packs (first, count) as first << 4 | count), so the
// depth stays < 64, the device's traversal stack. Node 0 is the root, node 1 padding; every child
// pair starts at an even index (64-B aligned). Primitive and node indices must be < 2^28.
// bins: SAH bins per axis (0 = the default 64; spt_tuning.bvh_bins, 2..64)
void build_bvh(const spt_prim* in, std::vector<DevPrim>& prims, std::vector<BvhNode>& nodes,
               uint32_t max_leaf = 4, uint32_t bins = 0);

// The leaf size the library builds with: SAH splits until a leaf holds at most this many
// primitives. Single-primitive leaves are fastest for C4 (82 K primitives: 7.27 vs 5.75 Gsamples/s
// with 4), two per leaf for C5 (1 M: 1.22 vs 1.11 with 1, 1.09 with 4): a 4-wide node tests 4 boxes
// in one traversal step, a leaf one primitive per step, and past ~256 K primitives the node array
// of single-primitive leaves outgrows the caches.
inline uint32_t bvh_max_leaf(uint32_t n_prims) { return n_prims <= (1u << 18) ? 1u : 2u; }

// W-wide BVH node (host form, fp32): the boxes of up to W children in SoA, their packed refs
// (first << 4 | count; count > 0: a leaf of primitives [first, first + count), count == 0: the node
// `first`), kRefEmpty for unused slots. Built by collapsing the binary BVH (children of the
// largest-area interior child are pulled up until W), so every child box is a box of the binary tree.
// The device traverses the quantized form of the 4-wide collapse (BvhNodeQ, 64 B); the 8-wide form was
// measured slower on every BVH configuration (round 5, profiles/r05_a_ab_bvh8.txt) and is not built.
template <int W>
struct BvhNodeW {
    float lo_x[W], lo_y[W], lo_z[W], hi_x[W], hi_y[W], hi_z[W];
    uint32_t ref[W];
};
using BvhNode4 = BvhNodeW<4>;
constexpr uint32_t kRefEmpty = 0xffffffffu;

template <int W>
void collapse_bvh_w(const std::vector<BvhNode>& bin, std::vector<BvhNodeW<W>>& out);
inline void collapse_bvh4(const std::vector<BvhNode>& bin, std::vector<BvhNode4>& out) { collapse_bvh_w<4>(bin, out); }
// The most entries a traversal stack of the W-wide tree below node i ever holds: a node pushes its
// hit children but the nearest (at most valid children - 1), and the entries of the ancestors of the
// node being visited are all that can be on the stack.
template <int W>
uint32_t bvh_w_stack_need(const std::vector<BvhNodeW<W>>& nodes, uint32_t i);
inline uint32_t bvh4_stack_need(const std::vector<BvhNode4>& nodes, uint32_t i) { return bvh_w_stack_need<4>(nodes, i); }
// The largest packed child ref (first << 4 | count) of a W-wide tree: what a 4-B traversal stack
// entry must hold above its entry-distance code (spt_kernels.h bvh_stack_t0_bits).
template <int W>
uint32_t bvh_w_max_ref(const std::vector<BvhNodeW<W>>& nodes);
inline uint32_t bvh4_max_ref(const std::vector<BvhNode4>& nodes) { return bvh_w_max_ref<4>(nodes); }

// Incremental edit (spt_update_prims): recompute every bound of `nodes` — a tree build_bvh made —
// bottom-up for the edited primitives `in` (original order; `prims` are the device records in leaf
// order, b.w = original index), keeping the topology. The padding follows build_bvh.
void refit_bvh(const spt_prim* in, uint32_t n, const std::vector<DevPrim>& prims, std::vector<BvhNode>& nodes);

// Quantized 4-wide node, 64 B (half a cache line): the children's boxes as 8-bit offsets from a
// per-node origin in units of a per-axis power of two. Decoding, origin + q * 2^e, is EXACT in
// fp32 (origin is a multiple of 2^e with |origin / 2^e| + 255 < 2^24), and the quantization rounds
// every lower bound down and every upper bound up, so each decoded box contains the (padded) box of
// the BvhNode4 it came from: the traversal visits a superset of nodes and finds the same hits.
//   origin[3] | exps: three biased exponents (e + 127, byte i = axis i)
//   qlo[3]: byte j = child j's lower bound on that axis; qhi[3] likewise (upper); pad[2]
//   ref[4]: as BvhNode4
struct BvhNodeQ {
    float origin[3];
    uint32_t exps;
    uint32_t qlo[3];
    uint32_t qhi[3];
    uint32_t pad[2];
    uint32_t ref[4];
};
static_assert(sizeof(BvhNodeQ) == 64, "BvhNodeQ must be 64 bytes");

void quantize_bvh4(const std::vector<BvhNode4>& in, std::vector<BvhNodeQ>& out);
// The decoded box of child j (what the device computes).
void dequantize_child(const BvhNodeQ& n, int j, float lo[3], float hi[3]);

// The most entries a traversal stack may hold (== spt_kernels.h kBvhStackEntries): spt_set_scene refuses
// a tree needing more (bvh_w_stack_need)
constexpr uint32_t kBvhStackMax = 96;

constexpr uint32_t kBvhMaxDepth = 31;
constexpr uint32_t kBvhMaxLeaf = 15;

// Scenes below this size are traced without a BVH (every ray tests every primitive; the records
// stay in the scalar cache as wave-uniform loads).
constexpr uint32_t kFlatSceneMax = 32;
static_assert(kFlatSceneMax < 64, "PassParams::flat_ends packs 6-bit offsets");

}  // namespace spt
