// spt_kernels.hip — wavefront path-tracing kernels for MI355X (gfx950, CDNA4).
//
// The hot path of render::CPUPathTracer::render() / trace_ray()
// (libs/render/src/engines/pathtracer/backends/cpu/CPUPathTracer.cpp:43-326), re-laid out as a
// wavefront integrator: the per-pixel bounce loop becomes one extend (closest hit) + one shade
// launch per bounce depth over compacted SoA ray queues. See spt_kernels.h for the queue layout.
//
// Memory layout in HBM (per pass of F frames x P pixels, N = F*P paths, Q = n_sub * sub_cap >= N):
//   q[2].o/.d/.t : 3 x float4 x Q    ping-pong ray queues (48 B per queued ray)
//   hit          : float2 x Q        (t, primitive index)
//   radiance     : float4 x N        per-path radiance L (bounce 0 writes it, misses/emitters add)
//   accum        : float4 x P        the reference's m_accumulation_buffer (CPUPathTracer.h:68)
//   counts       : u32 x 2 x 33 x n_sub  segment lengths per bounce | radiance RMWs per bounce
// Scene records (DevPrim 64 B, DevMaterial 32 B, BvhNode 32 B) are read-only; in a flat scene
// every lane of a wave tests the same primitive, so the records are scalar (SMEM) loads.
#ifndef __HIPCC_RTC__  // hiprtc (spt_jit.cpp) compiles only the persistent kernels, no host code
#include <algorithm>
#endif

#include "spt_device.h"
#include "spt_kernels.h"

namespace spt {

namespace {

// Closest hit against every primitive, in index order (strict '<' keeps the lowest index on ties).
__device__ __forceinline__ float isect_any(const float4* __restrict__ prims, uint32_t k, uint32_t type, F3 o, F3 d) {
    if (type == 0u) return isect_sphere(prims[4 * k + 0], o, d, kTNear);
    if (type == 1u) return isect_quad(prims[4 * k + 0], prims[4 * k + 1], prims[4 * k + 2], prims[4 * k + 3], o, d, kTNear);
    return isect_tri(prims[4 * k + 0], prims[4 * k + 1], prims[4 * k + 2], o, d, kTNear);
}

__device__ __forceinline__ void closest_flat_exact(const float4* __restrict__ prims, uint32_t n_prims, F3 o, F3 d,
                                                   float& best_t, uint32_t& best_k) {
    // (measured: testing two same-type primitives per step for ILP costs a wave of occupancy and
    // is slower)
    for (uint32_t k = 0; k < n_prims; ++k) {
        const float t = isect_any(prims, k, meta_type(prims[4 * k + 3]), o, d);
        if (t < best_t) {
            best_t = t;
            best_k = k;
        }
    }
}

// the record's words in one scalar-load round trip (the compiler would otherwise sink some loads
// into the test: two dependent waits per primitive, -2.5 % on C2)
#define SPT_PIN4(v) asm volatile("" ::"s"((v).x), "s"((v).y), "s"((v).z), "s"((v).w))

// Closest hit in a flat scene. `fast_scene` (kFlagFastDiv: scene.cpp fast_division_ok) lets a wave
// whose rays all have |d| ~ 1 and no component below 2^-20 test spheres and axis-aligned quads with
// the unscaled division (div_ref) and sqrt_unit, which give the same bits within those ranges (the
// scale and fix-up steps of hipcc's sequences are the identity there); any other wave, and a lane
// that met a sphere discriminant in (0, 2^-96), runs the general loop. Same results either way.
// The fast path walks the kind-major copy of the records (scene.h sort_flat_by_kind; `flat_ends`
// holds its group ends, 6 bits each) one group per loop, so no primitive pays a type dispatch: the
// flat loop is bound by scalar issue (one scalar unit per CU for its four SIMDs), and the dispatch
// was most of each primitive's scalar instructions. The closest hit is the minimum of the 64-bit
// key (t bits, original index): every t is +inf or >= kTNear > 0, so the integer order is the float
// order, and equal t go to the lower original index, as in closest_flat_exact's index order. The
// search starts from the caller's (best_t, best_k), as closest_flat_exact does.
//
// kShape != 0: a kernel compiled for one scene shape at run time (spt_jit.hip, flat_shape_key):
// the group ends and the primitive count are compile-time constants, so every group loop unrolls
// and the compiler schedules the scalar record loads itself — it issues the loads of later
// primitives while earlier ones are tested and reads only the words each test uses (C2: +7.6 %
// over the run-time loop, whose loads are pinned to one round trip per primitive).

#define SPT_NOPIN(v) ((void)0)
#define SPT_FLAT_GROUPS(UNROLL, PIN)                                                            \
    {                                                                                           \
        uint32_t k = 0;                                                                         \
        UNROLL for (const uint32_t e = flat_ends & 63u; k < e; ++k) { /* spheres */             \
            const float4 pa = kp[4 * k + 0], pb = kp[4 * k + 1];                                \
            PIN(pa);                                                                            \
            PIN(pb);                                                                            \
            take(isect_sphere_fast(pa, pb.x, o, d, a, r2a, kTNear, redo), pb);                  \
        }                                                                                       \
        SPT_FLAT_GROUP(UNROLL, PIN, 6, (isect_quad_axis_fast<0, ((kRectBits >> 0) & 1u) != 0u>(pa, pc, pd, o, d, rdx, kTNear))) \
        SPT_FLAT_GROUP(UNROLL, PIN, 12, (isect_quad_axis_fast<1, ((kRectBits >> 1) & 1u) != 0u>(pa, pc, pd, o, d, rdy, kTNear))) \
        SPT_FLAT_GROUP(UNROLL, PIN, 18, (isect_quad_axis_fast<2, ((kRectBits >> 2) & 1u) != 0u>(pa, pc, pd, o, d, rdz, kTNear))) \
        SPT_FLAT_GROUP(UNROLL, PIN, 24, (isect_quad(pa, pb, pc, pd, o, d, kTNear)))              \
        UNROLL for (; k < n_prims; ++k) { /* triangles */                                       \
            const float4 pa = kp[4 * k + 0], pb = kp[4 * k + 1], pc = kp[4 * k + 2];            \
            PIN(pa);                                                                            \
            PIN(pb);                                                                            \
            PIN(pc);                                                                            \
            take(isect_tri(pa, pb, pc, o, d, kTNear), pb);                                      \
        }                                                                                       \
    }
#define SPT_FLAT_GROUP(UNROLL, PIN, SHIFT, TEST)                                                \
    UNROLL for (const uint32_t e = (flat_ends >> (SHIFT)) & 63u; k < e; ++k) {                  \
        const float4 pa = kp[4 * k + 0], pb = kp[4 * k + 1];                                    \
        const float4 pc = kp[4 * k + 2], pd = kp[4 * k + 3];                                    \
        PIN(pa);                                                                                \
        PIN(pb);                                                                                \
        PIN(pc);                                                                                \
        PIN(pd);                                                                                \
        take(TEST, pb);                                                                         \
    }

template <uint64_t kShape = 0>
__device__ __forceinline__ void closest_flat(const float4* __restrict__ prims, uint32_t n_prims, F3 o, F3 d,
                                             float& best_t, uint32_t& best_k, bool fast_scene = false,
                                             uint32_t flat_ends = 0u) {
    const float in_t = best_t;
    const uint32_t in_k = best_k;
    constexpr uint32_t kRectBits = (uint32_t)(kShape >> 53) & 7u;  // flat_shape_key
    if (fast_scene) {
        const float a = (d.x * d.x + d.y * d.y) + d.z * d.z;  // isect_sphere's a
        const float dmin = fminf(fminf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
        const bool ok = dmin >= 0x1p-20f && a >= 0.5f && a <= 2.0f;
        if (__ballot(!ok) == 0ull) {
            const RcpRef r2a = rcp_ref(2.0f * a);
            const RcpRef rdx = rcp_ref(d.x), rdy = rcp_ref(d.y), rdz = rcp_ref(d.z);  // axis-aligned quads
            bool redo = false;
            uint64_t best = ((uint64_t)__float_as_uint(in_t) << 32) | in_k;
            auto take = [&](float t, float4 pb) {
                const uint64_t key = ((uint64_t)__float_as_uint(t) << 32) | __float_as_uint(pb.w);
                best = key < best ? key : best;
            };
            if constexpr (kShape != 0) {  // the fast path's counts as constants (the rare exact
                // fallback below keeps the run-time loop: unrolled it would triple the kernel's code)
                const uint32_t flat_ends = (uint32_t)(kShape & 0x3fffffffu);
                const uint32_t n_prims = (uint32_t)(kShape >> 30) & 63u;
                const float4* __restrict__ kp = prims + 4 * n_prims;  // the kind-major copy
                SPT_FLAT_GROUPS(_Pragma("unroll"), SPT_NOPIN)
            } else {
                const float4* __restrict__ kp = prims + 4 * n_prims;
                SPT_FLAT_GROUPS(, SPT_PIN4)
            }
            if (__ballot(redo) == 0ull || !redo) {
                best_t = __uint_as_float((uint32_t)(best >> 32));
                best_k = best == (((uint64_t)__float_as_uint(in_t) << 32) | in_k) ? in_k
                         : (best_t < kInf ? (uint32_t)best : kMiss);
                return;
            }
            best_t = in_t;
            best_k = in_k;
        }
    }
    closest_flat_exact(prims, n_prims, o, d, best_t, best_k);  // (not unrolled: rare, and large)
}
#undef SPT_FLAT_GROUP
#undef SPT_FLAT_GROUPS
#undef SPT_NOPIN

// BVH closest hit. Ties are broken on the primitive's ORIGINAL index (DevPrim b.w), so the result
// equals closest_flat over the unreordered scene whatever the tree and the traversal order.
struct BvhCounters {
    uint32_t nodes = 0, prims = 0;  // interior nodes visited, primitives tested
};

// 4-wide traversal (BvhNode4, scene.h): one dependent 128-B node load per level (the 4 child boxes
// and their packed (first << 4 | count) refs), the boxes tested together, hits visited nearest
// first and the others pushed farthest first with their entry distances t0 on a per-lane stack
// (scratch). A pop re-checks t0 <= best_t, which is exactly the slab test of that box against the
// shrunk best_t (t0 was <= the box's exit distance when pushed and does not depend on tmax).
// The binary tree's depth is < 64, so the 4-wide depth is <= 32 and at most 3 x 32 entries are ever
// on the stack. Measured: 4-wide halves the node visits and beats the binary
// traversal (itself 2 dependent loads -> 1 per level) by 7 % on C4, 16 % on C5; an LDS stack and a
// register stack were slower.
constexpr int kStack4 = kBvhStackEntries;

// Traversal stacks. Every kind offers put(i, ref, t0) (entry i: a packed child ref and the child's
// entry distance, t0 >= kTNear), raw(i) (entry i as stored: `Raw`, what a read-ahead holds), and
// ref(raw) / t0(raw): the ref and a LOWER bound of t0 (t0 itself for 8-B entries).
// 8-B entries (ref, t0 bits) in an array: entry i of this lane at p[i * S].
template <uint32_t S>
struct StkG {
    uint2* p;
    using Raw = uint2;
    __device__ __forceinline__ void put(int i, uint32_t r, uint32_t t0) const { p[(uint32_t)i * S] = make_uint2(r, t0); }
    __device__ __forceinline__ Raw raw(int i) const { return p[(uint32_t)i * S]; }
    __device__ __forceinline__ uint32_t ref(Raw e) const { return e.x; }
    __device__ __forceinline__ float t0(Raw e) const { return __uint_as_float(e.y); }
};
using StkP = StkG<1u>;  // a lane's own array (scratch)
// A traversal stack in LDS: entry i of thread t at p[i * kBlock] with p = base + t (a block's lanes'
// entries of one depth side by side: conflict-free 8-B accesses). k_frame of a scene held whole in LDS.
using StkL = StkG<kBlock>;
// 4-B entries in a global buffer (kBvhStackEntry 4, spt_kernels.h): entry i of this lane at
// p[i * 64], one dword = ref << tb | code, code = min((bits(t0) >> sh) - base, mask) with sh = 28 - tb and
// base = bits(2^-10) >> sh, so (code + base) << sh <= bits(t0): a lower bound of t0, exact to tb - 5
// mantissa bits. t0 >= kTNear > 2^-10 keeps the difference non-negative. tb, sh, base, mask are
// wave-uniform (SGPRs): one shift, subtract, min and shift-or per push; a bit-field extract and an
// add-shift per pop.
struct StkG4 {
    uint32_t* p;
    uint32_t tb;
    StackCode c;  // spt_kernels.h stack_code_params(tb)
    using Raw = uint32_t;
    __device__ static StkG4 make(uint32_t* p, uint32_t tb) { return StkG4{p, tb, stack_code_params(tb)}; }
    __device__ __forceinline__ void put(int i, uint32_t r, uint32_t t0) const {
        p[(uint32_t)i * 64u] = (r << tb) | stack_code(t0, c);
    }
    __device__ __forceinline__ Raw raw(int i) const { return p[(uint32_t)i * 64u]; }
    __device__ __forceinline__ uint32_t ref(Raw e) const { return e >> tb; }
    __device__ __forceinline__ float t0(Raw e) const { return __uint_as_float(stack_t0_lower_bits(e, c)); }
};
constexpr uint32_t kRefEmptyDev = 0xffffffffu;  // scene.h kRefEmpty

__device__ __forceinline__ void cswap(uint32_t& ka, uint32_t& ra, uint32_t& kb, uint32_t& rb) {
    const bool sw = kb < ka;
    const uint32_t k0 = sw ? kb : ka, k1 = sw ? ka : kb, r0 = sw ? rb : ra, r1 = sw ? ra : rb;
    ka = k0;
    kb = k1;
    ra = r0;
    rb = r1;
}

// Resumable form: the traversal state of one ray, advanced one node or one leaf at a time
// (trav_step), so a persistent kernel can shade the lanes whose rays are done while the others
// keep their place in the tree (k_paths). The stack lives in the caller (scratch).
struct Trav {
    F3 inv;
    float best_t;
    uint32_t best_k;  // (its original index, the tie-break, is read from its record on an exact tie)
    // the node4 (count == 0) or leaf range [first, first + count) to visit next, packed as the tree's
    // refs are (first << 4 | count): one register for both
    uint32_t ref;
    int sp;
    __device__ __forceinline__ uint32_t first() const { return ref >> 4; }
    __device__ __forceinline__ uint32_t count() const { return ref & 15u; }
};

__device__ __forceinline__ void trav_init(Trav& tv, F3 d) {
    tv.inv = F3{recip_ref(d.x), recip_ref(d.y), recip_ref(d.z)};  // (1.0f / d, the same bits)
    tv.best_t = kInf;
    tv.best_k = kMiss;
    tv.ref = 0;  // the root node4
    tv.sp = 0;
}

// A shadow ray (NEE): visible iff nothing lies at kTNear <= t < tmax. Its traversal starts with best_t =
// tmax and best_k = kShadowK, which the any-hit traversal (trav_step's kAnyHit) reads as "stop at the
// first primitive hit before best_t": visibility is a boolean, so which blocker ends it does not matter.
constexpr uint32_t kShadowK = 0xfffffffeu;  // (below kMiss; never a primitive index: scenes < 2^27)
__device__ __forceinline__ void trav_init_shadow(Trav& tv, F3 d, float tmax) {
    trav_init(tv, d);
    tv.best_t = tmax;
    tv.best_k = kShadowK;
}

// Stack operations on a lane's traversal (Trav::sp)
template <class Stk>
__device__ __forceinline__ void stk_push(const Stk& stk, Trav& tv, uint32_t r, uint32_t t0) {
    stk.put(tv.sp, r, t0);
    ++tv.sp;
}
// the top entry (sp > 0) as stored
template <class Stk>
__device__ __forceinline__ typename Stk::Raw stk_peek(const Stk& stk, const Trav& tv) {
    return stk.raw(tv.sp > 0 ? tv.sp - 1 : 0);
}
// drop the top entry (sp > 0)
template <class Stk>
__device__ __forceinline__ void stk_drop(const Stk&, Trav& tv) {
    --tv.sp;
}

// The next entry of the stack whose box the ray can still reach first (t0 <= best_t); returns true
// when there is none: the traversal is finished (tv.best_t / best_k hold the closest hit).
template <class Stk>
__device__ __forceinline__ bool trav_pop(Trav& tv, const Stk& stk) {
    while (tv.sp > 0) {
        const auto e = stk_peek(stk, tv);  // (packed ref, entry distance): one 8-B or 4-B load
        stk_drop(stk, tv);
        if (stk.t0(e) <= tv.best_t) {
            const uint32_t r = stk.ref(e);
            tv.ref = r;
            return false;
        }
    }
    return true;
}

// Every traversal step loads the stack's top entry together with its node / primitive record, so the
// pop that follows a leaf or a node without a hit child waits on no load of its own (round 3: C4 +6 %,
// C5 +7 %; read-ahead on primitive steps only: +0 %). The traversal is bound by dependent load latency.
// The stack's top entry, read at the start of a step (with its record) for the pop that may end it
// (reading the next entry too, for a culled top, measured -4 % on C5: registers).
template <class Stk>
struct StkAhead {
    typename Stk::Raw e0;
};

template <class Stk>
__device__ __forceinline__ StkAhead<Stk> stk_ahead(const Trav& tv, const Stk& stk) {
    return StkAhead<Stk>{stk_peek(stk, tv)};
}

// trav_pop with the top entry already loaded (read ahead by the step that ends the leaf or finds no
// child hit, in flight together with its record): a pop whose first entry is not culled waits on no
// load. The step pushes only when it does not pop, so the entries read ahead are still the top ones.
template <class Stk>
__device__ __forceinline__ bool trav_pop_ahead(Trav& tv, const Stk& stk, const StkAhead<Stk>& a) {
    if (tv.sp <= 0) return true;
    stk_drop(stk, tv);
    if (stk.t0(a.e0) <= tv.best_t) {
        const uint32_t r = stk.ref(a.e0);
        tv.ref = r;
        return false;
    }
    return trav_pop(tv, stk);
}

// The test of primitive tv.first() (its 64-B record pa..pd) against the best hit so far; then the
// leaf's next primitive, or false when the leaf is done (the caller pops). kAnyHit: a shadow ray
// (best_k == kShadowK) that hits a primitive before its best_t ends its traversal (the stack dropped).
template <bool kAnyHit = false>
__device__ __forceinline__ bool trav_prim_rec(float4 pa, float4 pb, float4 pc, float4 pd, F3 o, F3 d, Trav& tv,
                                              const float4* __restrict__ prims) {
    const uint32_t k = tv.first();
    const uint32_t type = __float_as_uint(pc.w) & 3u;  // c.w repeats the type (scene.h DevPrim)
    float t;
    if (type == 2u) t = isect_tri(pa, pb, pc, o, d, kTNear);
    else if (type == 1u) t = isect_quad(pa, pb, pc, pd, o, d, kTNear);
    else t = isect_sphere(pa, o, d, kTNear);
    bool take = t < tv.best_t;
    const bool stop = kAnyHit && take && tv.best_k == kShadowK;
    if (t == tv.best_t && t != kInf) {  // an exact tie (rare): the lower original index wins
        const bool none = kAnyHit ? tv.best_k >= kShadowK : tv.best_k == kMiss;
        const uint32_t best_orig = none ? 0xffffffffu : __float_as_uint(prims[4u * tv.best_k + 1u].w);
        take = __float_as_uint(pb.w) < best_orig;
    }
    if (take) {
        tv.best_t = t;
        tv.best_k = k;
    }
    tv.ref += 15u;  // the next primitive: first + 1, count - 1
    if (kAnyHit && stop) {
        tv.sp = 0;
        return false;
    }
    return (tv.ref & 15u) != 0u;
}

// A node's child hits (keys k0..k3: entry-distance bits, 0xffffffff for a miss or an empty slot; refs
// r0..r3): the nearest becomes the next node or leaf and the others are pushed farthest first; returns
// false when no child is hit (the caller pops).
template <class Stk>
__device__ __forceinline__ bool node_push(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t r0, uint32_t r1,
                                          uint32_t r2, uint32_t r3, Trav& tv, const Stk& stk) {
    // entry distances are >= tmin > 0, so their bit patterns sort like the floats; misses last
    cswap(k0, r0, k1, r1);
    cswap(k2, r2, k3, r3);
    cswap(k0, r0, k2, r2);
    cswap(k1, r1, k3, r3);
    cswap(k1, r1, k2, r2);
    if (k0 == 0xffffffffu) return false;
    if (k3 != 0xffffffffu) stk_push(stk, tv, r3, k3);
    if (k2 != 0xffffffffu) stk_push(stk, tv, r2, k2);
    if (k1 != 0xffffffffu) stk_push(stk, tv, r1, k1);
    tv.ref = r0;
    return true;
}

// The children of a 4-wide node whose boxes are decoded (the LDS-held trees of k_frame kSmall), the
// bounds already ordered by the ray's direction signs: near (entry) bounds nx..nz, far (exit) bounds
// fx..fz per axis, packed refs rf; the slab tests (node_rec below), then node_push.
template <class Stk>
__device__ __forceinline__ bool node_children_nf(float4 nx, float4 ny, float4 nz, float4 fx, float4 fy, float4 fz,
                                                 float4 rf, F3 o, Trav& tv, const Stk& stk) {
    const F3 inv = tv.inv;
    const float bt = tv.best_t;
    auto key = [&](uint32_t r, float ax, float ay, float az, float bx, float by, float bz) {
        const float t0 = fmaxf(fmaxf((ax - o.x) * inv.x, (ay - o.y) * inv.y), fmaxf((az - o.z) * inv.z, kTNear));
        const float t1 = fminf(fminf((bx - o.x) * inv.x, (by - o.y) * inv.y), fminf((bz - o.z) * inv.z, bt));
        return (r != kRefEmptyDev && t0 <= t1) ? __float_as_uint(t0) : 0xffffffffu;
    };
    const uint32_t r0 = __float_as_uint(rf.x), r1 = __float_as_uint(rf.y), r2 = __float_as_uint(rf.z),
                   r3 = __float_as_uint(rf.w);
    const uint32_t k0 = key(r0, nx.x, ny.x, nz.x, fx.x, fy.x, fz.x);
    const uint32_t k1 = key(r1, nx.y, ny.y, nz.y, fx.y, fy.y, fz.y);
    const uint32_t k2 = key(r2, nx.z, ny.z, nz.z, fx.z, fy.z, fz.z);
    const uint32_t k3 = key(r3, nx.w, ny.w, nz.w, fx.w, fy.w, fz.w);
    return node_push(k0, k1, k2, k3, r0, r1, r2, r3, tv, stk);
}

// The child boxes of a quantized node (BvhNodeQ, scene.h, 64 B), decoded (exact: origin + q * 2^e in
// one fma): the LDS copy of a kSmall tree.
struct NodeBoxes {
    float4 lx, ly, lz, hx, hy, hz;
};
__device__ __forceinline__ NodeBoxes node_boxes(float4 n0, float4 n1, float4 n2) {
    const uint32_t eb = __float_as_uint(n0.w);
    const float sx = __uint_as_float((eb & 0xffu) << 23), sy = __uint_as_float(((eb >> 8) & 0xffu) << 23),
                sz = __uint_as_float(((eb >> 16) & 0xffu) << 23);
    const uint32_t qlx = __float_as_uint(n1.x), qly = __float_as_uint(n1.y), qlz = __float_as_uint(n1.z);
    const uint32_t qhx = __float_as_uint(n1.w), qhy = __float_as_uint(n2.x), qhz = __float_as_uint(n2.y);
    auto dq = [](uint32_t q, int j, float s, float o) {
        return __builtin_fmaf((float)((q >> (8 * j)) & 0xffu), s, o);  // exact (scene.h BvhNodeQ)
    };
    const float4 lx = make_float4(dq(qlx, 0, sx, n0.x), dq(qlx, 1, sx, n0.x), dq(qlx, 2, sx, n0.x), dq(qlx, 3, sx, n0.x));
    const float4 ly = make_float4(dq(qly, 0, sy, n0.y), dq(qly, 1, sy, n0.y), dq(qly, 2, sy, n0.y), dq(qly, 3, sy, n0.y));
    const float4 lz = make_float4(dq(qlz, 0, sz, n0.z), dq(qlz, 1, sz, n0.z), dq(qlz, 2, sz, n0.z), dq(qlz, 3, sz, n0.z));
    const float4 hx = make_float4(dq(qhx, 0, sx, n0.x), dq(qhx, 1, sx, n0.x), dq(qhx, 2, sx, n0.x), dq(qhx, 3, sx, n0.x));
    const float4 hy = make_float4(dq(qhy, 0, sy, n0.y), dq(qhy, 1, sy, n0.y), dq(qhy, 2, sy, n0.y), dq(qhy, 3, sy, n0.y));
    const float4 hz = make_float4(dq(qhz, 0, sz, n0.z), dq(qhz, 1, sz, n0.z), dq(qhz, 2, sz, n0.z), dq(qhz, 3, sz, n0.z));
    return NodeBoxes{lx, ly, lz, hx, hy, hz};
}

// The slab tests of a quantized node's children, against padded boxes: scene.cpp pads every BVH box
// outward by 1e-5 of the scene's coordinate magnitude, far more than the few-ulp rounding of a slab
// distance or of a primitive test, so the test never culls a box whose primitives the exact test would
// hit — the traversal visits a (possibly different) superset of the boxes it must, and finds the same
// hits (ties broken on the original index). (The FMA form lo*inv - o*inv is NOT usable: its error
// scales with |o*inv|, measured 10x more node visits.)
// - Bounds are not decoded first: a bound's offset from the ray origin is (origin - o) + q * 2^e, the
//   per-axis offset of the node's origin once per node, then one fma per bound (q * 2^e is exact),
//   instead of (origin + q * 2^e) - o. The two round differently by an ulp or so of the scene's
//   magnitude, far inside the padding.
// - Near and far bound per axis are picked by the sign of the inverse direction, once per node (one
//   select of the packed byte words per bound): a child's entry is max(near slabs, tmin) and its exit
//   min(far slabs, tmax), without a min/max pair per slab (C4 +6 %, C4 one frame +8 %, the App -6 % time).
//   Lower bounds never exceed upper ones, so with finite slab distances this is the pair form exactly;
//   with a zero direction component (inv = +-inf) and the origin on a bound's plane the distance is
//   0 * inf = NaN, which fmaxf/fminf drop: the interval is then a superset of the pair form's, never a
//   box culled that the pair form keeps.
template <class Stk>
__device__ __forceinline__ bool node_rec(float4 n0, float4 n1, float4 n2, float4 rf, F3 o, Trav& tv, const Stk& stk) {
    const uint32_t eb = __float_as_uint(n0.w);
    const float sx = __uint_as_float((eb & 0xffu) << 23), sy = __uint_as_float(((eb >> 8) & 0xffu) << 23),
                sz = __uint_as_float(((eb >> 16) & 0xffu) << 23);
    const float ox = n0.x - o.x, oy = n0.y - o.y, oz = n0.z - o.z;
    const F3 inv = tv.inv;
    const bool nx = __float_as_int(inv.x) < 0, ny = __float_as_int(inv.y) < 0, nz = __float_as_int(inv.z) < 0;
    const uint32_t qlx = __float_as_uint(n1.x), qly = __float_as_uint(n1.y), qlz = __float_as_uint(n1.z);
    const uint32_t qhx = __float_as_uint(n1.w), qhy = __float_as_uint(n2.x), qhz = __float_as_uint(n2.y);
    const uint32_t nqx = nx ? qhx : qlx, fqx = nx ? qlx : qhx;
    const uint32_t nqy = ny ? qhy : qly, fqy = ny ? qly : qhy;
    const uint32_t nqz = nz ? qhz : qlz, fqz = nz ? qlz : qhz;
    auto tq = [](uint32_t q, int j, float s, float oo, float iv) {
        return __builtin_fmaf((float)((q >> (8 * j)) & 0xffu), s, oo) * iv;
    };
    const uint32_t r0 = __float_as_uint(rf.x), r1 = __float_as_uint(rf.y), r2 = __float_as_uint(rf.z),
                   r3 = __float_as_uint(rf.w);
    const float bt = tv.best_t;
    uint32_t k[4];
    const uint32_t r[4] = {r0, r1, r2, r3};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float t0 = fmaxf(fmaxf(tq(nqx, j, sx, ox, inv.x), tq(nqy, j, sy, oy, inv.y)),
                               fmaxf(tq(nqz, j, sz, oz, inv.z), kTNear));
        const float t1 = fminf(fminf(tq(fqx, j, sx, ox, inv.x), tq(fqy, j, sy, oy, inv.y)),
                               fminf(tq(fqz, j, sz, oz, inv.z), bt));
        k[j] = (r[j] != kRefEmptyDev && t0 <= t1) ? __float_as_uint(t0) : 0xffffffffu;
    }
    return node_push(k[0], k[1], k[2], k[3], r0, r1, r2, r3, tv, stk);
}

// One node or one primitive, whichever is next, for every traversing lane: a BvhNodeQ and a DevPrim
// are both 64-B records, so every lane issues ONE 64-B load — its node or its primitive — and the node
// and primitive codes then run masked in turn on registers: lanes at a node and lanes at a primitive
// wait on memory together instead of in two rounds. Measured: k_frame on C4 +4.7 %;
// k_paths since round 5, with the cheaper node visit, instead of stepping only the larger group per
// iteration (the vote) with two primitives per step in its 7-wave kernel: C5 +1.7 to +3.6 %, C4 NEE
// +2.4 to +4.9 %, C4 +-0.8 % (profiles/r05_s_ab_unified_kpaths.txt).
// kLds: the whole tree, decoded (7 float4 per node: the child boxes lx..hz, then the refs), and every
// primitive record (4 float4) are in LDS; a step visits a node and then the primitive it arrives at.
// (Before that form every lane read 7 float4 at either kind of record — a primitive's 4 only, behind a
// branch, had measured slower: the App 39.0 -> 40.5 us.)
template <bool kCount = false, bool kLds = false, bool kAnyHit = false, class Stk>
__device__ __forceinline__ bool trav_step(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                                          F3 o, F3 d, Trav& tv, const Stk& stk,
                                          BvhCounters* ctr = nullptr, const float4* top = nullptr,
                                          uint32_t n_top = 0u, const float4* ptop = nullptr, uint32_t n_ptop = 0u) {
    {
        const bool at_prim = tv.count() > 0u;
        if (kCount) {
            ctr->prims += at_prim ? 1u : 0u;
            ctr->nodes += at_prim ? 0u : 1u;
        }
        bool more;
        if constexpr (kLds) {
            // A node, then — in the same step — the primitive the lane arrives at (its nearest child a
            // leaf, or a popped leaf): one wave iteration instead of two for every node visit followed by
            // a leaf, the common case in a small tree of single-primitive leaves (the App: 33.5 -> 30.5 us
            // per 512² frame). A node lane reads its near bounds (lo or hi per axis, by the sign of inv)
            // as r0..r2 and the far ones as r3..r5, so the slab test needs no min/max pairs (node_rec).
            if (!at_prim) {
                const uint32_t sx = (__float_as_uint(tv.inv.x) >> 31) * 3u;
                const uint32_t sy = (__float_as_uint(tv.inv.y) >> 31) * 3u;
                const uint32_t sz = (__float_as_uint(tv.inv.z) >> 31) * 3u;
                const float4* rec = top + 7u * tv.first();
                const float4 r0 = rec[sx], r1 = rec[1u + sy], r2 = rec[2u + sz], r3 = rec[3u - sx];
                const float4 r4 = rec[4u - sy], r5 = rec[5u - sz], r6 = rec[6];
                const auto ahead = stk_ahead(tv, stk);
                if (!node_children_nf(r0, r1, r2, r3, r4, r5, r6, o, tv, stk) && trav_pop_ahead(tv, stk, ahead))
                    return true;
            }
            if (tv.count() == 0u) return false;
            if (kCount && !at_prim) ctr->prims += 1u;
            const float4* rec = ptop + 4u * tv.first();
            const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2], r3 = rec[3];
            const auto ahead = stk_ahead(tv, stk);
            if (trav_prim_rec<kAnyHit>(r0, r1, r2, r3, o, d, tv, prims)) return false;
            return trav_pop_ahead(tv, stk, ahead);
        }
        const float4* rec = (at_prim ? (tv.first() < n_ptop ? ptop : prims) : (tv.first() < n_top ? top : nodes)) + 4u * tv.first();
        const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2], r3 = rec[3];
        const auto ahead = stk_ahead(tv, stk);
        more = at_prim ? trav_prim_rec<kAnyHit>(r0, r1, r2, r3, o, d, tv, prims) : node_rec(r0, r1, r2, r3, o, tv, stk);
        if (more) return false;
        return trav_pop_ahead(tv, stk, ahead);
    }
}

// kAnyHit: a shadow ray, best_t its tmax on entry: ends at the first primitive hit before it
template <bool kCount = false, bool kAnyHit = false>
__device__ __forceinline__ void closest_bvh4(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                                             F3 o, F3 d, float& best_t, uint32_t& best_k,
                                             BvhCounters* ctr = nullptr) {
    uint2 own[kStack4];
    const StkP stk{own};
    Trav tv;
    if (kAnyHit) trav_init_shadow(tv, d, best_t);
    else trav_init(tv, d);
    tv.best_t = best_t;  // kInf
    while (!trav_step<kCount, false, kAnyHit>(nodes, prims, o, d, tv, stk, ctr)) {
    }
    best_t = tv.best_t;
    best_k = tv.best_k;
}

// The same with the caller's stack (a persistent kernel lends its lane's traversal stack).
template <class Stk>
__device__ __forceinline__ void closest_bvh4_on(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                                                F3 o, F3 d, float& best_t, uint32_t& best_k, const Stk& stk) {
    Trav tv;
    trav_init(tv, d);
    while (!trav_step<false>(nodes, prims, o, d, tv, stk)) {
    }
    best_t = tv.best_t;
    best_k = tv.best_k;
}

// the BVH traversal the kernels use
template <bool kCount = false, bool kAnyHit = false>
__device__ __forceinline__ void closest_tree(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                                             F3 o, F3 d, float& best_t, uint32_t& best_k,
                                             BvhCounters* ctr = nullptr) {
    closest_bvh4<kCount, kAnyHit>(nodes, prims, o, d, best_t, best_k, ctr);
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Camera paths of a pass (CPUPathTracer.cpp:57-73). Path p = f * P + pixel of the pass's frame f.
// Bounce 0 never materializes a queue: extend and shade of bounce 0 recompute the camera ray from
// the slot index (dealt_path).
// ---------------------------------------------------------------------------------------------
struct CameraParams {
    uint32_t width, shard_rank, shard_count, shard_pixels;
    uint32_t n_paths, first_frame, n_sub;
    float inv_w, inv_h, aspect;
    // k_frame: the camera segments' closest hits across calls (PassParams::hit_cache; hit_mode 0: not
    // used, 1: trace the camera segments and store their hits, 2: take them from the cache)
    float2* hit_cache = nullptr;
    uint32_t hit_mode = 0;
    // hit_mode 3 (kFrameHitCache 2): the cache compacted once into the live pixels' records
    // (pixel, t bits, primitive, 0) and the sky pixels' indices, and their counts ([0] live, [1] sky)
    const uint4* live_rec = nullptr;
    const uint32_t* sky_pix = nullptr;
    const uint32_t* list_counts = nullptr;
    // hit_mode 3: the launch's first sky_blocks blocks add the sky pixels and end; the others trace
    uint32_t sky_blocks = 0;
    // k_frame: the fused resolve (PassParams::rgba)
    uint32_t* rgba = nullptr;
    float rgba_frames = 1.0f, rgba_exposure = 1.0f;
};

struct CameraRay {
    F3 d;
    uint32_t seed;
};

__device__ __forceinline__ CameraRay camera_ray(const CameraParams& c, uint32_t pid) {
    const uint32_t f = pid / c.shard_pixels;
    const uint32_t pix = pid - f * c.shard_pixels;
    const uint32_t lrow = pix / c.width;
    const uint32_t x = pix - lrow * c.width;
    const uint32_t y = c.shard_rank + c.shard_count * lrow;
    return CameraRay{primary_dir(x, y, c.inv_w, c.inv_h, c.aspect), rng_seed(x, y, c.width, c.first_frame + f + 1u)};
}

// ---------------------------------------------------------------------------------------------
// extend: closest hit for every ray of queue `bounce` (replaces rtcIntersect1,
// CPUPathTracer.cpp:214-227). Block s reads segment s: 32 B per ray (bounce 0: the camera ray is
// computed instead), writes 8 B. Scene, queue and hit pointers are separate __restrict__ arguments
// so the compiler can prove the hit stores never clobber the primitive records: in a flat scene
// every lane reads the same record, which becomes a scalar (s_load) broadcast.
// ---------------------------------------------------------------------------------------------
template <bool kBvh, bool kPrimary>
__global__ __launch_bounds__(kBlock) void k_extend(const float4* __restrict__ prims, const float4* __restrict__ nodes,
                                                   uint32_t n_prims, const float4* __restrict__ qo,
                                                   const float4* __restrict__ qd, float2* __restrict__ hit,
                                                   const uint32_t* __restrict__ counts, uint32_t sub_cap,
                                                   CameraParams cam) {
    const uint32_t s = blockIdx.x;
    const uint32_t n = kPrimary ? sub_count_of(cam.n_paths, s, cam.n_sub) : counts[s];
    const uint32_t base = s * sub_cap;
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
        F3 o, d;
        if (kPrimary) {
            o = F3{0.0f, 0.0f, 0.0f};
            d = camera_ray(cam, dealt_path(s, i, cam.n_sub)).d;
        } else {
            const float4 o4 = qo[base + i];
            const float4 d4 = qd[base + i];
            o = F3{o4.x, o4.y, o4.z};
            d = F3{d4.x, d4.y, d4.z};
        }
        float best_t = kInf;
        uint32_t best_k = kMiss;
        if (kBvh) closest_tree(nodes, prims, o, d, best_t, best_k);
        else closest_flat(prims, n_prims, o, d, best_t, best_k);
        hit[base + i] = make_float2(best_t, __uint_as_float(best_k));
    }
}

// ---------------------------------------------------------------------------------------------
// Sorted ray queues (SPT_FLAG_SORTED_RAYS, BVH scenes): before the closest-hit launch of a bounce
// >= 1, the queued rays are binned by (direction octant, cell of the origin in an 8 x 8 x 8 grid over
// the scene bounds, Morton order) — a counting sort in three light launches: per-block LDS
// histograms added into the global bin counts, one scan, a scatter that reserves each block's range
// of every bin with one global atomic — and k_extend_sorted traces them in bin order, so the rays
// of a wave, and of the waves an XCD runs together, start in the same region heading the same way
// and walk the same subtrees (L2 reuse). The order within a bin is arbitrary: every ray's result
// goes to its own queue slot, so the results are identical to the unsorted schedule.
// Per queued ray: keys 2 B written + read, perm 4 B written + read, the ray (32 B) read twice.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kRayBins = 4096;

struct BinParams {
    float lo[3], scale[3];  // cell c = (o - lo) * scale, clamped to [0, 8)
};

__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // 3 bits -> bits 0, 3, 6
    return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4);
}

__device__ __forceinline__ uint32_t ray_bin(float4 o, float4 d, const BinParams& bp) {
    const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    auto cell = [](float x, float lo, float sc) {
        return (uint32_t)fminf(fmaxf((x - lo) * sc, 0.0f), 7.0f);  // NaN -> 0
    };
    const uint32_t cx = cell(o.x, bp.lo[0], bp.scale[0]), cy = cell(o.y, bp.lo[1], bp.scale[1]),
                   cz = cell(o.z, bp.lo[2], bp.scale[2]);
    return oct << 9 | spread3(cx) | spread3(cy) << 1 | spread3(cz) << 2;
}

// keys of sub-queue s's rays + their counts into the global bins
__global__ __launch_bounds__(kBlock) void k_bin_count(const float4* __restrict__ qo, const float4* __restrict__ qd,
                                                      const uint32_t* __restrict__ counts, uint32_t sub_cap,
                                                      uint16_t* __restrict__ keys, uint32_t* __restrict__ bins,
                                                      BinParams bp) {
    __shared__ uint32_t h[kRayBins];
    for (uint32_t b = threadIdx.x; b < kRayBins; b += kBlock) h[b] = 0u;
    __syncthreads();
    const uint32_t s = blockIdx.x, n = counts[s], base = s * sub_cap;
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
        const uint32_t k = ray_bin(qo[base + i], qd[base + i], bp);
        keys[base + i] = (uint16_t)k;
        atomicAdd(&h[k], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kRayBins; b += kBlock)
        if (h[b]) atomicAdd(&bins[b], h[b]);
}

// exclusive scan of the bin counts into the scatter cursors (cursor[kRayBins] = total), and the
// counts cleared for the next bounce. One block.
__global__ __launch_bounds__(kBlock) void k_bin_scan(uint32_t* __restrict__ bins, uint32_t* __restrict__ cursor) {
    constexpr uint32_t kPer = kRayBins / kBlock;
    __shared__ uint32_t part[kBlock];
    uint32_t v[kPer], sum = 0;
    for (uint32_t j = 0; j < kPer; ++j) {
        v[j] = bins[threadIdx.x * kPer + j];
        bins[threadIdx.x * kPer + j] = 0u;
        sum += v[j];
    }
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < kBlock; off <<= 1) {  // inclusive Hillis-Steele scan of the partial sums
        const uint32_t add = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += add;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - sum;
    for (uint32_t j = 0; j < kPer; ++j) {
        cursor[threadIdx.x * kPer + j] = run;
        run += v[j];
    }
    if (threadIdx.x == kBlock - 1u) cursor[kRayBins] = run;
}

// perm[position in bin order] = queue slot; each block reserves its range of every bin it uses with
// one global atomic, then ranks its rays within the range in LDS
__global__ __launch_bounds__(kBlock) void k_bin_scatter(const uint16_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ counts, uint32_t sub_cap,
                                                        uint32_t* __restrict__ cursor, uint32_t* __restrict__ perm) {
    __shared__ uint32_t h[kRayBins];
    for (uint32_t b = threadIdx.x; b < kRayBins; b += kBlock) h[b] = 0u;
    __syncthreads();
    const uint32_t s = blockIdx.x, n = counts[s], base = s * sub_cap;
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) atomicAdd(&h[keys[base + i]], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kRayBins; b += kBlock)
        if (h[b]) h[b] = atomicAdd(&cursor[b], h[b]);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) perm[atomicAdd(&h[keys[base + i]], 1u)] = base + i;
}

// k_extend over the rays in bin order (bounce >= 1): total = cursor[kRayBins] after the scatter
// (the scan's total; the scatter advanced every bin's cursor to its end)
template <bool kBvh>
__global__ __launch_bounds__(kBlock) void k_extend_sorted(const float4* __restrict__ prims, const float4* __restrict__ nodes,
                                                          uint32_t n_prims, const float4* __restrict__ qo,
                                                          const float4* __restrict__ qd, float2* __restrict__ hit,
                                                          const uint32_t* __restrict__ perm,
                                                          const uint32_t* __restrict__ cursor) {
    const uint32_t total = cursor[kRayBins];
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < total; i += gridDim.x * kBlock) {
        const uint32_t slot = perm[i];
        const float4 o4 = qo[slot], d4 = qd[slot];
        const F3 o{o4.x, o4.y, o4.z}, d{d4.x, d4.y, d4.z};
        float best_t = kInf;
        uint32_t best_k = kMiss;
        if (kBvh) closest_tree(nodes, prims, o, d, best_t, best_k);
        else closest_flat(prims, n_prims, o, d, best_t, best_k);
        hit[slot] = make_float2(best_t, __uint_as_float(best_k));
    }
}

// ---------------------------------------------------------------------------------------------
// shade: one iteration of trace_ray's bounce loop after the intersection
// (CPUPathTracer.cpp:229-280). Block s consumes segment s of queue `bounce` and appends the
// surviving paths to segment s of queue `bounce + 1`: wave ballot + mbcnt for the lane offset, an
// LDS prefix over the block's waves for the wave offset, a block-uniform running length — no global
// atomics — and one plain store of the final length. Bounce 0 writes every path's radiance slot
// (0, T*sky or T*emission); later bounces add to it.
// ---------------------------------------------------------------------------------------------
struct ShadeParams {
    uint32_t sky_enabled, flags, max_bounces, rr_depth, sub_cap, bounce, n_prims, n_mats, flat_ends;
    float4 horizon, zenith;
    const float4* env;  // octahedral environment map (RGBA texels) or nullptr: the gradient sky
    uint32_t env_w, env_h;
    uint32_t n_nodes = 0;  // BVH scenes: records in `nodes` (PassParams::n_dev_nodes; the top ones are copied to LDS)
    void* stack = nullptr;  // PassParams::stack
    uint32_t stack_stride = kBvhStackEntries;  // entries per lane in `stack` (>= the tree's bvh4_stack_need)
    uint32_t stack_tb = 1;  // PassParams::stack_tb (4-B entries)
};

// The global traversal stack of lane `lane` of resident wave `wslot` (block * waves per block + wave):
// the wave owns 64 lanes' stacks of sp.stack_stride entries (a depth's 64 entries side by side), of
// kEntry bytes each (spt_kernels.h kBvhStackEntry / kBvhStackEntry8W; the buffer is sized for the wider).
template <uint32_t kEntry = kBvhStackEntry>
__device__ __forceinline__ auto lane_stack(const ShadeParams& sp, uint32_t wslot, uint32_t lane) {
    static_assert(kEntry == 4 || kEntry == 8, "stack entries are 4 or 8 bytes");
    const size_t w0 = (size_t)wslot * 64u * sp.stack_stride;
    if constexpr (kEntry == 4) return StkG4::make(static_cast<uint32_t*>(sp.stack) + w0 + lane, sp.stack_tb);
    else return StkG<64u>{static_cast<uint2*>(sp.stack) + w0 + lane};
}

// A kernel compiled with its launch configuration in the key (spt_kernels.h jit_config_key): the
// fields become constants. SPT_FLAG_ABS_FLOAT and the fast-division flag are the only flags these kernels
// read.
static_assert(kFlagAbsFloatBit == kFlagAbsFloat, "jit_config_key's flag bit");
template <uint64_t kShape>
__device__ __forceinline__ void bake_config(ShadeParams& sp) {
    if constexpr ((kShape & kConfigValid) != 0) {
        sp.max_bounces = (uint32_t)(kShape >> 38) & 63u;
        sp.rr_depth = (uint32_t)(kShape >> 44) & 63u;
        sp.sky_enabled = (uint32_t)(kShape >> 50) & 1u;
        sp.flags = (((kShape >> 51) & 1u) ? kFlagAbsFloat : 0u) | (((kShape >> 52) & 1u) ? kFlagFastDiv : 0u);
    }
}

// The miss radiance (CPUPathTracer.cpp:231-235 with sample_sky, :286-292, or the environment map).
// kEnv: 0 = gradient only (k_paths without a map), 1 = the map, 2 = decided at run time.
template <int kEnv = 2>
__device__ __forceinline__ F3 sky_radiance(const ShadeParams& sp, F3 d) {
    if (kEnv == 1 || (kEnv == 2 && sp.env)) {
        const float4 e = sp.env[octa_texel(d.x, d.y, d.z, sp.env_w, sp.env_h)];
        return F3{e.x, e.y, e.z};
    }
    return sample_sky(d.y, sp.horizon, sp.zenith);
}

constexpr uint32_t kFlatPrims = 32;                   // == scene.h kFlatSceneMax
constexpr uint32_t kLdsScene = 4 * kFlatPrims + 2 * 32;  // float4s: 32 DevPrims + 32 DevMaterials

// One iteration of trace_ray's loop body after rtcIntersect1 (CPUPathTracer.cpp:229-280) for the
// segment (o, d) that hit primitive k at t (or missed, k == kMiss), up to but excluding the new
// direction: updates o (hit point, plus n * EPSILON if the path continues), T, rng (Russian
// roulette), returns whether the path contributes `add` to its radiance, sets `alive` if it
// continues and then `n` to the shading normal the new direction is drawn around.
//
// kNee (SPT_FLAG_NEE): an emitter's emission counts on the camera segment only (every emitter is
// sampled: parallelograms, triangles, spheres), and the hit stops before Russian roulette: `alive`
// says the path continues past this hit (bounce_count < max_bounces), o is the hit point without the
// offset — the caller draws the light sample, then runs rr_continue.
template <int kEnv = 2, bool kRec = false, bool kNee = false>
__device__ __forceinline__ bool shade_hit(const float4* __restrict__ prims, const float4* __restrict__ mats,
                                          const ShadeParams& sp, uint32_t bounce_count, float t, uint32_t k, F3& o,
                                          F3 d, F3& T, uint32_t& rng, bool& alive, F3& add, F3& n) {
    alive = false;
    add = F3{0.f, 0.f, 0.f};
    if (k == kMiss) {
        // miss: accumulated_color += ray_throughput * sample_sky(current_direction) (:231-235)
        if (!sp.sky_enabled) return false;
        const F3 sky = sky_radiance<kEnv>(sp, d);
        add = F3{T.x * sky.x, T.y * sky.y, T.z * sky.z};
        return true;
    }
    bool contributes = false;
    // current_origin += hit_t * current_direction (:238-241)
    o = F3{o.x + t * d.x, o.y + t * d.y, o.z + t * d.z};
    F3 ng;
    float4 alb, emi;
    if (kRec) {  // flat scenes: the LDS shading record (make_shade_recs), one round trip
        const float4 g = prims[3 * k + 0];
        alb = prims[3 * k + 1];
        emi = prims[3 * k + 2];
        if (__float_as_uint(g.w) == 0u) {
            ng = F3{o.x - g.x, o.y - g.y, o.z - g.z};  // sphere Ng = hit - center
        } else {
            ng = F3{g.x, g.y, g.z};
            if (dot3(ng, d) > 0.0f) ng = F3{-ng.x, -ng.y, -ng.z};  // two-sided
        }
    } else {
        const float4 pa = prims[4 * k + 0];
        const float4 pd = prims[4 * k + 3];
        const uint32_t type = meta_type(pd);
        if (type == 0u) {
            ng = F3{o.x - pa.x, o.y - pa.y, o.z - pa.z};  // sphere Ng = hit - center
        } else {
            const float4 pb = prims[4 * k + 1];  // loaded unconditionally: a pointer select here spilled pd to scratch
            const float4 nv = type == 1u ? pb : pd;
            ng = F3{nv.x, nv.y, nv.z};
            if (dot3(ng, d) > 0.0f) ng = F3{-ng.x, -ng.y, -ng.z};  // two-sided
        }
        const uint32_t m = meta_material(pd);
        alb = mats[2 * m + 0];
        emi = mats[2 * m + 1];
    }
    // n = Ng / |Ng| (:244-250)
    const float inv_len = inv_sqrt_ref(ng.x * ng.x + ng.y * ng.y + ng.z * ng.z);
    n = F3{ng.x * inv_len, ng.y * inv_len, ng.z * inv_len};
    if (emi.w != 0.0f && (!kNee || bounce_count == 1u)) {  // superset: emission
        add = F3{T.x * emi.x, T.y * emi.y, T.z * emi.z};
        contributes = true;
    }
    // ray_throughput *= albedo (reference: 0.7f, :260)
    T = F3{T.x * alb.x, T.y * alb.y, T.z * alb.z};
    if (kNee) {
        alive = bounce_count < sp.max_bounces;  // NEE, then rr_continue, run by the caller
        return contributes;
    }
    if (bounce_count < sp.max_bounces) {
        alive = true;
        if (bounce_count > sp.rr_depth) {  // Russian roulette (:264-270)
            const float cp = fmaxf(fmaxf(T.x, T.y), T.z);
            if (random_float(rng) > cp) {
                alive = false;
            } else {
                T = rr_divide(T, cp);
            }
        }
        if (alive) o = F3{o.x + n.x * kOriginEps, o.y + n.y * kOriginEps, o.z + n.z * kOriginEps};  // :277-280
    }
    return contributes;
}

// shade_hit plus the new direction (get_random_bounche, :273-274): the whole loop body.
__device__ __forceinline__ bool shade_segment(const float4* __restrict__ prims, const float4* __restrict__ mats,
                                              const ShadeParams& sp, uint32_t bounce_count, float t, uint32_t k,
                                              F3& o, F3& d, F3& T, uint32_t& rng, bool& alive, F3& add) {
    F3 n;
    const bool contributes = shade_hit(prims, mats, sp, bounce_count, t, k, o, d, T, rng, alive, add, n);
    if (alive) d = bounce_dir(n, rng, sp.flags);
    return contributes;
}

// ---- next-event estimation (SPT_FLAG_NEE; oracle ref_trace_ray's NEE block) ----
// The second half of shade_hit for a path past its light sample: Russian roulette (:264-270) with
// bounce_count (after the increment); false ends the path.
__device__ __forceinline__ bool rr_continue(const ShadeParams& sp, uint32_t bounce_count, F3& T, uint32_t& rng) {
    if (bounce_count > sp.rr_depth) {
        const float cp = fmaxf(fmaxf(T.x, T.y), T.z);
        if (random_float(rng) > cp) return false;
        T = rr_divide(T, cp);
    }
    return true;
}

// current_origin += normal * EPSILON (:277-280): the next ray's origin, and the shadow ray's
__device__ __forceinline__ F3 offset_origin(F3 o, F3 n) {
    return F3{o.x + n.x * kOriginEps, o.y + n.y * kOriginEps, o.z + n.z * kOriginEps};
}

// The shadow ray (o, w): true when nothing lies at 0.001 <= t < tmax (oracle ref_visible). The search
// started from best_t = tmax finds a t < tmax iff there is one (ties with tmax keep best_t = tmax); the
// BVH culls against it conservatively (padded boxes) and stops at the first such hit (any-hit).
template <bool kBvh>
__device__ __forceinline__ bool shadow_visible(const float4* __restrict__ prims, const float4* __restrict__ nodes,
                                               uint32_t n_prims, const ShadeParams& sp, F3 o, F3 w, float tmax) {
    float best_t = tmax;
    uint32_t best_k = kMiss;
    if (kBvh) closest_tree<false, true>(nodes, prims, o, w, best_t, best_k);
    else closest_flat(prims, n_prims, o, w, best_t, best_k, (sp.flags & kFlagFastDiv) != 0u, sp.flat_ends);
    return !(best_t < tmax);
}

// shade_segment with NEE, for the wavefront kernels: the hit, the light sample and its shadow ray
// (traced here, inline), Russian roulette and the new direction. Bit 0: `add` (emission or sky) is
// added to the path's radiance, bit 1: then `add2` (the light sample), in that order.
template <bool kBvh>
__device__ __forceinline__ uint32_t shade_segment_nee(const float4* sh_prims, const float4* sh_mats,
                                                      const float4* __restrict__ prims,
                                                      const float4* __restrict__ nodes, uint32_t n_prims,
                                                      const ShadeParams& sp, const NeeParams& nee,
                                                      uint32_t bounce_count, float t, uint32_t k, F3& o, F3& d,
                                                      F3& T, uint32_t& rng, bool& alive, F3& add, F3& add2) {
    F3 n;
    const bool c1 = shade_hit<2, false, true>(sh_prims, sh_mats, sp, bounce_count, t, k, o, d, T, rng, alive, add, n);
    bool c2 = false;
    if (alive) {
        o = offset_origin(o, n);
        F3 w;
        float tmax;
        if (light_sample(nee.emit, nee.n_emit, o, n, T, rng, w, tmax, add2))
            c2 = shadow_visible<kBvh>(prims, nodes, n_prims, sp, o, w, tmax);
        alive = rr_continue(sp, bounce_count, T, rng);
        if (alive) d = bounce_dir(n, rng, sp.flags);
    }
    return (c1 ? 1u : 0u) | (c2 ? 2u : 0u);
}

// kFused: the "bounce" kernel — the closest hit is computed here (extend + shade in one launch), so
// the 8 B hit record and the 32 B ray re-read of a separate extend launch disappear.
// kNee (SPT_FLAG_NEE): each hit's light sample and its shadow ray are traced here too (shade_segment_nee).
template <bool kPrimary, bool kFused, bool kBvh, bool kNee = false>
__global__ __launch_bounds__(kBlock) void k_shade(const float4* __restrict__ prims, const float4* __restrict__ mats,
                                                  const float4* __restrict__ nodes, uint32_t n_prims,
                                                  const float2* __restrict__ hit, QueueBufs cur, QueueBufs nxt,
                                                  float4* __restrict__ radiance, uint32_t* __restrict__ counts,
                                                  ShadeParams sp, CameraParams cam, NeeParams nee) {
    __shared__ uint32_t s_wave_cnt[2][kBlock / 64];
    __shared__ uint32_t s_contrib[kBlock / 64];
    const uint32_t s = blockIdx.x;
    const uint32_t n_sub = cam.n_sub;
    const uint32_t n = kPrimary ? sub_count_of(cam.n_paths, s, n_sub) : counts[sp.bounce * n_sub + s];
    const uint32_t base = s * sp.sub_cap;
    const uint32_t bounce_count = sp.bounce + 1u;  // trace_ray's bounce_count after `bounce_count++` (:263)
    const uint32_t wave = threadIdx.x / 64u;
    const uint32_t lane = __lane_id();
    uint32_t out_n = 0;  // block-uniform length of the output segment
    uint32_t parity = 0;
    uint32_t wave_rmw = 0;  // wave-uniform count of radiance read-modify-writes (statistics)

    // Flat scenes: the shading gathers (divergent primitive / material records) read an LDS copy of
    // the scene (<= 32 primitives, <= 32 materials after spt_set_scene's remap) instead of global
    // memory; the closest-hit loop keeps its wave-uniform scalar loads.
    __shared__ float4 s_scene[kBvh ? 1 : kLdsScene];
    const float4* sh_prims = prims;
    const float4* sh_mats = mats;
    if (!kBvh) {  // host guarantees a flat scene: n_prims <= kFlatPrims, n_mats <= 32
        for (uint32_t k = threadIdx.x; k < 4u * sp.n_prims; k += kBlock) s_scene[k] = prims[k];
        for (uint32_t k = threadIdx.x; k < 2u * sp.n_mats; k += kBlock) s_scene[4u * kFlatPrims + k] = mats[k];
        __syncthreads();
        sh_prims = s_scene;
        sh_mats = s_scene + 4u * kFlatPrims;
    }

    for (uint32_t i0 = 0; i0 < n; i0 += kBlock) {
        const uint32_t i = i0 + threadIdx.x;
        bool alive = false;
        bool did_rmw = false;
        F3 o{0.f, 0.f, 0.f}, d{0.f, 0.f, 0.f}, T{1.f, 1.f, 1.f};
        uint32_t pid = 0, rng = 0;
        if (i < n) {
            float2 h;
            if (!kFused) h = hit[base + i];
            if (kPrimary) {
                pid = dealt_path(s, i, n_sub);
                const CameraRay cr = camera_ray(cam, pid);
                d = cr.d;
                rng = cr.seed;
            } else {
                // (a software prefetch of the next entry measured -3.5 % on C2: occupancy)
                const float4 o4 = cur.o[base + i];
                const float4 d4 = cur.d[base + i];
                const float4 t4 = cur.t[base + i];
                o = F3{o4.x, o4.y, o4.z};
                d = F3{d4.x, d4.y, d4.z};
                T = F3{t4.x, t4.y, t4.z};
                pid = __float_as_uint(o4.w);
                rng = __float_as_uint(d4.w);
            }
            if (kFused) {
                float best_t = kInf;
                uint32_t best_k = kMiss;
                if (kBvh) closest_tree(nodes, prims, o, d, best_t, best_k);
                else closest_flat(prims, n_prims, o, d, best_t, best_k, (sp.flags & kFlagFastDiv) != 0u, sp.flat_ends);
                h = make_float2(best_t, __uint_as_float(best_k));
            }
            F3 add;
            if constexpr (kNee) {
                F3 add2;
                const uint32_t c = shade_segment_nee<kBvh>(sh_prims, sh_mats, prims, nodes, n_prims, sp, nee, bounce_count,
                                                           h.x, __float_as_uint(h.y), o, d, T, rng, alive, add, add2);
                // accumulated_color += emission (or sky), then += the light sample, in bounce order
                if (kPrimary || c) {
                    float4 L = kPrimary ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : radiance[pid];
                    did_rmw = !kPrimary;
                    if (c & 1u) L = make_float4(L.x + add.x, L.y + add.y, L.z + add.z, L.w);
                    if (c & 2u) L = make_float4(L.x + add2.x, L.y + add2.y, L.z + add2.z, L.w);
                    radiance[pid] = L;
                }
            } else {
            const bool contributes =
                shade_segment(sh_prims, sh_mats, sp, bounce_count, h.x, __float_as_uint(h.y), o, d, T, rng, alive, add);
            // accumulated_color += contribution, in bounce order (L starts at 0 in bounce 0)
            if (kPrimary) {
                radiance[pid] = contributes ? make_float4(0.0f + add.x, 0.0f + add.y, 0.0f + add.z, 0.0f)
                                            : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            } else if (contributes) {
                did_rmw = true;
                float4 L = radiance[pid];
                L.x = L.x + add.x;
                L.y = L.y + add.y;
                L.z = L.z + add.z;
                radiance[pid] = L;
            }
            }
        }
        // ---- compaction into this block's output segment (no global atomics) ----
        wave_rmw += (uint32_t)__popcll(__ballot(did_rmw));
        const unsigned long long mask = __ballot(alive);
        const uint32_t lane_off =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        if (lane == 0) s_wave_cnt[parity][wave] = (uint32_t)__popcll(mask);
        __syncthreads();  // one barrier per iteration: s_wave_cnt is double-buffered by parity
        uint32_t before = 0, total = 0;
#pragma unroll
        for (uint32_t w = 0; w < kBlock / 64; ++w) {
            const uint32_t c = s_wave_cnt[parity][w];
            before += w < wave ? c : 0u;
            total += c;
        }
        if (alive) {
            const uint32_t slot = base + out_n + before + lane_off;
            nxt.o[slot] = make_float4(o.x, o.y, o.z, __uint_as_float(pid));
            nxt.d[slot] = make_float4(d.x, d.y, d.z, __uint_as_float(rng));
            nxt.t[slot] = make_float4(T.x, T.y, T.z, 0.0f);
        }
        out_n += total;
        parity ^= 1u;
    }
    if (lane == 0) s_contrib[wave] = wave_rmw;
    __syncthreads();
    if (threadIdx.x == 0) {
        counts[(sp.bounce + 1u) * n_sub + s] = out_n;
        if (kPrimary) counts[s] = n;  // bounce-0 length, for the statistics tally
        uint32_t rmw = 0;
        for (uint32_t w = 0; w < kBlock / 64; ++w) rmw += s_contrib[w];
        counts[(kMaxBounces + 1u + sp.bounce) * n_sub + s] = rmw;  // second half: radiance RMWs
    }
}

// ---------------------------------------------------------------------------------------------
// trace_tail: the remaining bounces of every path in queue `bounce`, one thread per path (the rest
// of trace_ray's loop, CPUPathTracer.cpp:211-281). Once Russian roulette has thinned the queues
// (bounce >= 3 holds ~5 % of C2's rays) a launch pair per bounce costs more than its work.
// Per-bounce segment and radiance-update counts are tallied in LDS for the statistics.
// ---------------------------------------------------------------------------------------------
template <bool kBvh, bool kNee = false>
__global__ __launch_bounds__(kBlock) void k_trace_tail(const float4* __restrict__ prims,
                                                       const float4* __restrict__ nodes, uint32_t n_prims,
                                                       const float4* __restrict__ mats, QueueBufs cur,
                                                       float4* __restrict__ radiance, uint32_t* __restrict__ counts,
                                                       ShadeParams sp, uint32_t n_sub, NeeParams nee) {
    __shared__ uint32_t s_seg[kMaxBounces];
    __shared__ uint32_t s_rmw[kMaxBounces];

    const uint32_t s = blockIdx.x;
    if (threadIdx.x < kMaxBounces) {
        s_seg[threadIdx.x] = 0;
        s_rmw[threadIdx.x] = 0;
    }
    __syncthreads();
    const uint32_t n = counts[sp.bounce * n_sub + s];
    const uint32_t base = s * sp.sub_cap;
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
        const float4 o4 = cur.o[base + i];
        const float4 d4 = cur.d[base + i];
        const float4 t4 = cur.t[base + i];
        F3 o{o4.x, o4.y, o4.z}, d{d4.x, d4.y, d4.z}, T{t4.x, t4.y, t4.z};
        const uint32_t pid = __float_as_uint(o4.w);
        uint32_t rng = __float_as_uint(d4.w);
        for (uint32_t b = sp.bounce; b < sp.max_bounces; ++b) {
            atomicAdd(&s_seg[b], 1u);
            float best_t = kInf;
            uint32_t best_k = kMiss;
            if (kBvh) closest_tree(nodes, prims, o, d, best_t, best_k);
            else closest_flat(prims, n_prims, o, d, best_t, best_k, (sp.flags & kFlagFastDiv) != 0u, sp.flat_ends);
            bool alive;
            F3 add;
            if constexpr (kNee) {
                F3 add2;
                const uint32_t c = shade_segment_nee<kBvh>(prims, mats, prims, nodes, n_prims, sp, nee, b + 1u, best_t,
                                                           best_k, o, d, T, rng, alive, add, add2);
                if (c) {
                    atomicAdd(&s_rmw[b], 1u);
                    float4 L = radiance[pid];
                    if (c & 1u) L = make_float4(L.x + add.x, L.y + add.y, L.z + add.z, L.w);
                    if (c & 2u) L = make_float4(L.x + add2.x, L.y + add2.y, L.z + add2.z, L.w);
                    radiance[pid] = L;
                }
            } else if (shade_segment(prims, mats, sp, b + 1u, best_t, best_k, o, d, T, rng, alive, add)) {
                atomicAdd(&s_rmw[b], 1u);
                float4 L = radiance[pid];
                L.x = L.x + add.x;
                L.y = L.y + add.y;
                L.z = L.z + add.z;
                radiance[pid] = L;
            }
            if (!alive) break;
        }
    }
    __syncthreads();
    const uint32_t b = threadIdx.x;
    if (b >= sp.bounce && b < sp.max_bounces) {
        if (b > sp.bounce) counts[b * n_sub + s] = s_seg[b];  // queue `bounce` itself is already counted
        counts[(kMaxBounces + 1u + b) * n_sub + s] = s_rmw[b];
    }
}

// ---------------------------------------------------------------------------------------------
// paths: the persistent schedule for flat scenes — the whole of render()'s pixel loop for a call of
// F frames (CPUPathTracer.cpp:57-82 with trace_ray :197-284 inlined) in ONE launch, no ray queues.
//
// Wave w owns 64 consecutive shard pixels and all F frames of them: 64*F path slots q = f*64 + j
// (pixel j, frame f). Every lane traces one path at a time; a lane whose path ended takes the next
// slot (ballot + mbcnt, a wave-uniform cursor — no atomics), so the lanes stay busy until the wave's
// last frame. Frame order of the accumulation (:77-80) is kept exactly: a finished path parks its
// radiance in an LDS ring of kRing frames, and when all 64 paths of the oldest frame are in, lane j
// adds that frame's radiance to pixel j's accumulator (a register, read once and stored once per
// launch). A slot is only handed out while its frame fits in the ring, so a long path holds back
// at most kRing frames. HBM traffic per launch: 32 B per pixel (accum read + write).
//
// The camera ray of a pixel has no jitter (:63-69), so its first segment is the same in every
// frame: everything up to the random bounce direction (closest hit, Ng, n, emission, albedo, the
// tangent frame of get_random_bounche, the offset origin) is computed once per pixel at the start
// of the launch and kept in LDS. A frame's path starts from that state: only the RNG-dependent
// part of bounce 0 (Russian roulette when rr_depth == 0, the direction draw) runs per frame. The
// arithmetic is the same expressions on the same inputs, so the results are bit-identical to
// tracing the camera ray again; the statistics still count bounce 0 as one segment per path.
// ---------------------------------------------------------------------------------------------
// path slots in flight per wave (ring of finished radiances); a larger ring for BVH scenes (longer
// paths, no LDS scene copy) measured no better on C4/C5
template <bool kBvh>
constexpr uint32_t ring_slots() { return 256u; }

// Per-pixel primary state, 3 float4s in LDS (48 B per pixel):
//   r0 = (n.xyz, seed)          n: shading normal of the camera ray's hit; seed = x + y * width
//   r1 = (o1.xyz, m | kHitBit)  o1 = hit + n * EPSILON (the next ray's origin), m: the hit primitive
//                               (flat scenes: its LDS shading record) or its material (BVH scenes)
//        (L0.xyz, 0)            on a miss: the sky (or black) radiance the path ends with
//   r2 = (t.xyz, 0)             t: get_random_bounche's tangent for n
// On a hit the radiance and throughput after bounce 0 are re-derived from the material, with the
// expressions of shade_segment (0 + 1 * emission, 1 * albedo), so they need no storage.
constexpr uint32_t kHitBit = 0x80000000u;
constexpr uint32_t kConstPx = 0x80u;  // k_paths s_pix: a constant pixel (no path slots)

struct PrimaryState {
    float4 r0, r1, r2;
    float4 r3, r4;  // flat scenes, after a hit: (1 * albedo, 0) and (0 + 1 * emission or 0, 0)
};

// Flat scenes' LDS shading records, 3 float4s per primitive, everything shade_hit needs after the
// closest hit in ONE round of independent LDS reads (the primitive and then its material record
// were two dependent rounds): g = (sphere center | quad normal | triangle Ng, type),
// the material's albedo and emission records (DevMaterial).
__device__ __forceinline__ void make_shade_recs(const float4* __restrict__ prims, const float4* __restrict__ mats,
                                                uint32_t n_prims, float4* recs) {
    for (uint32_t k = threadIdx.x; k < n_prims; k += kBlock) {
        const float4 pa = prims[4 * k + 0], pb = prims[4 * k + 1], pd = prims[4 * k + 3];
        const uint32_t type = meta_type(pd), m = meta_material(pd);
        const float4 g = type == 0u ? pa : (type == 1u ? pb : pd);
        recs[3 * k + 0] = make_float4(g.x, g.y, g.z, __uint_as_float(type));
        recs[3 * k + 1] = mats[2 * m + 0];
        recs[3 * k + 2] = mats[2 * m + 1];
    }
}

// trace_ray's first iteration (CPUPathTracer.cpp:211-280) for a camera ray, without the RNG draws.
template <bool kBvh, int kEnv, uint64_t kShape = 0, class Stk = StkP>
__device__ __forceinline__ PrimaryState primary_state(const float4* __restrict__ prims,
                                                      const float4* __restrict__ nodes, uint32_t n_prims,
                                                      const float4* sh_prims, const float4* sh_mats,
                                                      const ShadeParams& sp, F3 d, uint32_t seed,
                                                      const Stk& stk) {
    PrimaryState ps;
    ps.r0 = make_float4(0.f, 0.f, 0.f, __uint_as_float(seed));
    ps.r1 = make_float4(0.f, 0.f, 0.f, 0.f);
    ps.r2 = make_float4(0.f, 0.f, 0.f, 0.f);
    ps.r3 = make_float4(0.f, 0.f, 0.f, 0.f);
    ps.r4 = make_float4(0.f, 0.f, 0.f, 0.f);
    F3 o{0.f, 0.f, 0.f};
    float best_t = kInf;
    uint32_t best_k = kMiss;
    if (kBvh) closest_bvh4_on(nodes, prims, o, d, best_t, best_k, stk);
    else closest_flat<kShape>(prims, n_prims, o, d, best_t, best_k, (sp.flags & kFlagFastDiv) != 0u, sp.flat_ends);
    if (best_k == kMiss) {
        if (sp.sky_enabled) {  // L = 0 + T * sky with T = 1 (:231-235)
            const F3 sky = sky_radiance<kEnv>(sp, d);
            ps.r1 = make_float4(0.0f + 1.0f * sky.x, 0.0f + 1.0f * sky.y, 0.0f + 1.0f * sky.z, 0.0f);
        }
        return ps;
    }
    o = F3{o.x + best_t * d.x, o.y + best_t * d.y, o.z + best_t * d.z};
    const float4 pa = sh_prims[4 * best_k + 0];
    const float4 pd = sh_prims[4 * best_k + 3];
    const uint32_t type = meta_type(pd);
    F3 ng;
    if (type == 0u) {
        ng = F3{o.x - pa.x, o.y - pa.y, o.z - pa.z};
    } else {
        const float4 pb = sh_prims[4 * best_k + 1];
        const float4 nv = type == 1u ? pb : pd;
        ng = F3{nv.x, nv.y, nv.z};
        if (dot3(ng, d) > 0.0f) ng = F3{-ng.x, -ng.y, -ng.z};
    }
    const float inv_len = inv_sqrt_ref(ng.x * ng.x + ng.y * ng.y + ng.z * ng.z);
    const F3 n{ng.x * inv_len, ng.y * inv_len, ng.z * inv_len};
    ps.r0 = make_float4(n.x, n.y, n.z, __uint_as_float(seed));
    const F3 o1{o.x + n.x * kOriginEps, o.y + n.y * kOriginEps, o.z + n.z * kOriginEps};
    // the tag: a flat scene's shading record (make_shade_recs) is per primitive, a BVH scene's
    // material record per material
    ps.r1 = make_float4(o1.x, o1.y, o1.z, __uint_as_float((kBvh ? meta_material(pd) : best_k) | kHitBit));
    if (!kBvh) {  // bounce 0's throughput and radiance after the hit, with the path start's expressions
        const uint32_t m = meta_material(pd);
        const float4 alb = sh_mats[2 * m + 0];
        const float4 emi = sh_mats[2 * m + 1];
        ps.r3 = make_float4(1.0f * alb.x, 1.0f * alb.y, 1.0f * alb.z, 0.0f);
        if (emi.w != 0.0f) ps.r4 = make_float4(0.0f + 1.0f * emi.x, 0.0f + 1.0f * emi.y, 0.0f + 1.0f * emi.z, 0.0f);
    }
    if (1u < sp.max_bounces) {
        const F3 t = bounce_tangent(n, sp.flags);
        ps.r2 = make_float4(t.x, t.y, t.z, 0.0f);
    }
    return ps;
}

// Launch-bound and LDS tuning of the persistent kernels (measured):
// flat k_paths keeps 3 per-pixel records (bounce 0's throughput and radiance are read from the hit
// primitive's LDS shading record at the path start), so 7 blocks fit per CU and it runs at 7 waves/SIMD
// (C2 +0.8 % over 5 records at 6 waves; 8 waves at 64 VGPRs: -11 %)
constexpr uint32_t kFlatPxRecs = 3;
constexpr int kPathsWaves = 6;      // __launch_bounds__ waves per SIMD: flat k_frame, NEE k_paths
constexpr int kPathsWavesFlat = 7;  // flat k_paths
constexpr int kPathsWavesBvh = 7;   // BVH k_paths / k_frame: the latency-bound traversal (C4 +4 %, C5 +6.5 % vs 6)
constexpr int kBvhSmallWaves = 8;   // BVH k_paths of scenes of <= kBvhSmall primitives (C4 +2.6 % over 7; C5: -5 %)
constexpr uint32_t kFrameTopPrims = 64;  // k_frame: a BVH scene of <= 64 primitives keeps their records in LDS
constexpr uint32_t kFrameTopNodes = 64;  // k_frame: LDS copy of the first 64 nodes (4 KB per block)
constexpr uint32_t kBvhTopNodes = 53;    // k_paths (7 waves/SIMD): LDS copy of the top 3 levels of the 4-wide tree and
                                         // half of the 4th (the LDS left at 7 blocks per CU: C5 +1.7 %, r05_zb)
constexpr uint32_t kBvhTopNodes8 = 5;    // ... with 8 waves/SIMD (less LDS per block): the top 2 levels
constexpr uint32_t kBvhSmall = 256u * 1024u;  // == scene.h bvh_max_leaf's one-primitive-leaf range
constexpr uint32_t kMaxChunkShift = 5;  // k_paths chunks of at most 32 pixels (LDS: 1.5 KB state per wave)
// and at least 1: a small row shard of an N-GPU run starts with 4-pixel chunks (N = 8: +2-5 % over 8) and
// ends with 2- and 1-pixel ones — a chunk runs all frames of a launch (N x 64), so its length, not its
// pixel count, sets the launch's tail
constexpr uint32_t kMinChunkShift = 0;

// Static profile builds (-DSPT_STATIC_PROFILE): asm comments between the sections of a k_paths step,
// counted by scripts/static_profile.py (the markers constrain scheduling a little; analysis only)
#ifdef SPT_STATIC_PROFILE
#define SPT_MARK(x) asm volatile("; SPT_MARK " #x)
#else
#define SPT_MARK(x) ((void)0)
#endif

// acc.w after k more frames: k additions of 1.0f, as one add while every partial sum is an integer
// below 2^24 (each +1 exact, so their sum is the one exact add), else one by one (CPUPathTracer.cpp:80)
__device__ __forceinline__ float add_count(float w, uint32_t k) {
    if (w + (float)k <= 16777216.0f) return w + (float)k;
    for (uint32_t i = 0; i < k; ++i) w = w + 1.0f;
    return w;
}
// channel c of an accumulator after n frames that each add v (c == 3: the count)
__device__ __forceinline__ float add_frames(float a, uint32_t c, float v, uint32_t n) {
    if (c == 3u) return add_count(a, n);
    for (uint32_t f = 0; f < n; ++f) a = a + v;
    return a;
}

// The lane id computed where it is used: an asm volatile is not hoisted out of a loop, so a lane-derived
// value does not occupy a VGPR across the loop (the persistent kernels' step loops run at the VGPR limit)
__device__ __forceinline__ uint32_t lane_id_here() {
    uint32_t v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
    return v;
}

// Work queue of the persistent kernels: units (chunks / runs) 0..n-1 dealt over kWorkHeads heads,
// head r handing out units r, r + 8, r + 16, ... in increasing order. A wave pulls from the head of
// its own XCD (HW_REG_XCC_ID; placement only affects speed) and, once that is empty, from the others
// in turn: one word saturates at ~88 dequeues/us (MI355X_MICROARCH.md, "dequeue"), which a 1-frame
// launch of 2M pixels would hit. `h` (wave-uniform, starts at 0) counts the heads found empty.
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}

__device__ __forceinline__ uint32_t pull_unit(uint32_t* __restrict__ work, uint32_t n, uint32_t xcc, uint32_t& h) {
    while (h < kWorkHeads) {
        const uint32_t r = (xcc + h) & (kWorkHeads - 1u);
        const uint32_t len = n > r ? (n - r + kWorkHeads - 1u) / kWorkHeads : 0u;  // units r + 8k < n
        uint32_t k = len;
        if (__lane_id() == 0u) {
            uint32_t* head = work + r * kWorkStride;
            // a head found empty by a plain (L2-bypassing) read is skipped without an atomic
            if (h == 0u || __hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < len)
                k = atomicAdd(head, 1u);
        }
        k = __builtin_amdgcn_readfirstlane(k);
        if (k < len) return r + k * kWorkHeads;
        ++h;
    }
    return n;
}

#ifdef SPT_TIMELINE
// measurement builds only (scripts/k_paths_timeline.py): every wave's start, last chunk and end
__device__ unsigned long long g_tl[8192 * 4];
#endif

// k_paths work plan: n[i] chunks of 1 << shift[i] pixels starting at pixel start[i] (start[0] = 0).
// Flat scenes: the first tier's chunks are handed out in `order` (chunk indices, longest first) once a
// launch has recorded each one's cost in `cost` (launch_paths, k_chunk_order); nullptr: pixel order,
// no recording.
struct ChunkPlan {
    uint32_t n[3];
    uint32_t start[3];
    uint32_t shift[3];
    const uint32_t* order;
    uint16_t* cost;
};

// BVH scenes: lanes advance their rays through the tree (trav_step) until this many lanes of the
// wave wait — ray done, or no path while new slots are free — then those are shaded and refilled
// while the others keep their place in the tree. Against 24, 16 and 32 measured C4 -1.8 % / -0.7 %
// and C5 -3.7 % / -0.1 % (profiles/r05_f_ab_batch_vote.txt); with the unified step (below) 16 / 32 / 40:
// C5 -1 / +0.2 / -3.5 %, C4 -3 / +0.5 / +0.7 % (profiles/r05_s_ab_unified_kpaths.txt). With NEE a
// waiting lane also has a shadow ray to start, and larger rounds pay (C4 NEE: 24 -> 40 +7 %, then with
// the unified step 40 -> 48 +2.3 %).
constexpr uint32_t kBvhBatch = 24;
constexpr uint32_t kBvhBatchNee = 48;

// The traversal phase of k_frame (BVH scenes): advance the rays of lanes with a path (`have`) whose
// traversal is not done, one node visit or one primitive test per iteration (the unified step: one
// shared record load), until `batch` lanes wait (ray done, or no path while `can_start`: new paths
// could start). k_paths writes its own loop with the vote between node and primitive steps.
template <bool kStats, bool kLds = false, bool kAnyHit = false, class Stk>
__device__ __forceinline__ void advance_rays(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                                             bool have, bool can_start, F3 o, F3 d, Trav& tv, bool& tdone,
                                             const Stk& stk, BvhCounters& ctr,
                                             uint32_t& lane_slots, uint32_t& lane_busy,
                                             const float4* top = nullptr, uint32_t n_top = 0u,
                                             const float4* ptop = nullptr, uint32_t n_ptop = 0u,
                                             uint32_t batch = kBvhBatch) {
    for (;;) {
        const bool trav = have && !tdone;
        const unsigned long long tm = __ballot(trav);
        if (tm == 0ull) break;
        if ((uint32_t)__popcll(__ballot(have ? tdone : can_start)) >= batch) break;
        if (kStats) {
            lane_slots += 64u;
            lane_busy += (uint32_t)__popcll(tm);
        }
        if (trav)
            tdone = trav_step<kStats, kLds, kAnyHit>(nodes, prims, o, d, tv, stk, &ctr, top, n_top, ptop, n_ptop);
    }
}

// kSimdWaves: __launch_bounds__' waves per SIMD, 0 = the default of the scene kind. BVH scenes of up
// to kBvhSmall primitives run with 8 (C4 +2.6 % over 7), larger ones with 7 (C5: 8 is -5 %).
// kChan: a flat scene's instantiation for chunks of <= 16 pixels (the small row shards of N-GPU runs),
// which keeps the accumulators in channel lanes as the BVH instantiations always do (§ chunk start).
// kNee: next-event estimation (SPT_FLAG_NEE, § the step's NEE state); run with kEnv = 2. kNeeAll samples
// every emitter kind; kNeeNoSpheres (BVH scenes whose emitter table holds no sphere) leaves the sphere
// sample out of the kernel: its fp64 registers cost the BVH step loop spills (C4 NEE -4.4 %, record
// r05_x), the flat kernels nothing.
template <bool kStats, bool kBvh, int kEnv, uint64_t kShape = 0, int kSimdWaves = 0, bool kChan = false, int kNee = 0>
__global__ __launch_bounds__(kBlock, kSimdWaves ? kSimdWaves : (kBvh ? kPathsWavesBvh : (kNee ? kPathsWaves : kPathsWavesFlat))) void k_paths(const float4* __restrict__ prims, const float4* __restrict__ mats,
                                                  const float4* __restrict__ nodes, uint32_t n_prims,
                                                  float4* __restrict__ accum,
                                                  unsigned long long* __restrict__ totals,
                                                  uint32_t* __restrict__ work, uint32_t* __restrict__ work_next,
                                                  ShadeParams sp, CameraParams cam, uint32_t n_frames, ChunkPlan plan,
                                                  NeeParams nee) {
    constexpr uint32_t kWaves = kBlock / 64u;
    bake_config<kShape>(sp);
    constexpr uint32_t kRingSlots = ring_slots<kBvh>();
    // flat scenes: launch-sized LDS shading records, 3 float4s per primitive (make_shade_recs)
    extern __shared__ float4 s_scene[];
    constexpr uint32_t kPxRecs = kBvh ? 3u : kFlatPxRecs;  // PrimaryState records kept per pixel
    __shared__ float4 s_px[kWaves][kPxRecs][1u << kMaxChunkShift];  // per-pixel primary state (PrimaryState)
    __shared__ float s_L[kWaves][3][kRingSlots];  // radiance of finished paths, ring of path slots
    // a done byte per ring entry (the slot's lap), read four at a time by the completion check
    __shared__ __attribute__((aligned(16))) uint32_t s_cnt[kWaves][64];
    __shared__ uint8_t s_pix[kWaves][1u << kMaxChunkShift];  // per pixel: live rank | kConstPx + entry of its Lc
    // BVH scenes: the tree's top nodes (breadth-first: the root and the levels below it), read from
    // LDS instead of L2 by every traversal — the LDS left over at this kernel's occupancy
    constexpr uint32_t kTop = kBvh ? (kSimdWaves == 8 ? kBvhTopNodes8 : kBvhTopNodes) : 0u;
    __shared__ float4 s_top[kTop ? 4u * kTop : 1u];
    const uint32_t n_top = min(kTop, sp.n_nodes);
    for (uint32_t k = threadIdx.x; k < 4u * n_top; k += kBlock) s_top[k] = nodes[k];
    __shared__ uint32_t s_seg[kStats ? kMaxBounces : 1u];
    __shared__ uint32_t s_rmw[kStats ? kMaxBounces : 1u];
    __shared__ uint32_t s_shadow[kStats && kNee ? 1u : 1u];  // NEE shadow rays traced (statistics)
    if (kStats && kNee && threadIdx.x == 0u) s_shadow[0] = 0u;
    if (!kBvh) make_shade_recs(prims, mats, sp.n_prims, s_scene);
    // the next launch's work heads (stream order: the previous user of that set has finished)
    if (blockIdx.x == 0u && threadIdx.x < kWorkHeads) work_next[threadIdx.x * kWorkStride] = 0u;
    if (kStats && threadIdx.x < kMaxBounces) {
        s_seg[threadIdx.x] = 0;
        s_rmw[threadIdx.x] = 0;
    }
    __syncthreads();
    // shading gathers: a flat scene's LDS shading records, global memory (L2/MALL) for a BVH scene
    // (BVH material records copied to LDS measured +-0 on C4/C5, round 3)
    const float4* sh_prims = kBvh ? prims : s_scene;
    const float4* sh_mats = mats;

    // (wave-uniform, made known to the compiler: the per-wave LDS bases then live in SGPRs)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64u);
    const uint32_t lane = __lane_id();
    // persistent grid: (block, wave) names one resident wave, which owns 64 lanes' stacks
    const auto stk = lane_stack<kSimdWaves == 8 ? kBvhStackEntry8W : kBvhStackEntry>(sp, blockIdx.x * kWaves + wave, lane);
    // Waves are persistent: each takes chunks from a launch-wide counter until none are left, so a
    // wave slot never idles behind a finished chunk (chunks differ a lot in cost: sky pixels end at
    // bounce 0). The plan's chunks shrink towards the end (32, then 16, then 8 pixels), so the
    // waves' last chunks — the launch's tail — are short.
    uint32_t lane_slots = 0, lane_busy = 0;  // statistics: lane utilization of the tracing steps
    BvhCounters bvh_ctr;                     // statistics: BVH work of this lane's traced segments
    const uint32_t n_chunks = plan.n[0] + plan.n[1] + plan.n[2];
    const uint32_t xcc = xcc_id();
    uint32_t heads_empty = 0;
    // The first tier is handed out longest first (ChunkPlan::order). A chunk's cost is its live pixels'
    // paths: a row of sky costs nothing, a row inside the Cornell box up to ~6 x the average — and one
    // such chunk handed out late held its wave past every other (the launch timeline,
    // scripts/k_paths_timeline.py: ~10 % of C2's wave slots idle in the tail). BVH scenes too since
    // round 6: C4's last waves traced fully live 16-pixel chunks of the bunny handed out at 60 % of the
    // launch for 40 % of it (10 % of the wave slots idle); in cost order C4 +4.5 %, C5 +-0
    // (profiles/r06_j_ab_bvh_chunk_order.txt; C5 had lost 8 % in round 5, before the unified step).
    // The BVH NEE kernels count their traversal iterations into the cost (below).
    constexpr bool kOrdered = true;
#ifdef SPT_TIMELINE
    const unsigned long long tl_start = wall_clock64();
    unsigned long long tl_last = tl_start;
    uint32_t tl_chunks = 0, tl_pxs = 0, tl_live = 0;
#endif
    for (;;) {
        const uint32_t chunk = pull_unit(work, n_chunks, xcc, heads_empty);
        if (chunk >= n_chunks) break;
#ifdef SPT_TIMELINE
        tl_last = wall_clock64();
        ++tl_chunks;
#endif
        uint32_t pxs, pix0;
        if (chunk < plan.n[0]) {
            pxs = plan.shift[0];
            pix0 = ((kOrdered && plan.order) ? __builtin_amdgcn_readfirstlane(plan.order[chunk]) : chunk) << pxs;
        } else if (chunk < plan.n[0] + plan.n[1]) {
            pxs = plan.shift[1];
            pix0 = plan.start[1] + ((chunk - plan.n[0]) << pxs);
        } else {
            pxs = plan.shift[2];
            pix0 = plan.start[2] + ((chunk - plan.n[0] - plan.n[1]) << pxs);
        }
        const uint32_t px = 1u << pxs;  // pixels of this chunk (4 to 32)
        const uint32_t npx = min(px, cam.shard_pixels - pix0);
        // Bounce 0 of every pixel, once per chunk. A pixel whose camera ray ends its path without an
        // RNG draw — a miss (the sky), or any hit when max_bounces <= 1 — is a *constant* pixel: every
        // frame's path of it returns the same radiance Lc, so it gets no path slots at all (C2: 61 %
        // of all paths are such sky pixels; each used to take a lane for a whole step). Only the live
        // pixels' slots are handed out; the constant ones' Lc is added per frame at accumulation, in
        // the same frame order, so the sums are the same bits.
        // The chunk's accumulators live in *channel lanes*: lane L holds channel c0 (and c0 + 1 for
        // 32-pixel chunks) of pixel L mod px — 32 pixels: lanes 0-31 (x, y), 32-63 (z, w); 4-16 pixels:
        // lane L channel L / px. An accumulation then adds one or two channels per lane and frame
        // instead of all four of one pixel (the same additions in the same frame order), and the
        // frame count w takes the k completed frames in one exact add. 2 VGPRs instead of 4.
        // Channel lanes for BVH scenes (2 accumulator VGPRs instead of 4: C4 +4 %, C5 +1.5 %) and, in
        // the kChan instantiation, for a flat scene's small shards (N = 8: +7 %); the flat kernel of a
        // whole image keeps one pixel per lane (channel lanes in the same kernel cost C2 3-4 %).
        constexpr bool chmode = kBvh || kChan;
        const uint32_t cp = lane & (px - 1u);                                // the channel lane's pixel
        const uint32_t c0 = pxs == kMaxChunkShift ? 2u * (lane >> pxs) : (lane >> pxs);  // its first channel
        const bool ch_on = chmode && c0 < 4u && cp < npx;
        // pixel lanes: pixel `lane`'s accumulator; channel lanes: .x = channel c0, .y = channel c0 + 1
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ch_on) {
            const float* af = reinterpret_cast<const float*>(accum) + 4u * (size_t)(pix0 + cp) + c0;
            acc.x = af[0];
            if (pxs == kMaxChunkShift) acc.y = af[1];
        }
        bool live_px = false;
        PrimaryState ps;
        if (lane < npx) {
            const uint32_t pix = pix0 + lane;
            if (!chmode) acc = accum[pix];
            const uint32_t lrow = pix / cam.width;
            const uint32_t x = pix - lrow * cam.width;
            const uint32_t y = cam.shard_rank + cam.shard_count * lrow;
            const F3 d = primary_dir(x, y, cam.inv_w, cam.inv_h, cam.aspect);
            // (a BVH scene's camera ray borrows the lane's traversal stack: empty between chunks)
            ps = primary_state<kBvh, kEnv, kShape>(prims, nodes, n_prims, prims, mats, sp, d, x + y * cam.width, stk);
            live_px = (__float_as_uint(ps.r1.w) & kHitBit) != 0u && 1u < sp.max_bounces;
        }
        // constant pixel's Lc: the sky radiance of a miss (0 + 1 * sky, or 0 without a sky), or after a hit
        // with max_bounces <= 1 bounce 0's emission
        F3 lc{ps.r1.x, ps.r1.y, ps.r1.z};
        if (!live_px && lane < npx && (__float_as_uint(ps.r1.w) & kHitBit)) {
            if (!kBvh) {
                lc = F3{ps.r4.x, ps.r4.y, ps.r4.z};
            } else {
                const float4 emi = sh_mats[2u * (__float_as_uint(ps.r1.w) & ~kHitBit) + 1u];
                lc = emi.w != 0.0f ? F3{0.0f + 1.0f * emi.x, 0.0f + 1.0f * emi.y, 0.0f + 1.0f * emi.z}
                                   : F3{0.f, 0.f, 0.f};
            }
        }
        if (kStats && lane == 0u) atomicAdd(&s_seg[0], n_frames * npx);  // bounce 0: one segment per path
        const uint32_t live_mask = (uint32_t)__ballot(live_px);  // bit j: pixel j is live (px <= 32)
        const uint32_t n_live = (uint32_t)__popc(live_mask);
#ifdef SPT_TIMELINE
        tl_pxs = pxs;
        tl_live = n_live;
#endif
        if (kOrdered && plan.cost && n_live == 0u && chunk < plan.n[0] && lane == 0u) plan.cost[chunk] = 0u;
        if (n_live == 0u) {  // a chunk of constant pixels (sky): every frame adds Lc, in order
            // (the channel lanes fetch their pixel's Lc from its pixel lane)
            const float lx = __shfl(lc.x, (int)cp, 64), ly = __shfl(lc.y, (int)cp, 64), lz = __shfl(lc.z, (int)cp, 64);
            const float v0 = c0 == 0u ? lx : (c0 == 1u ? ly : lz);
            const float v1 = c0 + 1u == 1u ? ly : lz;  // (32-pixel chunks: c0 + 1 is y or w)
            if (ch_on) {
                acc.x = add_frames(acc.x, c0, v0, n_frames);
                if (pxs == kMaxChunkShift) acc.y = add_frames(acc.y, c0 + 1u, v1, n_frames);
                float* af = reinterpret_cast<float*>(accum) + 4u * (size_t)(pix0 + cp) + c0;
                af[0] = acc.x;
                if (pxs == kMaxChunkShift) af[1] = acc.y;
            } else if (!chmode && lane < npx) {
                for (uint32_t f = 0; f < n_frames; ++f) acc = make_float4(acc.x + lc.x, acc.y + lc.y, acc.z + lc.z, acc.w + 1.0f);
                accum[pix0 + lane] = acc;
            }
            continue;
        }
        // the live pixels' states at their rank among the live pixels (the hand-out reads them by slot);
        // a constant pixel's Lc at record 0, entry n_live + (its rank among the constant pixels);
        // s_pix[j]: pixel j's live rank, or kConstPx | the entry of its Lc (read by accumulate)
        const uint32_t li = __builtin_amdgcn_mbcnt_lo(live_mask, 0u);  // live pixels below this lane
        if (live_px) {
            s_px[wave][0][li] = ps.r0;
            s_px[wave][1][li] = ps.r1;
            s_px[wave][2][li] = ps.r2;
        } else if (lane < npx) {
            s_px[wave][0][n_live + lane - li] = make_float4(lc.x, lc.y, lc.z, 0.f);
        }
        if (lane < px) s_pix[wave][lane] = (uint8_t)(live_px ? li : (kConstPx | (n_live + lane - li)));
        // Ring of kRingSlots path slots (slot s = frame * n_live + live rank; entry s mod kRingSlots):
        // the radiance of finished paths and a done byte per entry holding the slot's lap (s / kRingSlots
        // + 1, <= 128 for <= 1024 frames of <= 32 pixels), so entries are never cleared: a byte left by
        // the previous lap reads as not done.
        s_cnt[wave][lane] = 0;
        uint8_t* const ring_flg = reinterpret_cast<uint8_t*>(&s_cnt[wave][0]);
        // floor(s / n_live) for s < 2^15 as a high multiply by m = ceil(2^31 / n_live) (an SGPR):
        // (2s * m) >> 32 = floor(s / n_live + s * e / (n_live * 2^31)) with e < n_live, exact
        const uint32_t m_live = __builtin_amdgcn_readfirstlane((0x80000000u + n_live - 1u) / n_live);
        auto div_live = [&](uint32_t s) { return __umulhi(s << 1, m_live); };
        // kChan (small chunks, <= 16 live pixels): the ring's radiance entries are laid out per pixel —
        // pixel rank r owns the 2^sr_sh entries [r << sr_sh, (r + 1) << sr_sh), frame f at f mod 2^sr_sh
        // — so the accumulation of k frames reads each pixel's entries consecutively (unrolled, immediate
        // offsets) instead of at a stride of n_live slots with a wrap mask and an address per frame. The
        // window shrinks to 2^sr_sh frames of n_live slots (<= kRingSlots; the done bytes stay in slot
        // order). Other kernels keep slot order (entry = slot mod kRingSlots).
        constexpr bool kPixRing = kChan;
        const uint32_t sr_sh = kPixRing ? 8u - (32u - (uint32_t)__builtin_clz(2u * n_live - 1u) - 1u) : 0u;
        const uint32_t win = kPixRing ? (n_live << sr_sh) : kRingSlots;  // slots in flight past oldest_s
        auto ring_entry = [&](uint32_t s) {
            if (!kPixRing) return s & (kRingSlots - 1u);
            const uint32_t f = div_live(s);
            return ((s - f * n_live) << sr_sh) | (f & ((1u << sr_sh) - 1u));
        };
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // path state of this lane (bc = trace_ray's bounce_count); q = its slot
        uint32_t q = 0;
        bool have = false;
        F3 o{0.f, 0.f, 0.f}, d{0.f, 0.f, 0.f}, T{1.f, 1.f, 1.f}, L{0.f, 0.f, 0.f};
        uint32_t rng = 0, bc = 0;
        Trav tv;             // BVH scenes: the current ray's place in the tree
        bool tdone = false;  // ... and whether its traversal has finished
        // NEE (kNee): at a hit that continues, every random draw of the hit runs at once, in the
        // oracle's order — the light sample (3 draws), Russian roulette (1), the new direction (2) — so
        // the light sampling and the direction sampling run on the same lanes in the same step instead
        // of in alternate steps with the other lanes masked. The lane then traces its shadow ray — o =
        // the offset hit point, d = towards the sampled point, up to smax, an any-hit traversal in BVH
        // scenes — while the estimate waits in the slot's ring entry (the entry holds the path's radiance
        // only once the path has finished) and nd holds the continuation's direction. The step that
        // resolves it adds the estimate if nothing was hit, then the path goes on along nd (`after`) or
        // ends (Russian roulette ended it).
        // Flat scenes (kInline) trace the shadow ray in the step that drew it, at a site of its own after
        // the direction sampling, so every lane's step shades a hit (no lanes resolving a shadow ray while
        // the others shade); nd then holds the shadow ray's direction.
        constexpr bool kInline = kNee && !kBvh;
        bool shadow = false, after = false;
        float smax = 0.f;
        F3 nd{0.f, 0.f, 0.f};

        const uint32_t n_slots = n_frames * n_live;
        uint32_t next = 0;      // wave-uniform cursor: next slot to hand out
        uint32_t oldest_s = 0;  // the first slot not accumulated (a frame boundary: frame oldest_s / n_live)

        auto finish = [&](bool fin) {  // park L of a finished path in the ring and mark its entry done
            if (fin) {
                const uint32_t e = ring_entry(q);
                s_L[wave][0][e] = L.x;
                s_L[wave][1][e] = L.y;
                s_L[wave][2][e] = L.z;
                ring_flg[q & (kRingSlots - 1u)] = (uint8_t)((q / kRingSlots) + 1u);
            }
        };
        auto accumulate = [&]() {  // every completed frame, oldest first (the reference's frame order)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // the run of done slots from oldest_s: lane i reads the done bytes of slots a .. a + 3
            // (a = the 4-aligned slot below oldest_s, + 4i) in one LDS read; bytes of slots below
            // oldest_s are ignored (the next lap may have reused their entries)
            const uint32_t base = oldest_s & ~3u;
            const uint32_t a = base + 4u * lane_id_here();
            const uint32_t want = ((a / kRingSlots) + 1u) * 0x01010101u;
            const uint32_t w = reinterpret_cast<const uint32_t*>(ring_flg)[(a & (kRingSlots - 1u)) >> 2];
            const uint32_t keep = a == base ? ~0u << (8u * (oldest_s & 3u)) : ~0u;
            const uint32_t miss = (w ^ want) & keep;  // nonzero bytes: slots not done
            const unsigned long long full = __ballot(miss == 0u);
            const uint32_t dz = ~full == 0ull ? 64u : (uint32_t)__builtin_ctzll(~full);
            uint32_t run = 4u * dz;  // done slots from base
            if (dz < 64u)            // + the leading done bytes of the first dword that is not
                run += (uint32_t)__builtin_ctz((uint32_t)__builtin_amdgcn_readlane((int)miss, (int)dz)) >> 3;
            const uint32_t k = min(div_live(n_slots - oldest_s), div_live(run - (oldest_s & 3u)));  // complete frames
            if (k == 0u) return;
            if (ch_on) {
                // channel lanes: frames in pairs (both ring reads in flight at once), the adds in frame
                // order; a constant pixel adds its Lc (from LDS) where a live one reads its ring entry
                const uint32_t ix = s_pix[wave][cp];
                const bool lv = ix < kConstPx;
                const float* cl = reinterpret_cast<const float*>(&s_px[wave][0][ix & ((1u << kMaxChunkShift) - 1u)]);
                const uint32_t c1 = c0 + 1u;
                const bool two = pxs == kMaxChunkShift && c1 < 3u;  // a second radiance channel (x, y lanes)
                const float k0 = c0 < 3u ? cl[c0 < 3u ? c0 : 0u] : 0.f, k1 = cl[c1 < 3u ? c1 : 0u];
                if (kPixRing && c0 < 3u) {
                    // the pixel's k frames from f0 = the oldest frame: consecutive entries of its ring
                    // part, wrapping once at most (k <= 2^sr_sh); wave-uniform counts, four frames per
                    // round of reads, the adds in frame order (a constant pixel adds its Lc instead)
                    const uint32_t msk = (1u << sr_sh) - 1u;
                    const uint32_t j0 = div_live(oldest_s) & msk;
                    const uint32_t n1 = min(k, msk + 1u - j0);
                    const float* pr = &s_L[wave][c0 < 3u ? c0 : 0u][(lv ? ix : 0u) << sr_sh];
                    auto run = [&](const float* p, uint32_t n) {
                        uint32_t f = 0;
                        for (; f + 4u <= n; f += 4u) {
                            const float x0 = p[f], x1 = p[f + 1u], x2 = p[f + 2u], x3 = p[f + 3u];
                            // (an empty asm use: every lane loads, so the compiler does not sink each read
                            // into an exec-mask branch of its own for the live lanes)
                            asm volatile("" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3));
                            acc.x = (((acc.x + (lv ? x0 : k0)) + (lv ? x1 : k0)) + (lv ? x2 : k0)) + (lv ? x3 : k0);
                        }
                        for (; f < n; ++f) {
                            const float x0 = p[f];
                            asm volatile("" ::"v"(x0));
                            acc.x = acc.x + (lv ? x0 : k0);
                        }
                    };
                    run(pr + j0, n1);
                    run(pr, k - n1);
                } else if (c0 < 3u) {
                    const float* r0 = &s_L[wave][c0 < 3u ? c0 : 0u][0];
                    const float* r1 = &s_L[wave][c1 < 3u ? c1 : 0u][0];
                    uint32_t e = oldest_s + ix;
                    uint32_t f = 0;
                    // (the reads stay conditional here: unconditional ones measured C4 +0.4 % but C4 NEE
                    // -6 to -8 %, profiles/r06_h_ab_c4nee.txt)
                    for (; f + 2u <= k; f += 2u) {
                        const uint32_t e0 = e & (kRingSlots - 1u), e1 = (e + n_live) & (kRingSlots - 1u);
                        e += 2u * n_live;
                        const float x0 = lv ? r0[e0] : k0, x1 = lv ? r0[e1] : k0;
                        acc.x = (acc.x + x0) + x1;
                        if (two) {
                            const float y0 = lv ? r1[e0] : k1, y1 = lv ? r1[e1] : k1;
                            acc.y = (acc.y + y0) + y1;
                        }
                    }
                    if (f < k) {
                        const uint32_t e0 = e & (kRingSlots - 1u);
                        acc.x = acc.x + (lv ? r0[e0] : k0);
                        if (two) acc.y = acc.y + (lv ? r1[e0] : k1);
                    }
                } else {
                    acc.x = add_count(acc.x, k);  // w (4-16-pixel chunks: lanes 3 * px + p)
                }
                if (pxs == kMaxChunkShift && c1 == 3u) acc.y = add_count(acc.y, k);  // w (32-pixel chunks: z, w lanes)
            } else if (!chmode && lane < npx) {
                // pixel lanes (a flat scene's 32-pixel chunks): frames in pairs, all four channels (the reads
                // stay conditional here: unconditional ones measured C2 -0.4 %, profiles/r06_d_ab_acc_loads.txt)
                const uint32_t ix = s_pix[wave][lane];
                const bool lv = ix < kConstPx;
                const float4 c = s_px[wave][0][ix & ((1u << kMaxChunkShift) - 1u)];  // (live pixels: unused)
                uint32_t e = oldest_s + ix;
                uint32_t f = 0;
                for (; f + 2u <= k; f += 2u) {
                    const uint32_t e0 = e & (kRingSlots - 1u), e1 = (e + n_live) & (kRingSlots - 1u);
                    e += 2u * n_live;
                    const float x0 = lv ? s_L[wave][0][e0] : c.x, y0 = lv ? s_L[wave][1][e0] : c.y,
                                z0 = lv ? s_L[wave][2][e0] : c.z;
                    const float x1 = lv ? s_L[wave][0][e1] : c.x, y1 = lv ? s_L[wave][1][e1] : c.y,
                                z1 = lv ? s_L[wave][2][e1] : c.z;
                    acc.x = (acc.x + x0) + x1;
                    acc.y = (acc.y + y0) + y1;
                    acc.z = (acc.z + z0) + z1;
                    acc.w = (acc.w + 1.0f) + 1.0f;
                }
                if (f < k) {
                    const uint32_t e0 = e & (kRingSlots - 1u);
                    acc.x = acc.x + (lv ? s_L[wave][0][e0] : c.x);
                    acc.y = acc.y + (lv ? s_L[wave][1][e0] : c.y);
                    acc.z = acc.z + (lv ? s_L[wave][2][e0] : c.z);
                    acc.w = acc.w + 1.0f;
                }
            }
            oldest_s += k * n_live;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };

        // The loop runs on after the last path until every frame is accumulated (one call site of
        // accumulate), with a bound no correct run reaches (every path ends within max_bounces steps),
        // so that a wave always leaves it and the grid drains.
        uint32_t steps_left = (n_slots + 64u) * ((kNee ? 2u : 1u) * sp.max_bounces + 2u) + n_frames + 4096u;
        const uint32_t steps_init = steps_left;
        uint32_t titer = 0;  // BVH NEE kernels: the chunk's traversal iterations (its cost, with the steps)
        while ((__ballot(have) != 0ull || next < n_slots || oldest_s < n_slots) && steps_left-- != 0u) {
            // ---- one segment (bounce >= 1) for every lane with a live path ----
            SPT_MARK(step);
            bool fin = false;
            bool pend = false;  // a new direction is to be drawn around (dn, dt) below
            F3 dn{0.f, 0.f, 0.f}, dt{0.f, 0.f, 0.f};
            bool snew = false;  // kNee: a shadow ray starts (its direction in d; the continuation's goes to nd)
            // kNee: the hit's draws (o: its offset point, n: its normal, bc: the bounce count after the hit):
            // the light sample, then Russian roulette; the direction around (dn, dt) is drawn at the step's
            // sampling site below. A path that roulette ends with no shadow ray to trace ends here (fin).
            auto nee_hit = [&](F3 n, bool& fin) {
                F3 w, add;
                float tm;
                if (light_sample<kNee == kNeeAll>(nee.emit, nee.n_emit, o, n, T, rng, w, tm, add)) {
                    const uint32_t e = ring_entry(q);
                    s_L[wave][0][e] = add.x;
                    s_L[wave][1][e] = add.y;
                    s_L[wave][2][e] = add.z;
                    if (kInline) nd = w;
                    else d = w;
                    smax = tm;
                    shadow = true;
                    snew = true;
                    if (kStats) atomicAdd(&s_shadow[0], 1u);
                }
                after = rr_continue(sp, bc, T, rng);
                if (after) {
                    dn = n;
                    pend = true;
                } else if (!snew) {
                    have = false;
                    fin = true;
                }
            };
            if (kBvh) {
                // incoherent rays need very different numbers of traversal steps: advance them
                // until kBvhBatch lanes wait, instead of until the wave's slowest ray is done
                // (written out here rather than calling advance_rays: measured 4 % faster on C4)
                const bool can_start = next < min(n_slots, oldest_s + win);
                for (;;) {
                    const bool trav = have && !tdone;
                    const unsigned long long tm = __ballot(trav);
                    if (tm == 0ull) break;
                    if ((uint32_t)__popcll(__ballot(have ? tdone : can_start)) >= (kNee ? kBvhBatchNee : kBvhBatch)) break;
                    if (kStats) {
                        lane_slots += 64u;
                        lane_busy += (uint32_t)__popcll(tm);
                    }
                    if (kNee) ++titer;
                    if (trav) tdone = trav_step<kStats, false, kNee != 0>(nodes, prims, o, d, tv, stk, &bvh_ctr, s_top, n_top);
                }
            }
            const bool ready = kBvh ? (have && tdone) : have;
            const unsigned long long tracing = __ballot(ready);
            if (tracing != 0ull) {
                if (kStats && !kBvh) {
                    lane_slots += 64u;
                    lane_busy += (uint32_t)__popcll(tracing);
                }
                if (ready) {
                    float best_t = (kNee && !kInline && shadow) ? smax : kInf;
                    uint32_t best_k = kMiss;
                    if (kBvh) {
                        best_t = tv.best_t;
                        best_k = tv.best_k;
                    } else {
                        SPT_MARK(closest);
                        closest_flat<kShape>(prims, n_prims, o, d, best_t, best_k, (sp.flags & kFlagFastDiv) != 0u, sp.flat_ends);
                    }
                    if constexpr (kNee) {
                        if (!kInline && shadow) {  // the shadow ray: the estimate counts if nothing was hit before smax
                            shadow = false;
                            if (!(best_t < smax)) {
                                const uint32_t e = ring_entry(q);
                                L = F3{L.x + s_L[wave][0][e], L.y + s_L[wave][1][e], L.z + s_L[wave][2][e]};
                            }
                            if (after) {  // on along the direction drawn at the hit
                                d = nd;
                                if (kBvh) {
                                    trav_init(tv, d);
                                    tdone = false;
                                }
                            } else {
                                fin = true;
                                have = false;
                            }
                        } else {
                            bool alive;
                            F3 add, n;
                            const bool contributes = shade_hit<kEnv, !kBvh, true>(sh_prims, sh_mats, sp, bc + 1u, best_t,
                                                                                  best_k, o, d, T, rng, alive, add, n);
                            if (contributes) L = F3{L.x + add.x, L.y + add.y, L.z + add.z};
                            if (kStats) {
                                atomicAdd(&s_seg[bc], 1u);
                                if (contributes) atomicAdd(&s_rmw[bc], 1u);
                            }
                            ++bc;
                            fin = !alive;
                            have = alive;
                            if (alive) {
                                o = offset_origin(o, n);
                                nee_hit(n, fin);
                                if (pend) dt = bounce_tangent(n, sp.flags);
                            }
                        }
                    } else {
                    bool alive;
                    F3 add;
                    SPT_MARK(shade);
                    const bool contributes =
                        shade_hit<kEnv, !kBvh>(sh_prims, sh_mats, sp, bc + 1u, best_t, best_k, o, d, T, rng, alive, add, dn);
                    if (alive) {
                        dt = bounce_tangent(dn, sp.flags);
                        pend = true;
                    }
                    if (contributes) L = F3{L.x + add.x, L.y + add.y, L.z + add.z};
                    if (kStats) {
                        atomicAdd(&s_seg[bc], 1u);
                        if (contributes) atomicAdd(&s_rmw[bc], 1u);
                    }
                    ++bc;
                    fin = !alive;
                    have = alive;
                    }
                }
                finish(fin);
            }
            SPT_MARK(acc_check);
            // Lazy accumulation: completed frames only need adding (in order) once the ring window
            // limits the next hand-out; until then they wait in the ring and the step skips the check
            if (next + 64u > min(n_slots, oldest_s + win)) accumulate();
            SPT_MARK(handout);
            // ---- hand the next slots to lanes without a path; bounce 0 from the pixel's state ----
            const bool idle = !have;
            const unsigned long long m = __ballot(idle);
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint32_t limit = min(n_slots, oldest_s + win);
            bool fin0 = false;
            const bool take = idle && next + rank < limit;
            if (take) {
                q = next + rank;
                const uint32_t f = div_live(q);  // the slot's frame and its pixel's live rank
                const uint32_t r = q - f * n_live;
                const uint32_t frame = cam.first_frame + f + 1u;
                const float4 p0 = s_px[wave][0][r];
                const float4 p1 = s_px[wave][1][r];
                bool alive = true;  // a live pixel: a hit, and bounce_count 1 < max_bounces
                if (!kBvh) {  // ... from the hit primitive's LDS shading record (make_shade_recs)
                    const uint32_t k = __float_as_uint(p1.w) & ~kHitBit;
                    const float4 alb = s_scene[3u * k + 1u];
                    const float4 emi = s_scene[3u * k + 2u];
                    L = emi.w != 0.0f ? F3{0.0f + 1.0f * emi.x, 0.0f + 1.0f * emi.y, 0.0f + 1.0f * emi.z}
                                      : F3{0.f, 0.f, 0.f};
                    T = F3{1.0f * alb.x, 1.0f * alb.y, 1.0f * alb.z};
                } else {
                    const uint32_t mat = __float_as_uint(p1.w) & ~kHitBit;  // BVH scenes: the material record
                    const float4 alb = sh_mats[2 * mat + 0];
                    const float4 emi = sh_mats[2 * mat + 1];
                    L = emi.w != 0.0f ? F3{0.0f + 1.0f * emi.x, 0.0f + 1.0f * emi.y, 0.0f + 1.0f * emi.z}
                                      : F3{0.f, 0.f, 0.f};
                    T = F3{1.0f * alb.x, 1.0f * alb.y, 1.0f * alb.z};
                }
                rng = rng_seed(__float_as_uint(p0.w), 0u, 0u, frame);
                if constexpr (kNee) {  // bounce 0's draws from the camera hit's offset point
                    o = F3{p1.x, p1.y, p1.z};
                    bc = 1u;
                    have = true;
                    nee_hit(F3{p0.x, p0.y, p0.z}, fin0);
                    if (pend) {
                        const float4 p2 = s_px[wave][2][r];
                        dt = F3{p2.x, p2.y, p2.z};
                    }
                    alive = false;  // (the direction follows at the sampling site)
                } else
                if (1u > sp.rr_depth) {  // Russian roulette at bounce_count 1 (:264-270)
                    const float cp = fmaxf(fmaxf(T.x, T.y), T.z);
                    if (random_float(rng) > cp) alive = false;
                    else T = rr_divide(T, cp);
                }
                if (alive) {
                    const float4 p2 = s_px[wave][2][r];
                    dn = F3{p0.x, p0.y, p0.z};
                    dt = F3{p2.x, p2.y, p2.z};
                    pend = true;
                    o = F3{p1.x, p1.y, p1.z};
                    bc = 1u;
                    have = true;
                }
                if (!kNee) fin0 = !alive;
            }
            finish(fin0);
            next = min(limit, next + (uint32_t)__popcll(m));
            SPT_MARK(accumulate_handout_done);
            // ---- new directions (get_random_bounche, :273-274) for continuing and new paths alike:
            // one copy of the sampling code per step instead of one per branch ----
            if (pend) {
                SPT_MARK(sample);
                const F3 dir = bounce_dir_frame<true>(dn, dt, rng);
                if (kNee && !kInline && snew) {  // (a shadow ray is traced first: the continuation waits in nd)
                    nd = dir;
                } else {
                    d = dir;
                    if (kBvh) {
                        trav_init(tv, d);
                        tdone = false;
                    }
                }
            }
            if (kNee && kBvh && snew) {  // a shadow ray's any-hit traversal, culled against smax
                trav_init_shadow(tv, d, smax);
                tdone = false;
            }
            if constexpr (kInline) {  // flat scenes: this step's shadow rays (o, nd, up to smax)
                bool fin_s = false;
                if (shadow) {
                    SPT_MARK(shadow);
                    shadow = false;
                    float bt = smax;
                    uint32_t bk = kMiss;
                    closest_flat<kShape>(prims, n_prims, o, nd, bt, bk, (sp.flags & kFlagFastDiv) != 0u, sp.flat_ends);
                    if (!(bt < smax)) {
                        const uint32_t e = ring_entry(q);
                        L = F3{L.x + s_L[wave][0][e], L.y + s_L[wave][1][e], L.z + s_L[wave][2][e]};
                    }
                    if (!after) {  // Russian roulette ended the path at the hit
                        have = false;
                        fin_s = true;
                    }
                }
                finish(fin_s);
            }
        }
        // the bound reached (steps_left wrapped): a logic error, reported instead of a silent partial image
        if (steps_left == ~0u && lane == 0u) atomicAdd(&totals[kTotStalled], 1ull);
        // the chunk's cost: its step-loop iterations (the same in every launch of this scene and shape);
        // with NEE in a BVH scene its traversal iterations count too (a shadow ray's traversal takes no
        // step of its own: ordered by steps alone C4 NEE lost 3-4 %, by steps x 4 + traversal iterations it
        // gains 8 %, profiles/r06_p_ab_bvh_nee_cost.txt)
        if (kOrdered && plan.cost && chunk < plan.n[0] && lane == 0u)
            plan.cost[chunk] = (uint16_t)min(65535u, (kBvh && kNee) ? ((steps_init - steps_left) * 4u + titer) >> 2
                                                                    : steps_init - steps_left);
        if (ch_on) {
            float* af = reinterpret_cast<float*>(accum) + 4u * (size_t)(pix0 + cp) + c0;
            af[0] = acc.x;
            if (pxs == kMaxChunkShift) af[1] = acc.y;
        } else if (!chmode && lane < npx) {
            accum[pix0 + lane] = acc;
        }
    }
#ifdef SPT_TIMELINE
    if (lane == 0u) {
        unsigned long long* r = g_tl + 4u * (blockIdx.x * kWaves + wave);
        r[0] = tl_start;
        r[1] = tl_last;
        r[2] = wall_clock64();
        r[3] = tl_chunks | ((unsigned long long)xcc << 32) | ((unsigned long long)tl_pxs << 40) |
               ((unsigned long long)tl_live << 48);
    }
#endif
    if (kStats) {
        if (lane == 0u) {
            atomicAdd(&totals[2u * kMaxBounces], (unsigned long long)lane_slots);
            atomicAdd(&totals[2u * kMaxBounces + 1u], (unsigned long long)lane_busy);
        }
        if (kBvh) {
            atomicAdd(&totals[2u * kMaxBounces + 2u], (unsigned long long)bvh_ctr.nodes);
            atomicAdd(&totals[2u * kMaxBounces + 3u], (unsigned long long)bvh_ctr.prims);
        }
        __syncthreads();
        if (threadIdx.x < sp.max_bounces) {
            if (s_seg[threadIdx.x]) atomicAdd(&totals[threadIdx.x], (unsigned long long)s_seg[threadIdx.x]);
            if (s_rmw[threadIdx.x]) atomicAdd(&totals[kMaxBounces + threadIdx.x], (unsigned long long)s_rmw[threadIdx.x]);
        }
        if (kNee && threadIdx.x == 0u && s_shadow[0]) atomicAdd(&totals[kTotShadow], (unsigned long long)s_shadow[0]);
    }
}

// ---------------------------------------------------------------------------------------------
// resolve: get_render_result (CPUPathTracer.cpp:87-117) + rgba_to_uint32 (Color.h:7-10)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t to_u8(float v, float frames) {
    float c = v / frames;
    c = c < 0.0f ? 0.0f : (1.0f < c ? 1.0f : c);  // std::clamp(c, 0.0f, 1.0f)
    if (c != c) c = 0.0f;                          // NaN: defined as 0 here (UB in the reference)
    return (uint32_t)(uint8_t)(c * 255.0f);
}

// exposure: the reference's commented-out `r *= getExposure()` (:101-104) on r, g, b after the
// division; 1.0f (reference mode) is an exact identity
__device__ __forceinline__ uint32_t to_u8(float v, float frames, float exposure) {
    float c = v / frames;
    c = c * exposure;
    c = c < 0.0f ? 0.0f : (1.0f < c ? 1.0f : c);
    if (c != c) c = 0.0f;
    return (uint32_t)(uint8_t)(c * 255.0f);
}

// one pixel's RGBA8: rgba_to_uint32(r, g, b, a) of the resolved channels (alpha without exposure)
__device__ __forceinline__ uint32_t rgba8(float4 a, float frames, float exposure) {
    return (to_u8(a.x, frames, exposure) << 24) | (to_u8(a.y, frames, exposure) << 16) |
           (to_u8(a.z, frames, exposure) << 8) | to_u8(a.w, frames);
}

// ---------------------------------------------------------------------------------------------
// k_frame: ONE frame per launch (calls of 1-3 frames, e.g. the App's one frame per UI frame,
// CPUPathTracer.cpp:43-85), persistent waves like k_paths. A frame holds exactly one path per
// pixel, so a path that ends adds its radiance straight into the pixel's accumulator
// (CPUPathTracer.cpp:77-80, one read-modify-write, no ordering to keep inside the launch; frames of
// a multi-frame call are stream-ordered launches). No ring and no per-pixel primary cache: every
// camera ray is traced as an ordinary segment. Lanes take pixels one at a time from the wave's
// current run of frame_chunk() pixels, which the wave pulls from the per-XCD work heads.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kFrameRun = 128;          // k_frame: pixels per work unit, flat scenes
constexpr uint32_t kFrameRunBvh = 64;        // ... BVH scenes
constexpr uint32_t kFrameBvhBatch = 24;        // k_frame: BVH lanes waiting before a shading round
constexpr uint32_t kFrameBvhBatchLds = 64;   // ... for a scene held whole in LDS: one round per segment
constexpr uint32_t kFrameLdsStackMax = 16;   // k_frame kSmall: LDS stack entries per lane at most (8 B each)
// pixels per work unit of k_frame: BVH scenes take shorter runs (their paths' lengths vary more, so
// the frame's tail is shorter with finer units: App +4.5 %, C4 one frame per call +11 % at 64 vs 128;
// flat scenes lose 33 % at 64)
__host__ __device__ constexpr uint32_t frame_chunk(bool bvh) { return bvh ? kFrameRunBvh : kFrameRun; }

// kSmall (BVH scenes of <= kFrameTopNodes nodes and <= kFrameTopPrims primitives, the App's):
// the whole scene and every lane's traversal stack live in LDS (the stack in the dynamic LDS, sized by
// the host from the tree's deepest stack), so a traversal step touches no global memory: its LDS loads
// no longer wait on the global stack's stores and reads (one vector-memory counter for both).
constexpr int kFrameWavesSmall = 5;  // kSmall: its LDS (tree, primitives, stacks: ~31 KB per block) allows 5
// kNee: next-event estimation (SPT_FLAG_NEE; the shadow ray is the lane's next segment, as in k_paths;
// kNeeAll / kNeeNoSpheres as in k_paths);
// run with kEnv = 2.
// kRgba: the resolve fused into the launch (cam.rgba, spt_render_resolve_rgba8); a separate
// instantiation, so the frames that are not resolved keep their code
template <bool kStats, bool kBvh, int kEnv, uint64_t kShape = 0, bool kSmall = false, int kNee = 0, bool kRgba = false>
__global__ __launch_bounds__(kBlock, kSmall ? kFrameWavesSmall : (kBvh ? kPathsWavesBvh : kPathsWaves)) void k_frame(const float4* __restrict__ prims, const float4* __restrict__ mats,
                                                  const float4* __restrict__ nodes, uint32_t n_prims,
                                                  float4* __restrict__ accum,
                                                  unsigned long long* __restrict__ totals,
                                                  uint32_t* __restrict__ work, uint32_t* __restrict__ work_next,
                                                  ShadeParams sp, CameraParams cam, NeeParams nee) {
    bake_config<kShape>(sp);
    // the next launch's work heads (stream order: the previous user of that set has finished)
    if (blockIdx.x == 0u && threadIdx.x < kWorkHeads) work_next[threadIdx.x * kWorkStride] = 0u;
    // hit_mode 3: the live pixels' records are the launch's work units; the sky pixels — a camera miss,
    // the same radiance in every frame — are added by the first cam.sky_blocks blocks, which trace
    // nothing and end, so the tracing waves start their paths at once (the sky blocks run beside them)
    const bool lists = cam.hit_mode == 3u;
    const uint32_t sky_blocks = lists ? cam.sky_blocks : 0u;
    if (blockIdx.x < sky_blocks) {
        const uint32_t n_sky = __builtin_amdgcn_readfirstlane(cam.list_counts[1]);
        for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n_sky; i += sky_blocks * kBlock) {
            const uint32_t px = cam.sky_pix[i];
            const CameraRay cr = camera_ray(cam, px);
            float4 a = accum[px];
            // shade_hit's miss with T = 1 on L = 0 (CPUPathTracer.cpp:231-235), then :77-80
            F3 lc{0.f, 0.f, 0.f};
            if (sp.sky_enabled) {
                const F3 sky = sky_radiance<kEnv>(sp, cr.d);
                lc = F3{0.0f + 1.0f * sky.x, 0.0f + 1.0f * sky.y, 0.0f + 1.0f * sky.z};
            }
            a.x = a.x + lc.x;
            a.y = a.y + lc.y;
            a.z = a.z + lc.z;
            a.w = a.w + 1.0f;
            accum[px] = a;
            if (kRgba) cam.rgba[px] = rgba8(a, cam.rgba_frames, cam.rgba_exposure);
        }
        if (kStats && blockIdx.x == 0u && threadIdx.x == 0u) {  // their camera segments, counted as before
            atomicAdd(&totals[0], (unsigned long long)n_sky);
            if (sp.sky_enabled) atomicAdd(&totals[kMaxBounces], (unsigned long long)n_sky);
        }
        return;  // (the whole block: no barrier below is reached by part of it)
    }
    const uint32_t bx = blockIdx.x - sky_blocks;  // the tracing block's index
    const uint32_t n_blocks = gridDim.x - sky_blocks;
    extern __shared__ float4 s_scene[];
    __shared__ uint32_t s_seg[kMaxBounces];
    __shared__ uint32_t s_rmw[kMaxBounces];
    __shared__ uint32_t s_shadow[1];  // kStats && kNee: shadow rays traced
    if (kStats && kNee && threadIdx.x == 0u) s_shadow[0] = 0u;
    if (!kBvh) make_shade_recs(prims, mats, sp.n_prims, s_scene);  // flat scenes: LDS shading records
    // BVH scenes: the tree's top nodes in LDS (breadth-first numbering; this kernel has LDS to spare,
    // and a small tree — the App's 38 spheres — fits whole)
    constexpr uint32_t kTop = kBvh ? kFrameTopNodes : 0u;
    __shared__ float4 s_top[kTop ? (kSmall ? 7u : 4u) * kTop : 1u];
    const uint32_t n_top = min(kTop, sp.n_nodes);
    if constexpr (kSmall) {  // the whole tree, decoded once per block: no decode in the traversal steps
        for (uint32_t k = threadIdx.x; k < n_top; k += kBlock) {
            const NodeBoxes b = node_boxes(nodes[4u * k], nodes[4u * k + 1u], nodes[4u * k + 2u]);
            float4* t = s_top + 7u * k;
            t[0] = b.lx;
            t[1] = b.ly;
            t[2] = b.lz;
            t[3] = b.hx;
            t[4] = b.hy;
            t[5] = b.hz;
            t[6] = nodes[4u * k + 3u];
        }
    } else {
        for (uint32_t k = threadIdx.x; k < 4u * n_top; k += kBlock) s_top[k] = nodes[k];
    }
    // ... and a small scene's primitive records too (all of them or none: leaf order; padded by 3
    // float4 for the LDS-only step's 7-float4 reads); kSmall: its material records after them
    // (frame_small_scene checks they fit), so a path's chain of dependent loads — traversal steps and
    // shading gathers — touches no global memory after its first segment
    constexpr uint32_t kPTop = kBvh ? kFrameTopPrims : 0u;
    __shared__ float4 s_ptop[kPTop ? 4u * kPTop + 3u : 1u];
    const uint32_t n_ptop = sp.n_prims <= kPTop ? sp.n_prims : 0u;
    for (uint32_t k = threadIdx.x; k < 4u * n_ptop; k += kBlock) s_ptop[k] = prims[k];
    float4* const s_mtop = s_ptop + (4u * n_ptop + 3u);
    if (kSmall)
        for (uint32_t k = threadIdx.x; k < 2u * sp.n_mats; k += kBlock) s_mtop[k] = mats[k];
    if (kStats && threadIdx.x < kMaxBounces) {
        s_seg[threadIdx.x] = 0;
        s_rmw[threadIdx.x] = 0;
    }
    __syncthreads();
    const float4* sh_prims = kBvh ? (kSmall ? s_ptop : prims) : s_scene;
    const float4* sh_mats = kSmall ? s_mtop : mats;

    const uint32_t lane = __lane_id();
    const uint32_t P = lists ? __builtin_amdgcn_readfirstlane(cam.list_counts[0]) : cam.shard_pixels;
    uint32_t lane_slots = 0, lane_busy = 0;
    BvhCounters bvh_ctr;
    uint32_t cur = 0, end = 0;  // wave-uniform: pixels [cur, end) of the current run are not started yet
    bool more = true;           // wave-uniform: the work heads may still hand out runs
    constexpr uint32_t kFrameChunk = frame_chunk(kBvh);
    const uint32_t n_runs = (P + kFrameChunk - 1u) / kFrameChunk;
    const uint32_t xcc = xcc_id();
    uint32_t heads_empty = 0;
    // The first run of each wave is its global wave index, taken without an atomic; the work heads
    // deal only the runs past the grid's waves. A one-frame launch starts all its waves at once, and
    // their first pulls queued on the heads (one word serves ~88 dequeues/us): the App's 512² frame
    // (4096 runs, 4096 waves, so no queue at all now) 76 -> 51 us, Cornell 1080p one frame per call
    // +4 %. (k_paths keeps the queue for its first chunks: -1 % on C2 with them static — its
    // waves' first pulls are spread over the launch's start.)
    const uint32_t n_waves = n_blocks * (kBlock / 64u);
    const uint32_t n_queued = n_runs > n_waves ? n_runs - n_waves : 0u;
    bool first = true;
    uint32_t pix = 0, rng = 0, bc = 0;
    bool have = false;
    F3 o{0.f, 0.f, 0.f}, d{0.f, 0.f, 0.f}, T{1.f, 1.f, 1.f}, L{0.f, 0.f, 0.f};
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);  // the pixel's accumulator, loaded when the path starts
    // The camera has no jitter (CPUPathTracer.cpp:63-69), so a pixel's camera segment has the same closest
    // hit in every frame: the first launch after a scene or configuration change stores it per pixel
    // (hit_mode 1), later launches take it instead of tracing the segment (hit_mode 2). Same (t, k), so
    // the same bits; the counters still count the segment.
    // the fused resolve (cam.rgba): the lane's finished pixel waits for its RGBA8 store until the lane
    // starts its next pixel or leaves, so a wave whose lanes take one pixel each (the App's 512² frame)
    // stores its run in one coalesced write over PCIe instead of one partial line per ending round
    bool pend = false;
    bool cached = false;               // this path's camera hit comes from the cache
    float2 ch = make_float2(0.f, 0.f);  // ... (t, primitive index bits)
    const auto stk = lane_stack(sp, bx * (kBlock / 64u) + threadIdx.x / 64u, lane);  // BVH scenes
    const StkL stk_lds{reinterpret_cast<uint2*>(s_scene) + threadIdx.x};  // kSmall
    Trav tv;
    bool tdone = false;
    // kNee: the lane's shadow ray (o = the offset hit point, d = towards the sampled point, up to smax,
    // any-hit), its estimate sadd, and — every draw of the hit made at the hit, in the oracle's order:
    // light sample, roulette, direction — whether the path goes on after it (`after`) along nd
    bool shadow = false, after = false;
    float smax = 0.f;
    F3 nd{0.f, 0.f, 0.f}, sadd{0.f, 0.f, 0.f};
    // A scene held whole in LDS (its primitive records copied above) traverses in a few LDS round
    // trips, and then one shading round per segment for the whole wave beats rounds of kBvhBatch
    // lanes (the App's 512² frame 51 -> 46 us; C4, from global memory, loses 25 % with it)
    const uint32_t batch = n_ptop ? kFrameBvhBatchLds : kFrameBvhBatch;
    // the finished pixel's RGBA8 (k_resolve's), from the same sum the accumulator was stored with
    const auto put_rgba = [&]() {
        float4 a = acc;
        a.x = a.x + L.x;
        a.y = a.y + L.y;
        a.z = a.z + L.z;
        a.w = a.w + 1.0f;
        cam.rgba[pix] = rgba8(a, cam.rgba_frames, cam.rgba_exposure);
    };
    for (;;) {
        // ---- one segment for every lane with a live path (bounce 0 included) ----
        if constexpr (kSmall)
            advance_rays<kStats, true>(nodes, prims, have, more || cur < end, o, d, tv, tdone, stk_lds, bvh_ctr,
                                       lane_slots, lane_busy, s_top, n_top, s_ptop, n_ptop, batch);
        else if (kBvh)
            advance_rays<kStats, false, kNee != 0>(nodes, prims, have, more || cur < end, o, d, tv, tdone, stk, bvh_ctr,
                                 lane_slots, lane_busy, s_top, n_top, s_ptop, n_ptop, batch);
        const bool ready = kBvh ? (have && tdone) : have;
        const unsigned long long tracing = __ballot(ready);
        if (tracing != 0ull) {
            if (kStats && !kBvh) {
                lane_slots += 64u;
                lane_busy += (uint32_t)__popcll(tracing);
            }
            if (ready) {
                float best_t = (kNee && shadow) ? smax : kInf;
                uint32_t best_k = kMiss;
                if (cached) {  // the camera segment, from the cache
                    best_t = ch.x;
                    best_k = __float_as_uint(ch.y);
                    cached = false;
                } else if (kBvh) {
                    best_t = tv.best_t;
                    best_k = tv.best_k;
                } else {
                    closest_flat<kShape>(prims, n_prims, o, d, best_t, best_k, (sp.flags & kFlagFastDiv) != 0u, sp.flat_ends);
                }
                if (cam.hit_mode == 1u && bc == 0u && !(kNee && shadow))
                    cam.hit_cache[pix] = make_float2(best_t, __uint_as_float(best_k));
                if constexpr (kNee) {
                    bool done = false, trace = false;
                    if (shadow) {  // the estimate counts if nothing was hit before smax
                        shadow = false;
                        if (!(best_t < smax)) L = F3{L.x + sadd.x, L.y + sadd.y, L.z + sadd.z};
                        if (after) {  // on along the direction drawn at the hit
                            d = nd;
                            trace = true;
                        } else {
                            done = true;
                        }
                    } else {
                        bool alive;
                        F3 add, n;
                        const bool contributes = shade_hit<kEnv, !kBvh, true>(sh_prims, sh_mats, sp, bc + 1u, best_t,
                                                                              best_k, o, d, T, rng, alive, add, n);
                        if (contributes) L = F3{L.x + add.x, L.y + add.y, L.z + add.z};
                        if (kStats) {
                            atomicAdd(&s_seg[bc], 1u);
                            if (contributes) atomicAdd(&s_rmw[bc], 1u);
                        }
                        ++bc;
                        if (alive) {  // light sample, Russian roulette, then get_random_bounche (:264-274)
                            o = offset_origin(o, n);
                            F3 w;
                            float tm;
                            if (light_sample<kNee == kNeeAll>(nee.emit, nee.n_emit, o, n, T, rng, w, tm, sadd)) {
                                if (kStats) atomicAdd(&s_shadow[0], 1u);
                                if constexpr (!kBvh) {  // flat scenes: the shadow ray traced here, at once
                                    float bt = tm;
                                    uint32_t bk = kMiss;
                                    closest_flat<kShape>(prims, n_prims, o, w, bt, bk, (sp.flags & kFlagFastDiv) != 0u,
                                                         sp.flat_ends);
                                    if (!(bt < tm)) L = F3{L.x + sadd.x, L.y + sadd.y, L.z + sadd.z};
                                } else {
                                    d = w;
                                    smax = tm;
                                    shadow = true;
                                    trace = true;
                                }
                            }
                            after = rr_continue(sp, bc, T, rng);
                            if (after) {
                                const F3 dir = bounce_dir<true>(n, rng, sp.flags);
                                if (shadow) {
                                    nd = dir;
                                } else {
                                    d = dir;
                                    trace = true;
                                }
                            } else if (!shadow) {
                                done = true;
                            }
                        } else {
                            done = true;
                        }
                    }
                    if (done) {  // accumulation += color (:77-80)
                        float4 a = acc;
                        a.x = a.x + L.x;
                        a.y = a.y + L.y;
                        a.z = a.z + L.z;
                        a.w = a.w + 1.0f;
                        accum[pix] = a;
                        pend = kRgba;
                    }
                    if (kBvh && trace) {
                        if (shadow) trav_init_shadow(tv, d, smax);
                        else trav_init(tv, d);
                        tdone = false;
                    }
                    have = !done;
                } else {
                bool alive;
                F3 add, n;
                const bool contributes =
                    shade_hit<kEnv, !kBvh>(sh_prims, sh_mats, sp, bc + 1u, best_t, best_k, o, d, T, rng, alive, add, n);
                if (contributes) L = F3{L.x + add.x, L.y + add.y, L.z + add.z};
                if (kStats) {
                    atomicAdd(&s_seg[bc], 1u);
                    if (contributes) atomicAdd(&s_rmw[bc], 1u);
                }
                ++bc;
                if (alive) {
                    d = bounce_dir<true>(n, rng, sp.flags);  // get_random_bounche (:273-274)
                    if (kBvh) {
                        trav_init(tv, d);
                        tdone = false;
                    }
                } else {                               // accumulation += color (:77-80), color.a = 1 (:283)
                    float4 a = acc;
                    a.x = a.x + L.x;
                    a.y = a.y + L.y;
                    a.z = a.z + L.z;
                    a.w = a.w + 1.0f;
                    accum[pix] = a;
                    pend = kRgba;
                }
                have = alive;
                }
            }
        }
        // ---- idle lanes start the next pixels' camera paths (:57-73) ----
        const bool idle = !have;
        const unsigned long long m = __ballot(idle);
        const uint32_t n_idle = (uint32_t)__popcll(m);
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t rem = end - cur;
        uint32_t nc = 0;
        bool got = false;
        if (more && rem < n_idle) {  // the run cannot serve every idle lane: pull the next one too
            uint32_t run;
            if (first) {
                run = __builtin_amdgcn_readfirstlane(bx * (kBlock / 64u) + threadIdx.x / 64u);
                first = false;
            } else {
                run = n_queued ? pull_unit(work, n_queued, xcc, heads_empty) + (n_runs - n_queued) : n_runs;
            }
            if (run >= n_runs) {
                more = false;
            } else {
                nc = run * kFrameChunk;
                got = true;
            }
        }
        const uint32_t nend = got ? min(nc + kFrameChunk, P) : 0u;
        if (idle) {
            uint32_t slot = P;
            if (rank < rem) slot = cur + rank;
            else if (got && nc + (rank - rem) < nend) slot = nc + (rank - rem);
            if (slot < P) {
                if (kRgba && pend) {
                    put_rgba();
                    pend = false;
                }
                pix = slot;
                cached = cam.hit_mode == 2u;
                if (cached) ch = cam.hit_cache[slot];  // (in flight until the segment is shaded)
                if (lists) {  // a live pixel's record: its index and camera hit
                    const uint4 rec = cam.live_rec[slot];
                    pix = rec.x;
                    ch = make_float2(__uint_as_float(rec.y), __uint_as_float(rec.z));
                    cached = true;
                }
                acc = accum[pix];  // in flight while the path is traced
                const CameraRay cr = camera_ray(cam, pix);
                o = F3{0.f, 0.f, 0.f};
                d = cr.d;
                T = F3{1.f, 1.f, 1.f};
                L = F3{0.f, 0.f, 0.f};
                rng = cr.seed;
                bc = 0;
                have = true;
                if (kBvh) {
                    trav_init(tv, d);
                    tdone = cached;  // the camera segment's closest hit is known: no traversal
                }
            }
        }
        if (got) {
            cur = min(nc + (n_idle - rem), nend);
            end = nend;
        } else {
            cur += min(rem, n_idle);
        }
        if (!more && cur == end && __ballot(have) == 0ull) break;
    }
    if (kRgba && pend) put_rgba();
    if (kStats) {
        if (lane == 0u) {
            atomicAdd(&totals[2u * kMaxBounces], (unsigned long long)lane_slots);
            atomicAdd(&totals[2u * kMaxBounces + 1u], (unsigned long long)lane_busy);
        }
        if (kBvh) {
            atomicAdd(&totals[2u * kMaxBounces + 2u], (unsigned long long)bvh_ctr.nodes);
            atomicAdd(&totals[2u * kMaxBounces + 3u], (unsigned long long)bvh_ctr.prims);
        }
        __syncthreads();
        if (threadIdx.x < sp.max_bounces) {
            if (s_seg[threadIdx.x]) atomicAdd(&totals[threadIdx.x], (unsigned long long)s_seg[threadIdx.x]);
            if (s_rmw[threadIdx.x]) atomicAdd(&totals[kMaxBounces + threadIdx.x], (unsigned long long)s_rmw[threadIdx.x]);
        }
        if (kNee && threadIdx.x == 0u && s_shadow[0]) atomicAdd(&totals[kTotShadow], (unsigned long long)s_shadow[0]);
    }
}

// ---------------------------------------------------------------------------------------------
// The camera-hit cache compacted (kFrameHitCache 2), once per scene / configuration, in pixel
// order: blocks of 256 pixels count their live pixels (a hit), one block scans the counts, and each
// block scatters its live pixels' records and sky pixels' indices at the scanned offsets.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_hit_count(const float2* __restrict__ hits, uint32_t n,
                                                     uint32_t* __restrict__ block_live) {
    __shared__ uint32_t s_c[kBlock / 64u];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const bool live = i < n && __float_as_uint(hits[i].y) != kMiss;
    const unsigned long long b = __ballot(live);
    if (__lane_id() == 0u) s_c[threadIdx.x / 64u] = (uint32_t)__popcll(b);
    __syncthreads();
    if (threadIdx.x == 0u) {
        uint32_t c = 0;
        for (uint32_t w = 0; w < kBlock / 64u; ++w) c += s_c[w];
        block_live[blockIdx.x] = c;
    }
}

__global__ __launch_bounds__(1024) void k_hit_scan(uint32_t* __restrict__ block_live, uint32_t nb, uint32_t n,
                                                  uint32_t* __restrict__ counts) {
    __shared__ uint32_t s_part[1024];
    const uint32_t per = (nb + 1023u) / 1024u, b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; ++b) sum += block_live[b];
    s_part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {  // inclusive scan of the 1024 partial sums
        const uint32_t v = threadIdx.x >= off ? s_part[threadIdx.x - off] : 0u;
        __syncthreads();
        s_part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = s_part[threadIdx.x] - sum;  // exclusive
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t c = block_live[b];
        block_live[b] = run;
        run += c;
    }
    if (threadIdx.x == 1023u) {
        counts[0] = s_part[1023];
        counts[1] = n - s_part[1023];
    }
}

__global__ __launch_bounds__(kBlock) void k_hit_scatter(const float2* __restrict__ hits, uint32_t n,
                                                       const uint32_t* __restrict__ block_off,
                                                       uint4* __restrict__ live_rec, uint32_t* __restrict__ sky_pix) {
    __shared__ uint32_t s_c[kBlock / 64u];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const float2 h = i < n ? hits[i] : make_float2(0.f, 0.f);
    const bool live = i < n && __float_as_uint(h.y) != kMiss;
    const unsigned long long b = __ballot(live);
    const uint32_t w = threadIdx.x / 64u;
    if (__lane_id() == 0u) s_c[w] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t before = block_off[blockIdx.x];  // live pixels before this block
    for (uint32_t k = 0; k < w; ++k) before += s_c[k];
    before += __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    if (live) live_rec[before] = make_uint4(i, __float_as_uint(h.x), __float_as_uint(h.y), 0u);
    else if (i < n) sky_pix[i - before] = i;
}

// ---------------------------------------------------------------------------------------------
// accumulate: m_accumulation_buffer[4*i + c] += color[c] for each frame of the pass, in frame
// order (CPUPathTracer.cpp:77-80; color.a is always 1, :283). Blocks < 2*max_bounces also tally
// one bounce's segment lengths (first half of counts) or radiance RMWs (second half) for spt_get_stats.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_accumulate(PassParams p) {
    __shared__ unsigned long long s_sum[kBlock / 64];
    if (blockIdx.x < 2u * p.max_bounces) {
        const uint32_t half = blockIdx.x >= p.max_bounces ? 1u : 0u;
        const uint32_t b = blockIdx.x - half * p.max_bounces;
        const uint32_t* row = p.counts + (half * (kMaxBounces + 1u) + b) * p.n_sub;
        unsigned long long sum = 0;
        for (uint32_t s = threadIdx.x; s < p.n_sub; s += kBlock) sum += row[s];
        for (int off = 32; off > 0; off >>= 1) sum += __shfl_down(sum, off, 64);
        if (__lane_id() == 0) s_sum[threadIdx.x / 64] = sum;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long t = 0;
            for (uint32_t w = 0; w < kBlock / 64; ++w) t += s_sum[w];
            p.totals[half * kMaxBounces + b] += t;  // one block per (half, bounce): no race
        }
    }
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < p.shard_pixels; i += gridDim.x * kBlock) {
        float4 acc = p.accum[i];
        for (uint32_t f = 0; f < p.n_frames; ++f) {
            const float4 l = p.radiance[f * p.shard_pixels + i];
            acc.x = acc.x + l.x;
            acc.y = acc.y + l.y;
            acc.z = acc.z + l.z;
            acc.w = acc.w + 1.0f;
        }
        p.accum[i] = acc;
    }
}

__global__ __launch_bounds__(kBlock) void k_resolve(const float4* __restrict__ accum, uint32_t n, float frames,
                                                     float exposure, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    out[i] = rgba8(accum[i], frames, exposure);
}

// Root-side de-interleave of gathered row shards (multi-GPU).
__global__ __launch_bounds__(kBlock) void k_assemble_rows(const float4* __restrict__ g, float4* __restrict__ out,
                                                           uint32_t width, uint32_t height, uint32_t world,
                                                           uint32_t rows_max) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= width * height) return;
    const uint32_t y = i / width;
    const uint32_t x = i - y * width;
    const uint32_t r = y % world;
    const uint32_t lr = y / world;
    out[i] = g[((size_t)r * rows_max + lr) * width + x];
}

// ---------------------------------------------------------------------------------------------
// host launchers
#ifndef __HIPCC_RTC__
}  // namespace spt
#include "spt_jit.h"
namespace spt {
// ---------------------------------------------------------------------------------------------
namespace {
CameraParams camera_params(const PassParams& p) {
    return CameraParams{p.width,   p.shard_rank,  p.shard_count, p.shard_pixels, p.n_paths,
                        p.first_frame, p.n_sub, p.inv_w,       p.inv_h,        p.aspect, p.hit_cache, p.hit_mode,
                        p.live_rec, p.sky_pix, p.list_counts, 0u, p.rgba, p.rgba_frames, p.rgba_exposure};
}
}  // namespace

void launch_extend(const PassParams& p, uint32_t bounce, hipStream_t s) {
    const QueueBufs& q = p.q[bounce & 1u];
    const CameraParams cam = camera_params(p);
    const uint32_t* counts = p.counts + bounce * p.n_sub;
    const dim3 grid(p.n_sub), block(kBlock);
    if (bounce == 0) {
        if (p.nodes)
            k_extend<true, true><<<grid, block, 0, s>>>(p.prims, p.nodes, p.n_prims, q.o, q.d, p.hit, counts, p.sub_cap, cam);
        else
            k_extend<false, true><<<grid, block, 0, s>>>(p.prims, p.nodes, p.n_prims, q.o, q.d, p.hit, counts, p.sub_cap, cam);
    } else {
        if (p.nodes)
            k_extend<true, false><<<grid, block, 0, s>>>(p.prims, p.nodes, p.n_prims, q.o, q.d, p.hit, counts, p.sub_cap, cam);
        else
            k_extend<false, false><<<grid, block, 0, s>>>(p.prims, p.nodes, p.n_prims, q.o, q.d, p.hit, counts, p.sub_cap, cam);
    }
}

void launch_extend_sorted(const PassParams& p, uint32_t bounce, hipStream_t s) {
    const QueueBufs& q = p.q[bounce & 1u];
    const uint32_t* counts = p.counts + bounce * p.n_sub;
    BinParams bp;
    for (int a = 0; a < 3; ++a) {
        bp.lo[a] = p.bin_lo[a];
        bp.scale[a] = p.bin_scale[a];
    }
    k_bin_count<<<p.n_sub, kBlock, 0, s>>>(q.o, q.d, counts, p.sub_cap, p.ray_keys, p.ray_bins, bp);
    k_bin_scan<<<1, kBlock, 0, s>>>(p.ray_bins, p.ray_cursor);
    k_bin_scatter<<<p.n_sub, kBlock, 0, s>>>(p.ray_keys, counts, p.sub_cap, p.ray_cursor, p.ray_perm);
    if (p.nodes)
        k_extend_sorted<true><<<p.n_sub, kBlock, 0, s>>>(p.prims, p.nodes, p.n_prims, q.o, q.d, p.hit, p.ray_perm, p.ray_cursor);
    else
        k_extend_sorted<false><<<p.n_sub, kBlock, 0, s>>>(p.prims, p.nodes, p.n_prims, q.o, q.d, p.hit, p.ray_perm, p.ray_cursor);
}

void launch_shade(const PassParams& p, uint32_t bounce, hipStream_t s) {
    const ShadeParams sp{p.sky_enabled, p.flags, p.max_bounces, p.rr_depth, p.sub_cap, bounce, p.n_prims, p.n_mats, p.flat_ends, p.horizon, p.zenith, p.env, p.env_w, p.env_h};
    const QueueBufs& cur = p.q[bounce & 1u];
    const QueueBufs& nxt = p.q[(bounce + 1u) & 1u];
    const dim3 grid(p.n_sub), block(kBlock);
    const CameraParams cam = camera_params(p);
#define SPT_SHADE(P, F, B)                                                                                          \
    do {                                                                                                            \
        if (p.nee.n_emit)                                                                                           \
            k_shade<P, F, B, true><<<grid, block, 0, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.hit, cur, nxt,     \
                                                          p.radiance, p.counts, sp, cam, p.nee);                    \
        else                                                                                                        \
            k_shade<P, F, B><<<grid, block, 0, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.hit, cur, nxt, p.radiance, \
                                                    p.counts, sp, cam, p.nee);                                      \
    } while (0)
    // kBvh here only selects where the shading gathers read from: the LDS copy of a flat scene, or
    // global memory for a BVH scene (too many records to stage)
    if (p.nodes) {
        if (bounce == 0) SPT_SHADE(true, false, true);
        else SPT_SHADE(false, false, true);
    } else {
        if (bounce == 0) SPT_SHADE(true, false, false);
        else SPT_SHADE(false, false, false);
    }
}

void launch_bounce(const PassParams& p, uint32_t bounce, hipStream_t s) {
    const ShadeParams sp{p.sky_enabled, p.flags, p.max_bounces, p.rr_depth, p.sub_cap, bounce, p.n_prims, p.n_mats, p.flat_ends, p.horizon, p.zenith, p.env, p.env_w, p.env_h};
    const QueueBufs& cur = p.q[bounce & 1u];
    const QueueBufs& nxt = p.q[(bounce + 1u) & 1u];
    const dim3 grid(p.n_sub), block(kBlock);
    const CameraParams cam = camera_params(p);
    if (p.nodes) {
        if (bounce == 0) SPT_SHADE(true, true, true);
        else SPT_SHADE(false, true, true);
    } else {
        if (bounce == 0) SPT_SHADE(true, true, false);
        else SPT_SHADE(false, true, false);
    }
#undef SPT_SHADE
}

void launch_trace_tail(const PassParams& p, uint32_t bounce, hipStream_t s) {
    const ShadeParams sp{p.sky_enabled, p.flags, p.max_bounces, p.rr_depth, p.sub_cap, bounce, p.n_prims, p.n_mats, p.flat_ends, p.horizon, p.zenith, p.env, p.env_w, p.env_h};
    const QueueBufs& cur = p.q[bounce & 1u];
    const dim3 grid(p.n_sub), block(kBlock);
    if (p.nodes && p.nee.n_emit)
        k_trace_tail<true, true><<<grid, block, 0, s>>>(p.prims, p.nodes, p.n_prims, p.mats, cur, p.radiance, p.counts, sp, p.n_sub, p.nee);
    else if (p.nee.n_emit)
        k_trace_tail<false, true><<<grid, block, 0, s>>>(p.prims, p.nodes, p.n_prims, p.mats, cur, p.radiance, p.counts, sp, p.n_sub, p.nee);
    else if (p.nodes)
        k_trace_tail<true><<<grid, block, 0, s>>>(p.prims, p.nodes, p.n_prims, p.mats, cur, p.radiance, p.counts, sp, p.n_sub, p.nee);
    else
        k_trace_tail<false><<<grid, block, 0, s>>>(p.prims, p.nodes, p.n_prims, p.mats, cur, p.radiance, p.counts, sp, p.n_sub, p.nee);
}

// The first tier's chunks of a flat k_paths launch, longest first: chunk indices sorted by decreasing
// recorded cost (step-loop iterations) — a stable counting sort over 64 buckets relative to the
// longest, one block. (Splitting the longest chunks in halves as well cost more per chunk than it
// saved in the tail: C2 -2 to -6 %.)
__global__ __launch_bounds__(128) void k_chunk_order(const uint16_t* __restrict__ cost, uint32_t n,
                                                     uint32_t* __restrict__ order) {
    constexpr uint32_t kB = 64u, kT = 128u;
    __shared__ uint32_t h[kB][kT];
    __shared__ uint32_t mx[kT];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n + kT - 1u) / kT, b0 = min(n, t * per), b1 = min(n, b0 + per);
    uint32_t m = 1u;
    for (uint32_t i = b0; i < b1; ++i) m = max(m, (uint32_t)cost[i]);
    mx[t] = m;
    for (uint32_t b = 0; b < kB; ++b) h[b][t] = 0u;
    __syncthreads();
    if (t == 0u) {
        uint32_t v = 1u;
        for (uint32_t u = 0; u < kT; ++u) v = max(v, mx[u]);
        mx[0] = v;
    }
    __syncthreads();
    const uint32_t top = mx[0];
    auto bucket = [&](uint32_t c) { return kB - 1u - min(kB - 1u, (c * kB) / (top + 1u)); };
    for (uint32_t i = b0; i < b1; ++i) h[bucket(cost[i])][t] += 1u;
    __syncthreads();
    if (t == 0u) {  // exclusive offsets, bucket-major then thread (stable: pixel order within a bucket)
        uint32_t run = 0;
        for (uint32_t b = 0; b < kB; ++b)
            for (uint32_t u = 0; u < kT; ++u) {
                const uint32_t v = h[b][u];
                h[b][u] = run;
                run += v;
            }
    }
    __syncthreads();
    for (uint32_t i = b0; i < b1; ++i) order[h[bucket(cost[i])][t]++] = i;
}

bool launch_paths(const PassParams& p, bool stats, hipStream_t s) {
    const ShadeParams sp{p.sky_enabled, p.flags, p.max_bounces, p.rr_depth, p.sub_cap, 0u, p.n_prims, p.n_mats, p.flat_ends, p.horizon, p.zenith, p.env, p.env_w, p.env_h, p.n_dev_nodes, p.stack, p.stack_stride, p.stack_tb};
    const CameraParams cam = camera_params(p);
    const bool bvh = p.nodes != nullptr;
    const size_t lds_scene = bvh ? 0 : sizeof(float4) * 3u * p.n_prims;  // make_shade_recs
    const int env = p.env ? 1 : 0;
    const void* kernels[2][2][2] = {
        {{(const void*)k_paths<false, false, 0>, (const void*)k_paths<false, false, 1>},
         {(const void*)k_paths<false, true, 0>, (const void*)k_paths<false, true, 1>}},
        {{(const void*)k_paths<true, false, 0>, (const void*)k_paths<true, false, 1>},
         {(const void*)k_paths<true, true, 0>, (const void*)k_paths<true, true, 1>}}};
    // NEE (p.nee.n_emit > 0): the kNee instantiations, the sky's kind decided at run time (kEnv 2)
    const bool nee = p.nee.n_emit != 0u;
    const bool nee_bvh_all = p.nee.spheres != 0u;  // BVH: the sphere sample compiled in only when needed
    const void* nee_kernels[2][2] = {{(const void*)k_paths<false, false, 2, 0, 0, false, kNeeAll>,
                                      nee_bvh_all ? (const void*)k_paths<false, true, 2, 0, 0, false, kNeeAll>
                                                  : (const void*)k_paths<false, true, 2, 0, 0, false, kNeeNoSpheres>},
                                     {(const void*)k_paths<true, false, 2, 0, 0, false, kNeeAll>,
                                      nee_bvh_all ? (const void*)k_paths<true, true, 2, 0, 0, false, kNeeAll>
                                                  : (const void*)k_paths<true, true, 2, 0, 0, false, kNeeNoSpheres>}};
    // small BVH scenes: the 8-wave variant (k_paths kSimdWaves)
    const bool bvh8 = bvh && !stats && !nee && p.n_prims <= kBvhSmall;
    const void* kernel = nee ? nee_kernels[stats ? 1 : 0][bvh ? 1 : 0]
                         : bvh8 ? (env ? (const void*)k_paths<false, true, 1, 0, kBvhSmallWaves> : (const void*)k_paths<false, true, 0, 0, kBvhSmallWaves>)
                              : kernels[stats ? 1 : 0][bvh ? 1 : 0][env];
    // a flat scene's kernel compiled for its shape (spt_jit.hip), unless it cannot be built
    hipFunction_t fn = (p.jit_shape && !bvh && !stats)
                           ? jit_function(nee ? kJitPathsNee : kJitPaths, nee ? 2 : env, p.jit_shape, nullptr, p.jit_wait != 0u)
                           : nullptr;
    // persistent grid: as many blocks as are resident at once (the waves then pull chunks)
    int per_cu = 0;
    const hipError_t occ = fn ? hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, lds_scene)
                              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, lds_scene);
    if (occ != hipSuccess || per_cu < 1) per_cu = 1;
    const uint32_t resident_waves = (uint32_t)per_cu * p.cu_count * (kBlock / 64u);
    // chunk plan: the largest chunks (32/16/8 pixels) that still give every resident wave >= 8, then
    // ~chunks_per_wave chunks per wave of each smaller size at the end (a wave's last chunk is the
    // launch's tail). A small row shard of a multi-GPU run gets small chunks, which it needs to fill
    // the GPU at all. spt_tuning.px_shift forces one size.
    ChunkPlan plan{};
    const uint32_t P = p.shard_pixels;
    uint32_t s0 = kMaxChunkShift;
    while (s0 > kMinChunkShift && ((uint64_t)P >> s0) < 8ull * resident_waves) --s0;
    if (p.px_shift) s0 = std::max(kMinChunkShift, std::min(p.px_shift, kMaxChunkShift));
    const uint32_t s1 = std::max(kMinChunkShift, s0 - 1u), s2 = std::max(kMinChunkShift, s0 - 2u);
    plan.shift[0] = s0;
    plan.shift[1] = s1;
    plan.shift[2] = s2;
    if (p.px_shift || s0 == kMinChunkShift) {
        plan.n[0] = (P + (1u << s0) - 1u) >> s0;
    } else {
        const uint64_t tail = (uint64_t)p.chunks_per_wave * resident_waves;  // chunks per small tier
        const uint32_t c_px = (uint32_t)std::min<uint64_t>(P, tail << s2);
        const uint32_t b_px = (uint32_t)std::min<uint64_t>(P - c_px, tail << s1) & ~((1u << s1) - 1u);
        const uint32_t a_px = (P - c_px - b_px) & ~((1u << s0) - 1u);
        plan.n[0] = a_px >> s0;
        plan.n[1] = b_px >> s1;
        plan.start[1] = a_px;
        plan.start[2] = a_px + b_px;
        plan.n[2] = (P - a_px - b_px + (1u << s2) - 1u) >> s2;
    }
    const uint32_t chunks = plan.n[0] + plan.n[1] + plan.n[2];
    // A launch records each first-tier chunk's cost, k_chunk_order sorts them behind it (stream order),
    // and the launches of the same plan that follow hand the first tier out longest first (C2 +4 %, with
    // NEE +3 %, the simulated N = 8 shard +5 %: profiles/r05_n_ab_chunk_order.txt; BVH scenes since
    // round 6: C4 +4.5 %, C4 NEE +8 %, profiles/r06_j_ab_bvh_chunk_order.txt, r06_p_ab_bvh_nee_cost.txt).
    // The key names the plan (first-tier chunks, pixels, chunk size); a scene or configuration change
    // clears it (spt_capi.hip). The order changes which wave traces a chunk, never a result.
    plan.order = nullptr;
    plan.cost = nullptr;
    bool record = false;
    const uint64_t order_key = ((uint64_t)plan.n[0] << 37) | ((uint64_t)P << 5) | plan.shift[0];
    if (!p.px_shift && p.chunk_cost && p.chunk_order && plan.n[0] > 1u) {
        if (*p.chunk_order_key == order_key) {
            plan.order = p.chunk_order;
        } else {
            plan.cost = p.chunk_cost;
            record = true;
        }
    }
    auto after = [&]() {
        if (!record) return;
        k_chunk_order<<<1, 128, 0, s>>>(p.chunk_cost, plan.n[0], p.chunk_order);
        // the order is only valid once both launches were enqueued (peek: spt_render reports the error)
        if (hipPeekAtLastError() == hipSuccess) *p.chunk_order_key = order_key;
    };
    const uint32_t needed = (chunks + kBlock / 64u - 1u) / (kBlock / 64u);
    // a flat scene whose chunks are all <= 16 pixels (a small row shard): the channel-lane kernel
    const bool chan = !bvh && !stats && !nee && plan.shift[0] < kMaxChunkShift;
    if (chan) fn = p.jit_shape ? jit_function(kJitPathsChan, env, p.jit_shape, nullptr, p.jit_wait != 0u) : nullptr;
    // (a BVH scene's global traversal stacks are sized for kMaxResidentWaves per CU)
    if (bvh) per_cu = std::min<int>(per_cu, (int)(kMaxResidentWaves / (kBlock / 64u)));
    const uint32_t grid = std::min<uint32_t>(needed, (uint32_t)per_cu * p.cu_count);
    if (fn) {
        const float4 *prims = p.prims, *mats = p.mats, *nodes = p.nodes;
        uint32_t n_prims = p.n_prims, n_frames = p.n_frames;
        float4* accum = p.accum;
        unsigned long long* totals = p.totals;
        uint32_t *work = p.work, *work_next = p.work_next;
        ShadeParams sp_arg = sp;
        CameraParams cam_arg = cam;
        NeeParams nee_arg = p.nee;
        void* args[] = {&prims, &mats, &nodes, &n_prims, &accum, &totals, &work, &work_next,
                        &sp_arg, &cam_arg, &n_frames, &plan, &nee_arg};
        if (hipModuleLaunchKernel(fn, grid, 1, 1, kBlock, 1, 1, (unsigned)lds_scene, s, args, nullptr) == hipSuccess) {
            after();
            return true;
        }
    }
#define SPT_PATHS(S, B, E)                                                                                          \
    k_paths<S, B, E><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, \
                                                     cam, p.n_frames, plan, p.nee)
#define SPT_PATHS_NEE(S, B, N) \
    k_paths<S, B, 2, 0, 0, false, N><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.n_frames, plan, p.nee)
#define SPT_PATHS_ENV(S, B)      \
    do {                         \
        if (env) SPT_PATHS(S, B, 1); \
        else SPT_PATHS(S, B, 0); \
    } while (0)
    if (nee) {
        if (stats && bvh && nee_bvh_all) SPT_PATHS_NEE(true, true, kNeeAll);
        else if (stats && bvh) SPT_PATHS_NEE(true, true, kNeeNoSpheres);
        else if (stats) SPT_PATHS_NEE(true, false, kNeeAll);
        else if (bvh && nee_bvh_all) SPT_PATHS_NEE(false, true, kNeeAll);
        else if (bvh) SPT_PATHS_NEE(false, true, kNeeNoSpheres);
        else SPT_PATHS_NEE(false, false, kNeeAll);
    } else if (bvh8) {
        if (env) k_paths<false, true, 1, 0, kBvhSmallWaves><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.n_frames, plan, p.nee);
        else k_paths<false, true, 0, 0, kBvhSmallWaves><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.n_frames, plan, p.nee);
    } else if (bvh) {
        if (stats) SPT_PATHS_ENV(true, true);
        else SPT_PATHS_ENV(false, true);
    } else if (chan) {
        if (env) k_paths<false, false, 1, 0, 0, true><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.n_frames, plan, p.nee);
        else k_paths<false, false, 0, 0, 0, true><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.n_frames, plan, p.nee);
    } else {
        if (stats) SPT_PATHS_ENV(true, false);
        else SPT_PATHS_ENV(false, false);
    }
    after();
#undef SPT_PATHS_ENV
#undef SPT_PATHS_NEE
#undef SPT_PATHS
    return false;
}

constexpr uint32_t kFrameSkyPerLane = 4;  // k_frame hit_mode 3: sky pixels per sky-block lane

bool frame_small_scene(const PassParams& p, bool stats) {
    return p.nodes != nullptr && !stats && p.nee.n_emit == 0u && p.n_dev_nodes <= kFrameTopNodes &&
           p.n_prims <= kFrameTopPrims && 4u * p.n_prims + 2u * p.n_mats <= 4u * kFrameTopPrims &&
           p.stack_need <= kFrameLdsStackMax;
}

bool frame_small_scene_lists(const PassParams& p) {
    return p.shard_pixels / kFrameRunBvh > (uint32_t)kFrameWavesSmall * 4u * p.cu_count;
}

template <bool kRgba>
bool launch_frame_t(const PassParams& p, bool stats, hipStream_t s) {
    const ShadeParams sp{p.sky_enabled, p.flags, p.max_bounces, p.rr_depth, p.sub_cap, 0u, p.n_prims, p.n_mats, p.flat_ends, p.horizon, p.zenith, p.env, p.env_w, p.env_h, p.n_dev_nodes, p.stack, p.stack_stride, p.stack_tb};
    CameraParams cam = camera_params(p);
    const bool bvh = p.nodes != nullptr;
    // a BVH scene held whole in LDS, with every lane's traversal stack (k_frame kSmall)
    const bool nee = p.nee.n_emit != 0u;  // the kNee instantiations (kEnv 2, no LDS-only small-scene form)
    const bool nee_bvh_all = p.nee.spheres != 0u;  // (k_paths)
    const bool small = frame_small_scene(p, stats);
    const size_t lds_scene = bvh ? (small ? sizeof(uint2) * kBlock * std::max(1u, p.stack_need) : 0)
                                 : sizeof(float4) * 3u * p.n_prims;  // LDS stacks / make_shade_recs
    const int env = p.env ? 1 : 0;
    const void* kernels[2][2][2] = {
        {{(const void*)k_frame<false, false, 0>, (const void*)k_frame<false, false, 1>},
         {(const void*)k_frame<false, true, 0>, (const void*)k_frame<false, true, 1>}},
        {{(const void*)k_frame<true, false, 0>, (const void*)k_frame<true, false, 1>},
         {(const void*)k_frame<true, true, 0>, (const void*)k_frame<true, true, 1>}}};
    const void* nee_kernels[2][2] = {{(const void*)k_frame<false, false, 2, 0, false, kNeeAll>,
                                      nee_bvh_all ? (const void*)k_frame<false, true, 2, 0, false, kNeeAll>
                                                  : (const void*)k_frame<false, true, 2, 0, false, kNeeNoSpheres>},
                                     {(const void*)k_frame<true, false, 2, 0, false, kNeeAll>,
                                      nee_bvh_all ? (const void*)k_frame<true, true, 2, 0, false, kNeeAll>
                                                  : (const void*)k_frame<true, true, 2, 0, false, kNeeNoSpheres>}};
    hipFunction_t fn = (p.jit_shape && !bvh && !stats)
                           ? jit_function(kRgba ? (nee ? kJitFrameNeeRgba : kJitFrameRgba) : (nee ? kJitFrameNee : kJitFrame),
                                          nee ? 2 : env, p.jit_shape, nullptr, p.jit_wait != 0u)
                           : nullptr;
    int per_cu = 0;
    const hipError_t occ =
        fn ? hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, lds_scene)
           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu,
                                                          nee ? nee_kernels[stats ? 1 : 0][bvh ? 1 : 0]
                                                          : small ? (env ? (const void*)k_frame<false, true, 1, 0, true>
                                                                       : (const void*)k_frame<false, true, 0, 0, true>)
                                                                : kernels[stats ? 1 : 0][bvh ? 1 : 0][env],
                                                          kBlock, lds_scene);
    if (occ != hipSuccess || per_cu < 1) per_cu = 1;
    // persistent grid, but no more waves than runs of frame_chunk() pixels
    // (hit_mode 3: the live pixels are the work units; the sky pixels go to blocks of their own, below)
    const bool lists = p.hit_mode == 3u;
    const uint32_t units = lists ? p.live_pixels : p.shard_pixels;
    const uint32_t runs = (units + frame_chunk(bvh) - 1u) / frame_chunk(bvh);
    constexpr uint32_t kFrameRunsPerWave = 4;
    // Flat scenes: a one-frame launch is bound by its lanes' longest chains of path segments, not by
    // throughput (VALU issue ~0.34), so fewer resident waves, each taking ~kFrameRunsPerWave
    // runs, finish the frame sooner than full occupancy (Cornell one frame per call: 720p 90 -> 67 us,
    // 1080p 113 -> 98 us, 4K 238 -> 234 us). BVH scenes keep full occupancy (their latency-bound
    // traversal needs the waves: C4 -4 % with the rule).
    constexpr uint32_t kFrameListsRpw = 2;  // flat scenes with lists: runs per wave, counted over the whole image's runs
    if (!bvh) {
        // with lists (hit_mode 3) the rule counts the whole image's runs, so a wave takes about
        // kFrameListsRpw x the live fraction runs of live pixels
        const uint32_t rule_runs = lists ? (p.shard_pixels + frame_chunk(bvh) - 1u) / frame_chunk(bvh) : runs;
        const uint32_t rpw = lists ? kFrameListsRpw : kFrameRunsPerWave;
        const uint32_t want_blocks = rule_runs / (rpw * (kBlock / 64u));
        per_cu = std::max(1, std::min(per_cu, (int)((want_blocks + p.cu_count / 2u) / std::max(1u, p.cu_count))));
    }
    const uint32_t needed = (runs + kBlock / 64u - 1u) / (kBlock / 64u);
    if (bvh) per_cu = std::min<int>(per_cu, (int)(kMaxResidentWaves / (kBlock / 64u)));  // global stacks' sizing
    const uint32_t path_grid = std::max(1u, std::min<uint32_t>(needed, (uint32_t)per_cu * p.cu_count));
    // hit_mode 3: the sky pixels' blocks, kFrameSkyPerLane pixels per lane, launched ahead of the
    // tracing blocks (k_frame: blockIdx < sky_blocks)
    const uint32_t n_sky = lists ? p.shard_pixels - p.live_pixels : 0u;
    cam.sky_blocks = (n_sky + kBlock * kFrameSkyPerLane - 1u) / (kBlock * kFrameSkyPerLane);
    const uint32_t grid = path_grid + cam.sky_blocks;
    if (fn) {
        const float4 *prims = p.prims, *mats = p.mats, *nodes = p.nodes;
        uint32_t n_prims = p.n_prims;
        float4* accum = p.accum;
        unsigned long long* totals = p.totals;
        uint32_t *work = p.work, *work_next = p.work_next;
        ShadeParams sp_arg = sp;
        CameraParams cam_arg = cam;
        NeeParams nee_arg = p.nee;
        void* args[] = {&prims, &mats, &nodes, &n_prims, &accum, &totals, &work, &work_next, &sp_arg, &cam_arg, &nee_arg};
        if (hipModuleLaunchKernel(fn, grid, 1, 1, kBlock, 1, 1, (unsigned)lds_scene, s, args, nullptr) == hipSuccess)
            return true;
    }
    // (kRgba: launch_frame passes stats = false, and S && !kRgba keeps the stats kernels single)
#define SPT_FRAME(S, B, E) \
    k_frame<(S) && !kRgba, B, E, 0, false, 0, kRgba><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.nee)
#define SPT_FRAME_NEE(S, B, N) \
    k_frame<(S) && !kRgba, B, 2, 0, false, N, kRgba><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.nee)
#define SPT_FRAME_ENV(S, B)          \
    do {                             \
        if (env) SPT_FRAME(S, B, 1); \
        else SPT_FRAME(S, B, 0);     \
    } while (0)
    if (nee) {
        if (stats && bvh && nee_bvh_all) SPT_FRAME_NEE(true, true, kNeeAll);
        else if (stats && bvh) SPT_FRAME_NEE(true, true, kNeeNoSpheres);
        else if (stats) SPT_FRAME_NEE(true, false, kNeeAll);
        else if (bvh && nee_bvh_all) SPT_FRAME_NEE(false, true, kNeeAll);
        else if (bvh) SPT_FRAME_NEE(false, true, kNeeNoSpheres);
        else SPT_FRAME_NEE(false, false, kNeeAll);
    } else if (small) {
        if (env) k_frame<false, true, 1, 0, true, 0, kRgba><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.nee);
        else k_frame<false, true, 0, 0, true, 0, kRgba><<<grid, kBlock, lds_scene, s>>>(p.prims, p.mats, p.nodes, p.n_prims, p.accum, p.totals, p.work, p.work_next, sp, cam, p.nee);
    } else if (bvh) {
        if (stats) SPT_FRAME_ENV(true, true);
        else SPT_FRAME_ENV(false, true);
    } else {
        if (stats) SPT_FRAME_ENV(true, false);
        else SPT_FRAME_ENV(false, false);
    }
#undef SPT_FRAME_ENV
#undef SPT_FRAME_NEE
#undef SPT_FRAME
    return false;
}

bool launch_frame(const PassParams& p, bool stats, hipStream_t s) {
    return p.rgba ? launch_frame_t<true>(p, false, s) : launch_frame_t<false>(p, stats, s);
}

void launch_accumulate(const PassParams& p, hipStream_t s) {
    uint32_t blocks = (p.shard_pixels + kBlock - 1) / kBlock;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 2 * p.max_bounces) blocks = 2 * p.max_bounces;
    if (blocks < 1) blocks = 1;
    k_accumulate<<<blocks, kBlock, 0, s>>>(p);
}

void launch_hit_lists(const PassParams& p, uint32_t* block_scratch, hipStream_t s) {
    const uint32_t n = p.shard_pixels, nb = (n + kBlock - 1u) / kBlock;
    if (n == 0u) return;
    k_hit_count<<<nb, kBlock, 0, s>>>(p.hit_cache, n, block_scratch);
    k_hit_scan<<<1, 1024, 0, s>>>(block_scratch, nb, n, const_cast<uint32_t*>(p.list_counts));
    k_hit_scatter<<<nb, kBlock, 0, s>>>(p.hit_cache, n, block_scratch, const_cast<uint4*>(p.live_rec),
                                        const_cast<uint32_t*>(p.sky_pix));
}

void launch_resolve(const float4* accum, uint32_t n, float frames, float exposure, uint32_t* out, hipStream_t s) {
    if (n == 0) return;
    k_resolve<<<(n + kBlock - 1) / kBlock, kBlock, 0, s>>>(accum, n, frames, exposure, out);
}

#ifdef SPT_TIMELINE
extern "C" int spt_exp_timeline(void* out, size_t bytes) {  // measurement builds only
    if (bytes > sizeof(g_tl)) bytes = sizeof(g_tl);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tl), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
void launch_assemble_rows(const float4* gathered, float4* out, uint32_t width, uint32_t height, uint32_t world,
                          uint32_t rows_max, hipStream_t s) {
    const uint32_t n = width * height;
    if (n == 0) return;
    k_assemble_rows<<<(n + kBlock - 1) / kBlock, kBlock, 0, s>>>(gathered, out, width, height, world, rows_max);
}

#endif  // __HIPCC_RTC__

}  // namespace spt
