// spt_kernels.h — launch interface between the C-ABI (spt_capi.hip) and the wavefront kernels
// (spt_kernels.hip). Internal.
//
// Wavefront layout: one pass traces F frames x P shard pixels camera paths.
//   extend[b]  : closest hit of every queued ray -> hit[]                 (rtcIntersect1, :214-227)
//                (bounce 0 computes the camera rays of the pass itself,     CPUPathTracer.cpp:57-73)
//   shade[b]   : miss/sky, emission, albedo, RR, bounce -> queue b+1      (trace_ray body, :229-280)
//   accumulate : per pixel, add the pass's F frame radiances in frame order (:77-80)
//
// Queues are SoA float4 arrays in HBM cut into n_sub block-private sub-queues of capacity sub_cap.
// Block s of every extend/shade launch owns sub-queue s: it reads segment s of queue b and appends
// the surviving paths to segment s of queue b+1 (wave ballot + LDS prefix, no global atomics), then
// publishes the segment length with one plain store. Paths are dealt to the sub-queues in wave-sized
// chunks round-robin, so every sub-queue samples the whole image and the segment lengths stay
// balanced bounce after bounce.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

namespace spt {

constexpr uint32_t kBlock = 256;
constexpr uint32_t kChunk = 64;  // paths are dealt to sub-queues in wave-sized chunks
constexpr uint32_t kMaxBounces = 32;
constexpr uint32_t kFlagFastDiv = 1u << 30;  // internal ShadeParams flag: the scene passed fast_division_ok (scene.cpp)
// statistics counters (u64): segments per bounce | radiance updates per bounce | k_paths lane slots
// of its tracing steps | lanes that traced in them | BVH interior nodes visited | primitives tested |
// NEE shadow rays traced | waves stopped by the step bound
constexpr uint32_t kTotShadow = 2 * kMaxBounces + 4;
// k_paths waves that left their step loop at its safety bound with frames not yet accumulated (a logic
// error: every path ends within max_bounces steps); always counted, reported by spt_get_stats
constexpr uint32_t kTotStalled = 2 * kMaxBounces + 5;
constexpr uint32_t kTotals = 2 * kMaxBounces + 6;

// Next-event estimation (SPT_FLAG_NEE): the emitter records (scene.h DevEmitter, spt_device.h
// light_sample). Passed as every integrator kernel's LAST argument, so the kernels without NEE keep
// their argument offsets (and their machine code).
constexpr uint32_t kFlagNee = 1u << 4;  // SPT_FLAG_NEE
struct NeeParams {
    const float4* emit;  // kEmitRecs float4 per emitter
    uint32_t n_emit;     // 0: NEE off (no emitters, or the flag is not set)
    uint32_t spheres;    // sphere lights in the table (BVH scenes without any run the kNeeNoSpheres kernels)
};
// k_paths / k_frame kNee: 0 off; kNeeAll: every emitter kind; kNeeNoSpheres: no sphere sample compiled in
constexpr int kNeeAll = 1;
constexpr int kNeeNoSpheres = 2;

struct QueueBufs {
    float4* o;  // (origin.xyz, path id bits)
    float4* d;  // (direction.xyz, rng state bits)
    float4* t;  // (throughput.rgb, 0)
};

struct PassParams {
    // scene
    const float4* prims;  // DevPrim: 4 x float4 each
    const float4* mats;   // DevMaterial: 2 x float4 each
    const float4* nodes;  // BvhNode: 2 x float4 each (nullptr for a flat scene)
    uint32_t n_prims;
    uint32_t n_mats;
    uint32_t n_nodes;      // binary SAH nodes (statistics)
    uint32_t n_dev_nodes;  // records in `nodes` (the 4-wide device tree): bounds the LDS top-node copies
    uint32_t sky_enabled;
    uint32_t flags;
    uint32_t flat_ends;   // flat scene: its kind groups' end offsets, 6 bits each (scene.h sort_flat_by_kind);
                          // the kind-major copy of the records follows the n_prims originals in `prims`
    float4 horizon;
    float4 zenith;
    const float4* env;  // octahedral environment map or nullptr (gradient sky)
    uint32_t env_w, env_h;
    // image / shard
    uint32_t width, height;
    uint32_t shard_rank, shard_count;
    uint32_t shard_pixels;  // P: pixels this ctx owns
    float inv_w, inv_h, aspect;
    uint32_t max_bounces, rr_depth;
    // pass
    uint32_t first_frame;  // global frame index of the pass's frame 0 (seed uses frame + 1)
    uint32_t n_frames;     // F
    uint32_t n_paths;      // F * P
    uint32_t n_sub;        // sub-queues = blocks of every extend/shade launch
    uint32_t sub_cap;      // capacity of one sub-queue (multiple of kChunk)
    // buffers
    QueueBufs q[2];
    float2* hit;             // (t, prim index bits) per queue slot
    float4* radiance;        // (L.rgb, 0) per path, path id = f * P + pixel
    float4* accum;           // (rgba) per shard pixel
    uint32_t* counts;        // [kMaxBounces + 1][n_sub] segment lengths of this pass
    unsigned long long* totals;  // [kTotals] statistics, summed over passes
    uint32_t* work;              // k_paths / k_frame work heads of this launch (kWorkWords, zero)
    uint32_t* work_next;         // the other set: zeroed by this launch for the next one
    uint32_t cu_count;
    uint32_t chunks_per_wave;    // k_paths: chunks per resident wave in each small tail tier
    uint32_t px_shift;           // k_paths: forced log2(pixels per chunk), 0 = automatic
    void* stack;                 // BVH scenes: cu_count * kMaxResidentWaves * 64 lanes' stacks
                                 // (kBvhStackEntryBytes per entry)
    uint32_t stack_need;         // BVH scenes: the most entries a traversal of this tree holds (bvh4_stack_need)
    uint32_t stack_stride;       // entries per lane in `stack`: stack_need rounded up (<= kBvhStackEntries)
    uint32_t stack_tb;           // 4-B entries: the low bits holding the entry distance's lower bound
                                 // (bvh_stack_t0_bits of the tree's largest child ref)
    uint64_t jit_shape;          // flat scene: flat_shape_key of its kernels compiled at run time, 0 = generic
    uint32_t jit_wait;           // 1: compile the specialized kernel inside the launch call if it is not ready;
                                 // 0: run the generic kernel until the background compile has finished
    // sorted ray queues (SPT_FLAG_SORTED_RAYS): the origin grid over the scene bounds and the sort buffers
    float bin_lo[3], bin_scale[3];
    uint16_t* ray_keys;          // [n_sub * sub_cap] bin of each queued ray
    uint32_t* ray_perm;          // [n_sub * sub_cap] queue slots in bin order
    uint32_t* ray_bins;          // [4096] bin counts (zero between bounces)
    uint32_t* ray_cursor;        // [4097] bin starts, then ends; [4096] = rays queued
    NeeParams nee;               // SPT_FLAG_NEE with emitters: the sampled emitters; n_emit = 0 otherwise
    float2* hit_cache;           // k_frame: per shard pixel, its camera segment's closest hit (t, prim bits)
    uint32_t hit_mode;           // 0: unused, 1: k_frame stores the camera hits, 2: k_frame reads them,
                                 // 3: k_frame runs over the compacted lists below
    const uint4* live_rec;       // [shard pixels] live pixels' (pixel, t bits, prim, 0), in pixel order
    const uint32_t* sky_pix;     // [shard pixels] the camera misses' pixel indices, in pixel order
    const uint32_t* list_counts; // [2] live, sky
    uint32_t live_pixels;        // hit_mode 3: list_counts[0] as the host read it back (grid sizing)
    // k_frame: the resolve fused into the frame (spt_render_resolve_rgba8): each pixel's RGBA8, as
    // k_resolve computes it from the value just accumulated, stored into the caller's registered host
    // buffer (device-mapped) when its path ends; nullptr: no resolve in the launch
    uint32_t* rgba;
    float rgba_frames, rgba_exposure;  // the resolve's divisor (frames accumulated after the launch) and exposure
    // flat k_paths: the first tier's chunk costs, recorded by one launch, and their order (longest first)
    uint16_t* chunk_cost;        // [shard pixels] step-loop iterations per first-tier chunk
    uint32_t* chunk_order;       // [shard pixels] first-tier chunk indices, costliest first
    uint64_t* chunk_order_key;   // (host) the plan the order was sorted for, 0 = none (launch_paths)
};

// A flat scene's shape, the compile-time key of its specialized persistent kernels (spt_jit.hip):
// its kind groups' ends (PassParams::flat_ends, 30 bits), the primitive count (6 bits), a valid bit.
constexpr uint64_t kShapeValid = 1ull << 36;
// (round 4) ... and 3 bits (53-55): the axis groups made of rectangles only (scene.h flat_rect_bits),
// whose quads then take the short form without the per-quad scalar check
__host__ __device__ constexpr uint64_t flat_shape_key(uint32_t flat_ends, uint32_t n_prims, uint32_t rect_bits = 0u) {
    return kShapeValid | (uint64_t)(n_prims & 63u) << 30 | (flat_ends & 0x3fffffffu) | (uint64_t)(rect_bits & 7u) << 53;
}
// ... plus the launch configuration the kernels read in their step loop, baked in as constants too
// (round 4): max_bounces and rr_depth (6 bits each), the sky switch, SPT_FLAG_ABS_FLOAT and the scene's
// fast-division flag. As run-time values they live in SGPRs, which the C2 kernel's step loop had spilled
// to VGPR lanes (a v_readlane per use), and every comparison and flag select ran at run time. A key
// without kConfigValid runs on the run-time values (the kernels' ShadeParams).
constexpr uint64_t kConfigValid = 1ull << 37;
constexpr uint32_t kFlagAbsFloatBit = 1u;  // SPT_FLAG_ABS_FLOAT (spt.h) == spt_device.h kFlagAbsFloat
__host__ __device__ constexpr uint64_t jit_config_key(uint64_t shape, uint32_t max_bounces, uint32_t rr_depth,
                                                      uint32_t sky_enabled, uint32_t flags) {
    if (max_bounces > 63u || rr_depth > 63u) return shape;
    return shape | kConfigValid | (uint64_t)max_bounces << 38 | (uint64_t)rr_depth << 44 |
           (uint64_t)(sky_enabled != 0u) << 50 | (uint64_t)((flags & kFlagAbsFloatBit) != 0u) << 51 |
           (uint64_t)((flags & kFlagFastDiv) != 0u) << 52;
}

// BVH traversal stack of the persistent kernels: a global buffer (PassParams::stack), the 64 lanes'
// entries of one depth side by side (one store per push; a depth's entries share their lines).
// Measured (round 3, profiles/r03_b_stack_ab.txt), C5 / C4: a per-lane scratch array 1.457 / 9.05
// Gsamples/s with 268 / 17.4 GB written per launch; this layout 1.511 / 9.11, 152 / 13.2 GB; each lane's
// entries contiguous 1.492 / 9.01, 104 / 12.8 GB but 20 % more bytes read. (The scratch array's swizzle
// put the two dwords of an entry in two 256-B rows: two partial lines per push.) The other two layouts
// are retired (round 4).
// Entry width of the global stacks. 8: (packed child ref, entry distance t0).
// 4 (round 4): ONE dword, the ref above a tb-bit code of a LOWER bound of t0 (the float's bits from
// 2^-10 = kTNear's binade down, shifted so that 32 binades fit: tb - 5 mantissa bits; clamped at the
// top). A pop culls an entry when that bound exceeds best_t — then t0 does too — so the culling stays
// conservative and the closest hit exact; entries just past best_t are visited and cut there by their
// exact slab or primitive tests. Half the stack bytes per push, pop and read-ahead.
// Measured (round 4, profiles/r04_b_ab_stack_entry_reg.txt, PMC per launch): C5 (1 M triangles, 7
// waves/SIMD) 1.643 -> 1.687 Gsamples/s with 4-B entries, fabric reads 569 -> 415 GB, writes 155 -> 134 GB
// (node visits per segment 13.66 -> 13.93: the coarser culling); C5 one frame per call +4.4 %. C4 (82 K,
// the 8-waves instantiation at 64 VGPRs) loses 4 % with them (its stacks are short; the code's extra VALU
// and SGPRs cost more than the bytes save), so the 8-waves k_paths of scenes <= kBvhSmall keeps 8-B
// entries (kBvhStackEntry8W); every other kernel takes kBvhStackEntry.
constexpr uint32_t kBvhStackEntry = 4;
constexpr uint32_t kBvhStackEntry8W = 8;
// the global stacks are allocated for the wider of the two (a scene's kernels may use either)
constexpr uint32_t kBvhStackEntryBytes = kBvhStackEntry > kBvhStackEntry8W ? kBvhStackEntry : kBvhStackEntry8W;
// tb for a tree whose largest packed child ref (first << 4 | count) is max_ref: every bit above the
// ref, at most 28 (the shift 28 - tb stays >= 0), at least 1 (refs below 2^31; spt_set_scene refuses
// trees beyond). tb = 1 still gives a valid (coarse) lower bound.
inline __host__ __device__ constexpr uint32_t bvh_stack_t0_bits(uint32_t max_ref) {
    uint32_t rb = 0;
    while (rb < 32u && (max_ref >> rb) != 0u) ++rb;
    const uint32_t tb = 32u - rb;
    return tb > 28u ? 28u : tb;
}
// The 4-B entry's code of an entry distance t0 >= kTNear (its float bits), and the lower bound it
// decodes to, for tb code bits: sh = 28 - tb, base = bits(2^-10) >> sh, mask = 2^tb - 1.
// (code + base) << sh <= (bits >> sh) << sh <= bits: the bound never exceeds t0.
struct StackCode {
    uint32_t sh, base, mask;
};
inline __host__ __device__ constexpr StackCode stack_code_params(uint32_t tb) {
    return StackCode{28u - tb, 0x3a800000u >> (28u - tb), (1u << tb) - 1u};
}
inline __host__ __device__ constexpr uint32_t stack_code(uint32_t t0_bits, StackCode c) {
    const uint32_t q = (t0_bits >> c.sh) - c.base;
    return q < c.mask ? q : c.mask;
}
inline __host__ __device__ constexpr uint32_t stack_t0_lower_bits(uint32_t code, StackCode c) {
    return ((code & c.mask) + c.base) << c.sh;
}
// The most entries a lane's stack may need: the per-lane scratch stacks (the wavefront kernels) have this
// many; a scene whose tree needs more (bvh4_stack_need, a deep degenerate tree) is refused by
// spt_set_scene / spt_update_prims with SPT_ERR_CAPACITY. The persistent kernels' global stacks are
// sized by the tree's own need (PassParams::stack_stride).
constexpr uint32_t kBvhStackEntries = 96;
// the global stacks' lane stride for a tree needing `need` entries (the pop read-ahead reads entry 0 of
// an empty stack: at least 1)
inline __host__ __device__ constexpr uint32_t bvh_stack_stride(uint32_t need) { return need < 1u ? 1u : (need + 3u) & ~3u; }
constexpr uint32_t kMaxResidentWaves = 8 * 4;  // per CU: 8 waves per SIMD x 4 SIMDs (global stack sizing)
constexpr uint32_t kDevNodeBytes = 64u;  // sizeof(BvhNodeQ)

// k_frame's camera-hit cache, level 2 (levels measured in round 4: 0: k_frame traces every camera
// segment; 1: it takes the camera hits from a per-pixel cache written by
// the first launch after a change (A/B: the App's 512² frame 38.8 -> 35.4 us, C4 one frame per call
// +5 %); 2: also compacted once into live-pixel records and sky-pixel indices, so the sky pixels take no
// path and no lane step (k_hit_count / k_hit_scan / k_hit_scatter), for the scenes where that measured
// faster (frame_lists_scene, and then at least 1 / kFrameListsMinSkyDiv of the pixels sky)
constexpr uint32_t kFrameHitCache = 2;
// A/B against the per-pixel cache alone (profiles/r04_g_ab_frame_lists.txt, r04_j_ab_flat_lists.txt):
// C4 one frame per call +16 % (656 -> 575 us); Cornell one frame per call, with the flat scenes' wave
// rule counting the whole image (launch_frame kFrameListsRpw): 720p 60.4 -> 40.1 us, 1080p 87.3 -> 69.3 us,
// 4K 221 -> 199 us, with NEE +15 %; the App's LDS-held scene -4 to -5.6 % (not used there); C5 (an
// interior, no sky) -1.6 % (below the sky threshold)
constexpr uint32_t kFrameListsMinSkyDiv = 4;  // lists when sky pixels >= shard pixels / 4

// persistent kernels' work queue: one head per XCD, each on its own 128-B line
constexpr uint32_t kWorkHeads = 8;  // power of two, <= 8
constexpr uint32_t kWorkStride = 32;
constexpr uint32_t kWorkWords = kWorkHeads * kWorkStride;

#ifndef __HIPCC_RTC__
// host launchers (stream-ordered, no synchronisation)
void launch_extend(const PassParams& p, uint32_t bounce, hipStream_t s);
// bounce >= 1 of the sorted schedule: bin the queued rays (counting sort), then extend in bin order
void launch_extend_sorted(const PassParams& p, uint32_t bounce, hipStream_t s);
void launch_shade(const PassParams& p, uint32_t bounce, hipStream_t s);
// extend + shade of one bounce in a single launch (the closest hit never leaves registers)
void launch_bounce(const PassParams& p, uint32_t bounce, hipStream_t s);
void launch_trace_tail(const PassParams& p, uint32_t bounce, hipStream_t s);
void launch_accumulate(const PassParams& p, hipStream_t s);
// flat scenes, persistent schedule: every frame of the call in one launch, accumulated in frame
// order in registers (no queues, no radiance buffer); `stats` tallies segments per bounce
// (true: the flat scene's specialized kernel ran, spt_jit.hip; false: the generic one)
bool launch_paths(const PassParams& p, bool stats, hipStream_t s);
bool launch_frame(const PassParams& p, bool stats, hipStream_t s);
// k_frame holds this BVH scene whole in LDS (its kSmall form)
bool frame_small_scene(const PassParams& p, bool stats);
// ... and whether such a scene's one-frame launches take the live-pixel lists (frame_lists_scene)
bool frame_small_scene_lists(const PassParams& p);
// the scenes k_frame's compacted lists are built for: all but the BVH scenes it holds in LDS (lists for
// every scene measured slower)
inline bool frame_lists_scene(const PassParams& p, bool stats) {
    if (kFrameHitCache < 2) return false;
    // a scene held in LDS (the App's): lists only when the image has more runs than the grid has
    // resident waves (5 per SIMD) — at 512² every run has a wave of its own and the lists only add
    // their reads (30.5 -> 30.8 us); at 1024² the waves take several runs each and the compacted live
    // pixels save whole runs (94.8 -> 71.5 us, profiles/r05_o_ab_small_lists.txt)
    if (frame_small_scene(p, stats)) return frame_small_scene_lists(p);
    return true;
}
// compact p.hit_cache into p.live_rec / p.sky_pix / p.list_counts (block_scratch: shard pixels / 256 words)
void launch_hit_lists(const PassParams& p, uint32_t* block_scratch, hipStream_t s);
void launch_resolve(const float4* accum, uint32_t n, float frames, float exposure, uint32_t* out, hipStream_t s);
void launch_assemble_rows(const float4* gathered, float4* out, uint32_t width, uint32_t height,
                          uint32_t world, uint32_t rows_max, hipStream_t s);

#endif  // __HIPCC_RTC__

// Dealing of camera path p: chunk c = p / kChunk goes to sub-queue c % n_sub, at slot
// (c / n_sub) * kChunk + p % kChunk; dealt_path inverts it.
inline __host__ __device__ uint32_t deal_sub(uint32_t p, uint32_t n_sub) { return (p / kChunk) % n_sub; }
inline __host__ __device__ uint32_t deal_slot(uint32_t p, uint32_t n_sub) {
    return (p / (kChunk * n_sub)) * kChunk + (p % kChunk);
}
inline __host__ __device__ uint32_t dealt_path(uint32_t s, uint32_t i, uint32_t n_sub) {
    return ((i / kChunk) * n_sub + s) * kChunk + (i % kChunk);
}
// Number of the first n paths dealt to sub-queue s.
inline __host__ __device__ uint32_t sub_count_of(uint32_t n, uint32_t s, uint32_t n_sub) {
    const uint32_t per_round = kChunk * n_sub;
    const uint32_t full = (n / per_round) * kChunk;
    const uint32_t rem = n % per_round;
    const uint32_t lo = s * kChunk;
    const uint32_t extra = rem > lo ? (rem - lo < kChunk ? rem - lo : kChunk) : 0u;
    return full + extra;
}
inline uint32_t sub_capacity(uint64_t n_paths, uint32_t n_sub) {
    const uint64_t per_round = (uint64_t)kChunk * n_sub;
    return (uint32_t)(((n_paths + per_round - 1) / per_round) * kChunk);
}

}  // namespace spt
