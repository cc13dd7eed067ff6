// spt_capi.hip — the C-ABI of libspt_hip.so (declared in include/spt.h).
//
// Owns one HIP device's state for the integrator: scene records, ray queues, accumulation, and
// the pass driver that replaces CPUPathTracer::render()'s serial pixel loop
// (libs/render/src/engines/pathtracer/backends/cpu/CPUPathTracer.cpp:43-85) with wavefront
// launches. Never aborts: every failure is a negative spt_status + spt_last_error().
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "scene.h"
#include "spt.h"
#include "spt_jit.h"
#include "spt_kernels.h"

using namespace spt;

static_assert(kBvhStackMax == kBvhStackEntries, "scene.h and spt_kernels.h stack bounds");

namespace {

// The tree the device traverses for a binary SAH BVH: its 4-wide collapse, quantized (scene.h BvhNodeQ),
// the most traversal stack entries it needs and the 4-B stack entries' t0 bits (bvh_stack_t0_bits of its
// largest child ref).
struct DevTree {
    std::vector<uint8_t> bytes;
    uint32_t stack_need = 0, stack_tb = 0;
};
template <int W, class Q, class QuantFn>
DevTree make_dev_tree(const std::vector<BvhNode>& bin, QuantFn quantize) {
    static_assert(sizeof(Q) == kDevNodeBytes, "device node record size");
    DevTree t;
    std::vector<BvhNodeW<W>> wide;
    collapse_bvh_w<W>(bin, wide);
    if (wide.empty()) return t;
    t.stack_need = bvh_w_stack_need<W>(wide, 0u);
    t.stack_tb = bvh_stack_t0_bits(bvh_w_max_ref<W>(wide));  // refs < 2^31 here
    std::vector<Q> q;
    quantize(wide, q);
    t.bytes.resize(sizeof(Q) * q.size());
    std::memcpy(t.bytes.data(), q.data(), t.bytes.size());
    return t;
}
DevTree device_tree(const std::vector<BvhNode>& bin) { return make_dev_tree<4, BvhNodeQ>(bin, quantize_bvh4); }

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    int kind = 0;  // 0 extend, 1 shade, 2 other, 3 tail, 4 persistent
    uint32_t bounce = 0;
    uint32_t launches = 1;  // kind 4: the launches between a and b (> 1 for a SPT_PROFILE_SPAN pair)
};

}  // namespace

struct spt_ctx {
    int device = -1;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    uint32_t cu_count = 256;

    // scene
    float4* d_prims = nullptr;
    float4* d_mats = nullptr;
    float4* d_nodes = nullptr;
    float4* d_env = nullptr;  // octahedral environment map (spt_set_env_map) or nullptr
    float4* d_emit = nullptr;  // SPT_FLAG_NEE: the sampled emitters (scene.h DevEmitter), n_emit records
    uint32_t n_emit = 0;
    uint32_t n_emit_spheres = 0;  // ... of which spheres (NeeParams::spheres)
    uint32_t env_w = 0, env_h = 0;
    uint32_t n_prims = 0, n_nodes = 0, n_mats = 0;
    uint32_t n_dev_nodes = 0;  // records in d_nodes (4-wide, quantized): bounds the kernels' LDS top-node copies
    void* bvh_stack = nullptr;  // the persistent kernels' traversal stacks (global memory)
    uint32_t bvh_stack_need = 0;  // the most stack entries a traversal of the 4-wide tree holds (bvh4_stack_need)
    uint32_t bvh_stack_stride = 0;  // entries per lane in bvh_stack (bvh_stack_stride(need)); 0: none allocated
    uint32_t bvh_stack_tb = 1;      // 4-B stack entries: bits of the entry-distance code (bvh_stack_t0_bits)
    spt_env env{};
    bool has_scene = false;
    uint32_t flat_ends = 0;  // PassParams::flat_ends
    uint32_t flat_rect = 0;  // flat_rect_bits of the kind-major copy (part of the shape key)
    bool fast_div = false;  // scene.cpp fast_division_ok: the flat loop's unscaled divisions apply
    uint64_t scene_bytes = 0;
    uint64_t stack_bytes = 0;  // the persistent kernels' global traversal stacks (BVH scenes)

    // configuration
    spt_config cfg{};
    bool configured = false;
    uint32_t rows = 0;          // rows owned by this shard
    uint32_t pixels = 0;        // rows * width
    uint32_t frames_per_pass = 1;
    uint32_t n_sub = 0;         // block-private sub-queues (= blocks of every extend/shade launch)
    uint32_t sub_cap = 0;       // capacity of one sub-queue

    // device buffers
    float4* q_o[2] = {nullptr, nullptr};
    float4* q_d[2] = {nullptr, nullptr};
    float4* q_t[2] = {nullptr, nullptr};
    float2* hit = nullptr;
    float4* radiance = nullptr;
    float4* accum = nullptr;
    float2* hit_cache = nullptr;  // k_frame: each shard pixel's camera-segment closest hit (configure-sized)
    bool hit_cache_valid = false;  // it holds the current scene's and configuration's hits
    uint16_t* chunk_cost = nullptr;   // flat k_paths' first-tier chunk costs and order (PassParams)
    uint32_t* chunk_order = nullptr;
    uint64_t chunk_order_key = 0;     // 0: no order (cleared with the hit cache by a scene or size change)
    bool frame_lists = false;      // ... and k_frame takes the compacted lists (hit_mode 3)
    uint4* live_rec = nullptr;     // ... compacted: the live pixels' records (kFrameHitCache 2)
    uint32_t* sky_pix = nullptr;   // ... the sky pixels' indices
    uint32_t* list_counts = nullptr;  // [2] live, sky; then the compaction's per-block scratch
    uint32_t live_pixels = 0;         // list_counts[0], read back once per compaction
    uint32_t* counts = nullptr;
    unsigned long long* totals = nullptr;
    uint32_t* work = nullptr;  // k_paths / k_frame work heads: 2 sets of kWorkWords, alternating per launch
    uint32_t work_parity = 0;
    uint32_t chunks_per_wave = 0;  // k_paths: chunks per resident wave in each small tail tier (spt_tuning; 0 = auto)
    uint32_t px_shift = 0;         // k_paths forced chunk size, log2 pixels (spt_tuning.px_shift = 2..5, clamped to the build)
    uint32_t* resolved = nullptr;
    // spt_register_host_output: a caller's host image buffer, page-locked and mapped into the GPU's
    // address space, that the resolve kernel writes over PCIe directly (no device staging, no DMA copy)
    void* out_host = nullptr;
    void* out_dev = nullptr;
    size_t out_bytes = 0;
    // spt_render_resolve_rgba8: the resolve the next k_frame launch of spt_render fuses (fuse_frames != 0),
    // and whether a launch took it
    float fuse_frames = 0.0f, fuse_exposure = 1.0f;
    bool fused = false;

    uint32_t frame_count = 0;

    // stats
    uint64_t frames = 0, paths = 0, passes = 0;
    bool profiling = false;
    bool span = false;        // SPT_PROFILE_SPAN: one event pair around the persistent launches
    bool span_open = false;   // its begin event is recorded
    EventPair span_ev;
    std::vector<EventPair> pending;
    std::vector<EventPair> free_events;
    uint64_t ext_launches = 0, shade_launches = 0, ext_segments = 0;
    double ext_ms = 0.0, shade_ms = 0.0, other_ms = 0.0, tail_ms = 0.0;
    uint64_t tail_launches = 0;
    // Schedule (measured): flat scenes run one fused extend+shade launch per bounce
    // and finish paths from bounce 3 in k_trace_tail; BVH scenes run split extend/shade launches
    // for every bounce (traversal divergence makes the fused and tail kernels slower there).
    // Overrides: spt_tuning.fused / .tail_bounce (spt_set_tuning), or SPT_FLAG_SPLIT_KERNELS.
    int fused_override = -1;       // -1: automatic
    uint32_t tail_override = 0;    // 0: automatic
    double ext_ms_b[kMaxBounces] = {}, shade_ms_b[kMaxBounces] = {};
    // Calls of >= SPT_PERSISTENT_MIN_FRAMES frames run the persistent k_paths schedule instead
    // (SPT_FLAG_WAVEFRONT or spt_tuning.persistent = 0 keep the wavefront one).
    int persistent_override = -1;  // -1: automatic
    int frame_override = -1;       // spt_tuning.frame_kernel for calls of < SPT_PERSISTENT_MIN_FRAMES frames
    bool counters = false;         // SPT_PROFILE_COUNTERS: k_paths tallies segments per bounce
    double persist_ms = 0.0;
    uint64_t persist_launches = 0;
    uint32_t last_schedule = SPT_SCHEDULE_FUSED;
    uint32_t sub_alloc = 0;        // n_sub the queue buffers were sized for (spt_configure)
    uint32_t bvh_max_leaf = 0;     // spt_tuning: 0 = bvh_max_leaf(n)
    uint32_t bvh_bins = 0;         // spt_tuning: 0 = the builder's default
    int32_t specialize = 0;        // spt_tuning: flat scenes' kernels compiled for their shape: 0 = in the
                                   // background (generic kernels until ready), 1 = inside the first launch, -1 = never
    // sorted ray queues (SPT_FLAG_SORTED_RAYS): the binning grid over the BVH scene's bounds, buffers
    float scene_lo[3] = {0.f, 0.f, 0.f}, scene_hi[3] = {1.f, 1.f, 1.f};
    uint16_t* ray_keys = nullptr;
    // host copies of the current scene for spt_update_prims: the caller's arrays, and for a BVH scene
    // the device-order records and the binary tree (refitted, not rebuilt, on an edit)
    std::vector<spt_prim> h_prims;
    std::vector<spt_material> h_mats;
    std::vector<DevPrim> h_dp;
    std::vector<BvhNode> h_nodes;
    std::vector<uint32_t> h_pos;  // original primitive index -> its record's position on the device
    uint64_t node_alloc = 0;      // bytes allocated at d_nodes
    uint32_t* ray_perm = nullptr;
    uint32_t* ray_bins = nullptr;
    uint32_t* ray_cursor = nullptr;
    bool last_specialized = false; // the last persistent / frame launch ran the specialized kernel

    // multi-GPU (spt_comm_init / spt_gather_image)
    ncclComm_t comm = nullptr;
    int comm_ranks = 0, comm_rank = -1;
    float4* gather_buf = nullptr;  // rank 0: comm_ranks padded shards; other ranks: their padded shard
    size_t gather_elems = 0;       // floats in gather_buf
    // spt_gather_image_overlapped: the gather runs on a stream of its own while the ctx stream renders on
    hipStream_t comm_stream = nullptr;
    hipEvent_t snap_ready = nullptr;   // ctx stream: the shard snapshot is in gather_buf
    hipEvent_t gather_done = nullptr;  // comm stream: the last overlapped gather (and assembly) finished
    bool gather_pending = false;       // an overlapped gather was enqueued since the last wait
};

namespace {

int fail(spt_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define SPT_HIP(ctx, call)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail((ctx), SPT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <typename T>
void free_dev(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

void free_buffers(spt_ctx* c) {
    for (int k = 0; k < 2; ++k) {
        free_dev(c->q_o[k]);
        free_dev(c->q_d[k]);
        free_dev(c->q_t[k]);
    }
    free_dev(c->hit);
    free_dev(c->ray_keys);
    free_dev(c->ray_perm);
    free_dev(c->ray_bins);
    free_dev(c->ray_cursor);
    free_dev(c->radiance);
    free_dev(c->accum);
    free_dev(c->hit_cache);
    free_dev(c->chunk_cost);
    free_dev(c->chunk_order);
    c->chunk_order_key = 0;
    free_dev(c->live_rec);
    free_dev(c->sky_pix);
    free_dev(c->list_counts);
    c->hit_cache_valid = false;
    free_dev(c->resolved);
}

// RCCL, resolved at run time (spt.h): the copy already in the process (PyTorch loads its own
// librccl.so, soname librccl.so.1) or the ROCm install's. Linking one at build time could put two
// RCCLs in one process, whose exported symbols would interpose on each other.
struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    bool ok = false;
    std::string err;
};

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so"})
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            x.err = std::string("RCCL not found: ") + (e ? e : "dlopen failed");
            return x;
        }
        x.get_unique_id = (decltype(x.get_unique_id))dlsym(h, "ncclGetUniqueId");
        x.comm_init_rank = (decltype(x.comm_init_rank))dlsym(h, "ncclCommInitRank");
        x.gather = (decltype(x.gather))dlsym(h, "ncclGather");
        x.comm_destroy = (decltype(x.comm_destroy))dlsym(h, "ncclCommDestroy");
        x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
        x.ok = x.get_unique_id && x.comm_init_rank && x.gather && x.comm_destroy && x.error_string;
        if (!x.ok) x.err = "RCCL: ncclGather / ncclCommInitRank missing from the loaded library";
        return x;
    }();
    return r;
}

#define SPT_NCCL(ctx, call)                                                                          \
    do {                                                                                             \
        ncclResult_t r_ = (call);                                                                    \
        if (r_ != ncclSuccess)                                                                       \
            return fail((ctx), SPT_ERR_HIP, std::string(#call) + ": " + rccl().error_string(r_));      \
    } while (0)

void free_comm(spt_ctx* c) {
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    if (c->comm && rccl().ok) (void)rccl().comm_destroy(c->comm);
    if (c->snap_ready) (void)hipEventDestroy(c->snap_ready);
    if (c->gather_done) (void)hipEventDestroy(c->gather_done);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    c->snap_ready = c->gather_done = nullptr;
    c->comm_stream = nullptr;
    c->gather_pending = false;
    c->comm = nullptr;
    c->comm_ranks = 0;
    c->comm_rank = -1;
    free_dev(c->gather_buf);
    c->gather_elems = 0;
}

void free_scene(spt_ctx* c) {
    c->hit_cache_valid = false;  // (the camera hits were this scene's)
    c->chunk_order_key = 0;  // (the chunks' costs were this scene's)
    free_dev(c->bvh_stack);
    c->bvh_stack_stride = 0;
    free_dev(c->d_prims);
    free_dev(c->d_mats);
    free_dev(c->d_nodes);
    free_dev(c->d_emit);
    c->n_prims = c->n_nodes = c->n_dev_nodes = c->n_emit = c->n_emit_spheres = 0;
    c->has_scene = false;
}

int flush_events(spt_ctx* c) {
    if (c->pending.empty()) return SPT_OK;
    SPT_HIP(c, hipEventSynchronize(c->pending.back().b));
    for (auto& e : c->pending) {
        float ms = 0.0f;
        SPT_HIP(c, hipEventElapsedTime(&ms, e.a, e.b));
        if (e.kind == 0) {
            c->ext_ms += ms;
            c->ext_ms_b[e.bounce] += ms;
            c->ext_launches++;
        } else if (e.kind == 1) {
            c->shade_ms += ms;
            c->shade_ms_b[e.bounce] += ms;
            c->shade_launches++;
        } else if (e.kind == 3) {
            c->tail_ms += ms;
            c->tail_launches++;
        } else if (e.kind == 4) {
            c->persist_ms += ms;
            c->persist_launches += e.launches;
        } else {
            c->other_ms += ms;
        }
        c->free_events.push_back(e);
    }
    c->pending.clear();
    return SPT_OK;
}

int begin_event(spt_ctx* c, EventPair& out, int kind, uint32_t bounce = 0) {
    if (c->free_events.empty()) {
        EventPair e;
        SPT_HIP(c, hipEventCreate(&e.a));
        SPT_HIP(c, hipEventCreate(&e.b));
        c->free_events.push_back(e);
    }
    out = c->free_events.back();
    c->free_events.pop_back();
    out.kind = kind;
    out.bounce = bounce;
    out.launches = 1;  // (a pooled pair may have been a span)
    SPT_HIP(c, hipEventRecord(out.a, c->stream));
    return SPT_OK;
}

int end_event(spt_ctx* c, EventPair& e) {
    SPT_HIP(c, hipEventRecord(e.b, c->stream));
    c->pending.push_back(e);
    if (c->pending.size() >= 4096) return flush_events(c);
    return SPT_OK;
}

// A persistent (k_paths / k_frame) launch under profiling: its own event pair, or (SPT_PROFILE_SPAN)
// the span's begin before the first one and a launch counted
int begin_persistent(spt_ctx* c, EventPair& ev) {
    if (!c->profiling) return SPT_OK;
    if (!c->span) return begin_event(c, ev, 4);
    if (!c->span_open) {
        if (begin_event(c, c->span_ev, 4) != SPT_OK) return SPT_ERR_HIP;
        c->span_ev.launches = 0;
        c->span_open = true;
    }
    c->span_ev.launches++;
    return SPT_OK;
}

int end_persistent(spt_ctx* c, EventPair& ev) {
    if (!c->profiling || c->span) return SPT_OK;
    return end_event(c, ev);
}

// the span's end: after the last launch, recorded when the span mode is switched off
int close_span(spt_ctx* c) {
    if (!c->span_open) return SPT_OK;
    c->span_open = false;
    return end_event(c, c->span_ev);
}

bool schedule_fused(const spt_ctx* c) {
    if (c->cfg.flags & (SPT_FLAG_SPLIT_KERNELS | SPT_FLAG_SORTED_RAYS)) return false;
    if (c->fused_override >= 0) return c->fused_override != 0;
    return c->n_nodes == 0;
}

constexpr uint32_t kPersistentMaxFrames = 1024;

bool schedule_persistent(const spt_ctx* c, uint32_t n_frames) {
    if (c->cfg.max_bounces == 0) return false;
    if (c->cfg.flags & (SPT_FLAG_SPLIT_KERNELS | SPT_FLAG_WAVEFRONT | SPT_FLAG_SORTED_RAYS)) return false;
    if (c->persistent_override >= 0) return c->persistent_override != 0;
    // measured: C2 flat 18.5 -> 40+ Gsamples/s, C4 BVH 2.02 -> 2.34, C5 BVH even
    return n_frames >= SPT_PERSISTENT_MIN_FRAMES;
}

// calls of fewer frames: one persistent k_frame launch per frame (same conditions otherwise)
bool schedule_frame(const spt_ctx* c) {
    if (c->cfg.max_bounces == 0) return false;
    if (c->cfg.flags & (SPT_FLAG_SPLIT_KERNELS | SPT_FLAG_WAVEFRONT | SPT_FLAG_SORTED_RAYS)) return false;
    if (c->frame_override >= 0) return c->frame_override != 0;
    if (c->persistent_override >= 0) return c->persistent_override != 0;
    return true;
}

uint32_t schedule_tail(const spt_ctx* c) {
    if (c->tail_override) return c->tail_override;
    return c->n_nodes == 0 ? 3u : kMaxBounces;
}

// persistent launches use one zeroed set of work heads and zero the other for the next launch
void next_work_set(spt_ctx* c, PassParams& p) {
    p.work = c->work + c->work_parity * kWorkWords;
    p.work_next = c->work + (c->work_parity ^ 1u) * kWorkWords;
    c->work_parity ^= 1u;
}

// The run-time specialized kernels' key of the ctx's flat scene: its shape and, once configured, the
// launch configuration (spt_kernels.h jit_config_key).
static uint64_t flat_jit_key(const spt_ctx* c) {
    const uint64_t shape = flat_shape_key(c->flat_ends, c->n_prims, c->flat_rect);
    if (!c->configured) return shape;
    const uint32_t flags = (c->cfg.flags & ~spt::kFlagFastDiv) | (c->fast_div ? spt::kFlagFastDiv : 0u);
    return jit_config_key(shape, c->cfg.max_bounces, c->cfg.rr_depth, c->env.sky_enabled ? 1u : 0u, flags);
}

// The NEE kernels run: the flag is set AND the scene has an emitter to sample (launch_paths / launch_frame
// select them from NeeParams::n_emit, which base_params sets from this)
// the sphere records of an emitter table (DevEmitter base[3] == 2)
static uint32_t sphere_emitters(const std::vector<DevEmitter>& emit) {
    uint32_t k = 0;
    for (const DevEmitter& e : emit) {
        uint32_t kind;
        std::memcpy(&kind, &e.base[3], 4);
        k += kind == 2u ? 1u : 0u;
    }
    return k;
}
static bool nee_active(const spt_ctx* c) { return c->configured && (c->cfg.flags & SPT_FLAG_NEE) && c->n_emit != 0u; }

// Start compiling a configured flat scene's specialized kernels in the background (a new shape or a new
// configuration): frames rendered before they are ready run the generic kernels.
static void prefetch_flat(const spt_ctx* c) {
    if (!(c->has_scene && c->configured && c->n_prims && c->n_nodes == 0 && c->specialize == 0)) return;
    const uint64_t key = flat_jit_key(c);
    if (nee_active(c)) {  // (the NEE kernels decide the sky at run time: env = 2)
        jit_prefetch(kJitPathsNee, 2, key);
        jit_prefetch(kJitFrameNee, 2, key);
        return;
    }
    const int env_variant = c->d_env ? 1 : 0;
    jit_prefetch(kJitPaths, env_variant, key);
    jit_prefetch(kJitFrame, env_variant, key);
    jit_prefetch(kJitPathsChan, env_variant, key);
}

PassParams base_params(spt_ctx* c) {
    PassParams p{};
    p.prims = c->d_prims;
    p.mats = c->d_mats;
    p.nodes = c->d_nodes;
    p.n_prims = c->n_prims;
    p.n_mats = c->n_mats;
    p.n_nodes = c->n_nodes;
    p.n_dev_nodes = c->n_dev_nodes;
    p.sky_enabled = c->env.sky_enabled ? 1u : 0u;
    p.flags = (c->cfg.flags & ~spt::kFlagFastDiv) | (c->fast_div ? spt::kFlagFastDiv : 0u);
    p.flat_ends = c->flat_ends;
    // flat scenes: their shape's kernels compiled at run time (spt_jit.hip), unless tuned off
    for (int a = 0; a < 3; ++a) {  // sorted ray queues: an 8 x 8 x 8 grid over the scene bounds
        p.bin_lo[a] = c->scene_lo[a];
        const float ext = c->scene_hi[a] - c->scene_lo[a];
        p.bin_scale[a] = ext > 0.0f ? 8.0f / ext : 0.0f;
    }
    p.ray_keys = c->ray_keys;
    p.ray_perm = c->ray_perm;
    p.ray_bins = c->ray_bins;
    p.ray_cursor = c->ray_cursor;
    p.jit_shape = (c->n_prims && c->n_nodes == 0 && c->specialize >= 0) ? flat_jit_key(c) : 0ull;
    p.jit_wait = c->specialize > 0 ? 1u : 0u;
    p.horizon = make_float4(c->env.horizon[0], c->env.horizon[1], c->env.horizon[2], 0.0f);
    p.zenith = make_float4(c->env.zenith[0], c->env.zenith[1], c->env.zenith[2], 0.0f);
    p.env = c->d_env;
    p.env_w = c->env_w;
    p.env_h = c->env_h;
    p.width = c->cfg.width;
    p.height = c->cfg.height;
    p.shard_rank = c->cfg.shard_rank;
    p.shard_count = c->cfg.shard_count;
    p.shard_pixels = c->pixels;
    // CPUPathTracer.cpp:53-54, 65
    p.inv_h = 1.0f / (float)c->cfg.height;
    p.inv_w = 1.0f / (float)c->cfg.width;
    p.aspect = (float)c->cfg.width / (float)c->cfg.height;
    p.max_bounces = c->cfg.max_bounces;
    p.rr_depth = c->cfg.rr_depth;
    p.n_sub = c->n_sub;
    p.sub_cap = c->sub_cap;
    for (int k = 0; k < 2; ++k) p.q[k] = QueueBufs{c->q_o[k], c->q_d[k], c->q_t[k]};
    p.hit = c->hit;
    p.radiance = c->radiance;
    p.accum = c->accum;
    p.counts = c->counts;
    p.totals = c->totals;
    p.cu_count = c->cu_count;
    // (auto: 4 for BVH scenes of <= 256 K primitives — C4 +1.3 %, C4 NEE +1.6 % over 2; 6: +1.5 %, 8: +0.6 % —
    // 2 otherwise: the C2 1/8 shard -5 % at 4, C5 -0.4 %; profiles/r06_t_ab_chunks_per_wave.txt)
    p.chunks_per_wave = c->chunks_per_wave ? c->chunks_per_wave
                                           : ((c->n_nodes != 0 && c->n_prims <= 256u * 1024u) ? 4u : 2u);
    p.px_shift = c->px_shift;
    p.stack = c->bvh_stack;
    p.stack_need = c->bvh_stack_need;
    p.stack_stride = c->bvh_stack_stride;
    p.stack_tb = c->bvh_stack_tb;
    // NEE only with the flag and something to sample (otherwise the oracle's integrator is the plain one)
    p.nee = NeeParams{c->d_emit, nee_active(c) ? c->n_emit : 0u, c->n_emit_spheres};
    return p;
}


}  // namespace

extern "C" {

int spt_abi_version(void) { return SPT_ABI_VERSION; }

int spt_device_count(int* count) {
    if (!count) return SPT_ERR_INVALID;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return SPT_OK;
}

int spt_create(spt_ctx** out, int device_id) {
    if (!out) return SPT_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SPT_ERR_NO_DEVICE;
    if (device_id < 0 || device_id >= n) return SPT_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device_id) != hipSuccess) return SPT_ERR_NO_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SPT_ERR_NO_DEVICE;  // built for gfx950 only
    spt_ctx* c = new spt_ctx();
    c->device = device_id;
    c->cu_count = (uint32_t)std::max(prop.multiProcessorCount, 1);
    // Block-private sub-queues: 12 per CU (two rounds of 6 resident 256-thread shade blocks) measured
    // best on C2 among 4/6/8/12 per CU (scripts/gpu_sweep.sh).
    c->n_sub = c->cu_count * 12u;
    if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->counts, sizeof(uint32_t) * 2 * (kMaxBounces + 1) * c->n_sub) != hipSuccess ||
        hipMalloc(&c->totals, sizeof(unsigned long long) * kTotals) != hipSuccess ||
        hipMalloc(&c->work, sizeof(uint32_t) * 2 * kWorkWords) != hipSuccess ||
        hipMemset(c->work, 0, sizeof(uint32_t) * 2 * kWorkWords) != hipSuccess ||
        hipMemset(c->totals, 0, sizeof(unsigned long long) * kTotals) != hipSuccess ||
        hipMemset(c->counts, 0, sizeof(uint32_t) * 2 * (kMaxBounces + 1) * c->n_sub) != hipSuccess) {
        spt_destroy(c);
        return SPT_ERR_HIP;
    }
    c->stream = c->own_stream;
    *out = c;
    return SPT_OK;
}

void spt_destroy(spt_ctx* c) {
    if (!c) return;
    if (c->device >= 0) (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& e : c->pending) c->free_events.push_back(e);
    if (c->span_open) c->free_events.push_back(c->span_ev);
    for (auto& e : c->free_events) {
        if (e.a) (void)hipEventDestroy(e.a);
        if (e.b) (void)hipEventDestroy(e.b);
    }
    free_buffers(c);
    free_scene(c);
    free_comm(c);
    free_dev(c->counts);
    free_dev(c->totals);
    free_dev(c->d_env);
    free_dev(c->work);
    if (c->out_host) (void)hipHostUnregister(c->out_host);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char* spt_last_error(const spt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int spt_set_stream(spt_ctx* c, void* hip_stream) {
    if (!c) return SPT_ERR_INVALID;
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    c->stream = hip_stream ? (hipStream_t)hip_stream : c->own_stream;
    return SPT_OK;
}

int spt_set_scene(spt_ctx* c, const spt_prim* prims, uint32_t n_prims, const spt_material* mats, uint32_t n_mats,
                  const spt_env* env) {
    if (!c) return SPT_ERR_INVALID;
    if ((n_prims && !prims) || !mats || n_mats == 0 || !env) return fail(c, SPT_ERR_INVALID, "spt_set_scene: null array");
    SPT_HIP(c, hipSetDevice(c->device));
    std::vector<spt_prim> keep_prims(prims, prims + n_prims);  // (prims may alias c->h_prims)
    std::vector<spt_material> keep_mats(mats, mats + n_mats);
    // Flat scenes keep their records in LDS during shading (spt_kernels.hip): compact the materials
    // to the <= kFlatSceneMax ones the primitives use, in order of first use.
    std::vector<spt_prim> remapped;
    std::vector<spt_material> used_mats;
    if (n_prims <= kFlatSceneMax) {
        std::vector<uint32_t> map(n_mats, 0xffffffffu);
        remapped.assign(prims, prims + n_prims);
        for (auto& p : remapped) {
            if (p.material >= n_mats) return fail(c, SPT_ERR_INVALID, "primitive material index out of range");
            if (map[p.material] == 0xffffffffu) {
                map[p.material] = (uint32_t)used_mats.size();
                used_mats.push_back(mats[p.material]);
            }
            p.material = map[p.material];
        }
        if (used_mats.empty()) used_mats.push_back(mats[0]);
        prims = remapped.data();
        mats = used_mats.data();
        n_mats = (uint32_t)used_mats.size();
    }
    std::vector<DevPrim> dp;
    const char* msg = nullptr;
    if (!prepare_prims(prims, n_prims, n_mats, dp, &msg)) return fail(c, SPT_ERR_INVALID, msg);
    const bool fast_div = fast_division_ok(prims, n_prims, dp);  // before build_bvh reorders dp
    std::vector<DevMaterial> dm;
    prepare_materials(mats, n_mats, dm);
    std::vector<DevEmitter> emit;  // SPT_FLAG_NEE's emitters (built for every scene: the flag may come later)
    build_emitters(prims, n_prims, mats, emit);
    std::vector<BvhNode> nodes;
    if (n_prims >= (1u << 27)) return fail(c, SPT_ERR_CAPACITY, "scene too large (>= 2^27 primitives)");
    if (n_prims > kFlatSceneMax) {
        uint32_t max_leaf = bvh_max_leaf(n_prims);  // scene.h
        if (c->bvh_max_leaf >= 1 && c->bvh_max_leaf <= kBvhMaxLeaf) max_leaf = c->bvh_max_leaf;  // spt_tuning
        build_bvh(prims, dp, nodes, max_leaf, c->bvh_bins);
    }
    // the device traverses the W-wide collapse of the binary SAH tree (device_tree); a tree too deep for
    // the traversal stacks is refused before anything of the current scene is freed
    const DevTree tree = device_tree(nodes);
    const uint32_t stack_need = tree.stack_need;
    const uint32_t stack_tb = tree.stack_tb;
    if (stack_need > kBvhStackEntries)
        return fail(c, SPT_ERR_CAPACITY, "spt_set_scene: the BVH needs " + std::to_string(stack_need) +
                                             " traversal stack entries (at most " + std::to_string(kBvhStackEntries) + ")");
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    free_scene(c);
    uint32_t flat_ends = 0, flat_rect = 0;
    if (n_prims && n_prims <= kFlatSceneMax) {  // flat: the originals, then the kind-major copy
        std::vector<DevPrim> sorted;
        uint32_t ends[kFlatKinds - 1];
        sort_flat_by_kind(dp, sorted, ends);
        for (uint32_t g = 0; g + 1 < kFlatKinds; ++g) flat_ends |= ends[g] << (6 * g);
        flat_rect = flat_rect_bits(sorted, ends);
        dp.insert(dp.end(), sorted.begin(), sorted.end());
    }
    if (n_prims) {
        SPT_HIP(c, hipMalloc(&c->d_prims, sizeof(DevPrim) * dp.size()));
        SPT_HIP(c, hipMemcpy(c->d_prims, dp.data(), sizeof(DevPrim) * dp.size(), hipMemcpyHostToDevice));
    }
    SPT_HIP(c, hipMalloc(&c->d_mats, sizeof(DevMaterial) * n_mats));
    SPT_HIP(c, hipMemcpy(c->d_mats, dm.data(), sizeof(DevMaterial) * n_mats, hipMemcpyHostToDevice));
    if (!emit.empty()) {
        SPT_HIP(c, hipMalloc(&c->d_emit, sizeof(DevEmitter) * emit.size()));
        SPT_HIP(c, hipMemcpy(c->d_emit, emit.data(), sizeof(DevEmitter) * emit.size(), hipMemcpyHostToDevice));
    }
    const void* node_data = tree.bytes.data();  // quantized (scene.h), exact decode on the device
    const uint64_t node_bytes = tree.bytes.size();
    c->node_alloc = node_bytes;
    if (node_bytes) {
        SPT_HIP(c, hipMalloc(&c->d_nodes, node_bytes));
        SPT_HIP(c, hipMemcpy(c->d_nodes, node_data, node_bytes, hipMemcpyHostToDevice));
    }
    if (!nodes.empty()) {  // every resident lane's traversal stack (8 waves x 4 SIMDs per CU), as deep as the tree needs
        const uint32_t stride = bvh_stack_stride(stack_need);
        const size_t bytes = (size_t)kBvhStackEntryBytes * stride * 64u * kMaxResidentWaves * c->cu_count;
        SPT_HIP(c, hipMalloc(&c->bvh_stack, bytes));
        c->bvh_stack_stride = stride;
    }
    c->n_prims = n_prims;
    c->n_mats = n_mats;
    c->n_emit = (uint32_t)emit.size();
    c->n_emit_spheres = sphere_emitters(emit);
    c->n_nodes = (uint32_t)nodes.size();
    c->n_dev_nodes = (uint32_t)(node_bytes / kDevNodeBytes);
    c->bvh_stack_need = stack_need;
    c->bvh_stack_tb = stack_tb;
    c->env = *env;
    c->has_scene = true;
    c->fast_div = fast_div;
    c->flat_ends = flat_ends;
    c->flat_rect = flat_rect;
    c->h_prims.swap(keep_prims);
    c->h_mats.swap(keep_mats);
    if (n_prims > kFlatSceneMax) {  // what spt_update_prims refits
        c->h_dp = dp;
        c->h_nodes = nodes;
        c->h_pos.assign(n_prims, 0u);
        for (uint32_t i = 0; i < n_prims; ++i) {
            uint32_t orig;
            std::memcpy(&orig, &dp[i].b[3], sizeof orig);  // DevPrim b.w: the original index's bits
            c->h_pos[orig] = i;
        }
    } else {
        c->h_dp.clear();
        c->h_nodes.clear();
        c->h_pos.clear();
    }
    if (!nodes.empty()) {  // the root's bounds: the sorted schedule's binning grid
        for (int a = 0; a < 3; ++a) {
            c->scene_lo[a] = nodes[0].lo[a];
            c->scene_hi[a] = nodes[0].hi[a];
        }
    }
    c->scene_bytes = sizeof(DevPrim) * (uint64_t)dp.size() + node_bytes + sizeof(DevMaterial) * (uint64_t)n_mats +
                     sizeof(DevEmitter) * (uint64_t)emit.size();
    c->stack_bytes = (uint64_t)kBvhStackEntryBytes * c->bvh_stack_stride * 64u * kMaxResidentWaves * c->cu_count;
    // a flat scene of a new shape: its specialized kernels start compiling now, off the render thread
    // (rebuild_scene -> here); frames rendered before they are ready run the generic kernels
    prefetch_flat(c);
    // scene change -> m_frameCount = 0 (CPUPathTracer.cpp:122-131)
    if (c->configured) return spt_reset(c);
    return SPT_OK;
}

int spt_update_prims(spt_ctx* c, const uint32_t* indices, const spt_prim* prims, uint32_t n) {
    if (!c) return SPT_ERR_INVALID;
    if (!c->has_scene) return fail(c, SPT_ERR_NO_SCENE, "spt_update_prims before spt_set_scene");
    if (n && (!indices || !prims)) return fail(c, SPT_ERR_INVALID, "spt_update_prims: null array");
    const uint32_t total = (uint32_t)c->h_prims.size();
    std::vector<DevPrim> upd;
    const char* msg = nullptr;
    if (!prepare_prims(prims, n, (uint32_t)c->h_mats.size(), upd, &msg)) return fail(c, SPT_ERR_INVALID, msg);
    for (uint32_t j = 0; j < n; ++j)
        if (indices[j] >= total) return fail(c, SPT_ERR_INVALID, "spt_update_prims: index out of range");
    c->hit_cache_valid = false;  // (moved primitives: k_frame traces the camera segments again)
    c->chunk_order_key = 0;  // (the chunks' costs were this scene's)
    // the edits are staged and committed to the host mirror only once the device holds them, so a
    // failed call leaves the ctx's scene as it was
    std::vector<spt_prim> all = c->h_prims;
    for (uint32_t j = 0; j < n; ++j) all[indices[j]] = prims[j];
    if (c->h_nodes.empty()) {  // flat scene: its records are a few hundred bytes, re-prepare them all
        const std::vector<spt_material> mats = c->h_mats;
        const spt_env env = c->env;
        return spt_set_scene(c, all.data(), total, mats.data(), (uint32_t)mats.size(), &env);
    }
    // BVH scene: the changed records at their device positions, the tree refitted (same topology:
    // no rebuild), the 4-wide collapse and its quantization redone, the node array re-uploaded
    std::vector<DevPrim> dp = c->h_dp;
    std::vector<BvhNode> tree = c->h_nodes;
    uint32_t lo = UINT32_MAX, hi = 0;  // the device positions touched: uploaded as one range
    for (uint32_t j = 0; j < n; ++j) {
        DevPrim d = upd[j];
        std::memcpy(&d.b[3], &indices[j], sizeof(uint32_t));  // the original index stays the tie-break key
        const uint32_t at = c->h_pos[indices[j]];
        dp[at] = d;
        lo = std::min(lo, at);
        hi = std::max(hi, at);
    }
    refit_bvh(all.data(), total, dp, tree);
    std::vector<DevEmitter> emit;  // moved emitters move their samples
    build_emitters(all.data(), total, c->h_mats.data(), emit);
    const DevTree dtree = device_tree(tree);
    const uint32_t stack_need = dtree.stack_need;  // (the refit can change the collapse)
    if (stack_need > kBvhStackEntries)
        return fail(c, SPT_ERR_CAPACITY, "spt_update_prims: the refitted BVH needs " + std::to_string(stack_need) +
                                             " traversal stack entries (at most " + std::to_string(kBvhStackEntries) + ")");
    const void* node_data = dtree.bytes.data();
    const uint64_t node_bytes = dtree.bytes.size();
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    // Every allocation the edit needs comes first — a grown node array (the 4-wide collapse opens the
    // largest children first, so refitted areas can change its node count), the emitter array, deeper
    // traversal stacks — and only once all of them have succeeded is anything copied or swapped in: a
    // failed call leaves the device scene, the stacks and their sizes exactly as they were.
    const uint32_t stride = bvh_stack_stride(stack_need);
    const size_t stack_bytes = (size_t)kBvhStackEntryBytes * stride * 64u * kMaxResidentWaves * c->cu_count;
    float4* grown_nodes = nullptr;
    float4* new_emit = nullptr;
    void* grown_stack = nullptr;
    auto release = [&]() {
        free_dev(grown_nodes);
        free_dev(new_emit);
        free_dev(grown_stack);
    };
    hipError_t e = hipSuccess;
    if (node_bytes > c->node_alloc) e = hipMalloc(&grown_nodes, node_bytes);
    if (e == hipSuccess && emit.size() != c->n_emit && !emit.empty())  // (an edit can make an emitter degenerate, or not)
        e = hipMalloc(&new_emit, sizeof(DevEmitter) * emit.size());
    if (e == hipSuccess && stride > c->bvh_stack_stride) e = hipMalloc(&grown_stack, stack_bytes);  // deeper than allocated
    if (e != hipSuccess) {
        release();
        (void)hipGetLastError();
        return fail(c, SPT_ERR_HIP, std::string("spt_update_prims: allocation failed: ") + hipGetErrorString(e));
    }
    // the copies into the buffers that stay (new buffers are swapped in only after theirs succeeded)
    float4* nodes_dst = grown_nodes ? grown_nodes : c->d_nodes;
    float4* emit_dst = emit.size() != c->n_emit ? new_emit : c->d_emit;
    e = hipMemcpy(nodes_dst, node_data, node_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && !emit.empty()) e = hipMemcpy(emit_dst, emit.data(), sizeof(DevEmitter) * emit.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && n)
        e = hipMemcpy(c->d_prims + 4u * lo, &dp[lo], sizeof(DevPrim) * (hi - lo + 1u), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        // a copy into the kept buffers may have landed partly: the device no longer matches the host
        // mirror, so the scene is dropped (the next render fails with SPT_ERR_NO_SCENE, not wrong bits)
        release();
        (void)hipGetLastError();
        free_scene(c);
        c->has_scene = false;
        return fail(c, SPT_ERR_HIP, std::string("spt_update_prims: upload failed: ") + hipGetErrorString(e));
    }
    if (grown_nodes) {
        free_dev(c->d_nodes);
        c->d_nodes = grown_nodes;
        c->node_alloc = node_bytes;
    }
    if (emit.size() != c->n_emit) {
        free_dev(c->d_emit);
        c->d_emit = new_emit;
    }
    c->n_emit = (uint32_t)emit.size();
    c->n_emit_spheres = sphere_emitters(emit);
    c->n_dev_nodes = (uint32_t)(node_bytes / kDevNodeBytes);
    if (grown_stack) {
        free_dev(c->bvh_stack);
        c->bvh_stack = grown_stack;
        c->bvh_stack_stride = stride;
        c->stack_bytes = stack_bytes;
    }
    c->bvh_stack_need = stack_need;
    c->bvh_stack_tb = dtree.stack_tb;  // (the collapse can add nodes)
    c->h_prims.swap(all);
    c->h_dp.swap(dp);
    c->h_nodes.swap(tree);
    for (int a = 0; a < 3; ++a) {
        c->scene_lo[a] = c->h_nodes[0].lo[a];
        c->scene_hi[a] = c->h_nodes[0].hi[a];
    }
    // scene change -> m_frameCount = 0 (CPUPathTracer.cpp:122-131)
    if (c->configured) return spt_reset(c);
    return SPT_OK;
}

int spt_configure(spt_ctx* c, const spt_config* cfg) {
    if (!c || !cfg) return SPT_ERR_INVALID;
    if (cfg->width == 0 || cfg->height == 0) return fail(c, SPT_ERR_INVALID, "width and height must be > 0");
    if (cfg->max_bounces > kMaxBounces) return fail(c, SPT_ERR_INVALID, "max_bounces > 32");
    if (cfg->shard_count == 0 || cfg->shard_rank >= cfg->shard_count)
        return fail(c, SPT_ERR_INVALID, "shard_rank must be < shard_count");
    if ((uint64_t)cfg->width * cfg->height >= (1ull << 31)) return fail(c, SPT_ERR_INVALID, "image too large");
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    const uint32_t rows = cfg->shard_rank < cfg->height
                              ? (cfg->height - cfg->shard_rank + cfg->shard_count - 1) / cfg->shard_count
                              : 0u;
    const uint32_t pixels = rows * cfg->width;
    uint32_t fpp = cfg->frames_in_flight;
    if (fpp == 0) {
        // auto: about 2^24 paths per pass (8 frames at 1920x1080): fewer, fuller launches
        const uint32_t target = 1u << 24;
        fpp = pixels ? std::max(1u, std::min(256u, target / std::max(pixels, 1u))) : 1u;
    }
    if ((uint64_t)fpp * pixels >= (1ull << 31)) return fail(c, SPT_ERR_INVALID, "frames_in_flight * pixels too large");
    const uint32_t cap = sub_capacity((uint64_t)fpp * pixels, c->n_sub);
    const bool realloc = !c->configured || pixels != c->pixels || fpp != c->frames_per_pass || c->sub_alloc != c->n_sub;
    c->cfg = *cfg;
    c->rows = rows;
    c->pixels = pixels;
    c->frames_per_pass = fpp;
    c->sub_cap = cap;
    if (realloc) {
        free_buffers(c);
        c->sub_alloc = c->n_sub;
        const size_t qn = (size_t)cap * c->n_sub;
        if (qn) {
            for (int k = 0; k < 2; ++k) {
                SPT_HIP(c, hipMalloc(&c->q_o[k], sizeof(float4) * qn));
                SPT_HIP(c, hipMalloc(&c->q_d[k], sizeof(float4) * qn));
                SPT_HIP(c, hipMalloc(&c->q_t[k], sizeof(float4) * qn));
            }
            SPT_HIP(c, hipMalloc(&c->hit, sizeof(float2) * qn));
            SPT_HIP(c, hipMalloc(&c->radiance, sizeof(float4) * (size_t)fpp * pixels));
        }
        SPT_HIP(c, hipMalloc(&c->accum, sizeof(float4) * std::max<size_t>(pixels, 1)));
        SPT_HIP(c, hipMalloc(&c->hit_cache, sizeof(float2) * std::max<size_t>(pixels, 1)));
        SPT_HIP(c, hipMalloc(&c->chunk_cost, sizeof(uint16_t) * std::max<size_t>(pixels, 1)));
        SPT_HIP(c, hipMalloc(&c->chunk_order, sizeof(uint32_t) * std::max<size_t>(pixels, 1)));
        if (kFrameHitCache >= 2) {
            SPT_HIP(c, hipMalloc(&c->live_rec, sizeof(uint4) * std::max<size_t>(pixels, 1)));
            SPT_HIP(c, hipMalloc(&c->sky_pix, sizeof(uint32_t) * std::max<size_t>(pixels, 1)));
            SPT_HIP(c, hipMalloc(&c->list_counts, sizeof(uint32_t) * (2 + (pixels + kBlock - 1) / kBlock)));
        }
        SPT_HIP(c, hipMalloc(&c->resolved, sizeof(uint32_t) * std::max<size_t>(pixels, 1)));
    }
    c->hit_cache_valid = false;  // (a new image size, shard or flags: the camera hits are traced again)
    c->chunk_order_key = 0;
    const size_t qn = (size_t)cap * c->n_sub;
    if ((cfg->flags & SPT_FLAG_SORTED_RAYS) && qn && !c->ray_perm) {  // the sorted schedule's buffers
        SPT_HIP(c, hipMalloc(&c->ray_keys, sizeof(uint16_t) * qn));
        SPT_HIP(c, hipMalloc(&c->ray_perm, sizeof(uint32_t) * qn));
        SPT_HIP(c, hipMalloc(&c->ray_bins, sizeof(uint32_t) * 4096));
        SPT_HIP(c, hipMalloc(&c->ray_cursor, sizeof(uint32_t) * 4097));
        SPT_HIP(c, hipMemset(c->ray_bins, 0, sizeof(uint32_t) * 4096));
    }
    c->configured = true;
    prefetch_flat(c);  // (a flat scene's kernels are compiled for the configuration too)
    // settings dirty / resize -> m_frameCount = 0 and a zeroed accumulation (CPUPathTracer.cpp:132-154)
    return spt_reset(c);
}

int spt_reset(spt_ctx* c) {
    if (!c) return SPT_ERR_INVALID;
    if (!c->configured) return fail(c, SPT_ERR_NOT_CONFIGURED, "spt_reset before spt_configure");
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipMemsetAsync(c->accum, 0, sizeof(float4) * std::max<size_t>(c->pixels, 1), c->stream));
    c->frame_count = 0;
    return SPT_OK;
}

int spt_get_frame_count(const spt_ctx* c, uint32_t* fc) {
    if (!c || !fc) return SPT_ERR_INVALID;
    *fc = c->frame_count;
    return SPT_OK;
}

int spt_render(spt_ctx* c, uint32_t first_frame, uint32_t n_frames) {
    if (!c) return SPT_ERR_INVALID;
    if (!c->has_scene) return fail(c, SPT_ERR_NO_SCENE, "Scene not set before rendering");  // CPUPathTracer.cpp:46
    if (!c->configured) return fail(c, SPT_ERR_NOT_CONFIGURED, "spt_render before spt_configure");
    if (c->sub_alloc != c->n_sub) return fail(c, SPT_ERR_NOT_CONFIGURED, "spt_set_tuning(subqueues) takes effect at spt_configure");
    SPT_HIP(c, hipSetDevice(c->device));
    if (c->pixels == 0 || n_frames == 0) {
        c->frame_count += n_frames;
        return SPT_OK;
    }
    PassParams p = base_params(c);
    uint32_t done = 0;
    if (schedule_persistent(c, n_frames)) {
        // one launch per <= kPersistentMaxFrames frames: every path of the call, accumulated in frame
        // order in-kernel (fewer, longer launches amortize each launch's tail)
        c->last_schedule = SPT_SCHEDULE_PERSISTENT;
        while (done < n_frames) {
            const uint32_t f = std::min(kPersistentMaxFrames, n_frames - done);
            p.first_frame = first_frame + done;
            p.n_frames = f;
            p.n_paths = f * c->pixels;
            EventPair ev;
            if (begin_persistent(c, ev) != SPT_OK) return SPT_ERR_HIP;
            next_work_set(c, p);
            p.chunk_cost = c->chunk_cost;
            p.chunk_order = c->chunk_order;
            p.chunk_order_key = &c->chunk_order_key;
            c->last_specialized = launch_paths(p, c->counters, c->stream);
            // a failed launch leaves no chunk order behind (a retry must not read an unsorted buffer)
            const hipError_t le = hipGetLastError();
            if (le != hipSuccess) c->chunk_order_key = 0;
            if (end_persistent(c, ev) != SPT_OK) {
                c->chunk_order_key = 0;
                return SPT_ERR_HIP;
            }
            SPT_HIP(c, le);
            done += f;
            c->passes++;
        }
        c->frames += n_frames;
        c->paths += (uint64_t)n_frames * c->pixels;
        c->frame_count += n_frames;
        return SPT_OK;
    }
    if (schedule_frame(c)) {
        c->last_schedule = SPT_SCHEDULE_FRAME;
        for (; done < n_frames; ++done) {  // stream order keeps the frames' accumulation order
            p.first_frame = first_frame + done;
            p.n_frames = 1;
            p.n_paths = c->pixels;
            EventPair ev;
            if (begin_persistent(c, ev) != SPT_OK) return SPT_ERR_HIP;
            next_work_set(c, p);
            p.hit_cache = c->hit_cache;
            p.live_rec = c->live_rec;
            p.sky_pix = c->sky_pix;
            p.list_counts = c->list_counts;
            p.hit_mode = !c->hit_cache_valid ? 1u : (c->frame_lists ? 3u : 2u);
            p.live_pixels = c->live_pixels;
            if (c->fuse_frames != 0.0f && done + 1u == n_frames) {  // the call's last frame resolves as it ends
                p.rgba = (uint32_t*)c->out_dev;
                p.rgba_frames = c->fuse_frames;
                p.rgba_exposure = c->fuse_exposure;
                c->fused = true;
            }
            c->last_specialized = launch_frame(p, c->counters, c->stream);
            if (end_persistent(c, ev) != SPT_OK) return SPT_ERR_HIP;
            SPT_HIP(c, hipGetLastError());
            if (!c->hit_cache_valid) c->frame_lists = false;
            if (!c->hit_cache_valid && frame_lists_scene(p, c->counters)) {  // compacted once (stream order)
                launch_hit_lists(p, c->list_counts + 2, c->stream);
                SPT_HIP(c, hipGetLastError());
                // the live count sizes the next launches' grids: read back once per scene / configuration
                // (this waits for the frame just launched, ~0.1 ms, on the first frame after a change only)
                SPT_HIP(c, hipMemcpyAsync(&c->live_pixels, c->list_counts, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                          c->stream));
                SPT_HIP(c, hipStreamSynchronize(c->stream));
                c->frame_lists = c->pixels - c->live_pixels >= c->pixels / kFrameListsMinSkyDiv;
            }
            c->hit_cache_valid = true;  // (stream order: the next launch reads what this one stored)
            c->passes++;
        }
        c->frames += n_frames;
        c->paths += (uint64_t)n_frames * c->pixels;
        c->frame_count += n_frames;
        return SPT_OK;
    }
    c->last_schedule = schedule_fused(c) ? SPT_SCHEDULE_FUSED : SPT_SCHEDULE_SPLIT;
    c->last_specialized = false;
    while (done < n_frames) {
        const uint32_t f = std::min(c->frames_per_pass, n_frames - done);
        p.first_frame = first_frame + done;
        p.n_frames = f;
        p.n_paths = f * c->pixels;
        EventPair ev;
        if (c->cfg.max_bounces == 0) {  // no segment traced: every path's radiance is 0
            SPT_HIP(c, hipMemsetAsync(c->radiance, 0, sizeof(float4) * (size_t)p.n_paths, c->stream));
            SPT_HIP(c, hipMemsetAsync(c->counts, 0, sizeof(uint32_t) * 2 * (kMaxBounces + 1) * c->n_sub, c->stream));
        }
        const uint32_t wave_bounces = std::min(c->cfg.max_bounces, schedule_tail(c));
        const bool fused = schedule_fused(c);
        for (uint32_t b = 0; b < wave_bounces; ++b) {
            if (fused) {  // extend + shade in one launch (timed as "shade")
                if (c->profiling && !c->span && begin_event(c, ev, 1, b) != SPT_OK) return SPT_ERR_HIP;
                launch_bounce(p, b, c->stream);
                if (c->profiling && !c->span && end_event(c, ev) != SPT_OK) return SPT_ERR_HIP;
                continue;
            }
            if (c->profiling && !c->span && begin_event(c, ev, 0, b) != SPT_OK) return SPT_ERR_HIP;
            if ((c->cfg.flags & SPT_FLAG_SORTED_RAYS) && b > 0 && c->n_nodes && c->ray_perm)
                launch_extend_sorted(p, b, c->stream);  // the binning is timed with the extend it serves
            else
                launch_extend(p, b, c->stream);
            if (c->profiling && !c->span && end_event(c, ev) != SPT_OK) return SPT_ERR_HIP;
            if (c->profiling && !c->span && begin_event(c, ev, 1, b) != SPT_OK) return SPT_ERR_HIP;
            launch_shade(p, b, c->stream);
            if (c->profiling && !c->span && end_event(c, ev) != SPT_OK) return SPT_ERR_HIP;
        }
        if (wave_bounces < c->cfg.max_bounces) {  // thinned queues: finish every path in one launch
            if (c->profiling && !c->span && begin_event(c, ev, 3, wave_bounces) != SPT_OK) return SPT_ERR_HIP;
            launch_trace_tail(p, wave_bounces, c->stream);
            if (c->profiling && !c->span && end_event(c, ev) != SPT_OK) return SPT_ERR_HIP;
        }
        if (c->profiling && !c->span && begin_event(c, ev, 2) != SPT_OK) return SPT_ERR_HIP;
        launch_accumulate(p, c->stream);
        if (c->profiling && !c->span && end_event(c, ev) != SPT_OK) return SPT_ERR_HIP;
        SPT_HIP(c, hipGetLastError());
        done += f;
        c->passes++;
    }
    c->frames += n_frames;
    c->paths += (uint64_t)n_frames * c->pixels;
    c->frame_count += n_frames;
    return SPT_OK;
}

// The caller waits for the frame (spt_synchronize, the resolves)
// (polling an event recorded after the frame instead measured the same)
static hipError_t wait_frame(spt_ctx* c) { return hipStreamSynchronize(c->stream); }

int spt_synchronize(spt_ctx* c) {
    if (!c) return SPT_ERR_INVALID;
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, wait_frame(c));
    return SPT_OK;
}

int spt_shard_pixels(const spt_ctx* c, uint64_t* n) {
    if (!c || !n) return SPT_ERR_INVALID;
    if (!c->configured) return SPT_ERR_NOT_CONFIGURED;
    *n = c->pixels;
    return SPT_OK;
}

int spt_read_accum(spt_ctx* c, float* host_rgba) {
    if (!c || !host_rgba) return SPT_ERR_INVALID;
    if (!c->configured) return fail(c, SPT_ERR_NOT_CONFIGURED, "not configured");
    SPT_HIP(c, hipSetDevice(c->device));
    if (c->pixels == 0) return SPT_OK;
    SPT_HIP(c, hipMemcpyAsync(host_rgba, c->accum, sizeof(float4) * c->pixels, hipMemcpyDeviceToHost, c->stream));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    return SPT_OK;
}

int spt_accum_device_ptr(spt_ctx* c, void** dptr, size_t* bytes) {
    if (!c || !dptr || !bytes) return SPT_ERR_INVALID;
    if (!c->configured) return fail(c, SPT_ERR_NOT_CONFIGURED, "not configured");
    *dptr = c->accum;
    *bytes = sizeof(float4) * (size_t)c->pixels;
    return SPT_OK;
}

int spt_copy_accum_device(spt_ctx* c, void* dst) {
    if (!c || !dst) return SPT_ERR_INVALID;
    if (!c->configured) return fail(c, SPT_ERR_NOT_CONFIGURED, "not configured");
    SPT_HIP(c, hipSetDevice(c->device));
    if (c->pixels == 0) return SPT_OK;
    SPT_HIP(c, hipMemcpyAsync(dst, c->accum, sizeof(float4) * c->pixels, hipMemcpyDeviceToDevice, c->stream));
    return SPT_OK;
}

int spt_resolve_rgba8(spt_ctx* c, uint32_t frame_count, uint32_t* host_out) {
    return spt_resolve_rgba8_exposure(c, frame_count, 1.0f, host_out);
}

int spt_resolve_rgba8_exposure(spt_ctx* c, uint32_t frame_count, float exposure, uint32_t* host_out) {
    if (!c || !host_out) return SPT_ERR_INVALID;
    if (!c->configured) return fail(c, SPT_ERR_NOT_CONFIGURED, "not configured");
    if (frame_count == 0) return fail(c, SPT_ERR_INVALID, "No frames rendered yet");  // CPUPathTracer.cpp:89
    SPT_HIP(c, hipSetDevice(c->device));
    if (c->pixels == 0) return SPT_OK;
    if (host_out == c->out_host && sizeof(uint32_t) * (size_t)c->pixels <= c->out_bytes) {
        // the registered buffer: the kernel's stores go straight to host memory over PCIe
        launch_resolve(c->accum, c->pixels, (float)frame_count, exposure, (uint32_t*)c->out_dev, c->stream);
        SPT_HIP(c, hipGetLastError());
    } else {
        launch_resolve(c->accum, c->pixels, (float)frame_count, exposure, c->resolved, c->stream);
        SPT_HIP(c, hipGetLastError());
        SPT_HIP(c, hipMemcpyAsync(host_out, c->resolved, sizeof(uint32_t) * c->pixels, hipMemcpyDeviceToHost, c->stream));
    }
    SPT_HIP(c, wait_frame(c));
    return SPT_OK;
}

int spt_render_resolve_rgba8(spt_ctx* c, uint32_t first_frame, uint32_t n_frames, uint32_t frame_count, float exposure,
                             uint32_t* host_out) {
    if (!c || !host_out) return SPT_ERR_INVALID;
    if (frame_count == 0) return fail(c, SPT_ERR_INVALID, "No frames rendered yet");  // CPUPathTracer.cpp:89
    // fused only into the registered buffer (device-mapped host memory) and only by a k_frame launch;
    // any other call renders, then resolves as spt_resolve_rgba8_exposure does (same pixels)
    // (not while spt_set_profiling counts segments: the fused kernels carry no counters)
    const bool fuse = c->configured && !c->counters && host_out == c->out_host &&
                      sizeof(uint32_t) * (size_t)c->pixels <= c->out_bytes;
    c->fuse_frames = fuse ? (float)frame_count : 0.0f;
    c->fuse_exposure = exposure;
    c->fused = false;
    const int rc = spt_render(c, first_frame, n_frames);
    const bool fused = c->fused;
    c->fuse_frames = 0.0f;
    c->fused = false;
    if (rc != SPT_OK) return rc;
    if (!fused) return spt_resolve_rgba8_exposure(c, frame_count, exposure, host_out);
    SPT_HIP(c, wait_frame(c));  // (the frame's stores have reached host memory)
    return SPT_OK;
}

int spt_register_host_output(spt_ctx* c, void* host_out, size_t bytes) {
    if (!c) return SPT_ERR_INVALID;
    if ((host_out == nullptr) != (bytes == 0)) return fail(c, SPT_ERR_INVALID, "host output: pointer and size disagree");
    SPT_HIP(c, hipSetDevice(c->device));
    if (c->out_host) {
        SPT_HIP(c, hipStreamSynchronize(c->stream));  // no resolve may still be writing it
        const hipError_t e = hipHostUnregister(c->out_host);
        c->out_host = c->out_dev = nullptr;
        c->out_bytes = 0;
        if (e != hipSuccess) return fail(c, SPT_ERR_HIP, std::string("hipHostUnregister: ") + hipGetErrorString(e));
    }
    if (!host_out) return SPT_OK;
    SPT_HIP(c, hipHostRegister(host_out, bytes, hipHostRegisterMapped));
    void* dev = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&dev, host_out, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(host_out);
        return fail(c, SPT_ERR_HIP, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
    }
    c->out_host = host_out;
    c->out_dev = dev;
    c->out_bytes = bytes;
    return SPT_OK;
}

int spt_assemble_rows(spt_ctx* c, const void* gathered, void* out) {
    if (!c || !gathered || !out) return SPT_ERR_INVALID;
    if (!c->configured) return fail(c, SPT_ERR_NOT_CONFIGURED, "not configured");
    SPT_HIP(c, hipSetDevice(c->device));
    const uint32_t world = c->cfg.shard_count;
    const uint32_t rows_max = (c->cfg.height + world - 1) / world;
    launch_assemble_rows((const float4*)gathered, (float4*)out, c->cfg.width, c->cfg.height, world, rows_max, c->stream);
    SPT_HIP(c, hipGetLastError());
    return SPT_OK;
}

int spt_set_env_map(spt_ctx* c, const float* rgba, uint32_t width, uint32_t height) {
    if (!c) return SPT_ERR_INVALID;
    if (rgba && (width == 0 || height == 0 || (uint64_t)width * height >= (1ull << 28)))
        return fail(c, SPT_ERR_INVALID, "environment map: bad size");
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    free_dev(c->d_env);
    c->env_w = c->env_h = 0;
    if (rgba) {
        const size_t bytes = sizeof(float4) * (size_t)width * height;
        SPT_HIP(c, hipMalloc(&c->d_env, bytes));
        SPT_HIP(c, hipMemcpy(c->d_env, rgba, bytes, hipMemcpyHostToDevice));
        c->env_w = width;
        c->env_h = height;
    }
    if (c->configured) return spt_reset(c);  // a different sky: the accumulation restarts
    return SPT_OK;
}

int spt_env_octa_from_equirect(const float* src, uint32_t sw, uint32_t sh, float* dst, uint32_t dw, uint32_t dh) {
    if (!src || !dst || sw == 0 || sh == 0 || dw == 0 || dh == 0) return SPT_ERR_INVALID;
    const double kPi = 3.14159265358979323846;
    for (uint32_t iy = 0; iy < dh; ++iy) {
        for (uint32_t ix = 0; ix < dw; ++ix) {
            // octahedral decode of the texel centre (the inverse of octa_texel's projection)
            double px = 2.0 * (ix + 0.5) / dw - 1.0, pz = 2.0 * (iy + 0.5) / dh - 1.0;
            double y = 1.0 - std::fabs(px) - std::fabs(pz);
            if (y < 0.0) {
                const double fx = (1.0 - std::fabs(pz)) * (px >= 0.0 ? 1.0 : -1.0);
                const double fz = (1.0 - std::fabs(px)) * (pz >= 0.0 ? 1.0 : -1.0);
                px = fx;
                pz = fz;
            }
            const double len = std::sqrt(px * px + y * y + pz * pz);
            const double x = px / len, yy = y / len, z = pz / len;
            const double phi = std::atan2(x, -z);                              // [-pi, pi]
            const double theta = std::acos(std::max(-1.0, std::min(1.0, yy)));  // 0 at +y
            uint32_t sx = (uint32_t)((phi + kPi) / (2.0 * kPi) * sw), sy = (uint32_t)(theta / kPi * sh);
            sx = std::min(sx, sw - 1u);
            sy = std::min(sy, sh - 1u);
            const float* t = src + 3ull * ((size_t)sy * sw + sx);
            float* o = dst + 4ull * ((size_t)iy * dw + ix);
            o[0] = t[0];
            o[1] = t[1];
            o[2] = t[2];
            o[3] = 1.0f;
        }
    }
    return SPT_OK;
}

int spt_set_profiling(spt_ctx* c, int mode) {
    if (!c) return SPT_ERR_INVALID;
    SPT_HIP(c, hipSetDevice(c->device));
    const bool span = (mode & SPT_PROFILE_SPAN) != 0;
    if (!span && close_span(c) != SPT_OK) return SPT_ERR_HIP;  // (recorded before any flush waits)
    if (!(mode & (SPT_PROFILE_EVENTS | SPT_PROFILE_SPAN)) && flush_events(c) != SPT_OK) return SPT_ERR_HIP;
    c->profiling = (mode & (SPT_PROFILE_EVENTS | SPT_PROFILE_SPAN)) != 0;
    c->span = span;
    const bool counters = (mode & SPT_PROFILE_COUNTERS) != 0;
    // k_frame's compacted camera-hit lists were chosen for the kernels of the old counters setting
    // (frame_lists_scene: the counting kernels never hold a scene in LDS): decided again
    if (counters != c->counters) c->hit_cache_valid = false;
    c->counters = counters;
    return SPT_OK;
}

int spt_get_stats(spt_ctx* c, spt_stats* out) {
    if (!c || !out) return SPT_ERR_INVALID;
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    if (flush_events(c) != SPT_OK) return SPT_ERR_HIP;
    unsigned long long tot[kTotals];
    SPT_HIP(c, hipMemcpy(tot, c->totals, sizeof(tot), hipMemcpyDeviceToHost));
    std::memset(out, 0, sizeof(*out));
    out->frames = c->frames;
    out->paths = c->paths;
    out->passes = c->passes;
    for (uint32_t b = 0; b < kMaxBounces && b < SPT_MAX_BOUNCES; ++b) {
        out->segments[b] = tot[b];
        out->segments_total += tot[b];
        out->radiance_updates[b] = tot[kMaxBounces + b];
    }
    out->extend_launches = c->ext_launches;
    out->extend_ms = c->ext_ms;
    out->extend_segments = c->ext_launches ? out->segments_total : 0;
    out->shade_launches = c->shade_launches;
    out->shade_ms = c->shade_ms;
    out->other_ms = c->other_ms;
    out->tail_ms = c->tail_ms;
    out->tail_launches = c->tail_launches;
    out->tail_bounce = schedule_tail(c);
    out->fused = schedule_fused(c) ? 1u : 0u;
    out->persistent_ms = c->persist_ms;
    out->persistent_launches = c->persist_launches;
    out->schedule = c->last_schedule;
    out->lane_slots = tot[2 * kMaxBounces];
    out->lane_busy = tot[2 * kMaxBounces + 1];
    out->bvh_node_visits = tot[2 * kMaxBounces + 2];
    out->prim_tests = tot[2 * kMaxBounces + 3];
    out->flat_fast_path = (c->fast_div && c->n_prims <= kFlatSceneMax) ? 1u : 0u;
    out->specialized = c->last_specialized ? 1u : 0u;
    for (uint32_t b = 0; b < kMaxBounces && b < SPT_MAX_BOUNCES; ++b) {
        out->extend_ms_bounce[b] = c->ext_ms_b[b];
        out->shade_ms_bounce[b] = c->shade_ms_b[b];
    }
    out->bvh_nodes = c->n_nodes;
    out->scene_bytes = c->scene_bytes;
    out->shadow_rays = tot[kTotShadow];
    out->emitters = c->n_emit;
    out->stack_bytes = c->stack_bytes;
    out->stack_need = c->bvh_stack_need;
    out->stalled_waves = tot[kTotStalled];
    if (tot[kTotStalled])
        return fail(c, SPT_ERR_HIP, "k_paths: " + std::to_string(tot[kTotStalled]) +
                                        " wave(s) stopped at the step bound with frames unaccumulated (a bug)");
    return SPT_OK;
}

int spt_stats_clear(spt_ctx* c) {
    if (!c) return SPT_ERR_INVALID;
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    if (flush_events(c) != SPT_OK) return SPT_ERR_HIP;
    SPT_HIP(c, hipMemset(c->totals, 0, sizeof(unsigned long long) * kTotals));
    c->frames = c->paths = c->passes = 0;
    c->ext_launches = c->shade_launches = c->ext_segments = 0;
    c->ext_ms = c->shade_ms = c->other_ms = c->tail_ms = 0.0;
    c->tail_launches = 0;
    c->persist_ms = 0.0;
    c->persist_launches = 0;
    for (uint32_t b = 0; b < kMaxBounces; ++b) c->ext_ms_b[b] = c->shade_ms_b[b] = 0.0;
    return SPT_OK;
}

int spt_specialize_scene(spt_ctx* c) {
    if (!c) return SPT_ERR_INVALID;
    if (!c->has_scene) return fail(c, SPT_ERR_NO_SCENE, "spt_specialize_scene before spt_set_scene");
    if (c->n_prims == 0 || c->n_nodes != 0 || c->specialize < 0) return SPT_OK;  // nothing to specialize
    SPT_HIP(c, hipSetDevice(c->device));
    const uint64_t key = flat_jit_key(c);  // (before spt_configure: the shape alone)
    const int env = c->d_env ? 1 : 0;
    std::string err;
    const bool nee = nee_active(c);
    if (nee ? (!jit_function(kJitPathsNee, 2, key, &err) || !jit_function(kJitFrameNee, 2, key, &err))
            : (!jit_function(kJitPaths, env, key, &err) || !jit_function(kJitFrame, env, key, &err) ||
               !jit_function(kJitPathsChan, env, key, &err)))
        return fail(c, SPT_ERR_HIP, ("specialized kernels unavailable (the generic ones run): " + err).c_str());
    return SPT_OK;
}

int spt_compile_flat_kernels(const spt_prim* prims, uint32_t n_prims, int env_map, char* log, size_t log_bytes) {
    if (log && log_bytes) log[0] = 0;
    if ((!prims && n_prims) || n_prims == 0 || n_prims > kFlatSceneMax) return SPT_ERR_INVALID;
    uint32_t n_mats = 1;
    for (uint32_t i = 0; i < n_prims; ++i) n_mats = std::max(n_mats, prims[i].material + 1u);
    std::vector<DevPrim> dp, sorted;
    const char* msg = nullptr;
    if (!prepare_prims(prims, n_prims, n_mats, dp, &msg)) return SPT_ERR_INVALID;
    uint32_t ends[kFlatKinds - 1], flat_ends = 0;
    sort_flat_by_kind(dp, sorted, ends);
    for (uint32_t g = 0; g + 1 < kFlatKinds; ++g) flat_ends |= ends[g] << (6 * g);
    const uint64_t key = flat_shape_key(flat_ends, n_prims, flat_rect_bits(sorted, ends));
    std::string out;
    const int env = env_map ? 1 : 0;
    if (jit_compile(kJitPaths, env, key, &out) && jit_compile(kJitFrame, env, key, &out) &&
        jit_compile(kJitPathsChan, env, key, &out))
        return SPT_OK;
    if (log && log_bytes) {
        std::strncpy(log, out.c_str(), log_bytes - 1);
        log[log_bytes - 1] = 0;
    }
    return SPT_ERR_HIP;
}

int spt_set_tuning(spt_ctx* c, const spt_tuning* t) {
    if (!c || !t) return SPT_ERR_INVALID;
    if (t->fused < -1 || t->fused > 1 || t->persistent < -1 || t->persistent > 1 || t->frame_kernel < -1 ||
        t->frame_kernel > 1)
        return fail(c, SPT_ERR_INVALID, "spt_tuning: fused / persistent / frame_kernel must be -1, 0 or 1");
    if (t->px_shift && (t->px_shift < 2 || t->px_shift > 5)) return fail(c, SPT_ERR_INVALID, "spt_tuning: px_shift 2..5");
    if (t->chunks_per_wave > 1024 || t->subqueues > 65536 || t->tail_bounce > kMaxBounces ||
        t->bvh_max_leaf > kBvhMaxLeaf || (t->bvh_bins && (t->bvh_bins < 2 || t->bvh_bins > 64)) ||
        t->specialize < -1 || t->specialize > 1)
        return fail(c, SPT_ERR_INVALID, "spt_tuning: value out of range");
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    const uint32_t n_sub = t->subqueues ? t->subqueues : c->cu_count * 12u;
    if (n_sub != c->n_sub) {  // the wavefront schedule's per-sub-queue counters: the new buffer first,
        // swapped in only once it exists (a failed allocation leaves the ctx as it was)
        uint32_t* counts = nullptr;
        const size_t bytes = sizeof(uint32_t) * 2 * (kMaxBounces + 1) * n_sub;
        SPT_HIP(c, hipMalloc(&counts, bytes));
        if (hipMemset(counts, 0, bytes) != hipSuccess) {
            (void)hipFree(counts);
            return fail(c, SPT_ERR_HIP, "spt_set_tuning: hipMemset of the sub-queue counters failed");
        }
        free_dev(c->counts);
        c->counts = counts;
        c->n_sub = n_sub;
    }
    c->fused_override = t->fused;
    c->tail_override = t->tail_bounce;
    c->persistent_override = t->persistent;
    c->frame_override = t->frame_kernel;
    c->chunks_per_wave = t->chunks_per_wave;
    c->px_shift = t->px_shift;
    c->bvh_max_leaf = t->bvh_max_leaf;
    c->bvh_bins = t->bvh_bins;
    c->specialize = t->specialize;
    return SPT_OK;
}

int spt_comm_available(void) { return rccl().ok ? SPT_OK : SPT_ERR_NO_DEVICE; }

int spt_comm_unique_id(uint8_t id[SPT_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == SPT_COMM_ID_BYTES, "RCCL unique id size");
    if (!id) return SPT_ERR_INVALID;
    if (!rccl().ok) return SPT_ERR_NO_DEVICE;
    ncclUniqueId u;
    if (rccl().get_unique_id(&u) != ncclSuccess) return SPT_ERR_HIP;
    std::memcpy(id, &u, sizeof(u));
    return SPT_OK;
}

int spt_comm_init(spt_ctx* c, const uint8_t id[SPT_COMM_ID_BYTES], int n_ranks, int rank) {
    if (!c || !id) return SPT_ERR_INVALID;
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(c, SPT_ERR_INVALID, "spt_comm_init: rank out of range");
    if (!rccl().ok) return fail(c, SPT_ERR_NO_DEVICE, rccl().err);
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    free_comm(c);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    SPT_NCCL(c, rccl().comm_init_rank(&c->comm, n_ranks, u, rank));
    c->comm_ranks = n_ranks;
    c->comm_rank = rank;
    return SPT_OK;
}

int spt_comm_destroy(spt_ctx* c) {
    if (!c) return SPT_ERR_INVALID;
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamSynchronize(c->stream));
    free_comm(c);
    return SPT_OK;
}

namespace {
// Checks shared by both gathers; rows_max / shard_elems: the padded shard's rows and floats.
int gather_check(spt_ctx* c, void* root_image, const char* what, uint32_t& rows_max, size_t& shard_elems) {
    if (!c->configured) return fail(c, SPT_ERR_NOT_CONFIGURED, "not configured");
    if (!c->comm) return fail(c, SPT_ERR_INVALID, std::string(what) + " before spt_comm_init");
    const uint32_t world = c->cfg.shard_count;
    if ((int)world != c->comm_ranks || (int)c->cfg.shard_rank != c->comm_rank)
        return fail(c, SPT_ERR_INVALID, std::string(what) + ": shard_rank / shard_count differ from the communicator's rank / size");
    if (c->comm_rank == 0 && !root_image) return fail(c, SPT_ERR_INVALID, std::string(what) + ": rank 0 needs an output image");
    SPT_HIP(c, hipSetDevice(c->device));
    rows_max = (c->cfg.height + world - 1) / world;
    shard_elems = (size_t)rows_max * c->cfg.width * 4;
    return SPT_OK;
}

// gather_buf of `need` floats, its padding rows zeroed once (every copy into it writes the same rows)
int gather_buffer(spt_ctx* c, size_t need) {
    if (c->gather_elems == need) return SPT_OK;
    if (c->gather_pending) SPT_HIP(c, hipStreamWaitEvent(c->stream, c->gather_done, 0));
    SPT_HIP(c, hipStreamSynchronize(c->stream));  // (an earlier gather may still read the old buffer)
    free_dev(c->gather_buf);
    if (need) {
        SPT_HIP(c, hipMalloc(&c->gather_buf, sizeof(float) * need));
        SPT_HIP(c, hipMemsetAsync(c->gather_buf, 0, sizeof(float) * need, c->stream));
    }
    c->gather_elems = need;
    return SPT_OK;
}
}  // namespace

int spt_gather_image(spt_ctx* c, void* root_image) {
    if (!c) return SPT_ERR_INVALID;
    uint32_t rows_max = 0;
    size_t shard_elems = 0;
    int st = gather_check(c, root_image, "spt_gather_image", rows_max, shard_elems);
    if (st != SPT_OK) return st;
    // rank 0 receives world padded shards; a rank owning fewer than rows_max rows sends from a
    // zero-padded copy of its shard, the others straight from the accumulation buffer
    const bool root = c->comm_rank == 0;
    const bool padded = c->rows < rows_max;
    st = gather_buffer(c, root ? shard_elems * c->cfg.shard_count : (padded ? shard_elems : 0));
    if (st != SPT_OK) return st;
    if (c->gather_pending) SPT_HIP(c, hipStreamWaitEvent(c->stream, c->gather_done, 0));  // gather_buf is free
    const float4* send = c->accum;
    if (padded && !root) {
        if (c->pixels)
            SPT_HIP(c, hipMemcpyAsync(c->gather_buf, c->accum, sizeof(float4) * c->pixels, hipMemcpyDeviceToDevice, c->stream));
        send = c->gather_buf;
    }
    // one ncclGather for any world size (a 1-rank communicator copies: the single-GPU test runs the
    // same collective call the N-GPU run does)
    SPT_NCCL(c, rccl().gather(send, root ? c->gather_buf : nullptr, shard_elems, ncclFloat32, 0, c->comm, c->stream));
    if (root) {
        launch_assemble_rows(c->gather_buf, (float4*)root_image, c->cfg.width, c->cfg.height, c->cfg.shard_count,
                             rows_max, c->stream);
        SPT_HIP(c, hipGetLastError());
    }
    return SPT_OK;
}

int spt_gather_image_overlapped(spt_ctx* c, void* root_image) {
    if (!c) return SPT_ERR_INVALID;
    uint32_t rows_max = 0;
    size_t shard_elems = 0;
    int st = gather_check(c, root_image, "spt_gather_image_overlapped", rows_max, shard_elems);
    if (st != SPT_OK) return st;
    const bool root = c->comm_rank == 0;
    st = gather_buffer(c, root ? shard_elems * c->cfg.shard_count : shard_elems);  // every rank sends a snapshot
    if (st != SPT_OK) return st;
    if (!c->comm_stream) {
        SPT_HIP(c, hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
        SPT_HIP(c, hipEventCreateWithFlags(&c->snap_ready, hipEventDisableTiming));
        SPT_HIP(c, hipEventCreateWithFlags(&c->gather_done, hipEventDisableTiming));
    }
    // the snapshot, on the ctx stream after the frames rendered so far: rank 0's own shard goes to its
    // slot of the receive buffer (an in-place gather), the others' to their send buffer. The previous
    // overlapped gather must have finished reading that buffer first.
    if (c->gather_pending) SPT_HIP(c, hipStreamWaitEvent(c->stream, c->gather_done, 0));
    if (c->pixels)
        SPT_HIP(c, hipMemcpyAsync(c->gather_buf, c->accum, sizeof(float4) * c->pixels, hipMemcpyDeviceToDevice, c->stream));
    SPT_HIP(c, hipEventRecord(c->snap_ready, c->stream));
    // the collective and the assembly on the comm stream: the ctx stream renders on meanwhile
    SPT_HIP(c, hipStreamWaitEvent(c->comm_stream, c->snap_ready, 0));
    SPT_NCCL(c, rccl().gather(c->gather_buf, root ? c->gather_buf : nullptr, shard_elems, ncclFloat32, 0, c->comm,
                              c->comm_stream));
    if (root) {
        launch_assemble_rows(c->gather_buf, (float4*)root_image, c->cfg.width, c->cfg.height, c->cfg.shard_count,
                             rows_max, c->comm_stream);
        SPT_HIP(c, hipGetLastError());
    }
    SPT_HIP(c, hipEventRecord(c->gather_done, c->comm_stream));
    c->gather_pending = true;
    return SPT_OK;
}

int spt_gather_wait(spt_ctx* c) {
    if (!c) return SPT_ERR_INVALID;
    if (!c->gather_pending) return SPT_OK;
    SPT_HIP(c, hipSetDevice(c->device));
    SPT_HIP(c, hipStreamWaitEvent(c->stream, c->gather_done, 0));
    c->gather_pending = false;
    return SPT_OK;
}

}  // extern "C"
