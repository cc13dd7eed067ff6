"""GPU parity: the HIP wavefront integrator (through the C-ABI) vs the CPU oracle.

The bar: per-pixel L2 of the averaged radiance < 1e-4 RMS; in practice the two
agree bit for bit except where the device fp64 cos/sin differ from glibc's by an ulp that survives
the cast to float (rare), so the tests also require >= 99.9 % of pixels bit-identical.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4          # per-pixel L2 RMS bound on averaged radiance (north_star)
EXACT_FRAC = 0.999      # fraction of pixels whose float RGBA accumulation must be bit-identical


def parity(gpu_acc: np.ndarray, ref_acc: np.ndarray, frames: int):
    g = gpu_acc.reshape(-1, 4)
    r = ref_acc.reshape(-1, 4)
    exact = np.all(g.view(np.uint32) == r.view(np.uint32), axis=1)
    l2 = np.sqrt(np.sum(((g[:, :3].astype(np.float64) - r[:, :3]) / frames) ** 2, axis=1))
    return exact.mean(), float(np.sqrt(np.mean(l2 ** 2))) if l2.size else 0.0, float(l2.max()) if l2.size else 0.0


def render_both(spt, ref, ctx, scene, w, h, frames, bounces=4, rr=2, flags=0, fif=0, first=0):
    prims, mats, env = spt.build_scene(scene) if isinstance(scene, str) else scene
    ctx.set_scene(prims, mats, env)
    ctx.configure(w, h, bounces, rr, flags, 0, 1, fif)
    ctx.render(first, frames)
    g = ctx.read_accum().reshape(h, w, 4)
    r = ref.RefScene(prims, mats, env).render(w, h, first, frames, bounces, rr, flags, threads=0)
    return g, r


def assert_parity(g, r, frames):
    frac, rms, mx = parity(g, r, frames)
    assert rms < RMS_TOL, (frac, rms, mx)
    assert frac >= EXACT_FRAC, (frac, rms, mx)
    return frac, rms, mx


def test_c1_reference_config(spt, ref, gpu_ctx):
    """C1: sphere + ground (App.cpp:101-111), 256x256, 1 spp, 4 bounces, reference mode."""
    g, r = render_both(spt, ref, gpu_ctx, "c1", 256, 256, 1)
    assert_parity(g, r, 1)
    assert np.all(g[..., 3] == 1.0)


def test_c1_progressive_16(spt, ref, gpu_ctx):
    g, r = render_both(spt, ref, gpu_ctx, "c1", 256, 256, 16)
    assert_parity(g, r, 16)


def test_app_default_scene(spt, ref, gpu_ctx):
    g, r = render_both(spt, ref, gpu_ctx, "app", 320, 200, 8)
    assert_parity(g, r, 8)


@pytest.mark.parametrize("frames", [2, 5])  # k_frame (its LDS-only kernel for a scene this small) / k_paths
def test_small_mixed_bvh_scene(spt, ref, gpu_ctx, frames):
    """A 46-primitive BVH scene of quads, triangles and spheres (the Cornell walls and 30 triangles of
    the C4 mesh, 10 of the App's spheres): every primitive kind through the small-scene traversal."""
    b, bm, be = spt.build_scene("bunnylike")
    a, _, _ = spt.build_scene("app")
    spheres = a[:10].copy()
    spheres["material"] = 1
    prims = np.concatenate([b[:36], spheres])
    g, r = render_both(spt, ref, gpu_ctx, (prims, bm, be), 128, 96, frames, bounces=8)
    assert_parity(g, r, frames)


def test_cornell_full_res_8_bounces(spt, ref, gpu_ctx):
    """C2 geometry at the C2 resolution, 8 bounces, 2 frames (the oracle's share of the bench)."""
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 1920, 1080, 2, bounces=8)
    assert_parity(g, r, 2)


def test_abs_float_flag(spt, ref, gpu_ctx):
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 256, 144, 4, bounces=8, flags=spt.FLAG_ABS_FLOAT)
    assert_parity(g, r, 4)


def test_frames_in_flight_invariance(spt, gpu_ctx):
    """The pass size only changes scheduling: accumulations must be bit-identical."""
    prims, mats, env = spt.build_scene("cornell")
    out = []
    for fif in (1, 3, 0):
        gpu_ctx.set_scene(prims, mats, env)
        gpu_ctx.configure(200, 120, 8, 2, 0, 0, 1, fif)
        gpu_ctx.render(0, 7)
        out.append(gpu_ctx.read_accum())
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))
    assert np.array_equal(out[0].view(np.uint32), out[2].view(np.uint32))


def test_progressive_calls_equal_one_call(spt, gpu_ctx):
    prims, mats, env = spt.build_scene("cornell")
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(160, 90, 8, 2, 0, 0, 1, 0)
    gpu_ctx.render(0, 6)
    a = gpu_ctx.read_accum()
    gpu_ctx.reset()
    for f in range(6):
        gpu_ctx.render(f, 1)
    b = gpu_ctx.read_accum()
    assert gpu_ctx.frame_count == 6
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_row_shards_reassemble(spt, gpu_ctx):
    """Multi-GPU decomposition on one GPU: 3 row shards == the full image, bit for bit."""
    w, h, frames, world = 97, 61, 3, 3
    prims, mats, env = spt.build_scene("cornell")
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 8, 2, 0, 0, 1, 0)
    gpu_ctx.render(0, frames)
    full = gpu_ctx.read_accum().reshape(h, w, 4)
    for rank in range(world):
        gpu_ctx.configure(w, h, 8, 2, 0, rank, world, 0)
        gpu_ctx.render(0, frames)
        part = gpu_ctx.read_accum().reshape(-1, w, 4)
        assert np.array_equal(part.view(np.uint32), full[rank::world].view(np.uint32))


def test_resolve_rgba8_matches_reference_resolve(spt, ref, gpu_ctx):
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 128, 72, 5, bounces=8)
    px_gpu = gpu_ctx.resolve_rgba8(5)
    px_ref_of_gpu = ref.resolve_rgba8(g, 5)
    assert np.array_equal(px_gpu, px_ref_of_gpu)


@pytest.mark.parametrize("exposure", [1.0, 0.25, 1.7, 40.0])
def test_resolve_exposure_matches_oracle(spt, ref, gpu_ctx, exposure):
    """spt_resolve_rgba8_exposure (RenderSettings exposure, CPUPathTracer.cpp:101-104) vs the
    oracle's resolve of the same accumulation; exposure 1 equals the plain resolve."""
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 128, 72, 5, bounces=8)
    px = gpu_ctx.resolve_rgba8(5, exposure)
    assert np.array_equal(px, ref.resolve_rgba8(g, 5, exposure))
    if exposure == 1.0:
        assert np.array_equal(px, gpu_ctx.resolve_rgba8(5))


@pytest.mark.parametrize("progressive", [True, False])
def test_python_pathtracer_settings_mode(spt, ref, progressive):
    """settings_mode=True honours RenderSettings: bounces, RR depth, samples
    per render() call, progressive flag, exposure — vs the oracle."""
    tracer = spt.HIPPathTracer(settings_mode=True)
    scene = spt.Scene()
    s = scene.CreateNode(spt.SphereObject, "123"); s.SetRadius(1.0); s.SetPosition((0.0, -1.0, 5.0))
    s = scene.CreateNode(spt.SphereObject, "123"); s.SetRadius(100.0); s.SetPosition((0.0, -102.0, 5.0))
    settings = spt.RenderSettings()
    settings.setResolution(120, 80)
    settings.setSamplesPerPixel(6)
    settings.setMaxBounces(5)
    settings.setRussianRouletteDepth(1)
    settings.setExposure(1.5)
    settings.setProgressive(progressive)
    tracer.set_settings(settings)
    tracer.set_scene(scene)
    for _ in range(2):
        tracer.render()
    res = tracer.get_render_result()
    frames = 12 if progressive else 6
    prims = spt.sphere_prims([(0, -1, 5, 1), (0, -102, 5, 100)])
    r = ref.RefScene(prims, spt.reference_materials(), spt.reference_env()).render(120, 80, 0, frames, 5, 1)
    g = tracer.read_accumulation()
    assert_parity(g, r, frames)
    assert np.mean(res.image_buffer == ref.resolve_rgba8(r, frames, 1.5)) >= EXACT_FRAC


@pytest.mark.parametrize("frames", [3, 5])  # wavefront / persistent schedule
@pytest.mark.parametrize("w,h", [(1, 1), (1, 7), (7, 1), (65, 3)])
def test_ragged_sizes(spt, ref, gpu_ctx, w, h, frames):
    g, r = render_both(spt, ref, gpu_ctx, "cornell", w, h, frames, bounces=8)
    assert_parity(g, r, frames)


@pytest.mark.parametrize("frames", [2, 4])  # wavefront / persistent schedule
@pytest.mark.parametrize("bounces", [0, 1, 2, 3, 32])
def test_bounce_limits(spt, ref, gpu_ctx, bounces, frames):
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 96, 54, frames, bounces=bounces)
    assert_parity(g, r, frames)


def test_empty_scene_sky_only(spt, ref, gpu_ctx):
    prims = np.zeros(0, dtype=spt.PRIM_DTYPE)
    g, r = render_both(spt, ref, gpu_ctx, (prims, spt.reference_materials(), spt.reference_env(True)), 64, 48, 1)
    assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


def test_sky_off_is_black_without_emitters(spt, ref, gpu_ctx):
    prims, mats, _ = spt.build_scene("c1")
    g, r = render_both(spt, ref, gpu_ctx, (prims, mats, spt.reference_env(False)), 64, 64, 2)
    assert np.all(g[..., :3] == 0.0) and np.array_equal(g.view(np.uint32), r.view(np.uint32))


@pytest.mark.parametrize("frames", [2, 4])  # split wavefront / persistent schedule
def test_bvh_scene_bunnylike(spt, ref, gpu_ctx, frames):
    """C4 geometry (81,926 primitives, BVH on the GPU, independent BVH in the oracle)."""
    g, r = render_both(spt, ref, gpu_ctx, "bunnylike", 240, 135, frames, bounces=8)
    assert_parity(g, r, frames)


@pytest.mark.parametrize("frames", [1, 4])  # split wavefront / persistent schedule
def test_bvh_scene_interior_1m(spt, ref, gpu_ctx, frames):
    """C5 geometry (1,000,000 triangles), small resolution."""
    g, r = render_both(spt, ref, gpu_ctx, "interior1m", 160, 90, frames, bounces=8)
    assert_parity(g, r, frames)


def test_errors_fail_loudly(spt):
    ctx = spt.Context(0)
    with pytest.raises(spt.SptError, match="NOT_CONFIGURED|NO_SCENE"):
        ctx.render(0, 1)
    ctx.configure(8, 8)
    with pytest.raises(spt.SptError, match="NO_SCENE"):
        ctx.render(0, 1)
    with pytest.raises(spt.SptError, match="INVALID"):
        ctx.configure(0, 8)
    prims, mats, env = spt.build_scene("c1")
    bad = prims.copy()
    bad[0]["material"] = 5
    with pytest.raises(spt.SptError, match="INVALID"):
        ctx.set_scene(bad, mats, env)
    ctx.set_scene(prims, mats, env)
    with pytest.raises(spt.SptError, match="INVALID"):
        ctx.resolve_rgba8(0)
    ctx.close()


def test_python_pathtracer_mirror(spt, ref):
    """The reference interface mirror (App.cpp:98-133, :230-240) on the GPU_HIP backend."""
    tracer = spt.PathTracer.create_path_tracer(spt.BackendType.GPU_HIP)
    scene = spt.Scene()
    s = scene.CreateNode(spt.SphereObject, "123"); s.SetRadius(1.0); s.SetPosition((0.0, -1.0, 5.0))
    s = scene.CreateNode(spt.SphereObject, "123"); s.SetRadius(100.0); s.SetPosition((0.0, -102.0, 5.0))
    settings = spt.RenderSettings()
    settings.setResolution(128, 96)
    tracer.set_settings(settings)
    tracer.set_scene(scene)
    for _ in range(3):
        tracer.render()
        res = tracer.get_render_result()
    assert (res.width, res.height) == (128, 96)
    prims = spt.sphere_prims([(0, -1, 5, 1), (0, -102, 5, 100)])
    r = ref.RefScene(prims, spt.reference_materials(), spt.reference_env()).render(128, 96, 0, 3)
    assert np.mean(res.image_buffer == ref.resolve_rgba8(r, 3)) >= EXACT_FRAC
    with pytest.raises(RuntimeError, match="Unknown backend type"):
        spt.PathTracer.create_path_tracer(spt.BackendType.CPU_EMBREE)


@pytest.mark.parametrize("scene,w,h,bounces", [("cornell", 320, 180, 8), ("c1", 128, 128, 4),
                                               ("bunnylike", 160, 90, 8)])
def test_split_and_fused_schedules_agree(spt, scene, w, h, bounces):
    """Fused bounce kernel + tail kernel vs split extend/shade launches: bit-identical images
    (forced with spt_set_tuning's fused / tail_bounce, whatever the automatic schedule)."""
    prims, mats, env = spt.build_scene(scene)
    out = []
    for fused, tail in (("1", "3"), ("0", "32"), ("1", "32"), ("0", "2")):
        with spt.Context(0) as ctx:
            ctx.set_tuning(fused=int(fused), tail_bounce=int(tail), persistent=0, frame_kernel=0)
            ctx.set_scene(prims, mats, env)
            ctx.configure(w, h, bounces, 2, 0, 0, 1, 0)
            ctx.render(0, 3)
            out.append(ctx.read_accum())
            st = ctx.stats()
            assert bool(st.fused) == (fused == "1") and st.tail_bounce == int(tail)
    for o in out[1:]:
        assert np.array_equal(out[0].view(np.uint32), o.view(np.uint32))


def test_automatic_schedule(spt, gpu_ctx):
    """Flat scenes: fused + tail from bounce 3; BVH scenes: split, no tail."""
    for scene, fused, tail in (("cornell", 1, 3), ("bunnylike", 0, 32), ("app", 0, 32)):
        prims, mats, env = spt.build_scene(scene)
        gpu_ctx.set_scene(prims, mats, env)
        gpu_ctx.configure(64, 36, 8, 2, 0, 0, 1, 0)
        st = gpu_ctx.stats()
        assert st.fused == fused and st.tail_bounce == tail
        # calls of >= PERSISTENT_MIN_FRAMES frames run the persistent k_paths launch
        gpu_ctx.render(0, spt.PERSISTENT_MIN_FRAMES)
        assert gpu_ctx.stats().schedule == spt.SCHEDULE_PERSISTENT
        # fewer frames: one k_frame launch per frame
        gpu_ctx.render(0, spt.PERSISTENT_MIN_FRAMES - 1)
        assert gpu_ctx.stats().schedule == spt.SCHEDULE_FRAME
        gpu_ctx.configure(64, 36, 8, 2, spt.FLAG_WAVEFRONT, 0, 1, 0)
        gpu_ctx.render(0, 1)
        assert gpu_ctx.stats().schedule == (spt.SCHEDULE_FUSED if fused else spt.SCHEDULE_SPLIT)
    gpu_ctx.configure(64, 36, 8, 2, spt.FLAG_SPLIT_KERNELS, 0, 1, 0)
    assert gpu_ctx.stats().fused == 0


def test_split_schedule_parity(spt, ref, gpu_ctx):
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 480, 270, 4, bounces=8, flags=spt.FLAG_SPLIT_KERNELS)
    assert_parity(g, r, 4)


def test_persistent_cornell_full_res(spt, ref, gpu_ctx):
    """C2 at full resolution on the persistent schedule (k_paths), 4 frames vs the oracle."""
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 1920, 1080, 4, bounces=8, first=11)
    assert gpu_ctx.stats().schedule == spt.SCHEDULE_PERSISTENT
    assert_parity(g, r, 4)


@pytest.mark.parametrize("scene,w,h,bounces,frames,first,rank,world", [
    ("cornell", 320, 180, 8, 8, 0, 0, 1),
    ("cornell", 67, 33, 1, 9, 5, 0, 1),
    ("cornell", 64, 16, 32, 4, 0, 0, 1),
    ("cornell", 97, 61, 8, 1100, 0, 1, 3),  # > 1024 frames: two launches; a row shard
    ("c1", 97, 61, 4, 5, 2, 0, 1),
    ("cornell", 128, 72, 8, 6, 0, 0, 1),
    ("empty", 40, 30, 4, 4, 0, 0, 1),
    ("bunnylike", 96, 54, 8, 5, 3, 0, 1),    # BVH scenes: persistent vs split
    ("app", 128, 72, 4, 6, 0, 1, 2),
    ("interior1m", 64, 36, 8, 4, 0, 0, 1),
])
def test_persistent_matches_wavefront(spt, scene, w, h, bounces, frames, first, rank, world):
    """Persistent k_paths schedule vs the wavefront schedule: bit-identical accumulations and the
    same segment counts per bounce."""
    if scene == "empty":
        prims, mats, env = np.zeros(0, dtype=spt.PRIM_DTYPE), spt.reference_materials(), spt.reference_env(True)
    else:
        prims, mats, env = spt.build_scene(scene)
    out, segs = [], []
    wave_sched = spt.SCHEDULE_FUSED if len(prims) <= 32 else spt.SCHEDULE_SPLIT
    for flags, sched in ((0, spt.SCHEDULE_PERSISTENT), (spt.FLAG_WAVEFRONT, wave_sched)):
        with spt.Context(0) as ctx:
            ctx.set_scene(prims, mats, env)
            ctx.configure(w, h, bounces, 2, flags, rank, world, 0)
            ctx.set_profiling(False, counters=True)
            ctx.render(first, frames)
            out.append(ctx.read_accum())
            st = ctx.stats()
            assert st.schedule == sched
            segs.append((list(st.segments), list(st.radiance_updates)[1:]))
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))
    assert segs[0] == segs[1]


@pytest.mark.parametrize("scene,w,h,bounces,frames,first,rank,world", [
    ("cornell", 320, 180, 8, 1, 0, 0, 1),
    ("cornell", 67, 33, 1, 3, 5, 0, 1),
    ("cornell", 64, 16, 32, 2, 0, 0, 1),
    ("cornell", 97, 61, 8, 3, 2**32 - 2, 1, 3),  # frame index wraps; a row shard
    ("c1", 97, 61, 4, 1, 2, 0, 1),
    ("empty", 40, 30, 4, 2, 0, 0, 1),
    ("cornell", 7, 3, 8, 3, 0, 0, 1),            # fewer pixels than one run of 64
    ("bunnylike", 96, 54, 8, 2, 3, 0, 1),
    ("app", 128, 72, 4, 3, 0, 1, 2),
    ("interior1m", 64, 36, 8, 1, 0, 0, 1),
])
def test_frame_matches_wavefront(spt, scene, w, h, bounces, frames, first, rank, world):
    """k_frame (calls of < 4 frames, one launch per frame) vs the wavefront schedule: bit-identical
    accumulations and the same segment counts per bounce."""
    if scene == "empty":
        prims, mats, env = np.zeros(0, dtype=spt.PRIM_DTYPE), spt.reference_materials(), spt.reference_env(True)
    else:
        prims, mats, env = spt.build_scene(scene)
    out, segs = [], []
    wave_sched = spt.SCHEDULE_FUSED if len(prims) <= 32 else spt.SCHEDULE_SPLIT
    for flags, sched in ((0, spt.SCHEDULE_FRAME), (spt.FLAG_WAVEFRONT, wave_sched)):
        with spt.Context(0) as ctx:
            ctx.set_scene(prims, mats, env)
            ctx.configure(w, h, bounces, 2, flags, rank, world, 0)
            ctx.set_profiling(False, counters=True)
            ctx.render(first, frames)
            out.append(ctx.read_accum())
            st = ctx.stats()
            assert st.schedule == sched
            segs.append((list(st.segments), list(st.radiance_updates)[1:]))
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))
    assert segs[0] == segs[1]


@pytest.mark.parametrize("scene", ["cornell", "bunnylike"])
def test_frame_calls_match_one_persistent_call(spt, scene):
    """The App's pattern — one frame per call, 9 calls — accumulates the same bits as one call of
    9 frames on the k_paths schedule."""
    prims, mats, env = spt.build_scene(scene)
    out = []
    for per_call in (1, 9):
        with spt.Context(0) as ctx:
            ctx.set_scene(prims, mats, env)
            ctx.configure(150, 85, 8, 2, 0, 0, 1, 0)
            for f in range(0, 9, per_call):
                ctx.render(f, per_call)
            assert ctx.stats().schedule == (spt.SCHEDULE_FRAME if per_call == 1 else spt.SCHEDULE_PERSISTENT)
            out.append(ctx.read_accum())
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))


@pytest.mark.parametrize("w,h", [(512, 512), (1024, 640)])
def test_app_scene_frame_calls_with_and_without_lists(spt, w, h):
    """The App's LDS-held scene one frame per call: at 512² without the live-pixel lists, at 1024x640
    (more runs than resident waves) with them (frame_small_scene_lists) — 4 calls give the bits of one
    4-frame k_paths call either way."""
    prims, mats, env = spt.build_scene("app")
    out = []
    for per_call in (1, 4):
        with spt.Context(0) as ctx:
            ctx.set_scene(prims, mats, env)
            ctx.configure(w, h, 4, 2, 0, 0, 1, 0)
            for f in range(0, 4, per_call):
                ctx.render(f, per_call)
            out.append(ctx.read_accum())
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))


def test_persistent_counters_do_not_change_results(spt, gpu_ctx):
    """The counting k_paths variant (SPT_PROFILE_COUNTERS) renders the same bits as the lean one."""
    prims, mats, env = spt.build_scene("cornell")
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(160, 90, 8, 2, 0, 0, 1, 0)
    out = []
    for frames in (8, 2):  # k_paths, k_frame
        out = []
        for counters in (False, True):
            gpu_ctx.reset()
            gpu_ctx.clear_stats()
            gpu_ctx.set_profiling(False, counters=counters)
            gpu_ctx.render(0, frames)
            out.append(gpu_ctx.read_accum())
            st = gpu_ctx.stats()
            assert (st.segments_total > 0) == counters
            if counters:
                assert st.segments[0] == frames * 160 * 90 and 0 < st.lane_busy <= st.lane_slots
        gpu_ctx.set_profiling(False)
        assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))


@pytest.mark.parametrize("scene", ["cornell", "app"])
def test_span_profiling_counts_every_launch(spt, gpu_ctx, scene):
    """SPT_PROFILE_SPAN: one event pair around all the persistent launches (the bench's timing of
    one-frame calls) counts every launch, times a positive span, and changes no result."""
    prims, mats, env = spt.build_scene(scene)
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(96, 64, 4, 2, 0, 0, 1, 0)
    out = []
    for span in (False, True):
        gpu_ctx.reset()
        gpu_ctx.clear_stats()
        gpu_ctx.set_profiling(True, span=span)
        for f in range(5):
            gpu_ctx.render(f, 1)  # one-frame calls: k_frame
        gpu_ctx.set_profiling(False)  # closes the span
        st = gpu_ctx.stats()
        assert st.schedule == spt.SCHEDULE_FRAME
        assert st.persistent_launches == 5 and st.persistent_ms > 0.0
        out.append(gpu_ctx.read_accum())
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))


@pytest.mark.parametrize("scene,w,h", [("cornell", 133, 41), ("bunnylike", 80, 45)])
def test_persistent_chunk_sizes_agree(spt, scene, w, h):
    """k_paths with 4-, 8-, 16- and 32-pixel chunks (spt_set_tuning px_shift; the automatic choice
    depends on the shard size) renders the same bits; 133 px rows leave ragged last chunks."""
    prims, mats, env = spt.build_scene(scene)
    out = []
    for pxs in ("2", "3", "4", "5"):
        with spt.Context(0) as ctx:
            ctx.set_tuning(px_shift=int(pxs))
            ctx.set_scene(prims, mats, env)
            ctx.configure(w, h, 8, 2, 0, 0, 1, 0)
            ctx.render(2, 37)
            assert ctx.stats().schedule == spt.SCHEDULE_PERSISTENT
            out.append(ctx.read_accum())
    for o in out[1:]:
        assert np.array_equal(out[0].view(np.uint32), o.view(np.uint32))


@pytest.mark.parametrize("scene,w,h,nee", [("cornell", 320, 180, False), ("cornell", 133, 41, False),
                                            ("bunnylike", 96, 54, False), ("bunnylike", 320, 180, False),
                                            ("bunnylike", 160, 90, True), ("cornell", 200, 120, True)])
def test_chunk_order_changes_no_bits(spt, scene, w, h, nee):
    """The flat k_paths records its chunks' costs in one launch and hands them out longest first in
    the launches after it (launch_paths, k_chunk_order): calls of 8 frames (ordered from the second),
    one call of 24 (recording only), a forced chunk size (no order) switched back mid-way, and a scene
    change (the order cleared) all give the same bits, with NEE too. BVH scenes: in cost order too since
    round 6 (with NEE they keep the pixel order): same check."""
    prims, mats, env = spt.build_scene(scene)
    other = spt.build_scene("app")

    def run(calls, tuning_per_call=None, detour=False):
        with spt.Context(0) as ctx:
            ctx.set_scene(prims, mats, env)
            ctx.configure(w, h, 8, 2, spt.FLAG_NEE if nee else 0, 0, 1, 0)
            if detour:  # another scene's order first, then back (set_scene clears it)
                ctx.set_scene(*other)
                ctx.render(0, 8)
                ctx.render(8, 8)
                ctx.set_scene(prims, mats, env)
                ctx.reset()
            f = 0
            for i, n in enumerate(calls):
                if tuning_per_call is not None:
                    ctx.set_tuning(px_shift=tuning_per_call[i])
                ctx.render(f, n)
                assert ctx.stats().schedule == spt.SCHEDULE_PERSISTENT
                f += n
            return ctx.read_accum()

    ref = run([24])
    for acc in (run([8, 8, 8]), run([8, 8, 8], tuning_per_call=[3, 0, 0]), run([8, 8, 8], detour=True)):
        assert np.array_equal(ref.view(np.uint32), acc.view(np.uint32))


@pytest.mark.parametrize("frames", [2, 6])  # wavefront / persistent schedule
@pytest.mark.parametrize("rr", [0, 1, 5])
def test_rr_depths(spt, ref, gpu_ctx, rr, frames):
    """Russian roulette from bounce_count > rr (rr = 0: already after bounce 0, which k_paths runs
    from the cached primary state; rr = 5: late)."""
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 120, 68, frames, bounces=8, rr=rr)
    assert_parity(g, r, frames)


def mixed_flat_scene(spt, n_prims):
    """A flat (or just-BVH) scene with all three primitive types and emitters: a box of quads,
    a triangle fan and spheres, n_prims in total, several materials."""
    prims = np.zeros(n_prims, dtype=spt.PRIM_DTYPE)
    mats = np.zeros(5, dtype=spt.MATERIAL_DTYPE)
    mats["albedo"] = [(0.8, 0.8, 0.8), (0.7, 0.2, 0.2), (0.2, 0.7, 0.2), (0.9, 0.9, 0.5), (0.5, 0.5, 0.9)]
    mats["emission"][3] = (6.0, 5.0, 4.0)
    rng = np.random.default_rng(7)
    quads = [((-3, -2, 2), (6, 0, 0), (0, 0, 8)), ((-3, 3, 2), (0, 0, 8), (6, 0, 0)),
             ((-3, -2, 10), (6, 0, 0), (0, 5, 0)), ((-3, -2, 2), (0, 0, 8), (0, 5, 0)),
             ((3, -2, 2), (0, 5, 0), (0, 0, 8)), ((-0.5, 2.99, 5), (1, 0, 0), (0, 0, 1))]
    for i in range(n_prims):
        p = prims[i]
        if i < len(quads):
            q, u, v = quads[i]
            p["type"], p["material"] = spt.PRIM_QUAD, (3 if i == 5 else i % 3)
            p["p0"][:3], p["p1"][:3], p["p2"][:3] = q, u, v
        elif i % 2 == 0:
            c = rng.uniform((-2, -1.5, 4), (2, 1.5, 9))
            p["type"], p["material"] = spt.PRIM_TRIANGLE, 4
            p["p0"][:3], p["p1"][:3], p["p2"][:3] = c, c + rng.uniform(-0.6, 0.6, 3), c + rng.uniform(-0.6, 0.6, 3)
        else:
            p["type"], p["material"] = spt.PRIM_SPHERE, i % 5
            p["p0"] = (*rng.uniform((-2, -1.5, 4), (2, 1.5, 9)), rng.uniform(0.1, 0.4))
    env = spt.reference_env(True)
    return prims, mats, env


@pytest.mark.parametrize("frames", [2, 5])
@pytest.mark.parametrize("n_prims", [13, 32, 33])  # flat, largest flat, smallest BVH scene
def test_mixed_primitive_scenes(spt, ref, gpu_ctx, n_prims, frames):
    g, r = render_both(spt, ref, gpu_ctx, mixed_flat_scene(spt, n_prims), 160, 90, frames, bounces=6)
    assert_parity(g, r, frames)


def test_frame_index_wraps_like_the_reference(spt, ref, gpu_ctx):
    """Seeds are x + y*W + (frame+1)*982451653 mod 2^32 (CPUPathTracer.cpp:192-195): frame indices
    near 2^32 wrap identically on both sides (persistent schedule)."""
    g, r = render_both(spt, ref, gpu_ctx, "cornell", 64, 40, 6, bounces=8, first=2**32 - 3)
    assert_parity(g, r, 6)


@pytest.mark.parametrize("frames", [2, 5])  # k_frame (1-3 frames per call) / k_paths
@pytest.mark.parametrize("scene,w,h", [("cornell", 200, 112), ("c1", 128, 96), ("bunnylike", 96, 54),
                                       ("app", 96, 64)])  # app: k_frame's LDS-only small-scene kernel
def test_environment_map(spt, ref, gpu_ctx, scene, w, h, frames):
    """Miss radiance from an octahedral environment map vs the oracle."""
    prims, mats, env = spt.build_scene(scene)
    emap = spt.synthetic_env_map(128)
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 8, 2, 0, 0, 1, 0)
    gpu_ctx.set_env_map(emap)
    gpu_ctx.render(0, frames)
    g = gpu_ctx.read_accum().reshape(h, w, 4)
    gpu_ctx.set_env_map(None)
    rs = ref.RefScene(prims, mats, env)
    rs.set_env_map(emap)
    r = rs.render(w, h, 0, frames, 8, 2, 0, threads=0)
    assert_parity(g, r, frames)
    # and the map really changed the image
    rs.set_env_map(None)
    assert not np.array_equal(r, rs.render(w, h, 0, frames, 8, 2, 0, threads=0))


def scaled_scene(spt, name, s):
    """A flat scene with every coordinate (positions, edge vectors, radii) multiplied by s."""
    prims, mats, env = spt.build_scene(name)
    prims = prims.copy()
    for i in range(len(prims)):
        p = prims[i]
        if p["type"] == spt.PRIM_SPHERE:
            p["p0"] = p["p0"] * s
        else:
            for f in ("p0", "p1", "p2"):
                p[f][:3] = p[f][:3] * s
    return prims, mats, env


def coincident_flat_scene(spt):
    """A flat scene of exact and near ties across primitive kinds, each pair in the order the fast
    path's kind-major copy reverses: a triangle before the coplanar axis quad it halves, duplicate
    back walls and spheres with different materials, the two triangles of a slanted quad before the
    quad, and the emitter as a quad after its triangle copy."""
    Q, T, S = spt.PRIM_QUAD, spt.PRIM_TRIANGLE, spt.PRIM_SPHERE
    recs = [
        (T, 1, (-3, -2, 10), (3, -2, 10), (-3, 3, 10)),    # half of the back wall, red
        (Q, 2, (-3, -2, 10), (6, 0, 0), (0, 5, 0)),        # back wall, green
        (Q, 4, (-3, -2, 10), (6, 0, 0), (0, 5, 0)),        # the same wall again, blue
        (Q, 0, (-3, -2, 2), (6, 0, 0), (0, 0, 8)),         # floor
        (Q, 0, (-3, 3, 2), (0, 0, 8), (6, 0, 0)),          # ceiling
        (Q, 1, (-3, -2, 2), (0, 0, 8), (0, 5, 0)),         # left wall
        (Q, 2, (3, -2, 2), (0, 5, 0), (0, 0, 8)),          # right wall
        (S, 1, (-1.0, -1.2, 6.0, 0.8), None, None),        # sphere, red
        (S, 2, (-1.0, -1.2, 6.0, 0.8), None, None),        # the same sphere, green
        (T, 3, (-0.5, 2.99, 5), (0.5, 2.99, 5), (-0.5, 2.99, 6)),  # emitter half as a triangle
        (Q, 3, (-0.5, 2.99, 5), (1, 0, 0), (0, 0, 1)),     # the emitter quad
        (T, 4, (0.5, -2, 4), (2.5, -2, 4), (2.5, 0, 6)),   # slanted quad's two triangles ...
        (T, 1, (0.5, -2, 4), (2.5, 0, 6), (0.5, 0, 6)),
        (Q, 2, (0.5, -2, 4), (2, 0, 0), (0, 2, 2)),        # ... then the quad (general, not axis)
    ]
    prims = np.zeros(len(recs), dtype=spt.PRIM_DTYPE)
    for p, (ty, m, a, b, c) in zip(prims, recs):
        p["type"], p["material"] = ty, m
        if ty == S:
            p["p0"] = a
        else:
            p["p0"][:3], p["p1"][:3], p["p2"][:3] = a, b, c
    mats = np.zeros(5, dtype=spt.MATERIAL_DTYPE)
    mats["albedo"] = [(0.8, 0.8, 0.8), (0.7, 0.2, 0.2), (0.2, 0.7, 0.2), (0.9, 0.9, 0.5), (0.2, 0.2, 0.8)]
    mats["emission"][3] = (8.0, 7.0, 6.0)
    return prims, mats, spt.reference_env(True)


@pytest.mark.parametrize("frames", [1, 5])  # k_frame / k_paths
def test_flat_ties_across_kinds(spt, ref, gpu_ctx, frames):
    """The fast path tests the primitives kind by kind (scene.h sort_flat_by_kind) and resolves
    equal t on the original index; exact duplicates and coplanar pairs of different kinds, placed in
    the opposite order, give the oracle's lowest-index-wins image."""
    g, r = render_both(spt, ref, gpu_ctx, coincident_flat_scene(spt), 128, 72, frames, bounces=6)
    assert int(gpu_ctx.stats().flat_fast_path) == 1
    assert_parity(g, r, frames)


@pytest.mark.parametrize("frames", [1, 5])  # k_frame / k_paths
def test_flat_fast_path_boundaries(spt, ref, gpu_ctx, frames):
    """The flat loop's unscaled-division fast path covers the Cornell scene and a
    scene with a tiny (2^-11 x 2^-11) axis-aligned quad; the Cornell box scaled by 2^28 (past the
    coordinate bound) runs the general loop (spt_stats.flat_fast_path = 0). All match the oracle."""
    prims, mats, env = mixed_flat_scene(spt, 13)
    prims = prims.copy()
    prims[5]["p1"][:3] = (2.0 ** -11, 0.0, 0.0)  # u x v = (0, -2^-22, 0)
    prims[5]["p2"][:3] = (0.0, 0.0, 2.0 ** -11)
    cases = [("cornell", spt.build_scene("cornell"), 1),
             ("mixed", mixed_flat_scene(spt, 13), 1),
             ("cornell x 2^28", scaled_scene(spt, "cornell", 2.0 ** 28), 0),
             ("tiny axis quad", (prims, mats, env), 1)]
    for name, scene, fast in cases:
        g, r = render_both(spt, ref, gpu_ctx, scene, 96, 54, frames, bounces=8)
        assert int(gpu_ctx.stats().flat_fast_path) == fast, name
        assert_parity(g, r, frames)


@pytest.mark.parametrize("frames", [1, 6])  # k_frame / k_paths
@pytest.mark.parametrize("scene", ["cornell", "c1", "mixed13", "ties"])
def test_specialized_kernels_match_generic(spt, ref, gpu_ctx, scene, frames):
    """Flat scenes run k_paths / k_frame compiled at run time for their shape (spt_jit.hip,
    DESIGN.md §3.1c): spt_stats.specialized reports it, and the image is bit-identical to the
    generic kernel's (spt_tuning.specialize = -1) and to the oracle's."""
    sc = {"mixed13": lambda: mixed_flat_scene(spt, 13), "ties": lambda: coincident_flat_scene(spt)}.get(
        scene, lambda: spt.build_scene(scene))()
    w, h, b = 160, 90, 8
    gpu_ctx.set_tuning(specialize=1)  # compiled inside the first launch (the default compiles in the background)
    try:
        g, r = render_both(spt, ref, gpu_ctx, sc, w, h, frames, bounces=b)
    finally:
        gpu_ctx.set_tuning()
    assert int(gpu_ctx.stats().specialized) == 1, gpu_ctx.stats().schedule
    assert_parity(g, r, frames)
    try:
        gpu_ctx.set_tuning(specialize=-1)
        gpu_ctx.set_scene(*sc)
        gpu_ctx.configure(w, h, b, 2, 0, 0, 1, 0)
        gpu_ctx.render(0, frames)
        assert int(gpu_ctx.stats().specialized) == 0
        generic = gpu_ctx.read_accum().reshape(h, w, 4)
    finally:
        gpu_ctx.set_tuning()
    assert np.array_equal(g.view(np.uint32), generic.view(np.uint32))


def test_specialize_scene_precompiles(spt, gpu_ctx):
    """spt_specialize_scene loads the current flat scene's kernels ahead of the first frame; a BVH
    scene is a no-op; a moved sphere (same shape) re-uses the kernels and still matches the generic."""
    prims, mats, env = spt.build_scene("cornell")
    gpu_ctx.set_tuning()
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(96, 64, 8, 2, 0, 0, 1, 0)  # (the kernels are compiled for the configuration too)
    gpu_ctx.specialize_scene()
    moved = prims.copy()
    moved[-1]["p0"][:3] = (0.4, -1.2, 5.5)
    gpu_ctx.set_scene(moved, mats, env)
    gpu_ctx.render(0, 5)
    assert int(gpu_ctx.stats().specialized) == 1
    a = gpu_ctx.read_accum()
    gpu_ctx.set_tuning(specialize=-1)
    try:
        gpu_ctx.reset()
        gpu_ctx.render(0, 5)
        b = gpu_ctx.read_accum()
    finally:
        gpu_ctx.set_tuning()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    gpu_ctx.set_scene(*spt.build_scene("bunnylike"))
    gpu_ctx.specialize_scene()


def test_new_flat_shape_does_not_wait_for_the_compiler(spt, ref, gpu_ctx):
    """A flat scene of a shape never compiled in this process (the App adding a sphere): the first
    render() runs the generic kernel while hiprtc compiles the specialized one on a background thread
    (spt_set_scene starts it), so it does not wait for the compile and is bit-exact vs the oracle; once
    spt_specialize_scene has waited for the compile, the specialized kernel runs, with the same bits.
    Reference call pattern: App.cpp:230-240 (one render() per UI frame)."""
    import time

    prims, mats, env = spt.build_scene("app")  # 38 spheres: a BVH scene; keep 29 of them -> flat
    prims = prims[:29].copy()
    w, h = 256, 160
    gpu_ctx.set_tuning()
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 4, 2, 0, 0, 1, 1)
    gpu_ctx.render(0, 1)  # warm the generic kernel's code object load (not the compile)
    gpu_ctx.synchronize()
    extra = prims[:27].copy()  # a new shape: 27 spheres
    gpu_ctx.set_scene(extra, mats, env)
    gpu_ctx.configure(w, h, 4, 2, 0, 0, 1, 1)
    t0 = time.perf_counter()
    gpu_ctx.render(0, 1)
    gpu_ctx.synchronize()
    dt = time.perf_counter() - t0
    first_specialized = int(gpu_ctx.stats().specialized)
    g1 = gpu_ctx.read_accum().reshape(h, w, 4)
    r1 = ref.RefScene(extra, mats, env).render(w, h, 0, 1, 4, 2, 0, threads=0)
    assert_parity(g1, r1, 1)
    # the first render ran the generic kernel: it did not wait for the compile (~1-2 s), which the
    # loose time bound confirms without depending on a quiet box
    assert first_specialized == 0
    assert dt < 0.75, f"first render of a new flat shape took {dt * 1e3:.1f} ms"
    gpu_ctx.specialize_scene()  # waits for the background compile, loads the kernels
    gpu_ctx.reset()
    gpu_ctx.render(0, 1)
    assert int(gpu_ctx.stats().specialized) == 1
    g2 = gpu_ctx.read_accum().reshape(h, w, 4)
    assert np.array_equal(g1.view(np.uint32), g2.view(np.uint32)), first_specialized


@pytest.mark.parametrize("scene,w,h,frames", [("bunnylike", 240, 135, 3), ("interior1m", 160, 90, 2)])
def test_sorted_ray_queues(spt, ref, gpu_ctx, scene, w, h, frames):
    """SPT_FLAG_SORTED_RAYS (BVH scenes): rays binned by direction octant and origin cell before every
    bounce >= 1 closest-hit launch. The split schedule ran; the image is bit-identical to the
    persistent schedule's and matches the oracle."""
    g, r = render_both(spt, ref, gpu_ctx, scene, w, h, frames, bounces=8, flags=spt.FLAG_SORTED_RAYS)
    assert int(gpu_ctx.stats().schedule) == spt.SCHEDULE_SPLIT
    assert_parity(g, r, frames)
    gpu_ctx.configure(w, h, 8, 2, 0, 0, 1, 0)
    gpu_ctx.set_tuning(persistent=1)  # k_paths for these few frames too
    try:
        gpu_ctx.render(0, frames)
    finally:
        gpu_ctx.set_tuning()
    assert int(gpu_ctx.stats().schedule) == spt.SCHEDULE_PERSISTENT
    p = gpu_ctx.read_accum().reshape(h, w, 4)
    assert np.array_equal(g.view(np.uint32), p.view(np.uint32))


def test_sorted_ray_queues_many_passes(spt, gpu_ctx):
    """Several wavefront passes per call with the sorted schedule (the bin counts are cleared between
    bounces and passes): equal to the persistent schedule on the same frames."""
    prims, mats, env = spt.build_scene("bunnylike")
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(96, 54, 8, 2, spt.FLAG_SORTED_RAYS, 0, 1, 2)  # 2 frames per pass
    gpu_ctx.render(0, 7)
    a = gpu_ctx.read_accum()
    gpu_ctx.configure(96, 54, 8, 2, 0, 0, 1, 0)
    gpu_ctx.render(0, 7)
    b = gpu_ctx.read_accum()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("per_call", [4, 1])  # k_paths / k_frame (the App's one frame per call; for the
# App's scene the LDS-only kernel, whose stack size follows the refitted tree)
@pytest.mark.parametrize("scene,w,h", [("bunnylike", 160, 90), ("app", 160, 100), ("cornell", 128, 72)])
def test_update_prims_matches_a_fresh_scene(spt, ref, gpu_ctx, scene, w, h, per_call):
    """spt_update_prims: frames rendered, then primitives moved in place (a BVH
    scene keeps its tree and refits; a flat one re-uploads its records) and the accumulation restarts.
    The restarted image equals a fresh spt_set_scene of the edited array bit for bit, and the oracle's
    render of the edited scene (CPUPathTracer.cpp:119-161: a scene change resets m_frameCount)."""
    prims, mats, env = spt.build_scene(scene)
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 8, 2, 0, 0, 1, 0)
    gpu_ctx.render(0, 5)
    edited = prims.copy()
    step = max(1, len(prims) // 40)
    idx = np.arange(0, len(prims), step, dtype=np.uint32)
    for i in idx:  # translate: spheres' centers, triangles' and quads' base point (and triangle vertices)
        off = np.array([0.21, 0.13, -0.27], dtype=np.float32)
        edited[i]["p0"][:3] += off
        if edited[i]["type"] == spt.PRIM_TRIANGLE:
            edited[i]["p1"][:3] += off
            edited[i]["p2"][:3] += off
    gpu_ctx.update_prims(idx, edited[idx])
    assert gpu_ctx.frame_count == 0
    for f in range(0, 4, per_call):
        gpu_ctx.render(f, per_call)
    upd = gpu_ctx.read_accum().reshape(h, w, 4)
    gpu_ctx.set_scene(edited, mats, env)
    for f in range(0, 4, per_call):
        gpu_ctx.render(f, per_call)
    fresh = gpu_ctx.read_accum().reshape(h, w, 4)
    assert np.array_equal(upd.view(np.uint32), fresh.view(np.uint32))
    r = ref.RefScene(edited, mats, env).render(w, h, 0, 4, 8, 2, 0, threads=0)
    assert_parity(upd, r, 4)


def test_update_prims_rejects_bad_input(spt, gpu_ctx):
    prims, mats, env = spt.build_scene("bunnylike")
    gpu_ctx.set_scene(prims, mats, env)
    with pytest.raises(spt.SptError):
        gpu_ctx.update_prims([len(prims)], prims[:1])  # index out of range
    bad = prims[:1].copy()
    bad[0]["material"] = len(mats)
    with pytest.raises(spt.SptError):
        gpu_ctx.update_prims([0], bad)  # material out of range


@pytest.mark.parametrize("scene", ["cornell", "bunnylike"])
def test_frame_calls_follow_scene_changes(spt, ref, gpu_ctx, scene):
    """One-frame calls (k_frame) after a scene edit (spt_update_prims), a new sky map and a
    reconfiguration equal a fresh context's render of the edited scene and the oracle's."""
    prims, mats, env = spt.build_scene(scene)
    w, h = 96, 54
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 8, 2, 0, 0, 1, 0)
    for f in range(2):
        gpu_ctx.render(f, 1)
    assert int(gpu_ctx.stats().schedule) == spt.SCHEDULE_FRAME
    edited = prims.copy()
    edited[-1]["p0"][:3] += np.array([0.3, 0.25, -0.2], dtype=np.float32)
    gpu_ctx.update_prims([len(prims) - 1], edited[-1:])
    gpu_ctx.set_env_map(spt.synthetic_env_map(64))
    gpu_ctx.configure(w, h, 6, 1, 0, 0, 1, 0)
    for f in range(3):
        gpu_ctx.render(f, 1)
    a = gpu_ctx.read_accum().reshape(h, w, 4)
    with spt.Context(0) as fresh:
        fresh.set_scene(edited, mats, env)
        fresh.set_env_map(spt.synthetic_env_map(64))
        fresh.configure(w, h, 6, 1, 0, 0, 1, 0)
        for f in range(3):
            fresh.render(f, 1)
        b = fresh.read_accum().reshape(h, w, 4)
    gpu_ctx.set_env_map(None)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    rs = ref.RefScene(edited, mats, env)
    rs.set_env_map(spt.synthetic_env_map(64))
    assert_parity(a, rs.render(w, h, 0, 3, 6, 1, 0, threads=0), 3)


@pytest.mark.parametrize("scene", ["cornell", "app", "bunnylike"])
def test_frame_camera_hit_cache_follows_edits(spt, gpu_ctx, scene):
    """k_frame keeps each pixel's camera-segment hit across one-frame calls (the camera has no jitter,
    CPUPathTracer.cpp:63-69). After spt_update_prims alone, and after an spt_set_scene of the same shape
    alone (no reconfiguration in between), the next one-frame calls must trace the camera segments again:
    their images equal a fresh context's."""
    prims, mats, env = spt.build_scene(scene)
    w, h = 96, 54
    gpu_ctx.set_tuning()
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 4, 2, 0, 0, 1, 0)
    for f in range(3):  # the first call stores the camera hits, the next ones read them
        gpu_ctx.render(f, 1)
    assert int(gpu_ctx.stats().schedule) == spt.SCHEDULE_FRAME
    moved = prims.copy()
    i = len(prims) - 1
    moved[i]["p0"][:3] += np.array([0.35, -0.2, 0.15], dtype=np.float32)
    if moved[i]["type"] == spt.PRIM_TRIANGLE:
        moved[i]["p1"][:3] += np.array([0.35, -0.2, 0.15], dtype=np.float32)
        moved[i]["p2"][:3] += np.array([0.35, -0.2, 0.15], dtype=np.float32)
    gpu_ctx.update_prims([i], moved[i:i + 1])
    for f in range(2):
        gpu_ctx.render(f, 1)
    a = gpu_ctx.read_accum().reshape(h, w, 4)
    moved2 = moved.copy()
    moved2[0]["p0"][:3] += np.array([-0.1, 0.05, 0.3], dtype=np.float32)
    if moved2[0]["type"] == spt.PRIM_TRIANGLE:
        moved2[0]["p1"][:3] += np.array([-0.1, 0.05, 0.3], dtype=np.float32)
        moved2[0]["p2"][:3] += np.array([-0.1, 0.05, 0.3], dtype=np.float32)
    gpu_ctx.set_scene(moved2, mats, env)
    for f in range(2):
        gpu_ctx.render(f, 1)
    b = gpu_ctx.read_accum().reshape(h, w, 4)
    for scene_prims, got in ((moved, a), (moved2, b)):
        with spt.Context(0) as fresh:
            fresh.set_scene(scene_prims, mats, env)
            fresh.configure(w, h, 4, 2, 0, 0, 1, 0)
            for f in range(2):
                fresh.render(f, 1)
            want = fresh.read_accum().reshape(h, w, 4)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def _sparse_spheres(spt, n=120, seed=7):
    """n small spheres scattered in front of the camera (a BVH scene, too large for k_frame's LDS-held
    form, mostly sky pixels)."""
    rng = np.random.default_rng(seed)
    return spt.sphere_prims([(float(rng.uniform(-2.0, 2.0)), float(rng.uniform(-1.2, 1.2)), float(rng.uniform(5.0, 9.0)),
                              float(rng.uniform(0.05, 0.18))) for _ in range(n)])


@pytest.mark.parametrize("case", ["empty", "sky_off", "cornell", "spheres", "spheres_sky_off"])
def test_frame_calls_with_sky_pixels(spt, ref, gpu_ctx, case):
    """Several one-frame calls in a row (k_frame: the first stores the camera hits, the next ones run
    from them) on an empty scene (every pixel sky: no live pixel at all), a scene without sky, the
    Cornell box (61 % sky pixels), and a sparse BVH scene with sky on and off (the compacted lists:
    sky pixels added without a path, SPT_FRAME_HIT_CACHE 2): bit-exact against the oracle."""
    if case == "empty":
        scene = (np.zeros(0, dtype=spt.PRIM_DTYPE), spt.reference_materials(), spt.reference_env(True))
    elif case == "sky_off":
        prims, mats, _ = spt.build_scene("c1")
        scene = (prims, mats, spt.reference_env(False))
    elif case.startswith("spheres"):
        scene = (_sparse_spheres(spt), spt.reference_materials(), spt.reference_env(case == "spheres"))
    else:
        scene = spt.build_scene("cornell")
    w, h, frames = 72, 40, 4
    gpu_ctx.set_tuning()
    gpu_ctx.set_scene(*scene)
    gpu_ctx.configure(w, h, 6, 2, 0, 0, 1, 0)
    for f in range(frames):
        gpu_ctx.render(f, 1)
    assert int(gpu_ctx.stats().schedule) == spt.SCHEDULE_FRAME
    g = gpu_ctx.read_accum().reshape(h, w, 4)
    r = ref.RefScene(*scene).render(w, h, 0, frames, 6, 2, 0, threads=0)
    assert np.array_equal(g.view(np.uint32), r.view(np.uint32))
