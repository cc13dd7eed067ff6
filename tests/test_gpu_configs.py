"""GPU parity at the configurations' own shapes and against the committed golden fixtures.

* C3 (BASELINE.json configs[2]): Cornell 1920x1080, 4096 spp progressive, accumulated on the GPU in
  calls of 64 frames (the reference's frame k is seeded with k + 1, CPUPathTracer.cpp:61, and added
  in frame order, :77-80) — checked against the oracle over the same 4096 frames on a 64x64 centre
  crop and one full row (the oracle's `rect`: it traces only those pixels, with the full-image seeds).
* tests/golden/accum.npz (written by tests/golden/make_golden.py): the HIP accumulation and its
  device RGBA8 resolve vs the committed fixtures, no oracle call at run time.
* SURVEY.md 8f row 2 (scene upload / rebuild): a changed scene handed to the backend restarts the
  accumulation and renders the new geometry (CPUPathTracer.cpp:119-161, 328-404).
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
RMS_TOL = 1e-4          # per-pixel L2 RMS bound on averaged radiance (north_star)
EXACT_FRAC = 0.999      # fraction of pixels whose float RGBA accumulation must be bit-identical


def check(g, r, frames, what):
    g = np.ascontiguousarray(g, np.float32).reshape(-1, 4)
    r = np.ascontiguousarray(r, np.float32).reshape(-1, 4)
    exact = np.all(g.view(np.uint32) == r.view(np.uint32), axis=1)
    l2 = np.sqrt(np.sum(((g[:, :3].astype(np.float64) - r[:, :3]) / frames) ** 2, axis=1))
    l2 = np.where(exact, 0.0, l2)  # bit-identical pixels differ by 0 (also where both hold the same NaN)
    rms = float(np.sqrt(np.mean(l2 ** 2)))
    print(f"{what}: {exact.mean():.6f} bit-exact, rms L2 {rms:.3g}, max L2 {float(l2.max()):.3g}")
    assert rms < RMS_TOL, (what, rms)
    assert exact.mean() >= EXACT_FRAC, (what, exact.mean())


def test_c3_4096spp_progressive_in_calls_of_64(spt, ref, gpu_ctx):
    """C3: 1920x1080, 8 bounces, 4096 frames as 64 spt_render calls of 64 frames (k_paths)."""
    w, h, frames, call = 1920, 1080, 4096, 64
    prims, mats, env = spt.build_scene("cornell")
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 8, 2)
    for first in range(0, frames, call):
        gpu_ctx.render(first, call)
    assert gpu_ctx.frame_count == frames
    assert gpu_ctx.stats().schedule == spt.SCHEDULE_PERSISTENT
    g = gpu_ctx.read_accum().reshape(h, w, 4)
    assert np.all(g[..., 3] == float(frames))
    rs = ref.RefScene(prims, mats, env)
    x0, y0 = 928, 508  # 64x64 crop through the spheres and the back wall
    crop = rs.render(w, h, 0, frames, 8, 2, 0, rect=(x0, y0, x0 + 64, y0 + 64), threads=0)
    check(g[y0:y0 + 64, x0:x0 + 64], crop, frames, "C3 crop 64x64")
    row = 700  # a full row through the spheres, both side walls and the floor
    band = rs.render(w, h, 0, frames, 8, 2, 0, rect=(0, row, w, row + 1), threads=0)
    check(g[row:row + 1], band, frames, "C3 row 700")
    # and the resolve the App would display after 4096 frames (CPUPathTracer.cpp:87-117)
    px = gpu_ctx.resolve_rgba8(frames).reshape(h, w)
    assert np.array_equal(px[row:row + 1].reshape(-1), ref.resolve_rgba8(band, frames))


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(HERE, "golden", "accum.npz"))


@pytest.mark.parametrize("frames", [1, 16])
def test_golden_c1(spt, gpu_ctx, golden, frames):
    """C1 (App.cpp:101-111, 256x256, 4 bounces): frame 1 full image; 16 frames, the (96,96)-(160,160)
    crop — vs the committed fixtures."""
    gpu_ctx.set_scene(*spt.build_scene("c1"))
    gpu_ctx.configure(256, 256, 4, 2)
    gpu_ctx.render(0, frames)
    g = gpu_ctx.read_accum().reshape(256, 256, 4)
    if frames == 1:
        check(g, golden["c1_f1"], 1, "golden c1_f1")
    else:
        check(g[96:160, 96:160], golden["c1_f16_crop"], 16, "golden c1_f16_crop")


@pytest.mark.parametrize("frames_per_call", [1, 16])  # k_frame per frame / one k_paths launch
def test_golden_app_scene_and_rgba8(spt, gpu_ctx, golden, frames_per_call):
    """The App's default 38-sphere scene (App.cpp:98-122), 64x64 x 16 frames, and its RGBA8 resolve."""
    gpu_ctx.set_scene(*spt.build_scene("app"))
    gpu_ctx.configure(64, 64, 4, 2)
    for first in range(0, 16, frames_per_call):
        gpu_ctx.render(first, frames_per_call)
    check(gpu_ctx.read_accum(), golden["app_64_f16"], 16, "golden app_64_f16")
    px = gpu_ctx.resolve_rgba8(16)
    same = np.mean(px == golden["app_64_f16_rgba8"])
    print(f"golden app_64_f16_rgba8: {same:.6f} identical")
    assert same >= EXACT_FRAC


def test_registered_host_output_resolve(spt, golden):
    """spt_register_host_output: the resolve kernel writes a registered host buffer directly (no DMA
    copy) — the same RGBA8 as the staging-and-copy path and the golden fixture, with exposure too;
    unregistered or too-small buffers take the copy path; re-registration and unregistration work."""
    with spt.Context(0) as ctx:
        ctx.set_scene(*spt.build_scene("app"))
        ctx.configure(64, 64, 4, 2)
        ctx.render(0, 16)
        copied = ctx.resolve_rgba8(16)
        copied_exp = ctx.resolve_rgba8(16, 1.7)
        buf = np.full(ctx.shard_pixels, 0xdeadbeef, dtype=np.uint32)
        ctx.register_host_output(buf)
        assert ctx.resolve_rgba8(16, out=buf) is buf
        np.testing.assert_array_equal(buf, copied)
        assert np.mean(buf == golden["app_64_f16_rgba8"]) >= EXACT_FRAC
        np.testing.assert_array_equal(ctx.resolve_rgba8(16, 1.7, out=buf), copied_exp)
        other = np.zeros(ctx.shard_pixels, dtype=np.uint32)  # not registered: the copy path
        np.testing.assert_array_equal(ctx.resolve_rgba8(16, out=other), copied)
        big = np.zeros(2 * ctx.shard_pixels, dtype=np.uint32)  # re-registration replaces the first
        ctx.register_host_output(big)
        ctx.resolve_rgba8(16, out=big)
        np.testing.assert_array_equal(big[:ctx.shard_pixels], copied)
        assert not big[ctx.shard_pixels:].any()
        ctx.configure(96, 96, 4, 2)  # now larger than the registered 2 x 64 x 64: the copy path
        ctx.render(0, 2)
        grown = np.zeros(ctx.shard_pixels, dtype=np.uint32)
        ref2 = ctx.resolve_rgba8(2, out=grown)
        ctx.register_host_output(None)
        np.testing.assert_array_equal(ctx.resolve_rgba8(2), ref2)
        ctx.register_host_output(grown)  # and registered at the new size: direct again
        ctx.render(2, 2)
        np.testing.assert_array_equal(ctx.resolve_rgba8(4, out=grown), ctx.resolve_rgba8(4))
        with pytest.raises(spt.SptError):
            ctx.register_host_output(np.zeros(ctx.shard_pixels, dtype=np.float32))


@pytest.mark.parametrize("scene,w,h,bounces,flags", [
    ("app", 512, 512, 4, 0),          # the App's frame: k_frame kSmall, one pixel per lane
    ("cornell", 320, 180, 8, 0),      # flat (run-time specialized), camera hits cached then listed
    ("bunnylike", 160, 90, 8, 0),     # BVH from global memory
    ("cornell", 160, 90, 8, "nee"),   # next-event estimation
])
def test_render_resolve_fused(spt, scene, w, h, bounces, flags):
    """spt_render_resolve_rgba8 (the resolve fused into the frame's k_frame launch, each pixel stored
    into the registered host buffer as its path ends) gives exactly render() + resolve_rgba8() after
    every call: one-frame calls (camera hits stored, then read, then compacted), a 2-frame call (only
    the last launch resolves), an exposure, a 5-frame call (k_paths: render then resolve), and a
    buffer that is not the registered one (the staging-and-copy resolve)."""
    fl = spt.FLAG_NEE if flags == "nee" else flags
    calls = [(1, 1.0), (1, 1.0), (1, 1.0), (2, 1.0), (1, 1.7), (5, 1.0), (1, 1.0)]
    with spt.Context(0) as plain, spt.Context(0) as fused:
        for c in (plain, fused):
            c.set_scene(*spt.build_scene(scene))
            c.configure(w, h, bounces, 2, fl)
        buf = np.zeros(fused.shard_pixels, dtype=np.uint32)
        fused.register_host_output(buf)
        frame = 0
        for n, exposure in calls:
            plain.render(frame, n)
            want = plain.resolve_rgba8(frame + n, exposure)
            buf[:] = 0xdeadbeef
            assert fused.render_resolve_rgba8(frame, n, frame + n, exposure, out=buf) is buf
            np.testing.assert_array_equal(buf, want, err_msg=f"{scene} frames {frame}+{n}")
            frame += n
        np.testing.assert_array_equal(fused.read_accum(), plain.read_accum())
        other = np.zeros(fused.shard_pixels, dtype=np.uint32)  # not registered: render, then the copy path
        plain.render(frame, 1)
        fused.render_resolve_rgba8(frame, 1, frame + 1, out=other)
        np.testing.assert_array_equal(other, plain.resolve_rgba8(frame + 1))
        with pytest.raises(spt.SptError):
            fused.render_resolve_rgba8(frame + 1, 1, 0, out=buf)  # frame_count 0: "No frames rendered yet"


def test_render_resolve_fused_golden(spt, golden):
    """The App's scene at 64x64, 16 one-frame calls through spt_render_resolve_rgba8 into the registered
    buffer: the committed oracle fixture's RGBA8."""
    with spt.Context(0) as ctx:
        ctx.set_scene(*spt.build_scene("app"))
        ctx.configure(64, 64, 4, 2)
        buf = np.zeros(ctx.shard_pixels, dtype=np.uint32)
        ctx.register_host_output(buf)
        for k in range(16):
            ctx.render_resolve_rgba8(k, 1, k + 1, out=buf)
        assert np.mean(buf == golden["app_64_f16_rgba8"]) >= EXACT_FRAC


def test_golden_cornell_crop(spt, gpu_ctx, golden):
    """Cornell (build-defined superset scene), 1920x1080 x 4 frames, 8 bounces: the 64x64 crop at
    (928, 508) vs the committed fixture."""
    gpu_ctx.set_scene(*spt.build_scene("cornell"))
    gpu_ctx.configure(1920, 1080, 8, 2)
    gpu_ctx.render(0, 4)
    g = gpu_ctx.read_accum().reshape(1080, 1920, 4)
    check(g[508:572, 928:992], golden["cornell_crop_f4"], 4, "golden cornell_crop_f4")


def test_scene_change_restarts_accumulation(spt, ref):
    """SURVEY.md 8f row 2 through the PathTracer mirror: 6 frames of the C1 scene, then the App
    hands over a changed scene (one sphere moved, one added: a new Scene starts with
    m_has_changes = true, Scene.h:140-150) — the backend re-uploads it, restarts at frame 0
    (CPUPathTracer.cpp:122-131, 154-158) and renders the new geometry: oracle of the NEW scene."""
    w, h = 160, 120
    tracer = spt.PathTracer.create_path_tracer(spt.BackendType.GPU_HIP)
    settings = spt.RenderSettings()
    settings.setResolution(w, h)
    tracer.set_settings(settings)

    def scene_of(spheres):
        sc = spt.Scene()
        for x, y, z, r in spheres:
            s = sc.CreateNode(spt.SphereObject, "s")
            s.SetPosition((x, y, z))
            s.SetRadius(r)
        return sc

    first = [(0.0, -1.0, 5.0, 1.0), (0.0, -102.0, 5.0, 100.0)]
    second = [(0.7, -0.8, 4.5, 1.0), (0.0, -102.0, 5.0, 100.0), (-1.6, -0.5, 6.0, 0.5)]
    tracer.set_scene(scene_of(first))
    for _ in range(6):
        tracer.render()
    tracer.set_scene(scene_of(second))
    t0 = time.perf_counter()
    tracer.render()  # re-upload + frame 0 of the new scene
    print(f"scene change + first frame: {(time.perf_counter() - t0) * 1e3:.2f} ms")
    for _ in range(3):
        tracer.render()
    res = tracer.get_render_result()
    acc = tracer.read_accumulation().reshape(h, w, 4)
    assert np.all(acc[..., 3] == 4.0)  # restarted: 4 frames of the new scene, not 10
    prims = spt.sphere_prims(second)
    r = ref.RefScene(prims, spt.reference_materials(), spt.reference_env()).render(w, h, 0, 4)
    check(acc, r, 4, "scene change")
    assert np.mean(res.image_buffer == ref.resolve_rgba8(r, 4)) >= EXACT_FRAC
    # the same renderer, the scene object left unchanged: progressive accumulation continues
    tracer.render()
    assert np.all(tracer.read_accumulation().reshape(h, w, 4)[..., 3] == 5.0)


def test_rccl_gather_image_single_rank(spt):
    """spt_comm_init / spt_gather_image (the library's RCCL collective) with one rank:
    the gathered, de-interleaved image equals the accumulation. (More ranks need more GPUs: RCCL puts
    one rank per device; the driver's multi-GPU bench runs that path.)"""
    import torch

    w, h = 97, 61
    with spt.Context(0) as ctx:
        ctx.set_scene(*spt.build_scene("cornell"))
        ctx.configure(w, h, 8, 2)
        ctx.render(0, 5)
        ctx.comm_init(spt.comm_unique_id(), 1, 0)
        img = torch.full((w * h * 4,), -1.0, dtype=torch.float32, device="cuda")
        ctx.gather_image(img.data_ptr())
        ctx.synchronize()
        got = img.cpu().numpy().reshape(h, w, 4)
        assert np.array_equal(got.view(np.uint32), ctx.read_accum().reshape(h, w, 4).view(np.uint32))
        with pytest.raises(spt.SptError, match="INVALID"):
            ctx.comm_init(spt.comm_unique_id(), 2, 2)  # rank out of range
        ctx.comm_init(spt.comm_unique_id(), 1, 0)
        ctx.configure(w, h, 8, 2, 0, 0, 2)  # shard 0 of 2, but a 1-rank communicator
        with pytest.raises(spt.SptError, match="INVALID"):
            ctx.gather_image(img.data_ptr())
        ctx.comm_destroy()


def test_rccl_gather_overlapped_takes_a_snapshot(spt):
    """spt_gather_image_overlapped: the shard is snapshot on the integrator's stream and gathered on the
    ctx's comm stream while the next spt_render calls run; after spt_gather_wait the image holds the
    frames rendered BEFORE the call, not the later ones. Back-to-back gathers reuse the snapshot buffer
    only after the previous gather has read it. One rank (RCCL puts one rank per GPU)."""
    import torch

    w, h = 97, 61
    with spt.Context(0) as ctx:
        ctx.set_scene(*spt.build_scene("cornell"))
        ctx.configure(w, h, 8, 2)
        ctx.comm_init(spt.comm_unique_id(), 1, 0)
        imgs = [torch.full((w * h * 4,), -1.0, dtype=torch.float32, device="cuda") for _ in range(3)]
        expect = []
        ctx.render(0, 5)
        expect.append(ctx.read_accum().reshape(-1))  # (synchronizes)
        ctx.gather_image_overlapped(imgs[0].data_ptr())
        ctx.render(5, 64)  # overlaps the gather
        ctx.gather_image_overlapped(imgs[1].data_ptr())
        ctx.render(69, 3)
        ctx.gather_image_overlapped(imgs[2].data_ptr())
        ctx.gather_wait()
        ctx.synchronize()
        final = ctx.read_accum().reshape(-1)
        got = [i.cpu().numpy() for i in imgs]
        assert np.array_equal(got[0].view(np.uint32), expect[0].view(np.uint32))
        assert np.array_equal(got[2].view(np.uint32), final.view(np.uint32))
        assert np.all(got[1].reshape(h, w, 4)[..., 3] == 69.0)  # frames 0..68
        assert not np.array_equal(got[1].view(np.uint32), got[2].view(np.uint32))
        # the blocking gather after overlapped ones waits for them too
        ctx.gather_image(imgs[0].data_ptr())
        ctx.synchronize()
        assert np.array_equal(imgs[0].cpu().numpy().view(np.uint32), final.view(np.uint32))
        ctx.gather_wait()  # nothing pending: a no-op
        ctx.configure(w, h, 8, 2, 0, 0, 2)  # shard 0 of 2, but a 1-rank communicator
        with pytest.raises(spt.SptError, match="INVALID"):
            ctx.gather_image_overlapped(imgs[0].data_ptr())
        ctx.comm_destroy()
