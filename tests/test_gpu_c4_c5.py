"""GPU parity of the BVH configurations at their OWN sizes (BASELINE.json configs[3] and [4]).

* C4: the bunny-like mesh (81,920 triangles in the Cornell box) at 1920x1080, 8 bounces — two k_paths
  launches of 4 frames (the second hands its chunks out longest first, by the costs the first one
  recorded), then 2 single-frame k_frame launches (the App's one frame per render()).
* C5: the 1,000,000-triangle interior at 3840x2160, 8 bounces — 4 frames in one k_paths launch, then
  one k_frame launch.
* C5 row shard: rank 5 of an 8-GPU run at 3840x2160 (rows y = 5 mod 8) vs the oracle's
  row_step = 8, row_offset = 5 on a crop.

Each image is checked against the oracle's rect= renders (which trace only those pixels, with the
full-image seeds) on a 64x64 crop through the mesh and one full row, plus the device RGBA8 resolve of
that row. The pixel loop replaced: CPUPathTracer.cpp:57-82; the bounce loop :197-284 (rtcIntersect1
at :227 -> the quantized 4-wide BVH).
"""
import numpy as np
import pytest

from test_gpu_configs import check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c5_scene(spt, ref):
    prims, mats, env = spt.build_scene("interior1m")
    return prims, mats, env, ref.RefScene(prims, mats, env)


def test_c4_bunnylike_1080p(spt, ref, gpu_ctx):
    """C4 at 1920x1080 x 8 bounces: 2 x 4 frames (k_paths, the second launch in cost order) + 2 x 1 frame
    (k_frame)."""
    w, h = 1920, 1080
    prims, mats, env = spt.build_scene("bunnylike")
    gpu_ctx.set_tuning()
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 8, 2)
    gpu_ctx.render(0, 4)
    gpu_ctx.render(4, 4)
    assert gpu_ctx.stats().schedule == spt.SCHEDULE_PERSISTENT
    gpu_ctx.render(8, 1)
    gpu_ctx.render(9, 1)
    assert gpu_ctx.stats().schedule == spt.SCHEDULE_FRAME
    frames = 10
    g = gpu_ctx.read_accum().reshape(h, w, 4)
    assert np.all(g[..., 3] == float(frames))
    rs = ref.RefScene(prims, mats, env)
    x0, y0 = 928, 628  # 64x64 inside the mesh's silhouette (screen extent x 864-1056, y 552-768)
    crop = rs.render(w, h, 0, frames, 8, 2, 0, rect=(x0, y0, x0 + 64, y0 + 64), threads=0)
    check(g[y0:y0 + 64, x0:x0 + 64], crop, frames, "C4 crop 64x64")
    row = 660  # through the mesh, both side walls and the floor's far edge
    band = rs.render(w, h, 0, frames, 8, 2, 0, rect=(0, row, w, row + 1), threads=0)
    check(g[row:row + 1], band, frames, "C4 row 660")
    px = gpu_ctx.resolve_rgba8(frames).reshape(h, w)
    assert np.array_equal(px[row:row + 1].reshape(-1), ref.resolve_rgba8(band, frames))


def test_c5_interior_4k(spt, ref, gpu_ctx, c5_scene):
    """C5 at 3840x2160 x 8 bounces: 4 frames (k_paths) + 1 frame (k_frame)."""
    w, h = 3840, 2160
    prims, mats, env, rs = c5_scene
    gpu_ctx.set_tuning()
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 8, 2)
    gpu_ctx.render(0, 4)
    assert gpu_ctx.stats().schedule == spt.SCHEDULE_PERSISTENT
    gpu_ctx.render(4, 1)
    assert gpu_ctx.stats().schedule == spt.SCHEDULE_FRAME
    frames = 5
    g = gpu_ctx.read_accum().reshape(h, w, 4)
    assert np.all(g[..., 3] == float(frames))
    x0, y0 = 1888, 1048  # image centre: every primary ray of the crop hits a mesh triangle
    crop = rs.render(w, h, 0, frames, 8, 2, 0, rect=(x0, y0, x0 + 64, y0 + 64), threads=0)
    check(g[y0:y0 + 64, x0:x0 + 64], crop, frames, "C5 crop 64x64")
    row = 1440
    band = rs.render(w, h, 0, frames, 8, 2, 0, rect=(0, row, w, row + 1), threads=0)
    check(g[row:row + 1], band, frames, "C5 row 1440")
    px = gpu_ctx.resolve_rgba8(frames).reshape(h, w)
    assert np.array_equal(px[row:row + 1].reshape(-1), ref.resolve_rgba8(band, frames))


def test_c5_row_shard_rank5_of_8(spt, ref, gpu_ctx, c5_scene):
    """C5's 8-GPU partition, rank 5: rows y = 5 mod 8 of 3840x2160 (270 rows), 4 frames in one k_paths
    launch — vs the oracle's row_step = 8, row_offset = 5 over a 64-column crop of rows 1024..1279
    (global rows 1029, 1037, ..., 1277 = shard rows 128..159) and one full shard row."""
    w, h, rank, world, frames = 3840, 2160, 5, 8, 4
    prims, mats, env, rs = c5_scene
    gpu_ctx.set_tuning()
    gpu_ctx.set_scene(prims, mats, env)
    gpu_ctx.configure(w, h, 8, 2, 0, rank, world)
    assert gpu_ctx.shard_pixels == w * (h // world)
    gpu_ctx.render(0, frames)
    g = gpu_ctx.read_accum().reshape(h // world, w, 4)
    x0, y0, y1 = 1888, 1024, 1280
    crop = rs.render(w, h, 0, frames, 8, 2, 0, rect=(x0, y0, x0 + 64, y1), row_step=world, row_offset=rank,
                     threads=0)
    assert crop.shape == (32, 64, 4)
    check(g[y0 // world:y1 // world, x0:x0 + 64], crop, frames, "C5 shard 5/8 crop")
    lr = 180  # shard row 180 = global row 5 + 8 * 180 = 1445
    band = rs.render(w, h, 0, frames, 8, 2, 0, rect=(0, rank + world * lr, w, rank + world * lr + 1), threads=0)
    check(g[lr:lr + 1], band, frames, "C5 shard 5/8 row 1445")
