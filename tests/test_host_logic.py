"""Host-side logic without a GPU: scene builders, the reference-interface mirror, queue dealing,
row sharding."""
import hashlib

import numpy as np
import pytest

KCHUNK = 64


def deal_sub(p, n_sub):  # spt_kernels.h deal_sub
    return (p // KCHUNK) % n_sub


def deal_slot(p, n_sub):  # spt_kernels.h deal_slot
    return (p // (KCHUNK * n_sub)) * KCHUNK + (p % KCHUNK)


def dealt_path(s, i, n_sub):  # spt_kernels.h dealt_path
    return ((i // KCHUNK) * n_sub + s) * KCHUNK + (i % KCHUNK)


def sub_count_of(n, s, n_sub):  # spt_kernels.h sub_count_of
    per = KCHUNK * n_sub
    return (n // per) * KCHUNK + min(max(n % per - s * KCHUNK, 0), KCHUNK)


def sub_capacity(n, n_sub):  # spt_kernels.h sub_capacity
    per = KCHUNK * n_sub
    return ((n + per - 1) // per) * KCHUNK


@pytest.mark.parametrize("n_sub", [1, 8, 1536, 2048])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 511, 512, 513, 4097, 65536, 2073600])
def test_queue_dealing_is_a_bijection_within_capacity(n, n_sub):
    p = np.arange(n, dtype=np.int64)
    cap = sub_capacity(n, n_sub)
    sub, slot = deal_sub(p, n_sub), deal_slot(p, n_sub)
    idx = sub * cap + slot
    assert slot.max() < cap and idx.max() < n_sub * cap
    assert len(np.unique(idx)) == n
    assert np.array_equal(dealt_path(sub, slot, n_sub), p)
    counts = np.bincount(sub, minlength=n_sub)
    for s in range(0, n_sub, max(1, n_sub // 16)):
        assert counts[s] == sub_count_of(n, s, n_sub)
        assert np.all(slot[sub == s] < counts[s])  # each sub-queue is a dense prefix


@pytest.mark.parametrize("h,world", [(1080, 1), (1080, 2), (1080, 8), (7, 3), (2160, 8), (5, 8)])
def test_row_shards_partition_the_image(spt, h, world):
    dist = __import__("importlib").import_module("software-path-tracer_amd.distributed")
    seen = []
    for r in range(world):
        rows = dist.rows_of(h, r, world)
        assert len(rows) <= dist.rows_max(h, world)
        seen += rows
    assert sorted(seen) == list(range(h))


def test_scene_builders(spt):
    counts = {}
    for name in ("c1", "app", "cornell", "bunnylike", "interior1m"):
        p, m, e = spt.build_scene(name)
        counts[name] = (len(p), np.bincount(p["type"], minlength=3).tolist(), len(m), e.sky_enabled)
        assert np.all(p["material"] < len(m))
    assert counts["c1"] == (2, [2, 0, 0], 1, 1)
    assert counts["app"] == (38, [38, 0, 0], 1, 1)                 # App.cpp:101-122
    assert counts["cornell"] == (8, [2, 6, 0], 4, 1)               # 6 quads + 2 spheres
    assert counts["bunnylike"] == (81926, [0, 6, 81920], 5, 1)     # icosphere subdiv 6 + box
    assert counts["interior1m"][0] == 1_000_000 and counts["interior1m"][1] == [0, 0, 1_000_000]
    assert counts["interior1m"][3] == 0


def test_scene_builders_are_deterministic(spt):
    for name in ("cornell", "bunnylike"):
        a = hashlib.sha256(spt.build_scene(name)[0].tobytes()).hexdigest()
        b = hashlib.sha256(spt.build_scene(name)[0].tobytes()).hexdigest()
        assert a == b


def test_c1_matches_app_cpp(spt):
    p, m, e = spt.build_scene("c1")
    assert p[0]["p0"].tolist() == [0.0, -1.0, 5.0, 1.0]
    assert p[1]["p0"].tolist() == [0.0, -102.0, 5.0, 100.0]
    assert np.allclose(m[0]["albedo"], 0.7) and np.all(m[0]["emission"] == 0)
    assert list(e.horizon) == [1.0, 1.0, 1.0] and np.allclose(list(e.zenith), [0.5, 0.7, 1.0])


def test_render_settings_mirror(spt):
    s = spt.RenderSettings()
    assert s.isDirty() and (s.getWidth(), s.getHeight()) == (512, 512)
    s.clearDirty()
    s.setResolution(512, 512)
    s.setMaxBounces(8)
    assert not s.isDirty()
    s.setSamplesPerPixel(32)
    assert s.isDirty()


def test_factory_rejects_other_backends(spt):
    for b in (spt.BackendType.CPU_EMBREE, spt.BackendType.GPU_OPTIX, spt.BackendType.GPU_METAL):
        with pytest.raises(RuntimeError, match="Unknown backend type"):
            spt.PathTracer.create_path_tracer(b)


def test_host_assembly_restatement(spt):
    dist = __import__("importlib").import_module("software-path-tracer_amd.distributed")
    w, h, world = 5, 11, 3
    img = np.random.default_rng(0).random((h, w, 4)).astype(np.float32)
    gathered = np.concatenate([dist.pad_shard(img[r::world], h, world) for r in range(world)])
    assert np.array_equal(dist.assemble_rows_host(gathered, w, h, world), img)


def test_env_octa_from_equirect_constant_and_poles(spt):
    """spt_env_octa_from_equirect: a constant image stays constant; the +y pole (centre texel)
    takes the top row, the -y pole (corners) the bottom row."""
    src = np.ones((32, 64, 3), dtype=np.float32) * np.array([0.25, 0.5, 0.75], dtype=np.float32)
    octa = spt.env_octa_from_equirect(src, 16, 16)
    assert octa.shape == (16, 16, 4) and np.all(octa[..., :3] == src[0, 0]) and np.all(octa[..., 3] == 1.0)
    grad = np.zeros((32, 64, 3), dtype=np.float32)
    grad[:, :, 0] = np.arange(32, dtype=np.float32)[:, None]  # row index
    octa = spt.env_octa_from_equirect(grad, 33, 33)
    assert octa[16, 16, 0] == 0.0 and octa[0, 0, 0] == 31.0 and octa[32, 32, 0] == 31.0


def test_octa_texel_restatement(ref):
    """The oracle's octa_texel against an independent numpy float32 restatement."""
    rng = np.random.default_rng(3)
    dirs = rng.normal(size=(2000, 3)).astype(np.float32)
    dirs[:10] = [(0, 1, 0), (0, -1, 0), (1, 0, 0), (-1, 0, 0), (0, 0, 1), (0, 0, -1), (0, 0, 0),
                 (1, 1, 1), (-1, -1, -1), (0.5, -0.25, 0.25)]
    w, h = 37, 23
    for d in dirs:
        x, y, z = (np.float32(v) for v in d)
        with np.errstate(invalid="ignore", divide="ignore"):
            s = (np.abs(x) + np.abs(y)) + np.abs(z)
            px, pz = x / s, z / s
            if y < 0:
                px, pz = ((np.float32(1) - np.abs(pz)) * np.float32(1 if px >= 0 else -1),
                          (np.float32(1) - np.abs(px)) * np.float32(1 if pz >= 0 else -1))
            u = np.fmin(np.fmax(px * np.float32(0.5) + np.float32(0.5), np.float32(0)), np.float32(1))
            v = np.fmin(np.fmax(pz * np.float32(0.5) + np.float32(0.5), np.float32(0)), np.float32(1))
        ix, iy = min(int(u * np.float32(w)), w - 1), min(int(v * np.float32(h)), h - 1)
        assert ref.octa_texel(d, w, h) == iy * w + ix, d


def kchan_ring(n_live):
    """k_paths kChan's per-pixel ring layout (spt_kernels.hip, chunk set-up and ring_entry), restated:
    sub-ring size 2^sr_sh frames per live pixel, window n_live << sr_sh slots."""
    lg = (2 * n_live - 1).bit_length() - 1  # 32 - clz(2 n - 1) - 1 = ceil(log2 n)
    sr_sh = 8 - lg
    m_live = (0x80000000 + n_live - 1) // n_live
    div_live = lambda s: ((s << 1) * m_live) >> 32  # noqa: E731  (exact for s < 2^15)

    def entry(s):
        f = div_live(s)
        return ((s - f * n_live) << sr_sh) | (f & ((1 << sr_sh) - 1))

    return sr_sh, n_live << sr_sh, div_live, entry


@pytest.mark.parametrize("n_live", list(range(1, 17)))
def test_kchan_ring_layout_is_a_bijection_within_the_window(n_live):
    """Within any window of slots [oldest, oldest + win) starting at a frame boundary, the per-pixel
    ring entries are distinct and inside the 256-entry ring; a pixel's consecutive frames are
    consecutive entries (mod its sub-ring), which the accumulation reads four at a time."""
    sr_sh, win, div_live, entry = kchan_ring(n_live)
    assert 1 <= sr_sh <= 8 and win <= 256 and win > 128  # the window never shrinks below half the ring
    for s in range(1 << 15):
        assert div_live(s) == s // n_live
    for oldest in range(0, 2048 * n_live, n_live):  # frame boundaries over 2048 frames (laps included)
        es = [entry(s) for s in range(oldest, oldest + win)]
        assert len(set(es)) == win and max(es) < 256
    for r in range(n_live):
        for f in range(0, 40):
            e0, e1 = entry(f * n_live + r), entry((f + 1) * n_live + r)
            assert e1 == (e0 + 1 if (f + 1) % (1 << sr_sh) else r << sr_sh)
