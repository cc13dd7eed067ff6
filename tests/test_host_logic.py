"""Host-side logic without a GPU: scene builders, the reference-interface mirror, queue dealing,
row sharding."""
import hashlib

import numpy as np
import pytest

KCHUNK, KSHARDS = 64, 8


def deal_shard(p):  # spt_kernels.h deal_shard
    return (p // KCHUNK) % KSHARDS


def deal_slot(p):  # spt_kernels.h deal_slot
    return (p // (KCHUNK * KSHARDS)) * KCHUNK + (p % KCHUNK)


def cap_for(n):  # spt_capi.hip queue_cap_for
    per = KCHUNK * KSHARDS
    return ((n + per - 1) // per) * KCHUNK


@pytest.mark.parametrize("n", [1, 63, 64, 65, 511, 512, 513, 4097, 65536, 2073600])
def test_queue_dealing_is_a_bijection_within_capacity(n):
    p = np.arange(n, dtype=np.int64)
    cap = cap_for(n)
    idx = deal_shard(p) * cap + deal_slot(p)
    assert idx.max() < KSHARDS * cap
    assert len(np.unique(idx)) == n
    # per-shard counts match shard_count_of() in spt_kernels.hip
    per_round = KCHUNK * KSHARDS
    for s in range(KSHARDS):
        full = (n // per_round) * KCHUNK
        rem = n % per_round
        extra = min(max(rem - s * KCHUNK, 0), KCHUNK)
        assert np.sum(deal_shard(p) == s) == full + extra
        assert np.all(deal_slot(p[deal_shard(p) == s]) < full + extra)


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
