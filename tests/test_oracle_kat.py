"""CPU oracle vs known answers (no GPU).

Pins the oracle (oracle/cpu_ref.c) three ways:
  1. the reference's only known-answer case: the Embree demo rays of src/main.cpp:38-75, whose
     answers follow analytically from sphere.md:145-188 (table in SURVEY.md §4);
  2. independent pure-Python/numpy restatements of CPUPathTracer.cpp's integer and float code
     (get_rng_state :192-195, random_float :294-301, primary ray :53-73, get_random_bounche :303-326),
     evaluated with float32 numpy arithmetic (IEEE, no FMA) and Python's double math;
  3. regression against the committed golden fixtures (tests/golden/, made by make_golden.py).
"""
import json
import math
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
f32 = np.float32


# ---------------------------------------------------------------- independent restatements
def py_random_float(state: int):
    """CPUPathTracer::random_float (:294-301) in Python integers."""
    state = (state * 747796405 + 2891336453) & 0xFFFFFFFF
    result = (((state >> ((state >> 28) + 4)) ^ state) * 277803737) & 0xFFFFFFFF
    result = ((result >> 22) ^ result) & 0xFFFFFFFF
    return f32(f32(result) / f32(4294967295.0)), state


def py_primary_dir(x, y, w, h):
    """CPUPathTracer::render (:53-73) in float32."""
    inv_h = f32(1.0) / f32(h)
    inv_w = f32(1.0) / f32(w)
    aspect = f32(w) / f32(h)
    u = f32(x) * inv_w
    v = f32(1.0) - f32(y) * inv_h
    uvx = (u * f32(2.0) - f32(1.0)) * aspect
    uvy = v * f32(2.0) - f32(1.0)
    ln = np.sqrt(uvx * uvx + uvy * uvy + f32(1.0), dtype=np.float32)
    return np.array([uvx / ln, uvy / ln, f32(1.0) / ln], dtype=np.float32)


def py_bounce(n, state, abs_float=False):
    """CPUPathTracer::get_random_bounche (:303-326): sqrt/cos/sin in double (libstdc++ binding)."""
    n = np.asarray(n, dtype=np.float32)
    u1, state = py_random_float(state)
    u2, state = py_random_float(state)
    cos_t = f32(math.sqrt(float(u1)))
    sin_t = f32(math.sqrt(float(f32(1.0) - u1)))
    phi = f32(f32(2.0) * f32(math.pi)) * u2
    x = f32(float(sin_t) * math.cos(float(phi)))
    y = f32(float(sin_t) * math.sin(float(phi)))
    z = cos_t
    not_pole = (abs(float(n[2])) < 0.999) if abs_float else (abs(int(n[2])) < 0.999)
    up = np.array([0, 0, 1] if not_pole else [1, 0, 0], dtype=np.float32)

    def cross(a, b):
        return np.array([a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1]],
                        dtype=np.float32)

    c = cross(up, n)
    inv = f32(1.0) / np.sqrt((c[0] * c[0] + c[1] * c[1]) + c[2] * c[2], dtype=np.float32)
    t = c * inv
    b = cross(n, t)
    return np.array([(x * t[k] + y * b[k]) + z * n[k] for k in range(3)], dtype=np.float32), state


# ---------------------------------------------------------------- 1. Embree demo KATs
def test_embree_demo_rays_known_answers(spt, ref):
    """src/main.cpp:38-75: 3 spheres, 4 rays, tnear = 0 (main.cpp:84)."""
    prims = spt.sphere_prims([(0.0, 0.0, 0.0, 1.0), (2.5, 0.0, 1.0, 0.5), (-1.5, 1.0, -0.5, 0.8)])
    s = ref.RefScene(prims, spt.reference_materials(), spt.reference_env())
    h = s.intersect((0, 0, -5), (0, 0, 1), 0.0)
    assert h[0] == 4.0 and h[1] == 0 and np.array_equal(h[2], [0, 0, -1])
    h = s.intersect((2.5, 0, -5), (0, 0, 1), 0.0)
    assert h[0] == 5.5 and h[1] == 1 and np.array_equal(h[2], [0, 0, -0.5])
    assert s.intersect((10, 10, -5), (0, 0, 1), 0.0) is None
    h = s.intersect((-2, -2, -5), (0.5, 0.5, 1), 0.0)  # unnormalized direction
    assert h[0] == 4.0 and h[1] == 0
    hit = np.array([-2, -2, -5], np.float32) + f32(h[0]) * np.array([0.5, 0.5, 1], np.float32)
    assert np.array_equal(hit, [0, 0, -1])


def test_sphere_closed_forms(spt, ref):
    """sphere.md:145-188: inside origin -> far root; tangent-ish and behind-origin cases."""
    prims = spt.sphere_prims([(0.0, 0.0, 5.0, 1.0)])
    s = ref.RefScene(prims, spt.reference_materials(), spt.reference_env())
    assert s.intersect((0, 0, 0), (0, 0, 1))[0] == 4.0
    assert s.intersect((0, 0, 5), (0, 0, 1))[0] == 1.0        # origin inside: far root
    assert s.intersect((0, 0, 7), (0, 0, 1)) is None          # sphere behind the ray
    assert s.intersect((0, 2, 0), (0, 0, 1)) is None          # passes above
    # the C1 centre pixel ray hits the r=1 sphere at (0,-1,5)? no: it passes above (y = 0 line)
    d = py_primary_dir(128, 128, 256, 256)
    assert d[1] == 0.0


def test_tnear_excludes_self_hit(spt, ref):
    """rtcIntersect1 tnear = 0.001f (CPUPathTracer.cpp:221): roots below it are skipped."""
    prims = spt.sphere_prims([(0.0, 0.0, 0.0, 1.0)])
    s = ref.RefScene(prims, spt.reference_materials(), spt.reference_env())
    h = s.intersect((0, 0, -1.0005), (0, 0, 1), 0.001)
    assert h is not None and abs(h[0] - 0.0005) > 0  # near root 0.0005 < tnear -> far root
    assert h[0] > 1.9


# ---------------------------------------------------------------- 2. independent restatements
@pytest.mark.parametrize("seed", [0, 1, 982451653, 0xFFFFFFFF, 2891336453, 123456789])
def test_random_float_matches_python(ref, seed):
    vals, states = ref.random_floats(seed, 64)
    s = seed
    for i in range(64):
        v, s = py_random_float(s)
        assert vals[i] == v and states[i] == s


def test_random_float_can_return_one(ref):
    """4294967295.0f == 2^32, so result >= 2^32 - 128 gives exactly 1.0f."""
    # search a seed whose first draw hashes high, with the Python restatement
    for seed in range(200000):
        v, _ = py_random_float(seed)
        if v == 1.0:
            vals, _ = ref.random_floats(seed, 1)
            assert vals[0] == 1.0
            return
    pytest.skip("no seed in range produced 1.0")


def test_rng_seed(ref):
    """get_rng_state (:192-195): x + y*width + frame*982451653 mod 2^32."""
    for x, y, w, f in [(0, 0, 256, 1), (255, 255, 256, 1), (7, 3, 256, 64), (1919, 1079, 1920, 4096)]:
        assert ref.rng_seed(x, y, w, f) == (x + y * w + f * 982451653) & 0xFFFFFFFF


@pytest.mark.parametrize("x,y,w,h", [(0, 0, 256, 256), (255, 255, 256, 256), (17, 200, 256, 256),
                                     (0, 0, 1920, 1080), (1919, 1079, 1920, 1080), (960, 540, 1920, 1080),
                                     (3, 1, 7, 5)])
def test_primary_dir_matches_numpy(ref, x, y, w, h):
    assert np.array_equal(ref.primary_dir(x, y, w, h), py_primary_dir(x, y, w, h))


@pytest.mark.parametrize("abs_float", [False, True])
@pytest.mark.parametrize("n", [(0.0, 0.0, -1.0), (0.0, 1.0, 0.0), (0.6, 0.0, -0.8), (0.0, 0.0, 1.0),
                               (0.28, -0.96, 0.0), (0.0, 0.9995, 0.0316)])
def test_bounce_matches_python(ref, n, abs_float):
    for seed in (1, 982451653, 0xDEADBEEF, 42):
        d, s = ref.bounce_dir(n, seed, 1 if abs_float else 0)
        pd, ps = py_bounce(n, seed, abs_float)
        assert s == ps
        assert np.array_equal(d, pd), (n, seed, d, pd)


def test_bounce_is_cosine_hemisphere(ref):
    """Statistical sanity: directions lie in the hemisphere of n with E[cos] = 2/3."""
    n = (0.0, 1.0, 0.0)
    cos = []
    for seed in range(1, 4001):
        d, _ = ref.bounce_dir(n, seed * 2654435761 & 0xFFFFFFFF)
        assert d[1] >= -1e-6
        cos.append(d[1] / np.linalg.norm(d))
    assert abs(np.mean(cos) - 2.0 / 3.0) < 0.02


def test_abs_int_quirk(ref):
    """::abs(int) on a float (CPUPathTracer.cpp:320): |n.z| = 0.9995 keeps up = +z (float fabs flips it)."""
    n = (0.0, 0.0316, 0.9995)
    d_int, _ = ref.bounce_dir(n, 7, 0)
    d_flt, _ = ref.bounce_dir(n, 7, 1)
    assert not np.array_equal(d_int, d_flt)


# ---------------------------------------------------------------- 3. golden fixtures (regression)
def test_golden_vectors(ref):
    with open(os.path.join(GOLDEN, "vectors.json")) as fh:
        g = json.load(fh)
    for case in g["rng"]:
        assert ref.rng_seed(case["x"], case["y"], case["width"], case["frame1"]) == case["seed"]
        vals, states = ref.random_floats(case["seed"], 16)
        assert [f"{v:08x}" for v in vals.view(np.uint32)] == case["floats_hex"]
        assert [int(s) for s in states] == case["states"]
    for case in g["bounce"]:
        d, s = ref.bounce_dir(case["normal"], case["seed"], case["flags"])
        assert [f"{v:08x}" for v in d.view(np.uint32)] == case["dir_hex"] and s == case["state_after"]


def test_golden_images(spt, ref):
    gold = np.load(os.path.join(GOLDEN, "accum.npz"))
    p, m, e = spt.build_scene("c1")
    rs = ref.RefScene(p, m, e)
    assert np.array_equal(rs.render(256, 256, 0, 1, 4, 2, 0).view(np.uint32), gold["c1_f1"].view(np.uint32))
    crop = rs.render(256, 256, 0, 16, 4, 2, 0, rect=(96, 96, 160, 160))
    assert np.array_equal(crop.view(np.uint32), gold["c1_f16_crop"].view(np.uint32))
    p, m, e = spt.build_scene("app")
    app = ref.RefScene(p, m, e).render(64, 64, 0, 16, 4, 2, 0)
    assert np.array_equal(app.view(np.uint32), gold["app_64_f16"].view(np.uint32))
    assert np.array_equal(ref.resolve_rgba8(app, 16), gold["app_64_f16_rgba8"])
    p, m, e = spt.build_scene("cornell")
    cor = ref.RefScene(p, m, e).render(1920, 1080, 0, 4, 8, 2, 0, rect=(928, 508, 992, 572))
    assert np.array_equal(cor.view(np.uint32), gold["cornell_crop_f4"].view(np.uint32))


# ---------------------------------------------------------------- oracle properties
def test_alpha_counts_frames(spt, ref):
    p, m, e = spt.build_scene("c1")
    acc = ref.RefScene(p, m, e).render(32, 32, 0, 5)
    assert np.all(acc[..., 3] == 5.0)


def test_thread_count_invariance(spt, ref):
    p, m, e = spt.build_scene("cornell")
    rs = ref.RefScene(p, m, e)
    a = rs.render(96, 64, 0, 3, 8, threads=1)
    b = rs.render(96, 64, 0, 3, 8, threads=7)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_crop_and_row_shard_consistency(spt, ref):
    p, m, e = spt.build_scene("cornell")
    rs = ref.RefScene(p, m, e)
    full = rs.render(64, 40, 2, 3, 8)
    crop = rs.render(64, 40, 2, 3, 8, rect=(10, 5, 30, 25))
    assert np.array_equal(crop.view(np.uint32), full[5:25, 10:30].view(np.uint32))
    for r in range(3):
        part = rs.render(64, 40, 2, 3, 8, row_step=3, row_offset=r)
        assert np.array_equal(part.view(np.uint32), full[r::3].view(np.uint32))


def test_progressive_accumulation_order(spt, ref):
    """Frames are added one by one in order (CPUPathTracer.cpp:77-80): 0+c0+c1+... per pixel."""
    p, m, e = spt.build_scene("cornell")
    rs = ref.RefScene(p, m, e)
    acc = rs.render(48, 32, 0, 4, 8)
    manual = np.zeros_like(acc)
    for f in range(4):
        manual += rs.render(48, 32, f, 1, 8)
    assert np.array_equal(acc.view(np.uint32), manual.view(np.uint32))


def test_resolve_packing(ref):
    """get_render_result (:87-117): divide, clamp, truncate, R in the high byte (Color.h:7-10)."""
    acc = np.array([[2.0, 0.5, -1.0, 2.0], [0.999, 0.0, 0.25, 1.0]], dtype=np.float32)
    out = ref.resolve_rgba8(acc, 2)
    assert out[0] == (255 << 24) | (63 << 16) | (0 << 8) | 255
    assert out[1] == (127 << 24) | (0 << 16) | (31 << 8) | 127


def test_resolve_exposure(ref):
    """Exposure (the reference's commented-out :101-104) scales r, g, b after the division, before
    the clamp; alpha is untouched; 1.0 is the plain resolve."""
    acc = np.array([[1.0, 0.5, 0.1, 2.0], [0.2, 3.0, 0.0, 2.0]], dtype=np.float32)
    assert np.array_equal(ref.resolve_rgba8(acc, 2, 1.0), ref.resolve_rgba8(acc, 2))
    out = ref.resolve_rgba8(acc, 2, 1.5)
    c = lambda v: int(np.uint8(np.float32(min(max(np.float32(np.float32(v) / np.float32(2)) * np.float32(1.5), 0), 1)) * np.float32(255)))
    assert out[0] == (c(1.0) << 24) | (c(0.5) << 16) | (c(0.1) << 8) | 255
    assert out[1] == (c(0.2) << 24) | (c(3.0) << 16) | (0 << 8) | 255


def test_bvh_oracle_matches_flat(spt, ref):
    """The oracle's own BVH (used above 64 prims) returns exactly the flat closest hit."""
    p, m, e = spt.build_scene("bunnylike")
    flat = ref.RefScene(p[:64], m, e)       # 64 prims -> brute force in index order
    bvh = ref.RefScene(p[:65], m, e)        # 65 prims -> oracle BVH
    extra = ref.RefScene(p[64:65], m, e)    # the one extra primitive alone
    rng = np.random.default_rng(5)
    for _ in range(2000):
        o = rng.uniform([-2, -2, 3.5], [2, 2, 7.5]).astype(np.float32)
        d = rng.normal(size=3).astype(np.float32)
        a, b, c = flat.intersect(o, d), bvh.intersect(o, d), extra.intersect(o, d)
        # expected: closest of (flat hit, extra hit), ties to the lower index (the flat one)
        exp = a
        if c is not None and (a is None or c[0] < a[0]):
            exp = (c[0], 64, c[2])
        assert (b is None) == (exp is None)
        if b is not None:
            assert b[0] == exp[0] and b[1] == exp[1]
