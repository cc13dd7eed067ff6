"""CPU oracle: next-event estimation (SPT_FLAG_NEE; north_star's "BRDF + light sampling", SURVEY.md
§8a.6), no GPU.

The reference samples no lights (its bounce loop, CPUPathTracer.cpp:229-281, adds only the sky on a
miss), so the NEE integrator is this repo's superset and its parity with the reference binary is
unpinned. What is pinned here:
  1. ref_light_sample against an independent float32 numpy restatement, bit for bit (the draw order
     emitter / u / v, the uniform point on a parallelogram, a triangle or a sphere, the Lambertian
     estimate);
  2. the emitter table (which primitives are sampled) and the shadow ray's test on known geometry;
  3. the estimator: unbiased against the plain integrator on the same scene (statistically), and the
     flag without emitters is exactly the plain integrator.
"""
import math

import numpy as np
import pytest

from test_oracle_kat import py_random_float

f32 = np.float32
INV_PI = f32(0.318309886183790671538)


def py_light_sample(emitters, x, n, T, state):
    """ref_light_sample restated: emitters = list of (kind, base, e1, e2, Le) in primitive order (a
    sphere: ("sphere", center, radius, None, Le))."""
    dot = lambda a, b: (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]  # noqa: E731
    u0, state = py_random_float(state)
    u1, state = py_random_float(state)
    u2, state = py_random_float(state)
    ne = len(emitters)
    j = min(int(u0 * f32(ne)), ne - 1)
    kind, base, e1, e2, le = emitters[j]
    if kind == "sphere":
        c, r, le = np.asarray(base, np.float32), f32(e1), np.asarray(le, np.float32)
        wgt = ((((f32(4.0) * f32(math.pi)) * r) * r) * f32(ne)) * INV_PI
        z = f32(1.0) - f32(2.0) * u1
        sn = np.sqrt(f32(1.0) - z * z, dtype=np.float32)
        phi = (f32(2.0) * f32(math.pi)) * u2
        nl = np.array([f32(float(sn) * math.cos(float(phi))), f32(float(sn) * math.sin(float(phi))), z], np.float32)
        x = np.asarray(x, np.float32)
        v = np.array([(c[k] + r * nl[k]) - x[k] for k in range(3)], np.float32)
        d2 = dot(v, v)
        dist = np.sqrt(d2, dtype=np.float32)
        w = v * (f32(1.0) / dist)
        cs = dot(np.asarray(n, np.float32), w)
        xc = np.array([x[k] - c[k] for k in range(3)], np.float32)
        inside = dot(xc, xc) < r * r
        cl = dot(nl, w) if inside else -dot(nl, w)  # the side x sees: inside a dome, else outside
        if not (cs > 0 and cl > 0):
            return False, None, None, None, state
        g = ((cs * cl) * wgt) / d2
        add = np.array([f32(T[k]) * (le[k] * g) for k in range(3)], np.float32)
        return True, w, dist * f32(0.999), add, state
    base, e1, e2, le = (np.asarray(v, np.float32) for v in (base, e1, e2, le))
    if kind == "tri":
        e1, e2 = e1 - base, e2 - base
    nv = np.array([e1[1] * e2[2] - e2[1] * e1[2], e1[2] * e2[0] - e2[2] * e1[0], e1[0] * e2[1] - e2[0] * e1[1]],
                  np.float32)
    ln = np.sqrt(dot(nv, nv), dtype=np.float32)
    nl = nv * (f32(1.0) / ln)
    area = f32(0.5) * ln if kind == "tri" else ln
    wgt = (area * f32(ne)) * INV_PI
    a, b = u1, u2
    if kind == "tri":
        su = np.sqrt(u1, dtype=np.float32)
        a, b = su * (f32(1.0) - u2), su * u2
    x = np.asarray(x, np.float32)
    v = np.array([((base[k] + a * e1[k]) + b * e2[k]) - x[k] for k in range(3)], np.float32)
    d2 = dot(v, v)
    dist = np.sqrt(d2, dtype=np.float32)
    w = v * (f32(1.0) / dist)
    cs = dot(np.asarray(n, np.float32), w)
    cl = abs(dot(nl, w))
    if not (cs > 0 and cl > 0):
        return False, None, None, None, state
    g = ((cs * cl) * wgt) / d2
    add = np.array([f32(T[k]) * (le[k] * g) for k in range(3)], np.float32)
    return True, w, dist * f32(0.999), add, state


def cornell_emitters(spt, prims, mats):
    out = []
    for p in prims:
        le = mats[p["material"]]["emission"]
        if not le.any():
            continue
        if p["type"] == spt.PRIM_SPHERE:
            out.append(("sphere", p["p0"][:3], p["p0"][3], None, le))
            continue
        kind = "tri" if p["type"] == spt.PRIM_TRIANGLE else "quad"
        out.append((kind, p["p0"][:3], p["p1"][:3], p["p2"][:3], le))
    return out


@pytest.mark.parametrize("scene,count", [("c1", 0), ("app", 0), ("cornell", 1), ("bunnylike", 1)])
def test_emitter_table(spt, ref, scene, count):
    prims, mats, env = spt.build_scene(scene)
    assert ref.RefScene(prims, mats, env).emitter_count() == count


def test_light_sample_matches_restatement(spt, ref):
    """Bit-exact vs the numpy restatement on the Cornell light (a parallelogram) and a triangle pair."""
    prims, mats, env = spt.build_scene("cornell")
    tri = np.zeros(2, dtype=prims.dtype)
    mats2 = np.concatenate([mats, np.zeros(1, dtype=mats.dtype)])
    mats2[-1]["emission"] = (1.0, 2.0, 3.0)
    for i, (a, b, c) in enumerate([((-1, 1, 6), (0, 2, 6.5), (1, 1, 7)), ((2, -2, 4), (2, 0, 4), (2, -2, 6))]):
        tri[i]["type"] = spt.PRIM_TRIANGLE
        tri[i]["material"] = len(mats2) - 1
        tri[i]["p0"][:3], tri[i]["p1"][:3], tri[i]["p2"][:3] = a, b, c
    # an emissive sphere, one of radius 0 and a dome around the box (x inside it: its inner wall emits)
    sph = np.zeros(3, dtype=prims.dtype)
    for i, (c, r) in enumerate((((0.8, 1.2, 6.0), 0.45), ((-1.0, 0.0, 5.0), 0.0), ((0.0, 0.0, 5.0), 12.0))):
        sph[i]["type"] = spt.PRIM_SPHERE
        sph[i]["material"] = len(mats2) - 1
        sph[i]["p0"][:] = (*c, r)
    rng = np.random.default_rng(7)
    for scene_prims, scene_mats in ((prims, mats), (np.concatenate([prims, tri]), mats2),
                                    (np.concatenate([prims, sph, tri]), mats2)):
        rs = ref.RefScene(scene_prims, scene_mats, env)
        em = cornell_emitters(spt, scene_prims, scene_mats)
        assert rs.emitter_count() == len(em)
        n_ok = 0
        for _ in range(400):
            x = rng.uniform(-2.4, 2.4, 3).astype(np.float32)
            x[2] = f32(rng.uniform(3.1, 7.9))
            n = rng.normal(size=3).astype(np.float32)
            n = n * (f32(1.0) / np.sqrt(np.float32((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]), dtype=np.float32))
            T = rng.uniform(0.1, 1.0, 3).astype(np.float32)
            st = int(rng.integers(0, 2 ** 32))
            got = rs.light_sample(x, n, T, st)
            want = py_light_sample(em, x, n, T, st)
            assert got[0] == want[0] and got[4] == want[4]
            if want[0]:
                n_ok += 1
                assert np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32))
                assert np.float32(got[2]).view(np.uint32) == np.float32(want[2]).view(np.uint32)
                assert np.array_equal(got[3].view(np.uint32), want[3].view(np.uint32))
        assert n_ok > 50


def test_shadow_rays_on_known_geometry(spt, ref):
    prims, mats, env = spt.build_scene("cornell")
    rs = ref.RefScene(prims, mats, env)
    up = np.array([0, 1, 0], np.float32)
    # floor centre to the light's centre (0, 2.495, 5.5): open
    o = np.array([0.0, -2.4999, 5.5], np.float32)
    assert rs.visible(o, up, f32(4.9949) * f32(0.999))
    # under the sphere at (1, -1.7, 5): blocked
    assert not rs.visible(np.array([1.0, -2.4999, 5.0], np.float32), up, f32(4.99))
    # a short ray that stops before the sphere is not blocked
    assert rs.visible(np.array([1.0, -2.4999, 5.0], np.float32), up, f32(0.5))


def test_nee_without_emitters_is_the_plain_integrator(spt, ref):
    prims, mats, env = spt.build_scene("c1")
    rs = ref.RefScene(prims, mats, env)
    a = rs.render(48, 32, 0, 8, 4, 2, 0)
    b = rs.render(48, 32, 0, 8, 4, 2, ref.FLAG_NEE)
    assert rs.last_light_samples() == 0
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_nee_is_unbiased(spt, ref):
    """NEE and the plain integrator estimate the same image: batch means of the image sum (Cornell, sky
    off: the light carries the whole image) agree within 4 standard errors, and NEE's error is smaller."""
    prims, mats, env = spt.build_scene("cornell")
    env.sky_enabled = 0
    rs = ref.RefScene(prims, mats, env)
    w, h, fr, batches = 24, 14, 256, 8
    sums = {0: [], ref.FLAG_NEE: []}
    for flag in sums:
        for k in range(batches):
            acc = rs.render(w, h, 1000003 * k + (7 if flag else 0), fr, 6, 2, flag)
            sums[flag].append(acc[..., :3].sum(axis=(0, 1)) / fr)
    a, b = np.array(sums[0]), np.array(sums[ref.FLAG_NEE])
    se_a, se_b = a.std(0, ddof=1) / math.sqrt(batches), b.std(0, ddof=1) / math.sqrt(batches)
    z = np.abs(a.mean(0) - b.mean(0)) / np.sqrt(se_a ** 2 + se_b ** 2)
    print("plain", a.mean(0), se_a, "nee", b.mean(0), se_b, "z", z)
    assert np.all(z < 4.0), z
    assert np.all(se_b < se_a)


def sphere_lit_cornell(spt, center, radius, emission):
    """Cornell, sky off, the ceiling light switched off, lit by one emissive sphere."""
    prims, mats, env = spt.build_scene("cornell")
    env.sky_enabled = 0
    mats = np.concatenate([mats, np.zeros(2, dtype=mats.dtype)])
    mats[-2]["albedo"] = (0.7, 0.7, 0.7)  # the ceiling light, dark
    mats[-1]["albedo"] = (0.9, 0.9, 0.9)
    mats[-1]["emission"] = emission
    for p in prims:
        if mats[p["material"]]["emission"].any():
            p["material"] = len(mats) - 2
    sph = np.zeros(1, dtype=prims.dtype)
    sph[0]["type"] = spt.PRIM_SPHERE
    sph[0]["material"] = len(mats) - 1
    sph[0]["p0"][:] = (*center, radius)
    return np.concatenate([prims, sph]), mats, env


def nee_vs_plain(ref, rs, w=24, h=14, fr=256, batches=8):
    """Batch means of the image sum with and without NEE: (z scores, plain's and NEE's standard errors)."""
    sums = {0: [], ref.FLAG_NEE: []}
    for flag in sums:
        for k in range(batches):
            acc = rs.render(w, h, 1000003 * k + (7 if flag else 0), fr, 6, 2, flag)
            sums[flag].append(acc[..., :3].sum(axis=(0, 1)) / fr)
    a, b = np.array(sums[0]), np.array(sums[ref.FLAG_NEE])
    se_a, se_b = a.std(0, ddof=1) / math.sqrt(batches), b.std(0, ddof=1) / math.sqrt(batches)
    z = np.abs(a.mean(0) - b.mean(0)) / np.sqrt(se_a ** 2 + se_b ** 2)
    print("plain", a.mean(0), se_a, "nee", b.mean(0), se_b, "z", z)
    return z, se_a, se_b


def test_nee_sphere_light_is_unbiased(spt, ref):
    """A Cornell box lit only by an emissive sphere (the ceiling light switched off, sky off): NEE, which
    samples the sphere's area, and the plain integrator agree on the image sum within 4 standard errors."""
    rs = ref.RefScene(*sphere_lit_cornell(spt, (-0.6, 1.4, 5.2), 0.5, (6.0, 5.0, 4.0)))
    assert rs.emitter_count() == 1
    z, se_a, se_b = nee_vs_plain(ref, rs)
    assert np.all(z < 4.0), z
    assert np.all(se_b < se_a)


def test_nee_inside_an_emissive_sphere_is_unbiased(spt, ref):
    """The camera and the box inside a large emissive sphere (a dome, the only light): every point it
    samples is seen from inside, where its inner wall faces the hit point (sampling only the
    outward-facing side dropped every such sample, so the dome's light was lost after the camera
    segment). NEE and the plain integrator agree within 4 standard errors."""
    rs = ref.RefScene(*sphere_lit_cornell(spt, (0.0, 0.0, 5.0), 12.0, (0.6, 0.5, 0.4)))
    assert rs.emitter_count() == 1
    z, _, _ = nee_vs_plain(ref, rs)
    assert np.all(z < 4.0), z
