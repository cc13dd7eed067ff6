"""GPU: traversal stacks of deep, degenerate BVHs (the global stacks had a fixed 96-entry lane
stride with no bound check).

spt_set_scene now sizes the persistent kernels' global stacks by the tree's own bvh4_stack_need and
refuses a tree needing more than 96 entries (SPT_ERR_CAPACITY) — the per-lane scratch stacks of the
wavefront kernels hold 96. A chain of triangles doubling in size (SAH peels one off per level) needs 70
entries (tests/cpp/test_bvh.cpp); thousands of coincident triangles (no SAH split at all) need 34. Both
render bit-exact vs the oracle on every schedule, and no k_paths wave reaches its step bound
(spt_stats.stalled_waves, which spt_get_stats reports as an error).
Reference: rtcIntersect1, CPUPathTracer.cpp:214-227 (replaced by the BVH traversal).
"""
import numpy as np
import pytest

from test_gpu_configs import check

pytestmark = pytest.mark.gpu


def doubling_chain(spt, n=3000, z=5.0):
    p = np.zeros(n, dtype=spt.PRIM_DTYPE)
    for i in range(n):
        x = np.float32(np.ldexp(np.float32(1.0), i % 40 - 30) * np.float32(1 + i // 40))
        p[i]["type"] = spt.PRIM_TRIANGLE
        p[i]["p0"][:3] = (x, 0.0, z)
        p[i]["p1"][:3] = (2.0 * x, 0.0, z)
        p[i]["p2"][:3] = (x, x, z)
    return p


def coincident(spt, n=5000):
    p = np.zeros(n, dtype=spt.PRIM_DTYPE)
    p["type"] = spt.PRIM_TRIANGLE
    p["p0"][:, :3] = (-1.0, -1.0, 4.0)
    p["p1"][:, :3] = (1.0, -1.0, 4.5)
    p["p2"][:, :3] = (0.0, 1.0, 4.0)
    return p


@pytest.mark.parametrize("kind,need", [("chain", 70), ("coincident", 34)])
def test_deep_trees_on_every_schedule(spt, ref, gpu_ctx, kind, need):
    prims = doubling_chain(spt) if kind == "chain" else coincident(spt)
    mats, env = spt.reference_materials(), spt.reference_env()
    w, h, frames = 96, 64, 4
    rs = ref.RefScene(prims, mats, env)
    r = rs.render(w, h, 0, frames, 4, 2, 0)
    for flags, per_call in ((0, frames), (0, 1), (spt.FLAG_SPLIT_KERNELS, frames)):
        gpu_ctx.set_tuning()
        gpu_ctx.set_scene(prims, mats, env)
        gpu_ctx.configure(w, h, 4, 2, flags)
        for f in range(0, frames, per_call):
            gpu_ctx.render(f, per_call)
        st = gpu_ctx.stats()  # (raises if a wave stopped at its step bound)
        print(f"{kind}: stack need {st.stack_need} (host test_bvh: {need}), stack bytes {st.stack_bytes}")
        assert need - 8 <= st.stack_need <= 96 and st.stalled_waves == 0
        assert st.stack_bytes > 0
        check(gpu_ctx.read_accum().reshape(h, w, 4), r, frames, f"{kind} flags={flags} per_call={per_call}")
