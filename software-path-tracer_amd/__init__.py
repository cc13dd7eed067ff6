"""software-path-tracer_amd — MI355X (gfx950) path-tracing integrator, Python host side.

Binds the C-ABI of ``libspt_hip.so`` (``include/spt.h``) with ctypes and mirrors the reference's
backend interface ``render::PathTracer`` (reference ``libs/render/include/render/PathTracer.h:13-51``)
so that tests and ``bench.py`` read like the reference's own call sites (``src/App.cpp:98-133``,
``src/App.cpp:230-240``). The production host side is C++ (``csrc/HIPPathTracer.cpp``); this module is
the Python plumbing around the same C-ABI.

There is no CPU fallback: if ``libspt_hip.so`` is missing or no gfx950 device is usable, the calls
raise. The CPU oracle under ``oracle/`` is test infrastructure and is never imported from here.

Import with ``importlib.import_module("software-path-tracer_amd")`` (the directory name is not a
Python identifier).
"""
from __future__ import annotations

import ctypes
import enum
import os
from typing import Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPT_LIB_PATH") or os.path.join(_HERE, "libspt_hip.so")  # override: experiments only
RENDER_LIB_PATH = os.path.join(_HERE, "libspt_render.so")

# ---------------------------------------------------------------------------------------------
# C types (must match include/spt.h)
# ---------------------------------------------------------------------------------------------
SPT_OK = 0
SPT_ERR = {
    -1: "SPT_ERR_INVALID",
    -2: "SPT_ERR_HIP",
    -3: "SPT_ERR_NO_DEVICE",
    -4: "SPT_ERR_NO_SCENE",
    -5: "SPT_ERR_NOT_CONFIGURED",
    -6: "SPT_ERR_CAPACITY",
}

PRIM_SPHERE, PRIM_QUAD, PRIM_TRIANGLE = 0, 1, 2
FLAG_ABS_FLOAT = 1
FLAG_SPLIT_KERNELS = 2  # separate extend (closest hit) and shade launches per bounce
FLAG_WAVEFRONT = 4      # flat scenes: keep the wavefront schedule (no persistent k_paths launch)
FLAG_SORTED_RAYS = 1 << 3  # SPT_FLAG_SORTED_RAYS: BVH scenes, wavefront with binned (sorted) ray queues
FLAG_NEE = 1 << 4  # SPT_FLAG_NEE: next-event estimation (light sampling; superset of the reference)
SCHEDULE_SPLIT, SCHEDULE_FUSED, SCHEDULE_PERSISTENT, SCHEDULE_FRAME = 0, 1, 2, 3  # spt_stats.schedule
PERSISTENT_MIN_FRAMES = 4  # SPT_PERSISTENT_MIN_FRAMES
PROFILE_EVENTS, PROFILE_COUNTERS, PROFILE_SPAN = 1, 2, 4  # spt_set_profiling modes

SCENE_C1_SPHERE_GROUND = 0
SCENE_APP_DEFAULT = 1
SCENE_CORNELL = 2
SCENE_BUNNYLIKE = 3
SCENE_INTERIOR_1M = 4
SCENE_IDS = {
    "c1": SCENE_C1_SPHERE_GROUND,
    "app": SCENE_APP_DEFAULT,
    "cornell": SCENE_CORNELL,
    "bunnylike": SCENE_BUNNYLIKE,
    "interior1m": SCENE_INTERIOR_1M,
}

PRIM_DTYPE = np.dtype(
    [("type", "<u4"), ("material", "<u4"), ("reserved", "<u4", (2,)), ("p0", "<f4", (4,)), ("p1", "<f4", (4,)),
     ("p2", "<f4", (4,))],
    align=False,
)
MATERIAL_DTYPE = np.dtype([("albedo", "<f4", (3,)), ("emission", "<f4", (3,))])
assert PRIM_DTYPE.itemsize == 64 and MATERIAL_DTYPE.itemsize == 24


class SptEnv(ctypes.Structure):
    _fields_ = [("sky_enabled", ctypes.c_uint32), ("horizon", ctypes.c_float * 3), ("zenith", ctypes.c_float * 3)]


class SptConfig(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("max_bounces", ctypes.c_uint32),
        ("rr_depth", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("shard_rank", ctypes.c_uint32),
        ("shard_count", ctypes.c_uint32),
        ("frames_in_flight", ctypes.c_uint32),
    ]


SPT_MAX_BOUNCES = 32


class SptStats(ctypes.Structure):
    _fields_ = [
        ("frames", ctypes.c_uint64),
        ("paths", ctypes.c_uint64),
        ("segments", ctypes.c_uint64 * SPT_MAX_BOUNCES),
        ("segments_total", ctypes.c_uint64),
        ("passes", ctypes.c_uint64),
        ("extend_launches", ctypes.c_uint64),
        ("extend_ms", ctypes.c_double),
        ("extend_segments", ctypes.c_uint64),
        ("shade_launches", ctypes.c_uint64),
        ("shade_ms", ctypes.c_double),
        ("other_ms", ctypes.c_double),
        ("extend_ms_bounce", ctypes.c_double * SPT_MAX_BOUNCES),
        ("shade_ms_bounce", ctypes.c_double * SPT_MAX_BOUNCES),
        ("bvh_nodes", ctypes.c_uint64),
        ("scene_bytes", ctypes.c_uint64),
        ("radiance_updates", ctypes.c_uint64 * SPT_MAX_BOUNCES),
        ("tail_ms", ctypes.c_double),
        ("tail_launches", ctypes.c_uint64),
        ("tail_bounce", ctypes.c_uint64),
        ("fused", ctypes.c_uint64),
        ("persistent_ms", ctypes.c_double),
        ("persistent_launches", ctypes.c_uint64),
        ("schedule", ctypes.c_uint64),
        ("lane_slots", ctypes.c_uint64),
        ("lane_busy", ctypes.c_uint64),
        ("bvh_node_visits", ctypes.c_uint64),
        ("prim_tests", ctypes.c_uint64),
        ("flat_fast_path", ctypes.c_uint64),
        ("specialized", ctypes.c_uint64),
        ("shadow_rays", ctypes.c_uint64),
        ("emitters", ctypes.c_uint64),
        ("stack_bytes", ctypes.c_uint64),
        ("stack_need", ctypes.c_uint64),
        ("stalled_waves", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        d = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            d[k] = list(v) if isinstance(v, ctypes.Array) else v
        return d


# Every symbol include/spt.h declares (checked by tests/test_capi_symbols.py).
EXPORTED_SYMBOLS = (
    "spt_abi_version", "spt_device_count", "spt_create", "spt_destroy", "spt_last_error", "spt_set_stream",
    "spt_set_scene", "spt_configure", "spt_reset", "spt_get_frame_count", "spt_render", "spt_synchronize",
    "spt_shard_pixels", "spt_read_accum", "spt_accum_device_ptr", "spt_copy_accum_device", "spt_resolve_rgba8",
    "spt_resolve_rgba8_exposure", "spt_register_host_output", "spt_render_resolve_rgba8", "spt_assemble_rows",
    "spt_set_profiling", "spt_get_stats", "spt_stats_clear", "spt_build_scene",
    "spt_set_env_map", "spt_env_octa_from_equirect",
    "spt_comm_available", "spt_comm_unique_id", "spt_comm_init", "spt_gather_image", "spt_gather_image_overlapped", "spt_gather_wait",
    "spt_comm_destroy", "spt_set_tuning",
    "spt_specialize_scene", "spt_compile_flat_kernels", "spt_update_prims",
)
COMM_ID_BYTES = 128  # SPT_COMM_ID_BYTES


class SptTuning(ctypes.Structure):
    """spt_tuning: schedule knobs for measurement and tests (0 / -1 = automatic; results never change)."""
    _fields_ = [
        ("fused", ctypes.c_int32),
        ("tail_bounce", ctypes.c_uint32),
        ("persistent", ctypes.c_int32),
        ("frame_kernel", ctypes.c_int32),
        ("chunks_per_wave", ctypes.c_uint32),
        ("px_shift", ctypes.c_uint32),
        ("subqueues", ctypes.c_uint32),
        ("bvh_max_leaf", ctypes.c_uint32),
        ("bvh_bins", ctypes.c_uint32),
        ("specialize", ctypes.c_int32),
    ]

    def __init__(self, **kw):
        super().__init__(fused=-1, persistent=-1, frame_kernel=-1)
        for k, v in kw.items():
            if k not in dict(self._fields_):
                raise TypeError(f"unknown spt_tuning field {k}")
            setattr(self, k, v)

_lib: Optional[ctypes.CDLL] = None


class SptError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libspt_hip.so. Raises loudly if it is missing — there is no fallback path."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SptError(f"libspt_hip.so not built at {path} (run `make` or __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    P, U32, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    sig = {
        "spt_abi_version": ([], I),
        "spt_device_count": ([ctypes.POINTER(I)], I),
        "spt_create": ([ctypes.POINTER(P), I], I),
        "spt_destroy": ([P], None),
        "spt_last_error": ([P], ctypes.c_char_p),
        "spt_set_stream": ([P, P], I),
        "spt_set_scene": ([P, P, U32, P, U32, ctypes.POINTER(SptEnv)], I),
        "spt_configure": ([P, ctypes.POINTER(SptConfig)], I),
        "spt_reset": ([P], I),
        "spt_get_frame_count": ([P, ctypes.POINTER(U32)], I),
        "spt_render": ([P, U32, U32], I),
        "spt_synchronize": ([P], I),
        "spt_shard_pixels": ([P, ctypes.POINTER(ctypes.c_uint64)], I),
        "spt_read_accum": ([P, P], I),
        "spt_accum_device_ptr": ([P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)], I),
        "spt_copy_accum_device": ([P, P], I),
        "spt_resolve_rgba8": ([P, U32, P], I),
        "spt_resolve_rgba8_exposure": ([P, U32, ctypes.c_float, P], I),
        "spt_register_host_output": ([P, P, ctypes.c_size_t], I),
        "spt_render_resolve_rgba8": ([P, U32, U32, U32, ctypes.c_float, P], I),
        "spt_assemble_rows": ([P, P, P], I),
        "spt_set_profiling": ([P, I], I),
        "spt_set_env_map": ([P, P, U32, U32], I),
        "spt_env_octa_from_equirect": ([P, U32, U32, P, U32, U32], I),
        "spt_get_stats": ([P, ctypes.POINTER(SptStats)], I),
        "spt_stats_clear": ([P], I),
        "spt_build_scene": ([U32, P, ctypes.POINTER(U32), P, ctypes.POINTER(U32), ctypes.POINTER(SptEnv)], I),
        "spt_comm_available": ([], I),
        "spt_comm_unique_id": ([P], I),
        "spt_comm_init": ([P, P, I, I], I),
        "spt_gather_image": ([P, P], I),
        "spt_gather_image_overlapped": ([P, P], I),
        "spt_gather_wait": ([P], I),
        "spt_comm_destroy": ([P], I),
        "spt_set_tuning": ([P, ctypes.POINTER(SptTuning)], I),
        "spt_specialize_scene": ([P], I),
        "spt_update_prims": ([P, P, P, U32], I),
        "spt_compile_flat_kernels": ([P, U32, I, ctypes.c_char_p, ctypes.c_size_t], I),
    }
    for name, (args, res) in sig.items():
        if os.environ.get("SPT_LIB_PATH") and not hasattr(lib, name):
            continue  # an experiment library built from an older source (A/B runs only)
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def reference_env(sky: bool = True) -> SptEnv:
    """Reference sky gradient (CPUPathTracer.cpp:286-292)."""
    e = SptEnv()
    e.sky_enabled = 1 if sky else 0
    e.horizon[:] = (1.0, 1.0, 1.0)
    e.zenith[:] = (0.5, 0.7, 1.0)
    return e


def env_octa_from_equirect(equirect_rgb: np.ndarray, width: int, height: int) -> np.ndarray:
    """Resample an equirectangular (h, w, 3) float image into a (height, width, 4) octahedral map
    (spt_env_octa_from_equirect; host-only)."""
    src = np.ascontiguousarray(equirect_rgb, dtype=np.float32)
    dst = np.zeros((height, width, 4), dtype=np.float32)
    rc = load_library().spt_env_octa_from_equirect(src.ctypes.data, src.shape[1], src.shape[0], dst.ctypes.data,
                                                   width, height)
    if rc != 0:
        raise SptError(f"spt_env_octa_from_equirect: {rc}")
    return dst


def synthetic_env_map(size: int = 512, seed: int = 0x5eed) -> np.ndarray:
    """A deterministic HDR sky for tests and the bench (no image files offline): an equirectangular
    gradient with a bright sun disk and seeded noise, resampled to a size x size octahedral map."""
    h, w = size // 2, size
    theta = (np.arange(h, dtype=np.float64) + 0.5) / h * np.pi
    phi = (np.arange(w, dtype=np.float64) + 0.5) / w * 2 * np.pi - np.pi
    th, ph = np.meshgrid(theta, phi, indexing="ij")
    y = np.cos(th)
    base = np.stack([0.6 + 0.4 * y, 0.7 + 0.3 * y, 1.0 + 0.2 * y], axis=-1)
    sun = np.exp(-((th - 0.6) ** 2 + (ph - 0.8) ** 2) / 0.002)[..., None] * np.array([40.0, 36.0, 30.0])
    ground = (y < 0)[..., None] * np.array([-0.3, -0.35, -0.5])
    noise = np.random.default_rng(seed).uniform(0.0, 0.05, size=(h, w, 1))
    equirect = np.maximum(base + sun + ground + noise, 0.0).astype(np.float32)
    return env_octa_from_equirect(equirect, size, size)


def build_scene(scene: "int | str") -> Tuple[np.ndarray, np.ndarray, SptEnv]:
    """Deterministic synthetic scene (host-only, no GPU): (prims, materials, env)."""
    lib = load_library()
    sid = SCENE_IDS[scene] if isinstance(scene, str) else int(scene)
    n_p, n_m = ctypes.c_uint32(0), ctypes.c_uint32(0)
    env = SptEnv()
    rc = lib.spt_build_scene(sid, None, ctypes.byref(n_p), None, ctypes.byref(n_m), ctypes.byref(env))
    if rc != SPT_OK:
        raise SptError(f"spt_build_scene({sid}) -> {SPT_ERR.get(rc, rc)}")
    prims = np.zeros(n_p.value, dtype=PRIM_DTYPE)
    mats = np.zeros(n_m.value, dtype=MATERIAL_DTYPE)
    rc = lib.spt_build_scene(sid, _ptr(prims), ctypes.byref(n_p), _ptr(mats), ctypes.byref(n_m), ctypes.byref(env))
    if rc != SPT_OK:
        raise SptError(f"spt_build_scene({sid}) -> {SPT_ERR.get(rc, rc)}")
    return prims, mats, env


def compile_flat_kernels(prims: np.ndarray, env_map: bool = False) -> None:
    """spt_compile_flat_kernels (host only, no GPU): compile the persistent kernels specialized to
    the flat scene's shape into the process cache; raises with the compiler log on failure."""
    prims = np.ascontiguousarray(prims, dtype=PRIM_DTYPE)
    log = ctypes.create_string_buffer(1 << 16)
    rc = load_library().spt_compile_flat_kernels(_ptr(prims), len(prims), 1 if env_map else 0, log, len(log))
    if rc != SPT_OK:
        raise SptError(f"spt_compile_flat_kernels -> {SPT_ERR.get(rc, rc)}: {log.value.decode(errors='replace')}")


def sphere_prims(spheres: Sequence[Tuple[float, float, float, float]], material: int = 0) -> np.ndarray:
    p = np.zeros(len(spheres), dtype=PRIM_DTYPE)
    for i, (x, y, z, r) in enumerate(spheres):
        p[i]["type"] = PRIM_SPHERE
        p[i]["material"] = material
        p[i]["p0"] = (x, y, z, r)
    return p


def reference_materials() -> np.ndarray:
    """Reference mode: one gray Lambertian, throughput *= 0.7 (CPUPathTracer.cpp:260)."""
    m = np.zeros(1, dtype=MATERIAL_DTYPE)
    m[0]["albedo"] = (0.7, 0.7, 0.7)
    return m


class Context:
    """RAII wrapper of one spt_ctx (one HIP device)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.spt_create(ctypes.byref(h), device)
        if rc != SPT_OK:
            raise SptError(f"spt_create(device={device}) -> {SPT_ERR.get(rc, rc)} (needs a gfx950 GPU)")
        self.h = h
        self.width = self.height = 0
        self.cfg = SptConfig()
        self._out_reg = None  # the array registered by register_host_output

    def _check(self, rc: int, what: str) -> None:
        if rc != SPT_OK:
            msg = self.lib.spt_last_error(self.h)
            raise SptError(f"{what} -> {SPT_ERR.get(rc, rc)}: {msg.decode() if msg else ''}")

    def close(self) -> None:
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.spt_destroy(self.h)  # (unregisters the host output first)
            self.h = ctypes.c_void_p()
            self._out_reg = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_scene(self, prims: np.ndarray, mats: np.ndarray, env: SptEnv) -> None:
        prims = np.ascontiguousarray(prims, dtype=PRIM_DTYPE)
        mats = np.ascontiguousarray(mats, dtype=MATERIAL_DTYPE)
        self._check(self.lib.spt_set_scene(self.h, _ptr(prims), len(prims), _ptr(mats), len(mats), ctypes.byref(env)),
                    "spt_set_scene")

    def update_prims(self, indices, prims: np.ndarray) -> None:
        """spt_update_prims: replace primitives `indices` of the current scene (BVH: refit, no rebuild)."""
        idx = np.ascontiguousarray(indices, dtype=np.uint32)
        prims = np.ascontiguousarray(prims, dtype=PRIM_DTYPE)
        if len(idx) != len(prims):
            raise ValueError("indices and prims differ in length")
        self._check(self.lib.spt_update_prims(self.h, _ptr(idx), _ptr(prims), len(idx)), "spt_update_prims")

    def configure(self, width: int, height: int, max_bounces: int = 4, rr_depth: int = 2, flags: int = 0,
                  shard_rank: int = 0, shard_count: int = 1, frames_in_flight: int = 0) -> None:
        c = SptConfig(width, height, max_bounces, rr_depth, flags, shard_rank, shard_count, frames_in_flight)
        self._check(self.lib.spt_configure(self.h, ctypes.byref(c)), "spt_configure")
        self.cfg = c
        self.width, self.height = width, height

    def set_stream(self, hip_stream: int) -> None:
        self._check(self.lib.spt_set_stream(self.h, ctypes.c_void_p(hip_stream or 0)), "spt_set_stream")

    def reset(self) -> None:
        self._check(self.lib.spt_reset(self.h), "spt_reset")

    @property
    def frame_count(self) -> int:
        v = ctypes.c_uint32()
        self._check(self.lib.spt_get_frame_count(self.h, ctypes.byref(v)), "spt_get_frame_count")
        return v.value

    def render(self, first_frame: int, n_frames: int = 1) -> None:
        self._check(self.lib.spt_render(self.h, first_frame, n_frames), "spt_render")

    def synchronize(self) -> None:
        self._check(self.lib.spt_synchronize(self.h), "spt_synchronize")

    @property
    def shard_pixels(self) -> int:
        v = ctypes.c_uint64()
        self._check(self.lib.spt_shard_pixels(self.h, ctypes.byref(v)), "spt_shard_pixels")
        return v.value

    def read_accum(self) -> np.ndarray:
        out = np.zeros((self.shard_pixels, 4), dtype=np.float32)
        self._check(self.lib.spt_read_accum(self.h, _ptr(out)), "spt_read_accum")
        return out

    def accum_device_ptr(self) -> Tuple[int, int]:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(self.lib.spt_accum_device_ptr(self.h, ctypes.byref(p), ctypes.byref(n)), "spt_accum_device_ptr")
        return p.value or 0, n.value

    def copy_accum_device(self, dst_dev_ptr: int) -> None:
        self._check(self.lib.spt_copy_accum_device(self.h, ctypes.c_void_p(dst_dev_ptr)), "spt_copy_accum_device")

    def register_host_output(self, out: Optional[np.ndarray]) -> None:
        """spt_register_host_output: `out` (uint32, C-contiguous, >= shard_pixels) becomes the page-locked,
        GPU-mapped image buffer that resolve_rgba8(out=out) has the resolve kernel write directly; None
        unregisters. The Context keeps a reference to it while registered."""
        if out is None:
            self._check(self.lib.spt_register_host_output(self.h, None, 0), "spt_register_host_output")
            self._out_reg = None
            return
        if out.dtype != np.uint32 or not out.flags["C_CONTIGUOUS"] or out.size < self.shard_pixels:
            raise SptError("register_host_output: need a C-contiguous uint32 array of >= shard_pixels")
        self._check(self.lib.spt_register_host_output(self.h, _ptr(out), out.nbytes), "spt_register_host_output")
        self._out_reg = out

    def resolve_rgba8(self, frame_count: int, exposure: float = 1.0, out: Optional[np.ndarray] = None) -> np.ndarray:
        if out is None:
            out = np.zeros(self.shard_pixels, dtype=np.uint32)
        elif out.dtype != np.uint32 or not out.flags["C_CONTIGUOUS"] or out.size < self.shard_pixels:
            raise SptError("resolve_rgba8: out must be a C-contiguous uint32 array of >= shard_pixels")
        if exposure == 1.0:
            self._check(self.lib.spt_resolve_rgba8(self.h, frame_count, _ptr(out)), "spt_resolve_rgba8")
        else:
            self._check(self.lib.spt_resolve_rgba8_exposure(self.h, frame_count, exposure, _ptr(out)),
                        "spt_resolve_rgba8_exposure")
        return out

    def render_resolve_rgba8(self, first_frame: int, n_frames: int, frame_count: int, exposure: float = 1.0,
                             out: Optional[np.ndarray] = None) -> np.ndarray:
        """spt_render_resolve_rgba8: render(first_frame, n_frames), then resolve_rgba8(frame_count, exposure,
        out) — fused into the last frame's launch when `out` is the registered buffer and the call runs
        k_frame (the App's render() + get_render_result(), App.cpp:230-240)."""
        if out is None:
            out = np.zeros(self.shard_pixels, dtype=np.uint32)
        elif out.dtype != np.uint32 or not out.flags["C_CONTIGUOUS"] or out.size < self.shard_pixels:
            raise SptError("render_resolve_rgba8: out must be a C-contiguous uint32 array of >= shard_pixels")
        self._check(self.lib.spt_render_resolve_rgba8(self.h, first_frame, n_frames, frame_count, exposure, _ptr(out)),
                    "spt_render_resolve_rgba8")
        return out

    def assemble_rows(self, gathered_dev_ptr: int, out_dev_ptr: int) -> None:
        self._check(self.lib.spt_assemble_rows(self.h, ctypes.c_void_p(gathered_dev_ptr), ctypes.c_void_p(out_dev_ptr)),
                    "spt_assemble_rows")

    def set_tuning(self, **kw) -> None:
        """spt_set_tuning with the given SptTuning fields (the others automatic)."""
        self._check(self.lib.spt_set_tuning(self.h, ctypes.byref(SptTuning(**kw))), "spt_set_tuning")

    def specialize_scene(self) -> None:
        """spt_specialize_scene: compile and load the flat scene's shape-specialized kernels now."""
        self._check(self.lib.spt_specialize_scene(self.h), "spt_specialize_scene")

    def comm_init(self, comm_id: bytes, n_ranks: int, rank: int) -> None:
        """Join the RCCL communicator `comm_id` (from comm_unique_id() on rank 0) as rank / n_ranks."""
        if len(comm_id) != COMM_ID_BYTES:
            raise ValueError("communicator id must be 128 bytes")
        buf = ctypes.create_string_buffer(bytes(comm_id), COMM_ID_BYTES)
        self._check(self.lib.spt_comm_init(self.h, buf, n_ranks, rank), "spt_comm_init")

    def gather_image(self, root_image_dev_ptr: int = 0) -> None:
        """Collective: the ranks' row shards gathered to rank 0 over RCCL and assembled into the full
        float RGBA image at root_image_dev_ptr (device memory, rank 0; ignored elsewhere)."""
        self._check(self.lib.spt_gather_image(self.h, ctypes.c_void_p(root_image_dev_ptr or 0)), "spt_gather_image")

    def gather_image_overlapped(self, root_image_dev_ptr: int = 0) -> None:
        """spt_gather_image_overlapped: the same collective on the ctx's own comm stream, from a snapshot
        of the shard taken now, so that the next render() calls overlap it; gather_wait() orders the
        integrator's stream after it (root_image then holds the frames rendered before this call)."""
        self._check(self.lib.spt_gather_image_overlapped(self.h, ctypes.c_void_p(root_image_dev_ptr or 0)),
                    "spt_gather_image_overlapped")

    def gather_wait(self) -> None:
        self._check(self.lib.spt_gather_wait(self.h), "spt_gather_wait")

    def comm_destroy(self) -> None:
        self._check(self.lib.spt_comm_destroy(self.h), "spt_comm_destroy")

    def set_env_map(self, rgba: Optional[np.ndarray]) -> None:
        """Octahedral environment map (h, w, 4) float32 for the miss radiance, or None for the
        gradient sky (spt_set_env_map; resets the accumulation)."""
        if rgba is None:
            self._check(self.lib.spt_set_env_map(self.h, None, 0, 0), "spt_set_env_map")
            return
        a = np.ascontiguousarray(rgba, dtype=np.float32)
        if a.ndim != 3 or a.shape[2] != 4:
            raise ValueError("environment map must be (height, width, 4) float32")
        self._env_keep = a
        self._check(self.lib.spt_set_env_map(self.h, a.ctypes.data, a.shape[1], a.shape[0]), "spt_set_env_map")

    def set_profiling(self, enable, counters: bool = False, span: bool = False) -> None:
        """enable: HIP-event timing of every launch; counters: k_paths also counts segments per
        bounce (a slower kernel variant; the wavefront schedules always count); span: instead of
        per-launch events, one event pair around all k_paths / k_frame launches until profiling is
        switched off (SPT_PROFILE_SPAN; only with enable)."""
        mode = (PROFILE_EVENTS if enable and not span else 0) | (PROFILE_COUNTERS if counters else 0) | \
            (PROFILE_SPAN if span and enable else 0)
        self._check(self.lib.spt_set_profiling(self.h, mode), "spt_set_profiling")

    def stats(self) -> SptStats:
        s = SptStats()
        self._check(self.lib.spt_get_stats(self.h, ctypes.byref(s)), "spt_get_stats")
        return s

    def clear_stats(self) -> None:
        self._check(self.lib.spt_stats_clear(self.h), "spt_stats_clear")


def comm_available() -> bool:
    """True if this process can reach RCCL (spt_comm_available: symbols resolved; nothing created)."""
    return load_library().spt_comm_available() == SPT_OK


def comm_unique_id() -> bytes:
    """A new RCCL communicator id (rank 0; share it with the other ranks out of band)."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    rc = load_library().spt_comm_unique_id(buf)
    if rc != SPT_OK:
        raise SptError(f"spt_comm_unique_id -> {SPT_ERR.get(rc, rc)}")
    return buf.raw


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int()
    lib.spt_device_count(ctypes.byref(n))
    return n.value


# ---------------------------------------------------------------------------------------------
# Mirror of the reference interface (PathTracer.h:13-51, Types.h:43-95, Scene.h:123-227)
# ---------------------------------------------------------------------------------------------
class BackendType(enum.IntEnum):
    """PathTracer::BackendType (PathTracer.h:16-21) + the new GPU_HIP backend."""

    CPU_EMBREE = 0
    GPU_OPTIX = 1
    GPU_METAL = 2
    GPU_HIP = 3


class RenderSettings:
    """render::RenderSettings with its dirty flag (Types.h:43-95, RenderSettings.cpp:5-54)."""

    def __init__(self):
        self._width, self._height = 512, 512
        self._progressive = True
        self._spp, self._max_bounces, self._rr_depth = 64, 8, 3
        self._exposure = 1.0
        self._dirty = True  # dirty on construction

    def _set(self, name, value):
        if getattr(self, name) != value:
            setattr(self, name, value)
            self._dirty = True

    def setResolution(self, width: int, height: int) -> None:
        if (self._width, self._height) != (width, height):
            self._width, self._height = width, height
            self._dirty = True

    def setProgressive(self, v: bool) -> None:
        self._set("_progressive", v)

    def setSamplesPerPixel(self, v: int) -> None:
        self._set("_spp", v)

    def setMaxBounces(self, v: int) -> None:
        self._set("_max_bounces", v)

    def setRussianRouletteDepth(self, v: int) -> None:
        self._set("_rr_depth", v)

    def setExposure(self, v: float) -> None:
        self._set("_exposure", v)

    def getProgressive(self) -> bool:
        return self._progressive

    def getWidth(self) -> int:
        return self._width

    def getHeight(self) -> int:
        return self._height

    def getSamplesPerPixel(self) -> int:
        return self._spp

    def getMaxBounces(self) -> int:
        return self._max_bounces

    def getRussianRouletteDepth(self) -> int:
        return self._rr_depth

    def getExposure(self) -> float:
        return self._exposure

    def isDirty(self) -> bool:
        return self._dirty

    def clearDirty(self) -> None:
        self._dirty = False


class SphereObject:
    """render::SphereObject (Scene.h:123-133): position + radius."""

    def __init__(self, name: str = "Sphere"):
        self.name = name
        self.position = (0.0, 0.0, 0.0)
        self.radius = 1.0

    def SetPosition(self, p) -> None:
        self.position = tuple(float(v) for v in p)

    def SetRadius(self, r: float) -> None:
        self.radius = float(r)

    def GetPosition(self):
        return self.position

    def GetRadius(self) -> float:
        return self.radius


class Scene:
    """render::Scene (Scene.h:135-227): node registry + change flag."""

    def __init__(self):
        self._nodes = []
        self._has_changes = True

    def CreateNode(self, cls=SphereObject, name: str = "Sphere"):
        n = cls(name)
        self._nodes.append(n)
        return n

    def GetAllNodes(self):
        return list(self._nodes)

    def hasChanges(self) -> bool:
        return self._has_changes

    def markChangesProcessed(self) -> None:
        self._has_changes = False


class RenderResult:
    """PathTracer::RenderResult (PathTracer.h:23-28): RGBA8888 u32 per pixel, R in the high byte."""

    def __init__(self):
        self.image_buffer = np.zeros(0, dtype=np.uint32)
        self.width = 0
        self.height = 0


class PathTracer:
    """Abstract render::PathTracer (PathTracer.h:13-51)."""

    BackendType = BackendType

    @staticmethod
    def create_path_tracer(backend: BackendType) -> "PathTracer":
        # PathTracer.cpp:9-22; the reference's CPU_EMBREE backend is not part of this build
        if backend == BackendType.GPU_HIP:
            return HIPPathTracer()
        raise RuntimeError("Unknown backend type")


class HIPPathTracer(PathTracer):
    """GPU_HIP backend with CPUPathTracer's progressive-state semantics (CPUPathTracer.cpp:43-161).

    Reference mode (default): spheres of the Scene, albedo 0.7, sky on, 4 bounces, RR after bounce 2,
    one sample per pixel per render(); RenderSettings other than the resolution are ignored, as
    CPUPathTracer ignores them (CPUPathTracer.cpp:199, :264, :101-104).

    settings_mode=True honours RenderSettings instead: getMaxBounces,
    getRussianRouletteDepth, getSamplesPerPixel (frames traced per render() call — one spt_render
    call, so 64 spp run the persistent k_paths schedule), getProgressive (False: every render()
    starts a fresh accumulation) and getExposure (applied in the resolve).
    """

    def __init__(self, device: int = 0, max_bounces: int = 4, rr_depth: int = 2, flags: int = 0,
                 settings_mode: bool = False):
        self._ctx = Context(device)
        self._scene: Optional[Scene] = None
        self._settings = RenderSettings()
        self._result = RenderResult()
        self._frame_count = 0
        self._max_bounces, self._rr_depth, self._flags = max_bounces, rr_depth, flags
        self._settings_mode = settings_mode

    def set_scene(self, scene: Scene) -> None:
        self._scene = scene

    def set_settings(self, settings: RenderSettings) -> None:
        self._settings = settings

    def get_scene(self) -> Optional[Scene]:
        return self._scene

    def get_settings(self) -> RenderSettings:
        return self._settings

    def get_backend_name(self) -> str:
        return "GPU Path Tracer (HIP, gfx950)"

    def get_backend_type(self) -> BackendType:
        return BackendType.GPU_HIP

    def _invalidate(self) -> None:
        # CPUPathTracer.cpp:119-161
        needs_rebuild = False
        if self._scene.hasChanges():
            self._frame_count = 0
            needs_rebuild = True
        size_changed = (self._result.width, self._result.height) != (self._settings.getWidth(),
                                                                     self._settings.getHeight())
        if self._settings.isDirty() or size_changed:
            self._frame_count = 0
            self._settings.clearDirty()
            self._result.width, self._result.height = self._settings.getWidth(), self._settings.getHeight()
            bounces, rr = self._max_bounces, self._rr_depth
            if self._settings_mode:
                bounces, rr = self._settings.getMaxBounces(), self._settings.getRussianRouletteDepth()
            self._ctx.configure(self._result.width, self._result.height, bounces, rr, self._flags)
        if self._frame_count == 0:
            self._ctx.reset()
        if needs_rebuild:
            spheres = [(*n.GetPosition(), n.GetRadius()) for n in self._scene.GetAllNodes()
                       if isinstance(n, SphereObject)]
            self._ctx.set_scene(sphere_prims(spheres), reference_materials(), reference_env(True))
            self._scene.markChangesProcessed()

    def render(self) -> None:
        if self._scene is None:
            raise SptError("Scene not set before rendering")  # verify, CPUPathTracer.cpp:46
        if self._settings_mode and not self._settings.getProgressive():
            self._frame_count = 0  # a fresh accumulation every call
        self._invalidate()
        n = max(1, self._settings.getSamplesPerPixel()) if self._settings_mode else 1
        self._ctx.render(self._frame_count, n)
        self._frame_count += n

    def get_render_result(self) -> RenderResult:
        if self._frame_count <= 0:
            raise SptError("No frames rendered yet")  # CPUPathTracer.cpp:89
        exposure = self._settings.getExposure() if self._settings_mode else 1.0
        self._result.image_buffer = self._ctx.resolve_rgba8(self._frame_count, exposure)
        return self._result

    def read_accumulation(self) -> np.ndarray:
        return self._ctx.read_accum()
