"""ctypes binding of the CPU oracle (oracle/build/libcpu_ref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker / CPU baseline. The product (software-path-tracer_amd) never imports it.
See cpu_ref.h for what the oracle restates (CPUPathTracer.cpp:43-326) and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libcpu_ref.so")

FLAG_ABS_FLOAT = 1
FLAG_NEE = 1 << 4  # SPT_FLAG_NEE: next-event estimation (superset)


class RefConfig(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("max_bounces", ctypes.c_uint32),
                ("rr_depth", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class _Env(ctypes.Structure):  # == spt_env
    _fields_ = [("sky_enabled", ctypes.c_uint32), ("horizon", ctypes.c_float * 3), ("zenith", ctypes.c_float * 3)]


_lib: Optional[ctypes.CDLL] = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    P, U32, F = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float
    FP = ctypes.POINTER(ctypes.c_float)
    lib.ref_rng_seed.argtypes = [U32, U32, U32, U32]
    lib.ref_rng_seed.restype = U32
    lib.ref_random_float.argtypes = [ctypes.POINTER(U32)]
    lib.ref_random_float.restype = F
    lib.ref_primary_dir.argtypes = [U32, U32, U32, U32, FP]
    lib.ref_primary_dir.restype = None
    lib.ref_sample_sky.argtypes = [P, FP, FP]
    lib.ref_sample_sky.restype = None
    lib.ref_bounce_dir.argtypes = [FP, ctypes.POINTER(U32), U32, FP]
    lib.ref_bounce_dir.restype = None
    lib.ref_scene_create.argtypes = [P, U32, P, U32, P]
    lib.ref_scene_create.restype = P
    lib.ref_scene_destroy.argtypes = [P]
    lib.ref_scene_destroy.restype = None
    lib.ref_set_env_map.argtypes = [P, P, U32, U32]
    lib.ref_set_env_map.restype = None
    lib.ref_octa_texel.argtypes = [F, F, F, U32, U32]
    lib.ref_octa_texel.restype = U32
    lib.ref_intersect.argtypes = [P, FP, FP, F, FP, ctypes.POINTER(U32), FP]
    lib.ref_intersect.restype = ctypes.c_int
    lib.ref_trace_ray.argtypes = [P, ctypes.POINTER(RefConfig), FP, FP, ctypes.POINTER(U32), FP]
    lib.ref_trace_ray.restype = None
    lib.ref_render.argtypes = [P, ctypes.POINTER(RefConfig), U32, U32, U32, U32, U32, U32, U32, U32, P, ctypes.c_int]
    lib.ref_render.restype = ctypes.c_int
    lib.ref_resolve_rgba8.argtypes = [P, ctypes.c_uint64, U32, P]
    lib.ref_resolve_rgba8.restype = None
    lib.ref_resolve_rgba8_exposure.argtypes = [P, ctypes.c_uint64, U32, ctypes.c_float, P]
    lib.ref_resolve_rgba8_exposure.restype = None
    lib.ref_last_segments.argtypes = []
    lib.ref_last_segments.restype = ctypes.c_uint64
    lib.ref_last_light_samples.argtypes = []
    lib.ref_last_light_samples.restype = ctypes.c_uint64
    lib.ref_light_sample.argtypes = [P, FP, FP, FP, ctypes.POINTER(U32), FP, FP, FP]
    lib.ref_light_sample.restype = ctypes.c_int
    lib.ref_visible.argtypes = [P, FP, FP, F]
    lib.ref_visible.restype = ctypes.c_int
    lib.ref_emitter_count.argtypes = [P]
    lib.ref_emitter_count.restype = U32
    _lib = lib
    return lib


def _f3(v) -> ctypes.Array:
    return (ctypes.c_float * 3)(*[float(x) for x in v])


def _env(env) -> _Env:
    e = _Env()
    e.sky_enabled = env.sky_enabled
    e.horizon[:] = list(env.horizon)
    e.zenith[:] = list(env.zenith)
    return e


def rng_seed(x: int, y: int, width: int, frame1: int) -> int:
    return load().ref_rng_seed(x, y, width, frame1)


def random_floats(state: int, n: int) -> Tuple[np.ndarray, np.ndarray]:
    """n draws of random_float from `state`: (floats, states after each draw)."""
    lib = load()
    s = ctypes.c_uint32(state)
    vals = np.zeros(n, dtype=np.float32)
    states = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        vals[i] = lib.ref_random_float(ctypes.byref(s))
        states[i] = s.value
    return vals, states


def primary_dir(x: int, y: int, w: int, h: int) -> np.ndarray:
    out = (ctypes.c_float * 3)()
    load().ref_primary_dir(x, y, w, h, out)
    return np.array(out[:], dtype=np.float32)


def bounce_dir(n, state: int, flags: int = 0) -> Tuple[np.ndarray, int]:
    out = (ctypes.c_float * 3)()
    s = ctypes.c_uint32(state)
    load().ref_bounce_dir(_f3(n), ctypes.byref(s), flags, out)
    return np.array(out[:], dtype=np.float32), s.value


class RefScene:
    def __init__(self, prims: np.ndarray, mats: np.ndarray, env):
        self.lib = load()
        self._prims = np.ascontiguousarray(prims)
        self._mats = np.ascontiguousarray(mats)
        self._env = _env(env)
        self.h = self.lib.ref_scene_create(self._prims.ctypes.data if len(prims) else None, len(prims),
                                           self._mats.ctypes.data, len(mats), ctypes.byref(self._env))

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ref_scene_destroy(self.h)
            self.h = None

    def set_env_map(self, rgba: Optional[np.ndarray]) -> None:
        """Octahedral RGBA environment map (h, w, 4) float32, or None for the gradient sky."""
        if rgba is None:
            self.lib.ref_set_env_map(self.h, None, 0, 0)
            return
        a = np.ascontiguousarray(rgba, dtype=np.float32)
        self.lib.ref_set_env_map(self.h, a.ctypes.data, a.shape[1], a.shape[0])

    def intersect(self, o, d, tmin: float = 0.001):
        t = ctypes.c_float()
        prim = ctypes.c_uint32()
        ng = (ctypes.c_float * 3)()
        hit = self.lib.ref_intersect(self.h, _f3(o), _f3(d), tmin, ctypes.byref(t), ctypes.byref(prim), ng)
        if not hit:
            return None
        return float(t.value), int(prim.value), np.array(ng[:], dtype=np.float32)

    def render(self, width: int, height: int, first_frame: int, n_frames: int, max_bounces: int = 4,
               rr_depth: int = 2, flags: int = 0, rect: Optional[Tuple[int, int, int, int]] = None,
               row_step: int = 1, row_offset: int = 0, threads: int = 0) -> np.ndarray:
        """Accumulation buffer (rows, cols, 4) for frames [first_frame, first_frame+n_frames)."""
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, width, height)
        n_rows = max(0, (y1 - y0 - row_offset + row_step - 1) // row_step) if y1 > y0 + row_offset else 0
        acc = np.zeros((n_rows, x1 - x0, 4), dtype=np.float32)
        cfg = RefConfig(width, height, max_bounces, rr_depth, flags)
        rc = self.lib.ref_render(self.h, ctypes.byref(cfg), first_frame, n_frames, x0, y0, x1, y1, row_step,
                                 row_offset, acc.ctypes.data, threads)
        if rc != 0:
            raise ValueError("ref_render: bad arguments")
        return acc

    def last_segments(self) -> int:
        return int(self.lib.ref_last_segments())

    def last_light_samples(self) -> int:
        return int(self.lib.ref_last_light_samples())

    def emitter_count(self) -> int:
        return int(self.lib.ref_emitter_count(self.h))

    def light_sample(self, x, n, T, state: int):
        """NEE light sample at offset hit point x (normal n, throughput T): (valid, w, tmax, add, state)."""
        s = ctypes.c_uint32(state)
        w = (ctypes.c_float * 3)()
        tmax = ctypes.c_float()
        add = (ctypes.c_float * 3)()
        ok = self.lib.ref_light_sample(self.h, _f3(x), _f3(n), _f3(T), ctypes.byref(s), w, ctypes.byref(tmax), add)
        return bool(ok), np.array(w[:], np.float32), float(tmax.value), np.array(add[:], np.float32), s.value

    def visible(self, o, w, tmax: float) -> bool:
        return bool(self.lib.ref_visible(self.h, _f3(o), _f3(w), tmax))


def octa_texel(d, w: int, h: int) -> int:
    return int(load().ref_octa_texel(float(d[0]), float(d[1]), float(d[2]), w, h))


def resolve_rgba8(accum: np.ndarray, frame_count: int, exposure: float = 1.0) -> np.ndarray:
    a = np.ascontiguousarray(accum, dtype=np.float32).reshape(-1, 4)
    out = np.zeros(a.shape[0], dtype=np.uint32)
    if exposure == 1.0:
        load().ref_resolve_rgba8(a.ctypes.data, a.shape[0], frame_count, out.ctypes.data)
    else:
        load().ref_resolve_rgba8_exposure(a.ctypes.data, a.shape[0], frame_count, exposure, out.ctypes.data)
    return out
