#!/usr/bin/env python3
"""The App's per-frame pattern with the host hand-off included (src/App.cpp:231-238: render() one frame,
then get_render_result() -> SDL_UpdateTexture): per frame one spt_render(ctx, k, 1) and one
spt_resolve_rgba8 into a host buffer (4 B per pixel over PCIe), timed by the wall clock over N frames
after a warm-up, into a pageable, a page-locked (hipHostMalloc) and a registered host buffer
(spt_register_host_output: the resolve kernel writes it over PCIe directly, no DMA copy; the backend's
own RenderResult buffer is registered this way). Prints one JSON line per case:
microseconds per frame for the render alone (stream-synchronized) and with the resolve + device-to-host copy, and the host-inclusive Msamples/s.

    python scripts/app_pattern.py [--frames 200]

This is the PCIe-inclusive rate DESIGN.md quotes beside bench.py's device-resident `value`."""
import argparse
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [("app", 512, 512, 4), ("cornell", 1280, 720, 8), ("cornell", 1920, 1080, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    args = ap.parse_args()
    spt = importlib.import_module("software-path-tracer_amd")
    for (scene, w, h, bounces), mode in [(c, m) for c in CONFIGS for m in ("pageable", "pinned", "registered")]:
        prims, mats, env = spt.build_scene(scene)
        with spt.Context(0) as ctx:
            ctx.set_scene(prims, mats, env)
            ctx.configure(w, h, bounces, 2, 0, 0, 1, 0)
            if mode == "pinned":  # page-locked host memory (hipHostMalloc), as a caller can give the resolve
                hip = ctypes.CDLL("libamdhip64.so")
                pin = ctypes.c_void_p()
                if hip.hipHostMalloc(ctypes.byref(pin), ctypes.c_size_t(4 * w * h), ctypes.c_uint(0)) != 0:
                    raise RuntimeError("hipHostMalloc failed")
                optr = pin
            else:
                out = np.zeros(w * h, dtype=np.uint32)
                optr = out.ctypes.data_as(ctypes.c_void_p)
                if mode == "registered":
                    ctx.register_host_output(out)
            frame = 0
            for _ in range(args.warmup):
                ctx.render(frame, 1)
                frame += 1
                ctx.lib.spt_resolve_rgba8(ctx.h, frame, optr)
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.frames):
                ctx.render(frame, 1)
                frame += 1
            ctx.synchronize()
            t_render = (time.perf_counter() - t0) / args.frames
            t0 = time.perf_counter()
            for _ in range(args.frames):
                ctx.render(frame, 1)
                frame += 1
                rc = ctx.lib.spt_resolve_rgba8(ctx.h, frame, optr)  # synchronous: the image is on the host
                if rc != 0:
                    raise RuntimeError(f"spt_resolve_rgba8 -> {rc}")
            t_full = (time.perf_counter() - t0) / args.frames
            print(json.dumps({"scene": scene, "width": w, "height": h, "bounces": bounces, "frames": args.frames,
                              "host_buffer": mode,
                              "us_per_frame_render": round(t_render * 1e6, 2),
                              "us_per_frame_with_resolve_d2h": round(t_full * 1e6, 2),
                              "d2h_bytes_per_frame": 4 * w * h,
                              "msamples_per_s_host_inclusive": round(w * h / t_full / 1e6, 1)}), flush=True)
            if mode == "pinned":
                hip.hipHostFree(pin)


if __name__ == "__main__":
    main()
