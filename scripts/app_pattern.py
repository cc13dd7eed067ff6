#!/usr/bin/env python3
"""The App's per-frame pattern with the host hand-off included (src/App.cpp:231-238: render() one frame,
then get_render_result() -> SDL_UpdateTexture): per frame one spt_render(ctx, k, 1) and one
spt_resolve_rgba8 into a host buffer (4 B per pixel over PCIe), timed by the wall clock over N frames
after a warm-up, into a pageable, a page-locked (hipHostMalloc) and a registered host buffer
(spt_register_host_output: the resolve kernel writes it over PCIe directly, no DMA copy; the backend's
own RenderResult buffer is registered this way), and "fused": one spt_render_resolve_rgba8 per frame into
the registered buffer (the resolve rides in the frame's k_frame launch; what HIPPathTracer::render()
does with its registered buffer); "sync" is the floor: one spt_render + spt_synchronize per frame, no
hand-off. --modes picks the cases. Prints one JSON line per case:
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
    ap.add_argument("--modes", default="pageable,pinned,registered,fused,sync")
    args = ap.parse_args()
    spt = importlib.import_module("software-path-tracer_amd")
    for (scene, w, h, bounces), mode in [(c, m) for c in CONFIGS for m in args.modes.split(",")]:
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
                if mode in ("registered", "fused"):
                    ctx.register_host_output(out)
            def hand_off(k):  # one frame with this mode's hand-off; returns the next frame index
                if mode == "sync":  # no hand-off: the frame and the stream synchronization alone
                    ctx.render(k, 1)
                    ctx.synchronize()
                    return k + 1
                if mode == "fused":  # render + resolve in one call (and one launch); synchronous as well
                    rc = ctx.lib.spt_render_resolve_rgba8(ctx.h, k, 1, k + 1, ctypes.c_float(1.0), optr)
                else:
                    ctx.render(k, 1)
                    rc = ctx.lib.spt_resolve_rgba8(ctx.h, k + 1, optr)  # synchronous: the image is on the host
                if rc != 0:
                    raise RuntimeError(f"resolve -> {rc}")
                return k + 1

            frame = 0
            for _ in range(args.warmup):  # (also lets the run-time specialized kernels of this mode compile)
                frame = hand_off(frame)
            time.sleep(3.0)
            for _ in range(args.warmup):
                frame = hand_off(frame)
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.frames):
                ctx.render(frame, 1)
                frame += 1
            ctx.synchronize()
            t_render = (time.perf_counter() - t0) / args.frames
            t0 = time.perf_counter()
            for _ in range(args.frames):
                frame = hand_off(frame)
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
