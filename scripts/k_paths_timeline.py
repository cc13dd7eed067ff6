#!/usr/bin/env python3
"""Launch timeline of one k_paths launch from an instrumented build (measurement only):

    bash scripts/build_variant.sh tl "-DSPT_TIMELINE"
    SPT_LIB_PATH=build/libspt_exp_tl.so python scripts/k_paths_timeline.py [--frames 64] [--scene cornell]

Every resident wave of the generic (not run-time compiled) k_paths records wall_clock64() (100 MHz) at
its start, at its last chunk pull, at its end, and its chunk count. Prints one JSON line: the launch
span, the spread of wave starts (ramp), the spread of last-chunk starts and of wave ends (tail), and
the fraction of wave-slot time idle before the last wave ends."""
import argparse
import ctypes
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--show", type=int, default=12)
    ap.add_argument("--world", type=int, default=1, help="rank --rank's row shard of an N-GPU run")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--nee", action="store_true", help="SPT_FLAG_NEE")
    args = ap.parse_args()
    spt = importlib.import_module("software-path-tracer_amd")
    prims, mats, env = spt.build_scene(args.scene)
    with spt.Context(0) as ctx:
        ctx.set_tuning(specialize=-1)  # the offline-compiled kernel (its module holds the timeline)
        ctx.set_scene(prims, mats, env)
        ctx.configure(args.width, args.height, args.bounces, 2, spt.FLAG_NEE if args.nee else 0, args.rank, args.world, 0)
        f = 0
        for _ in range(args.warm):  # sustained clocks
            ctx.render(f, args.frames)
            f += args.frames
        ctx.synchronize()
        ctx.render(f, args.frames)
        ctx.synchronize()
        buf = np.zeros(8192 * 4, dtype=np.uint64)
        fn = ctx.lib.spt_exp_timeline
        fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        fn.restype = ctypes.c_int
        if fn(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) != 0:
            raise RuntimeError("spt_exp_timeline failed")
    r = buf.reshape(-1, 4)
    r = r[r[:, 0] != 0]
    t0 = r[:, 0].astype(np.float64) * 10e-3  # us (100 MHz)
    tlast = r[:, 1].astype(np.float64) * 10e-3
    tend = r[:, 2].astype(np.float64) * 10e-3
    chunks = (r[:, 3] & 0xffffffff).astype(np.int64)
    xcc = ((r[:, 3] >> 32) & 0xff).astype(np.int64)
    last_pxs = ((r[:, 3] >> 40) & 0xff).astype(np.int64)
    last_live = ((r[:, 3] >> 48) & 0xffff).astype(np.int64)
    base = t0.min()
    t0, tlast, tend = t0 - base, tlast - base, tend - base
    span = tend.max()
    pct = lambda a: [round(float(np.percentile(a, q)), 2) for q in (0, 10, 50, 90, 100)]
    idle_tail = float(np.sum(span - tend)) / (len(tend) * span)
    idle_ramp = float(np.sum(t0)) / (len(t0) * span)
    print(json.dumps({"scene": args.scene, "frames": args.frames, "world": args.world, "waves": int(len(r)), "span_us": round(float(span), 2),
                      "wave_start_us_pct_0_10_50_90_100": pct(t0),
                      "last_chunk_start_us_pct": pct(tlast),
                      "wave_end_us_pct": pct(tend),
                      "chunks_per_wave_pct": pct(chunks),
                      "idle_frac_ramp": round(idle_ramp, 4), "idle_frac_tail": round(idle_tail, 4)}))
    # the waves that end last: their last chunk (start, duration, size, live pixels) and XCD
    order = np.argsort(-tend)[:args.show]
    for i in order:
        print(json.dumps({"end_us": round(float(tend[i]), 1), "last_chunk_start_us": round(float(tlast[i]), 1),
                          "last_chunk_us": round(float(tend[i] - tlast[i]), 1), "last_chunk_px": int(1 << last_pxs[i]),
                          "last_chunk_live_px": int(last_live[i]), "xcc": int(xcc[i]), "chunks": int(chunks[i])}))
    # per XCD: when its waves took their last chunk and ended
    for x in range(8):
        m = xcc == x
        if m.any():
            print(json.dumps({"xcc": x, "waves": int(m.sum()), "last_pull_max_us": round(float(tlast[m].max()), 1),
                              "end_p50_us": round(float(np.percentile(tend[m], 50)), 1),
                              "end_max_us": round(float(tend[m].max()), 1)}))


if __name__ == "__main__":
    main()
