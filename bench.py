#!/usr/bin/env python3
"""bench.py — Msamples/s of the MI355X path-tracing integrator on the C2 Cornell config.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, N>1 under torch.distributed.run
(`--gpus N` without a launcher starts the N ranks itself as a child torch.distributed.run, before
anything touches a GPU, and exits with its status — it never silently runs on one GPU). Rank 0 prints
ONE JSON line. The untimed warm-up renders the W steps, repeated until the GPU has been busy for
--warmup-seconds (0.05 s), so the timed K steps run at sustained clocks.

Workload (BASELINE.json metric, configs[1] = C2): Cornell box (6 quads + 2 spheres), 1920x1080,
8 bounces, 64 spp. A *step* is one C2 image per GPU: --frames-per-step (64) full frames of camera
paths (one frame = one reference render() call, CPUPathTracer.cpp:43-85) in ONE spt_render call that
continues the progressive accumulation (step k traces frames 64k .. 64k+63, so K steps are the C3
progression at 64*K spp, and every step traces new samples). With N ranks the image rows are dealt
round-robin (row y -> rank y % N) and each rank traces 64*N frames of its rows per step, so per-GPU
work is fixed (weak scaling); after the last step the shards are gathered to rank 0 over RCCL by the
library's own collective (spt_gather_image: one ncclGather + a device de-interleave) inside the timed
region. At N=1 the accumulation buffer already is the image: nothing is gathered or copied.

`roofline` is the dominant kernel (k_paths, the persistent schedule; k_frame for
calls of < 4 frames), priced against the roof it actually runs against. `traffic` = HBM bytes per
launch from rocprofv3 PMC passes of THIS launch shape on THIS kernel source (profiles/pmc_r02.json,
keyed by configuration, frames per launch and a hash of the kernel sources; scripts/pmc_collect.py),
else null. The HBM figure is SURVEY.md §8d's: 40 B per traced ray segment x the segments one launch
traces / its HIP-event duration on the integrator's stream. When the measured traffic is below 10 %
of those algorithmic bytes (rays live in registers), `roofline.bound` is "valu" — VALU issue from
SQ_INSTS_VALU and the clock (GRBM_GUI_ACTIVE) of the same PMC record — and the §8d HBM figure is
`roofline.hbm_8d` (`algorithmic_gbps`: notional §8d bytes, not moved bytes; `measured_gbps`: the PMC
bytes per launch over the launch time). Every kernel with a PMC record also carries `measured_hbm`
(GB/s and fraction of 8 TB/s the kernel actually moves). `cpu_baseline` times the CPU oracle (a restatement of the
reference CPUPathTracer; oracle/) on this host, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SIMDS = 1024                   # 256 CUs x 4 SIMDs; a wave64 VALU instruction issues over 2 cycles
VALU_LANES_PER_CYCLE = 32      # per SIMD (MI355X_MICROARCH.md: 32 lanes/cycle x 2 cycles per wave64 op)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames-per-step", type=int, default=64,
                    help="full frames (spp) per GPU per step: 64 = one C2 image (BASELINE.json configs[1])")
    ap.add_argument("--warmup-seconds", type=float, default=0.05,
                    help="repeat the W warm-up steps until the GPU has been busy this long (sustained clocks)")
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--rr-depth", type=int, default=2)
    ap.add_argument("--frames-in-flight", type=int, default=0, help="frames per wavefront pass (0 = auto)")
    ap.add_argument("--frames-per-call", type=int, default=0,
                    help="frames per spt_render call (0 = one call per step)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--save-image", default="", help="rank 0: save the assembled float RGBA image (.npy)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL, one GPU per rank) or gloo (multi-rank rehearsal, ranks may share a GPU)")
    ap.add_argument("--gather", default="spt", choices=["spt", "torch"],
                    help="N>1 over nccl: spt_gather_image (RCCL inside the library) or torch.distributed.gather")
    ap.add_argument("--gather-every-step", action="store_true",
                    help="N>1 with --gather spt: every step's image to rank 0 (a progressive display), each "
                         "gather overlapped with the next step's rendering (spt_gather_image_overlapped)")
    ap.add_argument("--split", action="store_true", help="separate extend/shade launches (traversal kernel alone)")
    ap.add_argument("--wavefront", action="store_true", help="flat scenes: wavefront schedule instead of k_paths")
    ap.add_argument("--sorted", action="store_true",
                    help="BVH scenes: split wavefront with sorted (binned) ray queues (SPT_FLAG_SORTED_RAYS)")
    ap.add_argument("--nee", action="store_true",
                    help="next-event estimation (SPT_FLAG_NEE, light sampling; superset of the reference's integrator)")
    ap.add_argument("--env-map", type=int, default=0,
                    help="N > 0: miss radiance from a synthetic N x N octahedral environment map")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="single process: trace EVERY rank's row shard of an N-GPU run in turn (N x the frames "
                         "per step each) and the whole image at N = 1, to preview weak scaling on one GPU; "
                         "value = all ranks' samples / the slowest rank's time (the gather is not included)")
    ap.add_argument("--no-profile", action="store_true", help="skip per-launch HIP events (roofline)")
    ap.add_argument("--profile-mode", choices=("auto", "launch", "span"), default="auto",
                    help="kernel time of k_paths / k_frame: HIP events around every launch, or one event pair "
                         "around all the timed launches (span; default for one-frame launches, whose per-launch "
                         "events cost ~15 %%); auto = span for the frame schedule")
    ap.add_argument("--tuning", default="",
                    help="spt_tuning fields for experiments, e.g. px_shift=3,chunks_per_wave=4 (results never change)")
    ap.add_argument("--no-specialize", action="store_true",
                    help="flat scenes: the generic persistent kernels instead of the ones compiled for the scene's shape")
    ap.add_argument("--pmc-csv", default="",
                    help="rocprofv3 --pmc counter_collection.csv with FETCH_SIZE/WRITE_SIZE of this run's kernels")
    return ap.parse_args()


def kernel_source_hash() -> str:
    """Hash of the device code's sources: a committed PMC record applies only to the kernel it measured."""
    h = hashlib.sha256()
    for name in ("spt_kernels.hip", "spt_kernels.h", "spt_device.h", "spt_jit.hip"):
        with open(os.path.join(ROOT, "software-path-tracer_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_label(args, world: int, frames_per_launch: int) -> str:
    """Key of a launch shape in profiles/pmc_r02.json (scripts/pmc_collect.py writes the same key)."""
    env = f"-env{args.env_map}" if args.env_map else ""
    gen = "-generic" if args.no_specialize else ""
    nee = "-nee" if args.nee else ""
    return f"{args.scene}-{args.width}x{args.height}-b{args.bounces}-world{world}-f{frames_per_launch}{env}{gen}{nee}"


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher: run the N ranks as a child torch.distributed.run (this
    process has not touched a GPU) and return its exit status. Never falls back to one GPU."""
    import torch

    have = torch.cuda.device_count()  # counting devices does not initialise HIP
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {have} GPU(s) visible", file=sys.stderr)
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def committed_pmc(label: str, kernel: str):
    """The PMC record of `kernel` (HBM bytes, VALU instructions, clock) from rocprofv3 passes of exactly
    this launch shape on this kernel source (profiles/pmc_r02.json), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_r02.json")
    if not os.path.exists(path):
        return None
    entry = json.load(open(path)).get(label, {})
    if entry.get("kernel_source") != kernel_source_hash():
        return None
    for name, v in entry.get("kernels", {}).items():  # the timed variant, not the counting one
        if name.split("<")[0].endswith(kernel) and "<true" not in name:
            return v
    return None


def pmc_traffic(path: str, kernel: str):
    """HBM bytes per launch of `kernel` from rocprofv3 PMC csv (FETCH_SIZE x2 on gfx950 + WRITE_SIZE, KB)."""
    if not path or not os.path.exists(path):
        return None
    import csv

    fetch, write = [], []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            name = row.get("Counter_Name", "")
            val = float(row.get("Counter_Value", 0.0))
            if name == "FETCH_SIZE":
                fetch.append(val)
            elif name == "WRITE_SIZE":
                write.append(val)
    if not fetch:
        return None
    # MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of a wide streaming read on gfx950; units KB
    per_launch = (2.0 * np.mean(fetch) + (np.mean(write) if write else 0.0)) * 1024.0
    return float(per_launch)


def stats_diff(a, b):
    """b - a for the counters of two spt_stats snapshots (the schedule fields are b's)."""
    import ctypes

    out = type(b)()
    keep = {"tail_bounce", "fused", "schedule", "bvh_nodes", "scene_bytes", "flat_fast_path", "specialized", "emitters",
            "stack_bytes", "stack_need"}
    for name, typ in b._fields_:
        vb, va = getattr(b, name), getattr(a, name)
        if isinstance(vb, ctypes.Array):
            arr = getattr(out, name)
            for i in range(len(vb)):
                arr[i] = vb[i] - va[i]
        else:
            setattr(out, name, vb if name in keep else vb - va)
    return out


def traced_segments(st, bounces: int, pixels: int, frame_kernel: bool) -> int:
    """Ray segments the persistent kernels actually trace: k_frame the segments at bounce >= 1 (the
    camera segments' hits come from the per-pixel cache the first call after a change stored, DESIGN.md
    3.1b, and the timed calls follow the warm-up); k_paths the segments at bounce >= 1 + one camera
    segment per pixel per launch (bounce 0 is traced once per pixel and reused by every frame of the
    launch); + the NEE shadow rays."""
    if frame_kernel:
        return sum(int(x) for x in st.segments[1:bounces]) + int(st.shadow_rays)
    return sum(int(x) for x in st.segments[1:bounces]) + int(st.persistent_launches) * pixels + int(st.shadow_rays)


def kernel_rooflines(st, bounces: int, passes: int, pixels: int, pmc_csv: str, label: str = "",
                     frame_kernel: bool = False) -> dict:
    """Achieved algorithmic GB/s per kernel family over its HIP-event time.

    extend : 8 B hit write per camera ray (bounce 0 computes the ray) + 40 B per later ray
             (32 B ray read + 8 B hit write)
    shade  : bounce 0: 8 B hit + 16 B radiance write per path; bounce b>=1: 8 B hit + 48 B ray state
             per ray; every bounce: 48 B per surviving ray written + 32 B per radiance RMW
    accumulate (timed with nothing else in "other"): F x 16 B radiance + 32 B accum RMW per pixel
    """
    seg = [int(x) for x in st.segments[:bounces]] + [0]
    rmw = [int(x) for x in st.radiance_updates[:bounces]]
    wave = min(bounces, int(st.tail_bounce))  # bounces >= wave run in k_trace_tail
    out = {}
    if st.extend_launches and st.extend_ms > 0:
        b = seg[0] * 8 + sum(seg[k] * 40 for k in range(1, wave))
        out["k_extend"] = (b, st.extend_ms, st.extend_launches)
    if st.shade_launches and st.shade_ms > 0 and not st.fused:
        b = seg[0] * (8 + 16) + sum(seg[k] * 56 for k in range(1, wave))
        b += sum(seg[k + 1] * 48 for k in range(wave)) + sum(rmw[k] * 32 for k in range(wave))
        out["k_shade"] = (b, st.shade_ms, st.shade_launches)
    if st.shade_launches and st.shade_ms > 0 and st.fused:
        # fused extend+shade: bounce 0: 16 B radiance per path; b>=1: 48 B ray state read per ray;
        # 48 B per surviving ray written + 32 B per radiance RMW
        b = seg[0] * 16 + sum(seg[k] * 48 for k in range(1, wave))
        b += sum(seg[k + 1] * 48 for k in range(wave)) + sum(rmw[k] * 32 for k in range(wave))
        out["k_bounce"] = (b, st.shade_ms, st.shade_launches)
    if st.tail_launches and st.tail_ms > 0:
        # reads each queued path's 48 B state once; per segment only radiance RMWs touch memory
        b = seg[wave] * 48 + sum(rmw[k] * 32 for k in range(wave, bounces))
        out["k_trace_tail"] = (b, st.tail_ms, st.tail_launches)
    if st.persistent_launches and st.persistent_ms > 0 and frame_kernel:
        # k_frame (calls of < 4 frames, one launch per frame): the segments at bounce >= 1 are traced
        # (the camera hits are cached per pixel), 40 B each as for k_paths; its own HBM traffic is the
        # 32 B accumulator RMW per path plus the cached hits / live-pixel records
        traced = traced_segments(st, bounces, pixels, True)
        out["k_frame"] = (traced * 40, st.persistent_ms, st.persistent_launches)
    elif st.persistent_launches and st.persistent_ms > 0:
        # persistent k_paths: SURVEY.md §8d's per-unit traversal figure, 40 B per ray segment (32 B ray
        # read + 8 B hit write), x the segments the launches traced. The kernel itself keeps rays in
        # registers: its own HBM traffic is 32 B per pixel per launch. Only segments the kernel
        # actually traces count: bounce 0 is traced once per pixel per launch (its result is reused
        # for every frame of the pixel, spt_kernels.hip k_paths).
        traced = traced_segments(st, bounces, pixels, False)
        # BVH scenes: + §8d's scene bytes that are not cache-resident by construction, per node visited
        # (32 B) and triangle tested (48 B), from the counting re-render (bounce >= 1 segments)
        scene = int(st.bvh_node_visits) * 32 + int(st.prim_tests) * 48
        out["k_paths"] = (traced * 40 + scene, st.persistent_ms, st.persistent_launches)
    if passes and st.other_ms > 0:
        b = int(st.frames) * pixels * 16 + passes * pixels * 32
        out["k_accumulate"] = (b, st.other_ms, passes)
    res = {}
    for name, (nbytes, ms, launches) in out.items():
        achieved = nbytes / (ms * 1e-3) / 1e9
        traffic, source, pmc = pmc_traffic(pmc_csv, name), "this run's --pmc-csv", None
        if traffic is None:
            pmc = committed_pmc(label, name)
            traffic = pmc["traffic_bytes"] if pmc else None
            source = "profiles/pmc_r02.json: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, same launch shape and kernel source" \
                if pmc else "no PMC record for this launch shape and kernel source"
        res[name] = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": round(traffic, 1) if traffic is not None else None,
            "traffic_source": source,
            "kernel": name,
            "algorithmic_bytes_per_launch": round(nbytes / launches, 1),
            "avg_launch_us": round(ms * 1e3 / launches, 2),
            "launches": int(launches),
            "total_ms": round(ms, 4),
        }
        if traffic is not None:
            # the HBM (L2 <-> fabric) bytes the PMC passes measured for one launch of this shape, as a rate
            # over this run's average launch time: what the kernel actually moves, beside the 8(d) figure
            gbps = traffic / (ms * 1e-3 / launches) / 1e9
            res[name]["measured_hbm"] = {
                "gbps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBS, 4), "bytes_per_launch": round(traffic, 1),
                "basis": "PMC FETCH_SIZE x2 + WRITE_SIZE per launch (MI355X_MICROARCH.md gfx950 correction) / "
                         "this run's HIP-event average launch time"}
            if pmc and pmc.get("duration_ns"):
                res[name]["measured_hbm"]["pmc_duration_median_us"] = round(pmc["duration_ns"] / 1e3, 2)
                if pmc.get("duration_mean_ns"):
                    res[name]["measured_hbm"]["pmc_duration_mean_us"] = round(pmc["duration_mean_ns"] / 1e3, 2)
        if name in ("k_frame", "k_paths"):
            res[name]["basis"] = ("SURVEY.md 8d: 40 B per traced ray segment (ray 32 B + hit 8 B); traced = "
                                  + ("segments at bounce >= 1 (camera hits from the per-pixel cache)"
                                     if name == "k_frame" else
                                     "segments at bounce >= 1 + one camera segment per pixel per launch")
                                  + (" + NEE shadow rays" if st.shadow_rays else ""))
            res[name]["hbm_bytes_per_launch"] = 32 * pixels  # the accumulator RMW: the kernel's own traffic
            if name == "k_paths" and st.bvh_node_visits:
                L = max(1, int(launches))
                res[name]["basis"] += ("; + BVH scene bytes: 32 B per node visited + 48 B per triangle tested "
                                       "(SURVEY.md 8d)")
                res[name]["scene_bytes_8d_per_launch"] = round((int(st.bvh_node_visits) * 32 + int(st.prim_tests) * 48) / L, 1)
                # the records the device actually reads: 64-B quantized nodes, 64-B primitive records
                res[name]["scene_record_bytes_per_launch"] = round((int(st.bvh_node_visits) + int(st.prim_tests)) * 64 / L, 1)
                if traffic is not None:
                    res[name]["traffic_over_algorithmic"] = round(traffic / (nbytes / L), 3)
                if pmc:  # reads and writes apart (the traversal stack and spills are the kernel's writers)
                    res[name]["fetch_bytes_per_launch"] = pmc.get("fetch_bytes")
                    res[name]["write_bytes_per_launch"] = pmc.get("write_bytes")
            res[name]["note"] = ("rays live in registers: measured traffic is the accumulator plus scene "
                                 "reads, far below the algorithmic bytes; the kernel's binding limit is "
                                 "roofline_valu (VALU issue), DESIGN.md 5.1")
            if pmc and pmc.get("valu_insts") and pmc.get("duration_ns") and pmc.get("clock_ghz"):
                lane_ops = pmc["valu_insts"] * 64.0 / (pmc["duration_ns"] * 1e-9) / 1e12
                peak = SIMDS * VALU_LANES_PER_CYCLE * pmc["clock_ghz"] * 1e9 / 1e12
                res[name]["valu"] = {"bound": "valu", "achieved": round(lane_ops, 2), "peak": round(peak, 2),
                                     "unit": "T lane-ops/s", "frac": round(lane_ops / peak, 4),
                                     "valu_insts_per_launch": pmc["valu_insts"], "salu_insts_per_launch": pmc.get("salu_insts"),
                                     "clock_ghz": pmc["clock_ghz"], "pmc_duration_us": round(pmc["duration_ns"] / 1e3, 2),
                                     # active lanes per VALU instruction (divergence):
                                     # SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU), DESIGN.md 5.1
                                     "lane_density": (round(pmc["thread_cycles_valu"] / (64.0 * pmc["valu_insts"]), 4)
                                                      if pmc.get("thread_cycles_valu") else None),
                                     "basis": "SQ_INSTS_VALU x 64 lanes / kernel time vs 1024 SIMDs x 32 lanes/cycle "
                                              "x clock (GRBM_GUI_ACTIVE / 8 XCDs / time), same PMC record"}
    return res


def bound_from_evidence(r):
    """The roofline the kernel actually runs against. A persistent kernel keeps its
    rays in registers: when the measured HBM traffic is below 10 % of SURVEY.md 8(d)'s algorithmic
    bytes, the binding roof is VALU issue, so `roofline` carries the VALU figure (same PMC record, same
    launch shape and kernel source) and the 8(d) HBM figure moves to `roofline.hbm_8d`. Without a PMC
    record for this kernel source the HBM figure stays, marked as unverified."""
    if not r:
        return r
    traffic, algo, valu = r.get("traffic"), r.get("algorithmic_bytes_per_launch"), r.get("valu")
    # 8(d)'s figure: notional bytes (40 B per traced segment + scene bytes) over the launch time — named
    # algorithmic, never "achieved"; the measured rate (PMC bytes / time) beside it
    hbm = {"bound": "hbm", "algorithmic_gbps": r.get("achieved"), "peak": r.get("peak"), "unit": r.get("unit"),
           "algorithmic_frac": r.get("frac")}
    if r.get("measured_hbm"):
        hbm["measured_gbps"] = r["measured_hbm"]["gbps"]
        hbm["measured_frac"] = r["measured_hbm"]["frac"]
    if traffic is not None and algo and valu and traffic < 0.1 * algo:
        out = dict(r)
        out.update({"bound": "valu", "achieved": valu["achieved"], "peak": valu["peak"], "unit": valu["unit"],
                    "frac": valu["frac"], "hbm_8d": hbm,
                    "bound_evidence": f"measured traffic {traffic / algo:.3f} x the 8(d) algorithmic bytes (< 0.1): "
                                      "not HBM-bound; VALU issue from SQ_INSTS_VALU"})
        return out
    out = dict(r)
    out["bound_evidence"] = ("no PMC record of this launch shape and kernel source: bound not verified"
                             if traffic is None else f"measured traffic {traffic / max(algo, 1):.3f} x the 8(d) bytes")
    return out


def host_cpu() -> str:
    """CPU model and logical CPU count of this host (SURVEY.md 8d asks for both beside the baseline)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{model}, {os.cpu_count()} logical CPUs"


def cpu_threads() -> int:
    """This job's CPU share: OMP_NUM_THREADS when set (the GPU pool sets 16 per GPU and asks jobs to
    keep to it), else the CPUs this process may run on."""
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(env, share) if env > 0 else share)


def cpu_baseline(spt, args, scene_arrays, budget_s: float, max_frames: int, flags: int = 0):
    """Time the CPU oracle on this host: whole frames of the same workload until ~budget_s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref

    prims, mats, env = scene_arrays
    rs = cpu_ref.RefScene(prims, mats, env)
    if args.env_map > 0:
        rs.set_env_map(spt.synthetic_env_map(args.env_map))
    threads = cpu_threads()
    w, h = args.width, args.height
    # single-thread rate (the reference ships a serial loop, :57-82) on every 27th row of frame 0:
    # 40 full-width rows strided over the whole image (sky, walls, spheres and floor alike)
    stride = max(1, h // 40)
    t0 = time.perf_counter()
    rows = rs.render(w, h, 0, 1, args.bounces, args.rr_depth, flags, row_step=stride, threads=1)
    st_rate = rows.shape[0] * w / (time.perf_counter() - t0) / 1e6
    frames = 0
    acc = np.zeros((h, w, 4), np.float32)
    t0 = time.perf_counter()
    while True:
        acc += rs.render(w, h, frames, 1, args.bounces, args.rr_depth, flags, threads=threads)
        frames += 1
        el = time.perf_counter() - t0
        if el >= budget_s or frames >= max_frames:
            break
    rate = w * h * frames / el / 1e6
    return {
        "value": round(rate, 3),
        "unit": "Msamples/s",
        "cores": threads,
        "host": host_cpu(),
        "kind": "port",
        "sample": f"frames 0..{frames - 1} ({frames} spp) of the full {w}x{h} {args.scene} image, "
                  f"{args.bounces} bounces{', NEE' if flags else ''}, oracle/cpu_ref.c (-O3) OpenMP over rows",
        "threads_note": "this job's CPU share (OMP_NUM_THREADS; the GPU pool gives a 1-GPU job 16 of the "
                        "host's logical CPUs and asks it to stay within them)",
        "single_thread_value": round(st_rate, 3),
        "single_thread_sample": f"frame 0, every {stride}th row ({rows.shape[0]} rows x {w} px), 1 thread",
        "seconds": round(el, 2),
    }, frames, acc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    if world > 1:
        device = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:  # gloo: rehearsal of the multi-rank path on one GPU (ranks may share a device)
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)

    spt = importlib.import_module("software-path-tracer_amd")
    scene_arrays = spt.build_scene(args.scene)
    prims, mats, env = scene_arrays
    w, h = args.width, args.height
    # one stream for the integrator and torch's collectives/copies: a stream of our own (the default
    # stream's handle is NULL, which would leave the ctx on its private non-blocking stream, unordered
    # with torch's work on the default stream)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)

    ctx = spt.Context(torch.cuda.current_device())
    ctx.set_stream(stream.cuda_stream)
    tuning = {k: int(v) for k, v in (kv.split("=") for kv in args.tuning.split(",") if kv)}
    if args.no_specialize:
        tuning["specialize"] = -1
    if tuning:
        ctx.set_tuning(**tuning)
    ctx.set_scene(prims, mats, env)
    flags = (spt.FLAG_SPLIT_KERNELS if args.split else 0) | (spt.FLAG_WAVEFRONT if args.wavefront else 0) \
        | (spt.FLAG_SORTED_RAYS if args.sorted else 0) | (spt.FLAG_NEE if args.nee else 0)
    sim = args.simulate_world if (world == 1 and args.simulate_world > 1) else 0
    ctx.configure(w, h, args.bounces, args.rr_depth, flags, rank, sim or world, args.frames_in_flight)
    # weak scaling: one C2 image of samples per GPU per step (a 1/N row shard x N x 64 frames)
    frames_per_step = args.frames_per_step * (sim or world)
    chunk = args.frames_per_call or frames_per_step
    env_map = spt.synthetic_env_map(args.env_map) if args.env_map > 0 else None
    if env_map is not None:
        ctx.set_env_map(env_map)
    if not args.no_specialize:
        ctx.specialize_scene()  # a flat scene: wait for its shape's kernels (compiled in the background)

    use_spt_gather = world > 1 and args.dist_backend == "nccl" and args.gather == "spt"
    if use_spt_gather:  # the library's RCCL communicator; its id travels over the torch process group
        # Every rank first checks that the library can reach RCCL at all (spt_comm_available: the
        # symbols resolve, nothing is created), and all agree before any rank enters the collective
        # ncclCommInitRank: a rank failing before the collective would leave the others blocked inside it
        # (ADVICE r5). Rank 0 then makes the communicator's id.
        uid, usable = None, 1 if spt.comm_available() else 0
        if not usable:
            print(f"bench.py: rank {rank}: spt RCCL unavailable", file=sys.stderr)
        elif rank == 0:
            try:
                uid = spt.comm_unique_id()
            except Exception as e:  # e.g. no bootstrap interface
                print(f"bench.py: rank 0: ncclGetUniqueId failed ({e})", file=sys.stderr)
                usable = 0
        flag = torch.tensor([usable], dtype=torch.int32, device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        obj = [uid if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        if int(flag.item()) == 0 or obj[0] is None:
            print("bench.py: gathering with torch.distributed", file=sys.stderr)
            use_spt_gather = False
        else:
            ok = 1
            try:
                ctx.comm_init(obj[0], world, rank)
            except Exception as e:  # an RCCL error returned by ncclCommInitRank on this rank
                print(f"bench.py: rank {rank}: spt RCCL communicator failed ({e})", file=sys.stderr)
                ok = 0
            flag = torch.tensor([ok], dtype=torch.int32, device="cuda")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)  # every rank gathers the same way
            if int(flag.item()) == 0:
                print("bench.py: gathering with torch.distributed", file=sys.stderr)
                use_spt_gather = False
                if ok:  # this rank joined: leave the communicator the others could not join
                    try:
                        ctx.comm_destroy()
                    except Exception as e:
                        print(f"bench.py: rank {rank}: comm_destroy failed ({e})", file=sys.stderr)
    rows_max = (h + world - 1) // world
    shard_elems = rows_max * w * 4
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    send = gather_buf = gather_list = None
    if world > 1 and not use_spt_gather:
        send = torch.zeros(shard_elems, dtype=torch.float32, device="cuda")
        # rank 0 receives every shard straight into one buffer (per-rank views): no concatenation
        if rank == 0:
            gather_buf = torch.empty(world * shard_elems, dtype=torch.float32, device=coll_dev)
            gather_list = list(gather_buf.view(world, shard_elems).unbind(0))
    image = torch.empty(w * h * 4, dtype=torch.float32, device="cuda") if (rank == 0 and world > 1) else None

    every_step = use_spt_gather and args.gather_every_step

    def render_steps(n_steps: int, fps: int = 0, ch: int = 0) -> None:
        fps, ch = fps or frames_per_step, ch or chunk
        for step in range(n_steps):
            base = step * fps
            for first in range(base, base + fps, ch):
                ctx.render(first, min(ch, base + fps - first))
            if every_step:  # this step's image to rank 0 while the next step renders
                ctx.gather_image_overlapped(image.data_ptr() if rank == 0 else 0)

    def time_steps(fps: int, ch: int) -> float:
        """--simulate-world: the warm-up, then K timed steps of the current configuration (no profiling)."""
        render_steps(max(1, args.warmup), fps, ch)
        torch.cuda.synchronize()
        t_w = time.perf_counter()
        render_steps(max(1, args.warmup), fps, ch)
        torch.cuda.synchronize()
        one = max(time.perf_counter() - t_w, 1e-6)
        for _ in range(min(1000, int(args.warmup_seconds / one))):
            render_steps(max(1, args.warmup), fps, ch)
        ctx.reset()
        torch.cuda.synchronize()
        t = time.perf_counter()
        render_steps(args.steps, fps, ch)
        torch.cuda.synchronize()
        return time.perf_counter() - t

    # warm-up: the same launches, then the progressive accumulation restarts at frame 0. Everything
    # else is set up before it, so only a stats read-back separates the warm-up kernels from the timed
    # region (the GPU lowers its clock after ~1 ms idle).
    ctx.set_profiling(False)
    if args.warmup > 0:
        # W steps, repeated back to back until the warm-up has kept the GPU busy for at least
        # --warmup-seconds: a single 2 ms warm-up launch left the timed C2 launch 8 % slower than at
        # the sustained clocks of a longer run. Every repetition is the same launches.
        render_steps(args.warmup)  # first call: one-time set-up included
        torch.cuda.synchronize()
        t_w = time.perf_counter()
        render_steps(args.warmup)
        torch.cuda.synchronize()
        one = max(time.perf_counter() - t_w, 1e-6)
        for _ in range(min(1000, int(args.warmup_seconds / one))):
            render_steps(args.warmup)
        if use_spt_gather:
            ctx.gather_image(image.data_ptr() if rank == 0 else 0)  # collective set-up outside the timing
    ctx.reset()
    st0 = ctx.stats()  # synchronizes the integrator's stream
    # one-frame launches (k_frame) are timed with ONE event pair around the timed launches on their
    # stream: an event pair per ~40 us launch would cost the call ~15 %
    span = not args.no_profile and (args.profile_mode == "span" or
                                    (args.profile_mode == "auto" and st0.schedule == spt.SCHEDULE_FRAME))
    ctx.set_profiling(not args.no_profile, span=span)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    render_steps(args.steps)
    if span:  # the span's end event, on the stream right behind the last timed launch
        ctx.set_profiling(False)
    if every_step:  # the last step's gather is the image
        ctx.gather_wait()
    elif use_spt_gather:  # ncclGather of the padded shards + device de-interleave on rank 0
        ctx.gather_image(image.data_ptr() if rank == 0 else 0)
    elif world > 1:
        ctx.copy_accum_device(send.data_ptr())
        dist.gather(send if coll_dev == "cuda" else send.cpu(), gather_list, dst=0)
        if rank == 0:
            gathered = gather_buf if coll_dev == "cuda" else gather_buf.to("cuda")
            ctx.assemble_rows(gathered.data_ptr(), image.data_ptr())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_frames = args.steps * frames_per_step
    if rank == 0 and args.save_image:
        img = image.cpu().numpy() if image is not None else ctx.read_accum()
        np.save(args.save_image, img.reshape(h, w, 4))
    st = stats_diff(st0, ctx.stats())
    specialized = bool(st.specialized)  # the timed launches (the counting re-render below is generic)
    if st.schedule in (spt.SCHEDULE_PERSISTENT, spt.SCHEDULE_FRAME) and not args.no_profile:
        # The timed k_paths / k_frame launches do not count segments (that variant is slower); the rendering
        # is deterministic, so an untimed re-render of the same frames with counters gives the
        # exact segment counts of the timed work (kernel times are kept from the timed run).
        timed = st
        acc_keep = ctx.read_accum()
        ctx.set_profiling(False, counters=True)
        ctx.clear_stats()
        ctx.reset()
        render_steps(args.steps)
        st = ctx.stats()
        assert np.array_equal(ctx.read_accum().view(np.uint32), acc_keep.view(np.uint32))
        for name in ("persistent_ms", "persistent_launches", "passes", "frames", "paths"):
            setattr(st, name, getattr(timed, name))
        ctx.set_profiling(False)
    shard_px = ctx.shard_pixels  # (rank 0's shard: --simulate-world reconfigures the ctx below)
    # every rank traces all total_frames frames of its rows: the whole image at total_frames spp
    samples_total = total_frames * w * h
    value = samples_total / elapsed / 1e6
    sim_report = None
    if sim:
        # The N-GPU run previewed on one GPU: every rank's shard is rendered and timed in turn (the same
        # warm-up and K steps of N x frames_per_step frames each), then the whole image at N = 1 (K steps
        # of frames_per_step frames: one GPU's share of the work in the weak-scaling run). The N-GPU
        # step takes as long as its slowest rank; the gather is estimated apart (not in the preview).
        rank_t, rank_px = [], []
        for r in range(sim):
            ctx.configure(w, h, args.bounces, args.rr_depth, flags, r, sim, args.frames_in_flight)
            rank_px.append(ctx.shard_pixels)
            rank_t.append(time_steps(frames_per_step, chunk))
        ctx.configure(w, h, args.bounces, args.rr_depth, flags, 0, 1, args.frames_in_flight)
        one_fps = args.frames_per_step
        t1 = time_steps(one_fps, args.frames_per_call or one_fps)
        rate1 = args.steps * one_fps * w * h / t1
        # the same N = 1 image at the shards' frames per launch (N x frames_per_step): the baseline that
        # compares like with like — a shard's launch reuses each camera hit and chunk set-up over N x as
        # many frames, which alone makes the per-step comparison above super-linear
        t1m = time_steps(frames_per_step, chunk)
        rate1m = args.steps * frames_per_step * w * h / t1m
        t_max = max(rank_t)
        value = samples_total / t_max / 1e6
        rows_max = (h + sim - 1) // sim
        sim_report = {
            "world": sim,
            "rank_ms_per_step": [round(t * 1e3 / args.steps, 4) for t in rank_t],
            "rank_pixels": rank_px,
            "max_ms_per_step": round(t_max * 1e3 / args.steps, 4),
            "min_ms_per_step": round(min(rank_t) * 1e3 / args.steps, 4),
            "slowest_rank": int(np.argmax(rank_t)),
            "one_gpu_ms_per_step": round(t1 * 1e3 / args.steps, 4),
            "one_gpu_msamples_per_s": round(rate1 / 1e6, 3),
            "projected_speedup": round(samples_total / t_max / rate1, 3),
            "projected_efficiency": round(samples_total / t_max / rate1 / sim, 4),
            "one_gpu_matched_ms_per_step": round(t1m * 1e3 / args.steps, 4),
            "one_gpu_matched_msamples_per_s": round(rate1m / 1e6, 3),
            "projected_speedup_matched": round(samples_total / t_max / rate1m, 3),
            "projected_efficiency_matched": round(samples_total / t_max / rate1m / sim, 4),
            "matched_basis": f"N = 1 whole image at {frames_per_step} frames per step in {chunk}-frame calls, "
                             f"the shards' launch shape",
            "gather_estimate": {"bytes_per_rank": rows_max * w * 16, "bytes_into_rank0": (sim - 1) * rows_max * w * 16,
                                "note": "one ncclGather of the padded float RGBA shards after the last step "
                                        "(spt_gather_image), ~153 GB/s per xGMI link: not in value"},
            "basis": "value = all N ranks' samples / the slowest rank's measured time; every rank's shard timed "
                     "on this GPU in turn (weak scaling: N x frames_per_step frames of a 1/N row shard each)",
        }
        assert rank_px[0] == shard_px

    seg_total = st.segments_total
    frames_per_launch = 1 if st.schedule == spt.SCHEDULE_FRAME else min(chunk, 1024)
    label = pmc_label(args, sim or world, frames_per_launch)
    fams = kernel_rooflines(st, args.bounces, int(st.passes), shard_px, args.pmc_csv, label,
                            frame_kernel=st.schedule == spt.SCHEDULE_FRAME)
    for name in ("k_paths", "k_frame"):
        if name in fams:
            fams[name]["timing"] = ("one HIP event pair around all timed launches on the integrator's stream "
                                    "(span / launches; includes any gap between launches)" if span else
                                    "HIP events around every timed launch on the integrator's stream")
    # the dominant kernel family by measured time carries `roofline`; the traversal kernel's figure
    # (the north_star's target) is reported beside it
    roofline = max(fams.values(), key=lambda r: r["total_ms"]) if fams else None
    roofline = bound_from_evidence(roofline)
    roofline_extend = fams.get("k_paths") or fams.get("k_frame") or fams.get("k_extend") or fams.get("k_bounce")

    result = {
        "metric": "Msamples/sec (whole node), 1920x1080 x 8-bounce Cornell box" + (", NEE" if args.nee else ""),
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"{args.scene} {w}x{h}, {args.bounces} bounces, {args.frames_per_step} spp per GPU per "
                        f"step ({frames_per_step} frame(s) of a 1/{sim or world} row shard per GPU per step, "
                        f"{chunk} frames per spt_render call), {args.steps * args.frames_per_step * (sim or world)} "
                        f"spp image in total",
            "scene": args.scene,
            "width": w,
            "height": h,
            "bounces": args.bounces,
            "rr_depth": args.rr_depth,
            "spp_per_step": args.frames_per_step,
            "frames_per_call": chunk,
            "parallelism": f"row-shard{world}" + ((f"+{'spt' if use_spt_gather else 'torch'}-rccl-gather"
                                                   + ("-every-step-overlapped" if every_step else ""))
                                                  if world > 1 else ""),
            "env_map": args.env_map or None,
        },
        "roofline": roofline,
        "roofline_valu": (roofline or {}).get("valu"),
        "roofline_extend": roofline_extend,
        "rooflines": fams,
        "cpu_baseline": None,
        "pmc_label": label,
        "kernel_source": kernel_source_hash(),
        "segments_per_sample": round(seg_total / max(1, st.paths), 4),
        # traced work beside `value`: the camera ray has no jitter (CPUPathTracer.cpp:62-73), so k_paths
        # traces bounce 0 once per pixel per launch and adds the sky pixels' constant radiance without
        # tracing; `value` counts samples (paths), this counts the segments traced
        "traced_segments_per_s": (round(traced_segments(st, args.bounces, shard_px,
                                                        st.schedule == spt.SCHEDULE_FRAME) / elapsed, 1)
                                  if st.schedule in (spt.SCHEDULE_PERSISTENT, spt.SCHEDULE_FRAME) and not sim
                                  and not args.no_profile else None),
        # paths ended by their camera segment (misses): 1 - bounce-1 segments / paths
        "camera_only_path_frac": (round(1.0 - int(st.segments[1]) / max(1, int(st.segments[0])), 4)
                                  if args.bounces > 1 and st.segments[0] else None),
        "nee": {"shadow_rays": int(st.shadow_rays), "emitters": int(st.emitters),
                "shadow_rays_per_sample": round(int(st.shadow_rays) / max(1, st.paths), 4)} if args.nee else None,
        "simulate_world": sim_report,
        "schedule": ["split", "fused", "persistent", "frame"][int(st.schedule)],
        "specialized": specialized,
        "lane_utilization": round(st.lane_busy / st.lane_slots, 4) if st.lane_slots else None,
        # BVH work per segment at bounce >= 1 (k_paths' counters skip the cached camera segments)
        "bvh_per_traced_segment": ({"nodes": round(st.bvh_node_visits / max(1, sum(int(x) for x in st.segments[1:args.bounces])), 2),
                                    "prims": round(st.prim_tests / max(1, sum(int(x) for x in st.segments[1:args.bounces])), 2)}
                                   if st.bvh_node_visits else None),
        "kernel_ms": {"paths": round(st.persistent_ms, 3), "extend": round(st.extend_ms, 3), "shade": round(st.shade_ms, 3),
                      "trace_tail": round(st.tail_ms, 3), "accumulate": round(st.other_ms, 3)},
        "tail_bounce": int(st.tail_bounce),
        "per_bounce": [{"segments": int(st.segments[b]), "extend_ms": round(st.extend_ms_bounce[b], 3),
                        "shade_ms": round(st.shade_ms_bounce[b], 3)} for b in range(args.bounces)],
        "passes": int(st.passes),
    }

    if rank == 0 and world == 1 and not sim and not args.no_cpu_baseline:
        base, cpu_frames, r = cpu_baseline(spt, args, scene_arrays, args.cpu_seconds, total_frames,
                                           flags & spt.FLAG_NEE)
        result["cpu_baseline"] = base
        # parity on the same sub-budget: GPU frames 0..cpu_frames-1 vs the oracle's accumulation
        # (per-frame buffers summed in frame order == the oracle's own in-place accumulation)
        ctx.set_profiling(False)
        ctx.reset()
        ctx.render(0, cpu_frames)
        g = ctx.read_accum().reshape(h, w, 4)
        exact = np.all(g.view(np.uint32) == r.view(np.uint32), axis=-1)
        l2 = np.sqrt(np.sum(((g[..., :3].astype(np.float64) - r[..., :3]) / cpu_frames) ** 2, axis=-1))
        result["parity"] = {"frames": cpu_frames, "rms_l2": float(np.sqrt(np.mean(l2 ** 2))),
                            "max_l2": float(l2.max()), "p999_l2": float(np.quantile(l2, 0.999)),
                            "pixels_l2_over_1e-4": int(np.count_nonzero(l2 > 1e-4)),
                            "exact_pixel_frac": float(exact.mean())}

    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
