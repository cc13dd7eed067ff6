"""bench.py's launch contract on the host: `--gpus N` (N > 1) without a launcher starts the N ranks
itself as a child torch.distributed.run (before anything touches a GPU) or fails loudly — it never
silently measures one GPU and reports it as N."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_gpus_2_without_launcher_and_gpus_fails_loudly():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""  # whatever the host has: no GPU visible to this run
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
    assert '"metric"' not in r.stdout


def test_gpus_n_without_launcher_spawns_n_ranks(monkeypatch):
    bench = load_bench()
    import torch

    calls = []
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: calls.append(cmd) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    args = bench.parse()
    assert bench.launch_ranks(args) == 0
    (cmd,) = calls
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-5:] == [BENCH, "--gpus", "4", "--steps", "3"]


def test_world_size_mismatch_is_an_error(monkeypatch):
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1"], capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE 2" in r.stderr


def test_pmc_records_are_keyed_by_shape_and_kernel_source(tmp_path, monkeypatch):
    """roofline.traffic comes only from a PMC record of the same launch shape on the same kernel
    source; anything else reports null."""
    bench = load_bench()
    label = "cornell-1920x1080-b8-world1-f64"
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    os.makedirs(tmp_path / "profiles")
    os.makedirs(tmp_path / "software-path-tracer_amd" / "csrc")
    for n in ("spt_kernels.hip", "spt_kernels.h", "spt_device.h", "spt_jit.hip"):
        (tmp_path / "software-path-tracer_amd" / "csrc" / n).write_text(n)
    rec = {"traffic_bytes": 1.0e8, "valu_insts": 1.0e9, "duration_ns": 2.0e6, "clock_ghz": 2.1}
    import json
    (tmp_path / "profiles" / "pmc_r02.json").write_text(json.dumps(
        {label: {"kernel_source": bench.kernel_source_hash(), "kernels": {"spt::k_paths<false, false, 0>": rec}}}))
    assert bench.committed_pmc(label, "k_paths") == rec
    assert bench.committed_pmc(label.replace("f64", "f20"), "k_paths") is None
    (tmp_path / "software-path-tracer_amd" / "csrc" / "spt_kernels.hip").write_text("changed")
    assert bench.committed_pmc(label, "k_paths") is None


def test_pmc_collect_and_bench_hash_the_same_sources():
    """scripts/pmc_collect.py stamps records with the hash bench.py checks: the two must agree."""
    import importlib.util

    def load(path, name):
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bench = load(os.path.join(root, "bench.py"), "bench_for_hash")
    pmc = load(os.path.join(root, "scripts", "pmc_collect.py"), "pmc_for_hash")
    assert bench.kernel_source_hash() == pmc.kernel_source_hash()


def test_traced_segments_accounting():
    """SURVEY.md 8(d)'s traced work: k_paths traces bounce 0 once per pixel per launch, k_frame none of
    its camera segments (their hits come from the per-pixel cache); both add every later
    segment and the NEE shadow rays."""
    bench = load_bench()

    class St:
        segments = [1000, 400, 150, 50] + [0] * 28
        persistent_launches = 3
        shadow_rays = 7

    assert bench.traced_segments(St, 4, 100, frame_kernel=True) == 400 + 150 + 50 + 7
    assert bench.traced_segments(St, 4, 100, frame_kernel=False) == 400 + 150 + 50 + 3 * 100 + 7
    assert bench.traced_segments(St, 2, 100, frame_kernel=True) == 400 + 7  # only bounces < max_bounces
