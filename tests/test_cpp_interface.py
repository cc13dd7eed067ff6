"""The C++ render::PathTracer backend (libspt_render.so) driven the way the reference App drives
its backend (tests/cpp/test_pathtracer.cpp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "test_pathtracer")


@pytest.fixture(scope="module")
def exe(spt):
    subprocess.run(["make", "-s", "-C", ROOT, "cpp-tests"], check=True)
    return EXE


def test_cpp_interface_cpu(exe):
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


@pytest.mark.gpu
def test_cpp_app_scene_on_gpu(exe):
    r = subprocess.run([exe, "gpu", "256", "192", "8"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ("160", "96", "3", "5", "6", "1", "1.7", "1"),   # progressive: 15 frames, k_paths calls of 5
    ("96", "64", "2", "2", "8", "3", "0.5", "0"),    # not progressive: every call frames 0..1 (k_frame)
])
def test_cpp_settings_mode_on_gpu(exe, args):
    """HIPPathTracer::set_settings_mode(true): RenderSettings bounces / RR / spp / progressive /
    exposure honoured, vs the oracle; then back to reference mode."""
    r = subprocess.run([exe, "settings", *args], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_bvh_quantized_nodes_contain_fp32_boxes(exe):
    """The device's 64-B quantized BVH nodes decode exactly and contain every fp32 child box they
    came from (C4, C5 and App scenes; scene.h BvhNodeQ) — so traversal finds the same hits."""
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "test_bvh")], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


def test_device_sincos_matches_glibc(exe):
    """spt_device.h sincos_2pi (host build) vs glibc cos/sin on 2e7 reference-RNG draws: the float
    products the integrator uses must be identical."""
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "test_sincos"), "20000000"], capture_output=True,
                       text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_device_sqrt_unit_exhaustive(exe):
    """spt_device.h on the GPU: sqrt_unit == sqrtf on 0 and [2^-96, 2^96), inv_sqrt_ref == 1/sqrtf on all
    2^32 inputs, div_ref == n / s for every divisor in [2^-40, 2^20) (the flat loop's fast-path ranges)."""
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "test_device_math")], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr
