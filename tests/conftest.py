"""pytest configuration: the `gpu` marker, and import helpers for the package and the oracle.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, C-ABI exports, gloo ranks.
`-m gpu` runs on an MI355X: parity of the HIP path (through the C-ABI) against the oracle.
"""
import importlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
ORACLE_DIR = os.path.join(ROOT, "oracle")
if ORACLE_DIR not in sys.path:
    sys.path.insert(0, ORACLE_DIR)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path through the C-ABI")


def _ensure_built():
    lib = os.path.join(ROOT, "software-path-tracer_amd", "libspt_hip.so")
    orc = os.path.join(ORACLE_DIR, "build", "libcpu_ref.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        subprocess.run(["make", "-s", "-j8", "-C", ROOT, "all", "oracle"], check=True)


@pytest.fixture(scope="session")
def spt():
    _ensure_built()
    return importlib.import_module("software-path-tracer_amd")


@pytest.fixture(scope="session")
def ref():
    _ensure_built()
    import cpu_ref

    return cpu_ref


@pytest.fixture(scope="session")
def gpu_ctx(spt):
    """One spt context for the whole GPU session (tests reconfigure it)."""
    ctx = spt.Context(0)
    yield ctx
    ctx.close()
