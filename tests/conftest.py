import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: long-running (multi-second) test")


def _ensure_built():
    lib = os.path.join(REPO, "go-pbrt_amd", "lib", "libpbrt_gpu.so")
    orc = os.path.join(REPO, "oracle", "_build", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "go-pbrt_amd")], check=True)


_ensure_built()


@pytest.fixture(autouse=True)
def _no_schedule_cache(monkeypatch):
    """Every context a test creates learns its own schedule: the process-wide
    schedule cache (render.hip, on by default) would otherwise hand one test's
    measured order to the next test's fresh context and change which frames
    split. tests/test_gpu_schedule_cache.py turns it back on."""
    monkeypatch.setenv("PBRT_CI_ORDER_CACHE", "0")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    return oracle_lib


@pytest.fixture(scope="session")
def pbrtgpu():
    import pbrtgpu as G
    return G
