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


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    return oracle_lib


@pytest.fixture(scope="session")
def pbrtgpu():
    import pbrtgpu as G
    return G
