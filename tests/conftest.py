import os
import sys

import pytest

# torch bundles its own libamdhip64.so.7; if librt_hip.so is loaded first the
# process binds /opt/rocm's copy and torch then finds no GPU.  Load torch's
# runtime first so both share it (bench.py does the same).
try:
    import torch  # noqa: F401
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "se-195-project-ray-tracer_amd")
for p in (PKG, os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running exhaustive check")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    oracle_lib.lib()
    return oracle_lib


@pytest.fixture(scope="session")
def rt():
    """The product library; a GPU test fails (not skips) if it cannot load."""
    import rtamd
    rtamd.lib()
    if rtamd.device_count() < 1:
        pytest.fail("no HIP device visible to a gpu-marked test")
    return rtamd
