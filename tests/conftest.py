import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "multi-cluster-simulator_amd")
for p in (PKG_DIR, REPO, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libmcs.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running")


def _hip_device_present() -> bool:
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine():
    """One engine on device 0 for the whole GPU session (one process, one GPU)."""
    if not _hip_device_present():
        pytest.fail("gpu test selected but no HIP device is visible")
    from mcs_amd import Engine

    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="session")
def assets_dir():
    return os.path.join(REPO, "assets")
