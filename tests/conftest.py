"""Shared test setup: import paths, GPU marker, small helpers."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# libmrt honours its diagnostic MRT_* overrides (MRT_INFLIGHT, MRT_BATCH,
# MRT_KERNEL, ...) only under MRT_DIAG=1; the tests set them
os.environ["MRT_DIAG"] = "1"
for sub in ("", "metal-renderer_amd", "oracle", "tests"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    if not os.path.exists(oracle.LIB_PATH):
        oracle.build()
    return oracle


@pytest.fixture(scope="session")
def mrt_mod():
    import mrt
    return mrt


@pytest.fixture(scope="session")
def gpu(mrt_mod):
    """Skip-free GPU gate: a -m gpu run on a box without a device must FAIL."""
    import torch
    assert torch.cuda.is_available(), "gpu test run without a visible HIP device"
    torch.cuda.init()   # torch's bundled HIP runtime must initialise before libmrt's
    torch.zeros(1, device="cuda")
    assert mrt_mod.device_count() > 0, "libmrt.so sees no HIP device"
    return torch
