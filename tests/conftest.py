"""Shared pytest setup: markers, import paths, golden-fixture loader."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "hmc-stellar-toy-model_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a real GPU; skips only when no GPU is visible."""
    from rhmc_amd import capi
    if not capi.device_available():
        pytest.skip("no GPU visible")
    return capi
