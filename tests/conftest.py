"""Test configuration.  `-m gpu` tests need an MI355X (run through gpurun); everything else runs on
CPU and covers the oracle against golden/KAT vectors, host logic and the C-ABI surface."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct MI355X (gfx950)")


@pytest.fixture(scope="session")
def root():
    return ROOT


@pytest.fixture(scope="session")
def data_dir():
    return os.path.join(ROOT, "data")
