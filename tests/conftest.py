import os
import sys

import pytest

try:  # torch before libjpge: torch brings its own HIP runtime, and a process must load
    import torch  # noqa: F401  (one copy of it — loaded second, it finds no GPU)
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP path)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def encoder():
    import jpgenc_amd
    enc = jpgenc_amd.Encoder(0)
    yield enc
    enc.close()
