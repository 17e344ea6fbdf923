import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "tests"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long CPU run (minutes)")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN
