import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


# JoinHash's output chunk builders split into a job per 64 partitions (default 2048), so that the small joins of the
# tests run several builder jobs too (operators.cpp; read once when the first JoinHash executes)
os.environ.setdefault("HY_OP_PARTS_PER_JOB", "64")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def hy():
    import helpers

    return helpers.load_pkg()


@pytest.fixture(scope="session")
def oracle():
    import helpers

    return helpers.load_oracle()
