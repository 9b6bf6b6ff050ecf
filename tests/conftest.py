import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"
HAS_REFERENCE = os.path.isdir(os.path.join(REFERENCE, "src"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    if not os.path.exists(oracle_lib.LIB):
        oracle_lib.build()
    return oracle_lib


@pytest.fixture(scope="session")
def kdpt():
    """The product library (host builder + C-ABI); built in-tree if missing."""
    from kdtreepathtraceroptimization_amd import _build, runtime
    if not os.path.exists(runtime.LIB_PATH):
        _build.build()
    runtime.load_library()
    return runtime


@pytest.fixture(scope="session")
def anchors():
    import json
    with open(os.path.join(TESTS, "golden", "anchors.json")) as f:
        return json.load(f)


needs_reference = pytest.mark.skipif(not HAS_REFERENCE, reason="/root/reference not present")
