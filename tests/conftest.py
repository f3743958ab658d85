import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "rendering-algorithms-raytracer_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_MODELS = "/root/reference/Models"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU check")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(scope="session", autouse=True)
def _oracle_reference_libm():
    """Every GPU-vs-oracle comparison uses the reference's libm convention (glibc's atan2f /
    acosf / sinf / cosf / powf, oracle.LIBM_FLOAT): the device restates those five functions
    bit for bit (csrc/mrt_libm.h, pinned by tests/test_libm.py)."""
    import oracle
    prev = oracle.set_default_libm(oracle.LIBM_FLOAT)
    yield
    oracle.set_default_libm(prev)
