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
def _oracle_device_libm():
    """The oracle's default libm convention is the reference's (glibc sinf / cosf / powf,
    oracle.LIBM_FLOAT).  The bit-exact GPU-vs-oracle tests compare under the device's
    convention for those three functions (double, rounded once: oracle.LIBM_DEVICE) --
    atan2f / acosf are glibc's in both (csrc/mrt_libm.h).  Tests that compare against
    the reference's convention pass libm=oracle.LIBM_FLOAT explicitly and hold the
    north_star tolerance (tests/test_full_size.py, tests/test_final_scene.py)."""
    import oracle
    prev = oracle.set_default_libm(oracle.LIBM_DEVICE)
    yield
    oracle.set_default_libm(prev)
