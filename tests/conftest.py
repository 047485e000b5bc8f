import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: CPU tests at BASELINE sizes (quick suite: -m 'not gpu and not slow')")


@pytest.fixture(scope="session")
def counter():
    """One GPU context for the whole GPU test session (product path only)."""
    import approx_counter_amd as ac

    c = ac.ApproxCounter()
    yield c
    c.close()
