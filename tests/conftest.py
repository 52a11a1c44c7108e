import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools", "synth")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests of the HIP backend")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def native_lib():
    from av1dec_amd import native
    native.build()
    return native.lib()
