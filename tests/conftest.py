import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def validator():
    from comdb2_amd.hsc import Validator
    v = Validator(0)
    yield v
    v.close()
