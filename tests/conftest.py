import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def h3c():
    return importlib.import_module("3fs_amd")


@pytest.fixture(scope="session")
def orc():
    import oracle_lib

    return oracle_lib


@pytest.fixture
def hooks(h3c):
    """set(key, value) forces an engine path through h3c_test_hook; every key set is reset to
    its default when the test ends."""
    used = []

    def set_(key, value):
        used.append(key)
        h3c.set_test_hook(key, value)

    yield set_
    for k in used:
        h3c.set_test_hook(k, 0)
