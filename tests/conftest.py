import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def native():
    from simplepathtracer_amd import _native
    _native.build()
    _native.lib()
    return _native


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def golden_scenes():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "scenes.npz"), allow_pickle=False))
