import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X, gfx950)")


def pytest_collection_modifyitems(session, config, items):
    # torch's wheel bundles its own HIP runtime; when a process uses both torch and
    # libfsx_hip.so (/opt/rocm runtime), torch must initialise the device first.
    if any(it.get_closest_marker("gpu") for it in items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def native():
    """The in-tree libfsx_hip.so (built only if missing: on the GPU box the libraries
    built in the source container are used as shipped)."""
    from flowsentryx_amd import build, lib
    build.build_all(only_missing=True)
    return lib
