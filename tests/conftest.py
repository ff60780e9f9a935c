import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture
def knobs(monkeypatch):
    """Set MMDX_* launch-heuristic knobs for one test: the environment variable plus
    mmdx_reload_config (libmmdx_hip.so reads the knobs once per process); knobs(name, None)
    unsets one.  Undone, and the library re-read, after the test."""
    from mmdx import _lib as L

    def set_(name, value):
        if value is None:
            monkeypatch.delenv(name, raising=False)
        else:
            monkeypatch.setenv(name, str(value))
        L.reload_config()
    yield set_
    monkeypatch.undo()
    L.reload_config()
