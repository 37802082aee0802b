import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdlq.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from dlq_amd import lib  # raises loudly if libdlq.so is missing
    return lib


@pytest.fixture
def knobs():
    """Set libdlq knobs (dlq_set_knob) for one test; restored afterwards."""
    from dlq_amd import lib as L
    saved = {}

    def set_(name, value):
        old = L.set_knob(name, value)
        saved.setdefault(name, old)

    yield set_
    for name, old in saved.items():
        L.set_knob(name, old)
