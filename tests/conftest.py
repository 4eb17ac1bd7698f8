import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()


def pytest_collection_modifyitems(session, config, items):
    """The eight-rank one-GPU rehearsal (test_tp8_gpu.py) runs first: its eight processes take
    one hardware queue each, and a pytest process that already initialised HIP for earlier GPU
    tests holds four more - queues past the scheduler's slots are time-sliced, which stretches
    every collective hand-off between the ranks (tools/p2p_latency.py, r4)."""
    first = [it for it in items if it.nodeid.startswith("tests/test_tp8_gpu.py")]
    if first:
        rest = [it for it in items if it not in first]
        items[:] = first + rest
