"""Shared test setup: the `gpu` marker, import paths, and the oracle build."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def orc():
    from oracle import pyoracle
    if not os.path.exists(pyoracle.LIB):
        pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def hw():
    import hwbloomradixjoin_amd as hw
    hw.lib()  # raises if libhwbrj.so is missing: no silent fallback
    return hw


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture
def hook(hw):
    """hook(HOOK, value): hwbrj_set_test_hook for this test only (switched off at teardown)."""
    done = []

    def set_hook(h, value):
        hw.set_test_hook(h, int(value))
        done.append(h)
    yield set_hook
    for h in done:
        hw.set_test_hook(h, hw._HOOK_OFF[h])
