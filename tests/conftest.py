"""Shared pytest configuration.

Markers
-------
gpu : needs a real MI355X (gfx950) and the built `_sda_gpu` extension. The driver
      runs `-m "not gpu"` on CPU-only machines and `-m gpu` on a GPU box.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU and the HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def native():
    from sda_amd._native import native as _n
    return _n()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sda_amd._native import gpu
    gpu()  # must load: a GPU box without the extension is a failure, not a skip
    return torch.device("cuda")
