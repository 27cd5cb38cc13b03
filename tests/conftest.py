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


def _host_build_is_stale() -> bool:
    """True when the host module or a CLI binary is missing or older than a source."""
    import glob

    from sda_amd._native import bin_path, lib_dir

    outs = glob.glob(os.path.join(lib_dir(), "_sda_native*.so"))
    outs += [bin_path(b) for b in ("sda", "sdad", "sda_selftest", "sda_cpu_bench")]
    if not outs or not all(os.path.exists(o) for o in outs) or len(outs) < 5:
        return True
    built = min(os.path.getmtime(o) for o in outs)
    srcs = []
    for pat in ("csrc/src/*.cc", "csrc/bin/*.cc", "csrc/python/*.cc", "csrc/include/sda/*.hpp"):
        srcs += glob.glob(os.path.join(ROOT, pat))
    return any(os.path.getmtime(s) > built for s in srcs)


@pytest.fixture(scope="session")
def native():
    # the binaries and the extension are build products (not tracked): tests
    # always run what the sources in this checkout produce
    if _host_build_is_stale() and os.access(ROOT, os.W_OK):
        import subprocess

        subprocess.run(["make", "-C", ROOT, "-j8", "host"], check=True, capture_output=True)
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
