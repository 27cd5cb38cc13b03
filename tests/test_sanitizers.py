"""Host control plane under AddressSanitizer+UBSan and ThreadSanitizer.

Builds csrc/bin/sda_selftest.cc with the sanitizers (make asan / make tsan) and
runs it: crypto round trips, wire codec, every store backend, full in-process
loops with real client crypto, and concurrent REST clients against the HTTP
server. Host code only -- GPU sanitizers are not available on the GPU pool.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("target", ["asan", "tsan"])
def test_selftest_under_sanitizer(target):
    r = subprocess.run(["make", "-C", ROOT, target], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sda_selftest: all ok" in r.stdout


def test_selftest_plain(native):
    exe = os.path.join(ROOT, "sda_amd", "_lib", "bin", "sda_selftest")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "all ok" in r.stdout, r.stderr
