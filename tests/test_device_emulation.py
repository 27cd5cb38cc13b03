"""The device algorithms on the CPU: `csrc/kernels/host_emul.cpp` compiles the kernels'
own header code (Salsa20 / HSalsa20 / BLAKE2b / X25519 ladders, the chunked and the
matrix-core Poly1305 formulations with their tables, the per-tile MAC of the encode
kernel, the 24-bit Barrett step, the packed varint pairs) for the host and checks it
against the host crypto library (sealed boxes as sodiumoxide makes them,
client/src/crypto/encryption/sodium.rs:36-43) on random and edge-case inputs."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_device_algorithms_on_the_host(native):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not (os.path.exists(hipcc) or shutil.which("hipcc")):
        pytest.skip("no hipcc: the emulation is built from the kernels' headers")
    for _ in range(3):  # inputs are drawn fresh on every run
        out = subprocess.run(["make", "-C", ROOT, "emul"], capture_output=True, text=True, timeout=500)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
        assert "host_emul: all ok" in out.stdout
