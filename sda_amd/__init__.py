"""sda_amd -- an MI355X-native Secure Distributed Aggregation framework.

Capabilities of Snips' SDA (`sanyaade-machine-learning/sda`): private sums of
integer vectors from many participants via masking, additive / packed-Shamir
secret sharing and libsodium sealed boxes, coordinated by a REST server.

Layout
------
``sda_amd.protocol``  resources / schemes / JSON wire format (C++ codec)
``sda_amd.server``    in-process server, stores (memory / JFS / document), HTTP
``sda_amd.client``    agent roles (participant, clerk, recipient) over any service
``sda_amd.ops``       gfx950 HIP kernels (share, seal, open, combine, reconstruct)
``sda_amd.engine``    device aggregation engine (simulated participants/clerks)
``sda_amd.parallel``  multi-GPU engine over torch.distributed (RCCL / xGMI)
``sda_amd.models``    aggregation scheme presets (the "model zoo" of job specs)
``sda_amd.utils``     timing, env, keys helpers
"""
from __future__ import annotations

__version__ = "0.1.0"

from ._native import native, gpu  # noqa: F401
