"""gfx950 HIP kernel ops (see csrc/kernels)."""
from . import gpu  # noqa: F401
from .sealed import Arena, seal, open_  # noqa: F401
