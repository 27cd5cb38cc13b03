"""gfx950 HIP kernel ops (see csrc/kernels)."""
from . import gpu  # noqa: F401
from .sealed import Arena, seal, open_, seal_setup, seal_data, open_setup, open_data  # noqa: F401
