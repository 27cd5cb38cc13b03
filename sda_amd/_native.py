"""Loader for the in-tree native extensions.

* ``_sda_native`` -- C++ control plane + host crypto (always required)
* ``_sda_gpu``    -- HIP/CDNA4 kernels for gfx950 (required on a GPU box)

Both live in ``sda_amd/_lib`` and are built by ``make`` (see ``__graft_entry__``).
A missing GPU extension on a machine that *has* a GPU is an error, never a silent
fallback: every GPU op calls :func:`gpu` which raises.
"""
from __future__ import annotations

import importlib
import os
import sys

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
_cache: dict = {}


def _load(name: str):
    if name in _cache:
        return _cache[name]
    if _LIB_DIR not in sys.path:
        sys.path.insert(0, _LIB_DIR)
    try:
        mod = importlib.import_module(name)
    except ImportError as e:  # pragma: no cover - exercised only when unbuilt
        raise ImportError(
            f"sda_amd native extension {name!r} is not built; run `make -j8` "
            f"(or __graft_entry__.build()) in the repository root: {e}"
        ) from e
    _cache[name] = mod
    return mod


def native():
    """The host control-plane / crypto module."""
    return _load("_sda_native")


def gpu():
    """The gfx950 kernel module. Raises loudly if it is missing."""
    if "_sda_gpu" not in _cache:
        # torch first: it brings its own copy of the HIP runtime, and the module must
        # bind to the runtime torch's streams and tensors belong to. Loaded ahead of
        # torch, the module pulled in the system's runtime and its first launch failed
        # with "no ROCm-capable device is detected" once torch had initialised its own.
        import torch  # noqa: F401
    return _load("_sda_gpu")


def lib_dir() -> str:
    return _LIB_DIR


def bin_path(name: str) -> str:
    return os.path.join(_LIB_DIR, "bin", name)
