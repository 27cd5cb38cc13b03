"""Utilities: tracing switches."""
from .trace import tracing_enabled  # noqa: F401
