"""Stage tracing for the aggregation engines (the reference has no tracing of its own).

* ``SDA_TRACE=1``: every engine stage boundary (participate / exchange / clerk /
  reduce / reveal / waves) is a roctx marker -- PyTorch's nvtx API is backed by
  roctx on ROCm -- so ``rocprofv3 --marker-trace`` timelines show the protocol
  stages between the kernels;
* ``time_stages=True`` on an engine: HIP events at the same boundaries,
  reported as ``stage_ms`` in round results and in the bench JSON.
"""
from __future__ import annotations

import os


def tracing_enabled() -> bool:
    return os.environ.get("SDA_TRACE", "0") not in ("", "0", "false", "no")
