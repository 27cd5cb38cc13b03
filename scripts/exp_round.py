#!/usr/bin/env python3
"""Timing-only harness for kernel experiments: headline-shaped rounds with the
output and error checks off (an experimental kernel variant may compute garbage),
meant to run under `rocprofv3 --kernel-trace --stats`. Prints nothing of value
itself; read the per-kernel times from the profiler output (scripts/kstats.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd.engine import DeviceAggregator  # noqa: E402
from sda_amd.models.schemes import Additive, AggregationSpec  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
agg = DeviceAggregator(AggregationSpec(1_000_000, 433, Additive(3, 433)))
x = torch.randint(0, 433, (1000, 1_000_000), dtype=torch.int32, device="cuda")
for _ in range(rounds):
    agg.run_round(x, check=False)
torch.cuda.synchronize()
print("rounds", rounds)
