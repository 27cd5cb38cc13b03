#!/usr/bin/env python3
"""Experiment: headline rounds with the encode kernel's LDS tile sized for two-byte codes
(16-bit values below 2^13: 17 KB, eight workgroups a CU) or for three-byte ones (25 KB, six),
alternating in one process.  python scripts/exp_encode_tile2.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from sda_amd._native import gpu
from sda_amd.engine import DeviceAggregator, reference_sum
from sda_amd.models import Additive, AggregationSpec

dev = torch.device("cuda", 0)
agg = DeviceAggregator(AggregationSpec(1_000_000, 433, Additive(3, 433)), dev)
x = torch.randint(0, 433, (1000, 1_000_000), dtype=torch.int32, device=dev)
ref = reference_sum(x, 433)


def timed(n):
    t0 = time.perf_counter()
    for _ in range(n):
        r = agg.run_round(x, check=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    assert torch.equal(r.output, ref)
    return dt


timed(6)
res = {1: [], 0: []}
for rep in range(5):
    for flag in (1, 0):
        gpu().set_encode_tile2(flag)
        timed(4)
        res[flag].append(timed(16))
gpu().set_encode_tile2(1)
assert int(agg.take_errors().item()) == 0
for flag in (1, 0):
    print(f"tile for {'two' if flag else 'three'}-byte codes: min {min(res[flag]):.3f} ms  (" +
          " ".join(f"{v:.3f}" for v in res[flag]) + ")", flush=True)
