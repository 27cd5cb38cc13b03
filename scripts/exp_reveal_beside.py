#!/usr/bin/env python3
"""Experiment: headline rounds with the result path on its own stream or on the main stream,
alternating in one process (boxes differ by more than the effect).
python scripts/exp_reveal_beside.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

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
res = {True: [], False: []}
for rep in range(5):
    for flag in (True, False):
        agg.overlap_reveal = flag
        timed(4)  # keeps the card at its clocks; the next loop starts right behind it
        res[flag].append(timed(16))
assert int(agg.take_errors().item()) == 0
for flag in (True, False):
    print(f"result path {'on its own stream' if flag else 'on the main stream'}: min {min(res[flag]):.3f} ms  (" +
          " ".join(f"{v:.3f}" for v in res[flag]) + ")", flush=True)
