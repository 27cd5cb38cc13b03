#!/usr/bin/env python3
"""Experiment: the headline round with the lean decode-sum's accumulator rows plain
(default for m = 433) and padded: wall time per round, outputs checked."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd._native import gpu  # noqa: E402
from sda_amd.engine import DeviceAggregator, reference_sum  # noqa: E402
from sda_amd.models.schemes import Additive, AggregationSpec  # noqa: E402

agg = DeviceAggregator(AggregationSpec(1_000_000, 433, Additive(3, 433)))
x = torch.randint(0, 433, (1000, 1_000_000), dtype=torch.int32, device="cuda")
ref = reference_sum(x, 433)
for mode in (-1, 1, -1, 1):
    gpu().set_decode_swz(mode)
    for _ in range(3):
        assert torch.equal(agg.run_round(x).output, ref)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        agg.run_round(x, check=False)
    torch.cuda.synchronize()
    print(f"decode swz {mode}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/round", flush=True)
gpu().set_decode_swz(-1)
