#!/usr/bin/env python3
"""Experiment: a benchmark configuration's rounds with the lean decode-sum's accumulator
rows plain and padded (usage: exp_cfg_swz.py CONFIG): wall time per round."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd._native import gpu  # noqa: E402
from sda_amd.engine import DeviceAggregator  # noqa: E402
from sda_amd.models.configs import bench_config  # noqa: E402

cfg = bench_config(int(sys.argv[1]))
spec = cfg.spec()
eng = DeviceAggregator(spec)
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.randint(0, spec.field_modulus, (cfg.participants, spec.dimension), dtype=torch.int32,
                  device="cuda", generator=g)
for mode in (0, 1, 0, 1):
    gpu().set_decode_swz(mode)
    for _ in range(2):
        eng.run_round(x, check=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        eng.run_round(x, check=False)
    torch.cuda.synchronize()
    print(f"config {cfg.number if hasattr(cfg, 'number') else sys.argv[1]} decode swz {mode}: "
          f"{(time.perf_counter() - t0) / 5 * 1e3:.2f} ms/round", flush=True)
gpu().set_decode_swz(-1)
