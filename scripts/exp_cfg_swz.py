#!/usr/bin/env python3
"""Experiment: a benchmark configuration's rounds with the lean decode-sum's accumulator
rows plain and padded, or (with `long`) its byte-wise and value-wise long-code kernels
(usage: exp_cfg_swz.py CONFIG [long]): wall time per round."""
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
which = "long" if len(sys.argv) > 2 and sys.argv[2] == "long" else "swz"
setter = gpu().set_decode_long if which == "long" else gpu().set_decode_swz
for mode in (0, 1, 0, 1):
    setter(mode)
    for _ in range(2):
        eng.run_round(x, check=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        eng.run_round(x, check=False)
    torch.cuda.synchronize()
    print(f"config {sys.argv[1]} decode {which} {mode}: "
          f"{(time.perf_counter() - t0) / 5 * 1e3:.2f} ms/round", flush=True)
setter(-1)
