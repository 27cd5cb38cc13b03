#!/usr/bin/env python3
"""Experiment: consecutive rounds alternating between LANES streams (each round with
its own key-agreement side stream), against the same rounds on one stream.

  python scripts/exp_two_lanes.py CONFIG [LANES] [STEPS] [INFLIGHT_PER_LANE]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import sda_amd.engine as E
from sda_amd.engine import DeviceAggregator
from sda_amd.models.configs import bench_config

c = int(sys.argv[1])
lanes_n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
E._MAX_INFLIGHT = int(sys.argv[4]) if len(sys.argv) > 4 else 1
cfg = bench_config(c)
spec = cfg.spec()
dev = torch.device("cuda", 0)
x = torch.randint(0, spec.field_modulus, (cfg.participants, cfg.dimension), dtype=torch.int32, device=dev)
ref = torch.remainder(x.to(torch.int64).sum(0), spec.field_modulus).to(torch.int32)
clerks = list(cfg.clerks) if cfg.clerks is not None else None
engs = [DeviceAggregator(spec, device=dev, pss_backend=cfg.pss_backend) for _ in range(lanes_n)]
lanes = [torch.cuda.Stream(device=dev) for _ in range(lanes_n)]
torch.cuda.synchronize()


def run(n):
    outs = []
    for i in range(n):
        l = i % lanes_n
        with torch.cuda.stream(lanes[l]):
            outs.append(engs[l].run_round(x, clerks=clerks, check=False))
    torch.cuda.synchronize()
    return outs


for r in run(2 * lanes_n):
    assert int(r.err.item()) == 0 and torch.equal(r.output, ref)
t0 = time.perf_counter()
outs = run(steps)
dt = time.perf_counter() - t0
for r in outs:
    assert int(r.err.item()) == 0 and torch.equal(r.output, ref)
print(f"config {c} lanes {lanes_n} inflight/lane {E._MAX_INFLIGHT}: {dt / steps * 1e3:.2f} ms/round "
      f"(high water {torch.cuda.max_memory_allocated() / 1e9:.1f} GB)", flush=True)
