#!/usr/bin/env python3
"""Experiment: the committee round on one rank with the clerks' key agreement queued behind
the first wave's share kernel or beside it, alternating in one process (boxes differ by more
than the effect).  python scripts/exp_committee_open_keys.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29561", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")

import torch
import torch.distributed as dist

from sda_amd.engine import reference_sum
from sda_amd.models import Additive, AggregationSpec
from sda_amd.parallel.engine import DistributedAggregator

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
spec = AggregationSpec(1_000_000, 433, Additive(3, 433))
x = torch.randint(0, 433, (1000, 1_000_000), dtype=torch.int32, device="cuda")
ref = reference_sum(x, 433)
agg = DistributedAggregator(spec, engine="device", device=torch.device("cuda", 0), layout="committee",
                            waves=4, force_pipeline=True)
cm = agg._committee


def timed(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        r = agg.run_round(x, check=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    assert torch.equal(r.output, ref)
    return dt


for waves in (1, 2, 4, 8):
    agg.set_waves(waves)
    for _ in range(4):
        agg.run_round(x, check=False)
    res = {True: [], False: []}
    for rep in range(4):
        for flag in (True, False):
            cm.open_keys_behind_share = flag
            timed(3)
            res[flag].append(timed(10))
    print(f"waves {waves}: behind the share kernel {min(res[True]):.2f} ms (" +
          " ".join(f"{v:.2f}" for v in res[True]) + f"), beside it {min(res[False]):.2f} ms (" +
          " ".join(f"{v:.2f}" for v in res[False]) + ")", flush=True)
assert int(agg.engine.take_errors().item()) == 0
dist.destroy_process_group()
