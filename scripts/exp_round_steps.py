#!/usr/bin/env python3
"""Per-round times inside a bench-like loop of unchecked headline rounds (an event on the
main stream after every round): what the first rounds after a synchronisation cost more
than the later ones.  python scripts/exp_round_steps.py [STEPS] [IDLE_MS]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from sda_amd.engine import DeviceAggregator, reference_sum
from sda_amd.models import Additive, AggregationSpec

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
idle_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
dev = torch.device("cuda", 0)
spec = AggregationSpec(1_000_000, 433, Additive(3, 433))
agg = DeviceAggregator(spec, dev)
x = torch.randint(0, 433, (1000, 1_000_000), dtype=torch.int32, device=dev)
ref = reference_sum(x, 433)
warm = [agg.run_round(x, check=False) for _ in range(5)]
for r in warm:
    assert int(r.err.item()) == 0 and torch.equal(r.output, ref)
del warm
for trial in range(3):
    agg.take_errors()
    torch.cuda.synchronize()
    time.sleep(idle_ms / 1e3)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    host = []
    for i in range(steps):
        th = time.perf_counter()
        res = agg.run_round(x, check=False)
        host.append((time.perf_counter() - th) * 1e3)
        evs[i + 1].record()
    e = agg.take_errors()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    assert int(e.item()) == 0 and torch.equal(res.output, ref)
    gaps = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
    print(f"trial {trial}: wall {wall / steps:.3f} ms/round; per round on the main stream:",
          " ".join(f"{g:.2f}" for g in gaps), "| host ms:", " ".join(f"{h:.1f}" for h in host), flush=True)
