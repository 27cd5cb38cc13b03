#!/usr/bin/env python3
"""Soak of the round loop: hundreds of unchecked rounds over fresh inputs and several
aggregation kinds, results read one round late, now and then at once or through a checked
round, every output compared with the plain sum and the engines' running error words zero.
python scripts/soak_rounds.py [ROUNDS]"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from sda_amd.engine import DeviceAggregator, reference_sum
from sda_amd.models import PSS_4_8_3, Additive, AggregationSpec, ChaChaMask, FullMask

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 300
headline = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # that many headline-shape rounds too
dev = torch.device("cuda", 0)
m = 433
rng = random.Random(7)
kinds = {
    "additive": lambda D: AggregationSpec(D, m, Additive(3, m)),
    "fullmask": lambda D: AggregationSpec(D, m, Additive(3, m), FullMask(m)),
    "chacha": lambda D: AggregationSpec(D, m, Additive(3, m), ChaChaMask(m, D)),
    "pss": lambda D: AggregationSpec(D, m, PSS_4_8_3),
}
engines = {}
for name, mk in kinds.items():
    for D, P in ((200_003, 64), (30_011, 12)):
        engines[(name, D, P)] = DeviceAggregator(mk(D), dev)
keys = list(engines)
pending = []  # (result, reference, label)
bad = 0


def settle(upto):
    global bad
    while len(pending) > upto:
        res, ref, label = pending.pop(0)
        if not torch.equal(res.output, ref):
            bad += 1
            print("WRONG OUTPUT", label, flush=True)


for i in range(rounds):
    key = rng.choice(keys)
    name, D, P = key
    agg = engines[key]
    x = torch.randint(0, m, (P, D), dtype=torch.int32, device=dev)
    ref = reference_sum(x, m)
    mode = rng.random()
    if mode < 0.1:
        res = agg.run_round(x)  # checked: raises on an error word
        pending.append((res, ref, f"round {i} {key} checked"))
    else:
        res = agg.run_round(x, check=False)
        pending.append((res, ref, f"round {i} {key}"))
    settle(0 if mode > 0.9 else 1)  # mostly one round late, sometimes at once
    if i % 50 == 49:
        print(f"{i + 1} rounds", flush=True)
settle(0)
if headline:
    big = DeviceAggregator(AggregationSpec(1_000_000, m, Additive(3, m)), dev)
    engines[("additive", 1_000_000, 1000)] = big
    xs = [torch.randint(0, m, (1000, 1_000_000), dtype=torch.int32, device=dev) for _ in range(3)]
    refs = [reference_sum(x, m) for x in xs]
    for i in range(headline):
        res = big.run_round(xs[i % 3], check=False)
        pending.append((res, refs[i % 3], f"headline round {i}"))
        settle(1)
    settle(0)
torch.cuda.synchronize()
errs = {k: int(a.take_errors().item()) for k, a in engines.items()}
assert not any(errs.values()), errs
assert bad == 0, f"{bad} wrong outputs"
print(f"soak ok: {rounds} rounds over {len(engines)} engines, all outputs right, no error words", flush=True)
