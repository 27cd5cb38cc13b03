#!/usr/bin/env python3
"""Clerk-stage micro-benchmark: open + combine of the headline round's inbox
(1000 participants x 3 clerks x 1M values, m = 433), old path (open_data +
colsum) vs the fused path (open_sum).

python scripts/bench_clerk.py [--participants P] [--dim D] [--reps R]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--participants", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from sda_amd.engine import DeviceAggregator
    from sda_amd.models.schemes import Additive, AggregationSpec
    from sda_amd.ops import gpu as G
    from sda_amd.ops.sealed import open_data, open_sum

    m, n, P, D = 433, 3, args.participants, args.dim
    dev = torch.device("cuda")
    agg = DeviceAggregator(AggregationSpec(D, m, Additive(n, m)), dev)
    x = torch.randint(0, m, (P, D), dtype=torch.int32, device=dev)
    err = agg.new_error_word()
    st = agg._participate(x, list(range(n)), err, 0, local_clerks=True)
    torch.cuda.synchronize()
    inbox, keys = st["inbox"], st["ko_clerk"][0]
    saved = inbox.ct.clone()
    res = {}

    def timed(fn):
        ts = []
        out = None
        for _ in range(args.reps):
            inbox.ct.copy_(saved)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            out = fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return sorted(ts)[len(ts) // 2], out

    def old():
        vals = open_data(inbox, keys, err, out_dtype=agg.vdtype)
        out = torch.empty(n, D, dtype=torch.int32, device=dev)
        G.colsum(vals.view(n, P, D), m, out)
        return out

    res["old_open_data_colsum_ms"], ref = timed(old)
    out = torch.empty(n, D, dtype=torch.int32, device=dev)
    res["open_sum_ms"], out = timed(lambda: open_sum(inbox, keys, err, rows=n, out=out))
    res["open_sum_correct"] = bool(torch.equal(out, ref))
    res["err"] = int(err.item())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
