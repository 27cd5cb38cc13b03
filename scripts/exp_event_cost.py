#!/usr/bin/env python3
"""What an event recorded on a busy stream costs that stream: a chain of small kernels with
and without `other.wait_stream(main)` (an event record on main + a wait on the other stream)
or `main.wait_event(done)` (a wait for something long finished) between them."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

dev = torch.device("cuda", 0)
main = torch.cuda.current_stream(dev)
other = torch.cuda.Stream(device=dev)
x = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
big = torch.zeros(1 << 28, dtype=torch.int32, device=dev)  # 1 GiB: leaves the caches dirty
done = torch.cuda.Event()
done.record(main)
torch.cuda.synchronize()


def run(mode, n=200, dirty=False):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        if dirty:
            big.add_(1)
        else:
            x.add_(1)
        if mode == "record+wait_other":
            other.wait_stream(main)
        elif mode == "wait_done":
            main.wait_event(done)
        elif mode == "record_only":
            torch.cuda.Event().record(main)
        x.add_(1)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


for dirty in (False, True):
    base = None
    for mode in ("none", "record_only", "record+wait_other", "wait_done"):
        run(mode, 20, dirty)
        us = min(run(mode, 200, dirty) for _ in range(3))
        base = us if mode == "none" else base
        print(f"{'1 GiB kernel' if dirty else 'small kernel'} + {mode:18s}: {us:8.1f} us per pair"
              f"  (+{us - base:.1f})", flush=True)
