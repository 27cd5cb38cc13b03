#!/usr/bin/env python3
"""Which of a process's streams stand behind each other? For the main stream and a row of
fresh streams: stream A spins 300 us, stream B is made to wait for an event behind A's spin,
stream C runs a no-op; C's no-op ending with the spin means C sits in B's hardware queue."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from sda_amd.ops import gpu as G

dev = torch.device("cuda", 0)
main = torch.cuda.current_stream(dev)
gate = torch.zeros(1, dtype=torch.int32, device=dev)
streams = [torch.cuda.Stream(device=dev) for _ in range(10)]
print("stream handles", [hex(s.cuda_stream) for s in streams], flush=True)


def blocked(b, c):
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    torch.cuda.synchronize(dev)
    e0.record(main)
    G.gate_wait((gate, 1), timeout_us=300)
    spun = torch.cuda.Event()
    spun.record(main)
    b.wait_event(spun)
    with torch.cuda.stream(c):
        G.gate_wait((gate, 0), timeout_us=1)
        e1.record(c)
    e2.record(main)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / e0.elapsed_time(e2)


for i, b in enumerate(streams[:6]):
    row = []
    for j, c in enumerate(streams):
        row.append("  . " if i == j else f"{blocked(b, c):4.2f}")
    print(f"waiting stream {i}: no-op on stream j ends at (fraction of the spin)", " ".join(row), flush=True)
