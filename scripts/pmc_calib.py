#!/usr/bin/env python3
"""Known-traffic kernels for calibrating rocprofv3's memory counters: a 1 GiB copy
(reads 1 GiB, writes 1 GiB), a 1 GiB sum (reads 1 GiB) and a 1 GiB fill (writes
1 GiB), three times each. Run under `rocprofv3 --pmc ...`; scripts/gpu_pmc_calib.sh
prints the counters per kernel next to these byte counts."""
import torch

n = 1 << 28  # int32 elements: 1 GiB
x = torch.arange(n, dtype=torch.int32, device="cuda")
y = torch.empty_like(x)
torch.cuda.synchronize()
for _ in range(3):
    y.copy_(x)
    torch.cuda.synchronize()
    s = x.sum()
    torch.cuda.synchronize()
    y.fill_(7)
    torch.cuda.synchronize()
print("ok", int(s.item()) & 0xFFFF)
