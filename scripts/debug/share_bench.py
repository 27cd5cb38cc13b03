import sys, os; sys.path.insert(0, os.getcwd())
import torch
from sda_amd.ops import gpu as G
from sda_amd._native import gpu
P, D, n, m = 1000, 1_000_000, 3, 433
x = torch.randint(0, m, (P, D), dtype=torch.int32, device="cuda")
shares = torch.empty(n, P, D, dtype=torch.int16, device="cuda")
cnt = torch.empty(n * P * G.tiles(D), dtype=torch.int32, device="cuda")
err = torch.zeros(1, dtype=torch.int32, device="cuda")
names = {0: "share32", 1: "share48 (3 draws/word)", 2: "share16 (u16 halves)"}
for mode in (0, 1, 2, 1, 2):
    gpu().set_share16(mode)
    for _ in range(2):
        G.share_additive(x, n, m, shares, cnt, G.MASK_NONE, bytes(32), 0, err=err)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        G.share_additive(x, n, m, shares, cnt, G.MASK_NONE, bytes(32), 0, err=err)
    b.record(); torch.cuda.synchronize()
    print(names[mode], f"{a.elapsed_time(b)/5:.3f} ms", flush=True)
