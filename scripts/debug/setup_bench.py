"""Seal-setup latency vs message count, alone and next to the share kernel."""
import sys, os; sys.path.insert(0, os.getcwd())
import torch
from sda_amd.ops import gpu as G
from sda_amd.ops.sealed import Arena, seal_setup
from sda_amd.engine import DeviceAggregator
from sda_amd.models import Additive, AggregationSpec

P, D, n, m = 1000, 1_000_000, 3, 433
eng = DeviceAggregator(AggregationSpec(D, m, Additive(n, m)))
pks = eng.keys.pks
x = torch.randint(0, m, (P, D), dtype=torch.int32, device="cuda")
shares = torch.empty(n, P, D, dtype=torch.int16, device="cuda")
cnt = torch.empty(n * P * G.tiles(D), dtype=torch.int32, device="cuda")
err = torch.zeros(1, dtype=torch.int32, device="cuda")
side = torch.cuda.Stream(priority=-1)


def ev():
    return torch.cuda.Event(enable_timing=True)


for M in (3, 64, 512, 3000, 6000):
    arena = Arena.empty(M, 16, m)
    kidx = torch.zeros(M, dtype=torch.int32, device="cuda")
    for conc in (False, True, False, True):
        torch.cuda.synchronize()
        a, b, c, d = ev(), ev(), ev(), ev()
        c.record()
        if conc:
            G.share_additive(x, n, m, shares, cnt, G.MASK_NONE, bytes(32), 0, err=err)
        d.record()
        side.wait_stream(torch.cuda.current_stream()) if not conc else None
        with torch.cuda.stream(side):
            a.record(side)
            seal_setup(arena, kidx, pks, bytes(32), 0, err)
            b.record(side)
        torch.cuda.synchronize()
        print(f"M={M:5d} {'with share' if conc else 'alone     '} setup {a.elapsed_time(b):7.3f} ms"
              f"  share {c.elapsed_time(d):7.3f} ms", flush=True)
