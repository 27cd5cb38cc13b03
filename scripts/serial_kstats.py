#!/usr/bin/env python3
"""A benchmark configuration with the key-agreement side stream folded into the
main stream, so that no two kernels overlap: under `rocprofv3 --kernel-trace
--stats` every kernel's time is then its time alone on the card (in the product
schedule the X25519 ladders share the CUs with the share / encode kernels and
both look slower than they are).

  python scripts/serial_kstats.py CONFIG [STEPS]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from sda_amd.engine import DeviceAggregator
from sda_amd.models.configs import bench_config

DeviceAggregator._side_stream = lambda self: torch.cuda.current_stream(self.device)

c = int(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = bench_config(c)
spec = cfg.spec()
dev = torch.device("cuda", 0)
eng = DeviceAggregator(spec, device=dev, pss_backend=cfg.pss_backend)
x = torch.randint(0, spec.field_modulus, (cfg.participants, cfg.dimension), dtype=torch.int32, device=dev)
clerks = list(cfg.clerks) if cfg.clerks is not None else None
ref = torch.remainder(x.to(torch.int64).sum(0), spec.field_modulus).to(torch.int32)
for i in range(steps + 1):
    res = eng.run_round(x, clerks=clerks, check=True)
    if i == 0 and not torch.equal(res.output, ref):
        raise SystemExit("serial_kstats: wrong aggregate")
    torch.cuda.synchronize()
print("ok", flush=True)
