#!/bin/bash
# Per-round times of the FIRST GPU process on a fresh box (60 rounds), then of a second one.
set -e
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python - <<'PY'
import sys, time, torch
sys.path.insert(0, ".")
t00 = time.perf_counter()
from sda_amd.engine import DeviceAggregator
from sda_amd.models.schemes import Additive, AggregationSpec
agg = DeviceAggregator(AggregationSpec(1_000_000, 433, Additive(3, 433)))
x = torch.randint(0, 433, (1000, 1_000_000), dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
print(f"setup {time.perf_counter() - t00:.2f} s")
ts, hs = [], []
for i in range(60):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    agg.run_round(x, check=False)
    h = time.perf_counter() - t0
    torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) * 1e3); hs.append(h * 1e3)
print("round ms:", " ".join(f"{t:.1f}" for t in ts))
print("host  ms:", " ".join(f"{t:.1f}" for t in hs))
PY
done
