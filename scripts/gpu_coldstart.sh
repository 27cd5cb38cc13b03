#!/bin/bash
# Is the first bench process on a fresh box slower? Six back-to-back runs, then per-round times of a fresh process.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for i in 1 2 3 4; do
  timeout -k 10 120 python $R/bench.py --steps 10 --warmup 3 > gpurun_out/cold_$i.log 2>&1 || { tail -20 gpurun_out/cold_$i.log; exit 1; }
  echo "run $i $(tail -1 gpurun_out/cold_$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 120 python - <<'PY'
import sys, time, torch
sys.path.insert(0, ".")
from sda_amd.engine import DeviceAggregator
from sda_amd.models.schemes import Additive, AggregationSpec
agg = DeviceAggregator(AggregationSpec(1_000_000, 433, Additive(3, 433)))
x = torch.randint(0, 433, (1000, 1_000_000), dtype=torch.int32, device="cuda")
ts = []
for i in range(40):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    agg.run_round(x, check=False)
    torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) * 1e3)
print("per-round ms:", " ".join(f"{t:.1f}" for t in ts))
PY
