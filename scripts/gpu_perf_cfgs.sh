#!/bin/bash
# Kernel + share tests, then wall times of the many-clerk configurations and the headline.
set -e
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pss.py -x -q --timeout 120 --timeout-method thread > $O/perf_tests.log 2>&1 || { tail -30 $O/perf_tests.log; exit 1; }
tail -2 $O/perf_tests.log
for c in "$@"; do
  timeout -k 10 300 python bench_configs.py --config $c --steps 5 --warmup 2 --check > $O/perf_cfg$c.json 2> $O/perf_cfg$c.err || { tail -20 $O/perf_cfg$c.err; exit 1; }
  python - "$O/perf_cfg$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("config", d["config"], "ms/round", round(d["ms_per_round"], 2), "correct", d["correct"], flush=True)
PY
done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/perf_bench.log 2>&1 || { tail -30 $O/perf_bench.log; exit 1; }
tail -1 $O/perf_bench.log | cut -c1-200
