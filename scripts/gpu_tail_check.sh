#!/bin/bash
# Round tests, then the headline bench three times and configs 2 and 3 (run-to-run spread).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread -k "unchecked or round or bench" 2>&1 | tail -3
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_e_single$i.log 2>&1 || { tail -20 gpurun_out/r3_e_single$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_e_single$i.log
done
timeout -k 10 120 python bench.py 2>&1 | grep -o '"ms_per_step": [0-9.]*'
bash scripts/gpu_final_configs.sh 2 3
