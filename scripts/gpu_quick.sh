#!/bin/bash
# Kernel tests, then the headline bench (10 timed rounds).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || { tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
timeout -k 10 120 python bench.py --steps 10 --warmup 3 > gpurun_out/quick_bench.log 2>&1 || { tail -30 gpurun_out/quick_bench.log; exit 1; }
tail -1 gpurun_out/quick_bench.log | cut -c1-330
