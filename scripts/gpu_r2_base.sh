#!/bin/bash
# Bench at the default hardware-queue count, at 16 and at 2, then the GPU suite.
set -e
mkdir -p gpurun_out
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
timeout -k 10 120 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_q_default.log 2>&1 && tail -1 gpurun_out/bench_q_default.log
timeout -k 10 120 python bench.py --steps 10 --warmup 3 --hw-queues 16 > gpurun_out/bench_q16.log 2>&1 && tail -1 gpurun_out/bench_q16.log
timeout -k 10 120 python bench.py --steps 10 --warmup 3 --hw-queues 2 > gpurun_out/bench_q2.log 2>&1 && tail -1 gpurun_out/bench_q2.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; tail -3 gpurun_out/gpu_tests.log
