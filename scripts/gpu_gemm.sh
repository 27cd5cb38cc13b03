#!/bin/bash
# Modular GEMM: numerics tests, then a micro-benchmark at the PSS_155_728_100 share shape.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_modgemm.py tests/test_gpu_pss.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 300 python scripts/bench_modgemm.py | tee gpurun_out/bench_modgemm.txt
