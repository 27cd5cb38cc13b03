#!/bin/bash
# Config 5 (5-of-8 with clerk dropout) on the register kernel and the MFMA GEMM, p = 433 (u16
# shares) and p = 241 (u8 shares); PSS tests first.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pss.py tests/test_gpu_modgemm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pss_tests.log 2>&1 || { tail -40 gpurun_out/pss_tests.log; exit 1; }
tail -2 gpurun_out/pss_tests.log
for c in 5 7; do for b in valu mfma; do
timeout -k 10 300 python bench_configs.py --config $c --pss-backend $b --check --steps 5 --warmup 2 | tee gpurun_out/config${c}_$b.json | cut -c1-60,330-700
done; done
timeout -k 10 300 python bench_configs.py --config 3 --check --steps 5 --warmup 2 | tee gpurun_out/config3.json | cut -c1-60,330-700
