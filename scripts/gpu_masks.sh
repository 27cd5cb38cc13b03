#!/bin/bash
# ChaCha-mask kernels under rejections, masked rounds, and the three masked presets.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "chacha or mask" -x -v --timeout 120 --timeout-method thread > gpurun_out/mask_tests.log 2>&1 || { tail -40 gpurun_out/mask_tests.log; exit 1; }
tail -12 gpurun_out/mask_tests.log
for c in 2 9 10 11; do
timeout -k 10 300 python bench_configs.py --config $c --check --steps 5 --warmup 2 > gpurun_out/r3_config$c.json 2> gpurun_out/r3_config$c.err || { tail -20 gpurun_out/r3_config$c.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r3_config$c.json')); print($c, d['name'], round(d['ms_per_round'],2), 'ms', d['correct'])"
done
