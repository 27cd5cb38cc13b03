#!/bin/bash
# Config 4: 10k participants x 125M values, PSS_4_8_3, streamed in waves on one GPU, output checked.
set -e
mkdir -p gpurun_out
( while true; do sleep 60; echo "config 4 still running $(date +%T)"; done ) &
HB=$!
timeout -k 10 900 python -u bench_configs.py --config 4 --check > gpurun_out/config4.json 2> gpurun_out/config4.err || { kill $HB; tail -20 gpurun_out/config4.err; exit 1; }
kill $HB
cut -c1-60,250-900 gpurun_out/config4.json
