#!/bin/bash
# The reference's largest packed-Shamir set (19,682 clerks) end to end: first 4, then 16 participants x 1M.
set -e
mkdir -p gpurun_out
echo "config 8, 4 participants"; 
timeout -k 10 400 python -u bench_configs.py --config 8 --participants 4 --check --steps 2 --warmup 1 > gpurun_out/config8_p4.json 2> gpurun_out/config8_p4.err || { tail -20 gpurun_out/config8_p4.err; exit 1; }
cut -c1-60,300-800 gpurun_out/config8_p4.json
echo "config 8, 16 participants";
timeout -k 10 500 python -u bench_configs.py --config 8 --check --steps 2 --warmup 1 > gpurun_out/config8.json 2> gpurun_out/config8.err || { tail -20 gpurun_out/config8.err; exit 1; }
cut -c1-60,300-800 gpurun_out/config8.json
