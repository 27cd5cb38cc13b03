#!/bin/bash
# Distributed engine on one GPU: tests, then world-1 committee/owner overhead vs the plain round.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_dist_tests.log 2>&1 || { tail -40 gpurun_out/gpu_dist_tests.log; exit 1; }
tail -3 gpurun_out/gpu_dist_tests.log
timeout -k 10 120 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_single.log 2>&1 && tail -1 gpurun_out/bench_single.log | cut -c1-300
for lay in committee owner; do
  timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --force-dist --layout $lay --steps 10 --warmup 3 --stages > gpurun_out/bench_dist_${lay}_w1.log 2>&1 || { tail -30 gpurun_out/bench_dist_${lay}_w1.log; exit 1; }
  grep -h "stage_ms\|^{" gpurun_out/bench_dist_${lay}_w1.log | cut -c1-400
done
