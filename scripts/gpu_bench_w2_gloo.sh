#!/bin/bash
# bench.py's N > 1 path (wave autotuning, committee exchange, liveness rendezvous) rehearsed with two
# gloo ranks sharing the one GPU (device tensors staged through host memory): small shapes, correctness only.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --dist-backend gloo --participants 24 --dim 50000 --steps 3 --warmup 1 --check > gpurun_out/bench_w2_gloo.log 2>&1 || { tail -30 gpurun_out/bench_w2_gloo.log; exit 1; }
tail -1 gpurun_out/bench_w2_gloo.log | cut -c1-1500
