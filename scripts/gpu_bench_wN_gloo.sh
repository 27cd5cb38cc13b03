#!/bin/bash
# bench.py's N > 1 path (wave autotuning, committee exchange, clerk-internal partials, liveness
# rendezvous, sealed results) rehearsed with N gloo ranks sharing the one GPU (device tensors staged
# through host memory): small shapes, correctness only. usage: gpu_bench_wN_gloo.sh N [N ...]
set -e
mkdir -p gpurun_out
for N in "$@"; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2953$N \
  bench.py --gpus $N --dist-backend gloo --participants 24 --dim 50000 --steps 3 --warmup 1 --check > gpurun_out/bench_w${N}_gloo.log 2>&1 || { tail -30 gpurun_out/bench_w${N}_gloo.log; exit 1; }
echo "N=$N $(tail -1 gpurun_out/bench_w${N}_gloo.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/bench_w${N}_gloo.log | grep -o '"xgmi.*timed_steps' | cut -c1-420)"
done
