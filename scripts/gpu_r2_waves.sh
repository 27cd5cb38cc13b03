#!/bin/bash
# Committee round at world 1: wave-count sweep, then the whole GPU suite.
set -e
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for w in 1 2 3 4 8; do
timeout -k 10 180 python bench.py --gpus 1 --force-dist --layout committee --waves $w --steps 10 --warmup 3 > gpurun_out/bench_committee_w1_waves$w.log 2>&1 || { tail -30 gpurun_out/bench_committee_w1_waves$w.log; exit 1; }
echo "waves=$w $(tail -1 gpurun_out/bench_committee_w1_waves$w.log | cut -c100-230)"
done
timeout -k 10 180 python bench.py --gpus 1 --force-dist --layout owner --steps 10 --warmup 3 > gpurun_out/bench_owner_w1.log 2>&1 && echo "owner $(tail -1 gpurun_out/bench_owner_w1.log | cut -c100-230)"
unset MASTER_ADDR MASTER_PORT RANK WORLD_SIZE LOCAL_RANK
timeout -k 10 120 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_single.log 2>&1 && echo "single $(tail -1 gpurun_out/bench_single.log | cut -c100-230)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
