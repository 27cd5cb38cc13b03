#!/bin/bash
# Committee round at world 1 (RCCL group of one): hardware-queue count A/B with the probed side stream.
set -e
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for q in 0 8 16; do for w in 4 2; do
timeout -k 10 180 python bench.py --gpus 1 --force-dist --layout committee --waves $w --hw-queues $q --steps 10 --warmup 3 > gpurun_out/bench_committee_w1_q${q}_waves$w.log 2>&1 || { tail -30 gpurun_out/bench_committee_w1_q${q}_waves$w.log; exit 1; }
echo "queues=$q waves=$w $(tail -1 gpurun_out/bench_committee_w1_q${q}_waves$w.log | cut -c100-230)"
done; done
timeout -k 10 120 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_single.log 2>&1 && tail -1 gpurun_out/bench_single.log | cut -c100-230
