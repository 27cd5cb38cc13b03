#!/bin/bash
# Repeated headline benches (single engine, then the committee round on one rank) for run-to-run spread.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for i in 1 2 3; do
  timeout -k 10 120 python $R/bench.py --steps 20 --warmup 3 > gpurun_out/rep_single_$i.log 2>&1 || { tail -20 gpurun_out/rep_single_$i.log; exit 1; }
  echo "single $i $(tail -1 gpurun_out/rep_single_$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
for w in 1 2 4 8; do
  timeout -k 10 180 python $R/bench.py --gpus 1 --force-dist --layout committee --waves $w --steps 20 --warmup 3 > gpurun_out/rep_committee_w$w.log 2>&1 || { tail -20 gpurun_out/rep_committee_w$w.log; exit 1; }
  echo "committee waves=$w $(tail -1 gpurun_out/rep_committee_w$w.log | grep -o '"ms_per_step": [0-9.]*')"
done
