#!/bin/bash
# Tapered wave schedule: committee round on one rank (overhead), then the N = 2 gloo rehearsal with autotuning.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for w in 4 taper; do
  timeout -k 10 180 python $R/bench.py --gpus 1 --force-dist --layout committee --waves $w --steps 20 --warmup 3 > gpurun_out/rep_committee_w$w.log 2>&1 || { tail -20 gpurun_out/rep_committee_w$w.log; exit 1; }
  echo "committee waves=$w $(tail -1 gpurun_out/rep_committee_w$w.log | grep -o '"ms_per_step": [0-9.]*')"
done
unset MASTER_ADDR MASTER_PORT RANK WORLD_SIZE LOCAL_RANK
bash $R/scripts/gpu_bench_wN_gloo.sh 2
