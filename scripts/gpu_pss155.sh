#!/bin/bash
# PSS_155_728_100 (728 clerks) on the int8-limb MFMA GEMM: scaled check, then 1k x 1M, then kernel stats.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench_configs.py --config 6 --participants 40 --check --steps 2 --warmup 1 | tee gpurun_out/pss155_p40.json
timeout -k 10 600 python bench_configs.py --config 6 --check --steps 2 --warmup 1 | tee gpurun_out/pss155_1kx1m.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pss155_prof -o p -- python $R/bench_configs.py --config 6 --participants 250 --steps 2 --warmup 1 > $R/gpurun_out/pss155_prof.log 2>&1 || { tail -20 $R/gpurun_out/pss155_prof.log; exit 1; }
f=$(find $R/gpurun_out/pss155_prof -name "*kernel_stats.csv" | head -1)
head -14 $f | cut -c1-160
cp $f $R/gpurun_out/pss155_kernel_stats.csv
rm -rf $R/gpurun_out/pss155_prof
