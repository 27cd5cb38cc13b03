#!/bin/bash
# Per-kernel times of a bench_configs.py configuration: usage gpu_kstats_cfg.sh CONFIG [extra args]
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
c=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rtc -o rt -- python $R/bench_configs.py --config $c --steps 5 --warmup 2 "$@" > $O/kstats_cfg$c.log 2>&1 || { tail -20 $O/kstats_cfg$c.log; exit 1; }
python $R/scripts/kstats.py $(find $O/rtc -name "*kernel_stats.csv" | head -1) 7 > $O/kstats_cfg$c.txt
rm -rf $O/rtc
head -14 $O/kstats_cfg$c.txt
