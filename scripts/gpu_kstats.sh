#!/bin/bash
# Per-kernel times of the headline round (rocprofv3 --kernel-trace --stats, 5 timed + 2 warm-up rounds).
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rt -o rt -- python $R/bench.py --steps 5 --warmup 2 > $O/kstats.log 2>&1 || { tail -20 $O/kstats.log; exit 1; }
python $R/scripts/kstats.py $(find $O/rt -name "*kernel_stats.csv" | head -1) 7 > $O/kstats.txt
python $R/scripts/round_timeline.py $(find $O/rt -name "*kernel_trace.csv" | head -1) --min-us 15 > $O/ktimeline.txt
rm -rf $O/rt
head -12 $O/kstats.txt
