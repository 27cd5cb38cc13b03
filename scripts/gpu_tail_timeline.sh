#!/bin/bash
# Kernel timeline of a headline round, every kernel with its queue: shows where a round's
# result path runs against the next round's kernels, and what stands between the big grids.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tt -o tt -- python $R/bench.py --steps 8 --warmup 3 > $O/tail_trace.log 2>&1 || { tail -20 $O/tail_trace.log; exit 1; }
python $R/scripts/round_timeline.py $(find $O/tt -name "*kernel_trace.csv" | head -1) --min-us 0 > $O/tail_timeline_all.txt
head -1 $O/tail_timeline_all.txt
rm -rf $O/tt
