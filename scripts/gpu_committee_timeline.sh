#!/bin/bash
# Full kernel timeline (every kernel, no duration cut-off) of one committee round at world 1, 4 waves.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
W=${1:-4}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tlc -o tl -- python $R/bench.py --gpus 1 --force-dist --layout committee --waves $W --steps 3 --warmup 2 > $R/gpurun_out/tlc.log 2>&1 || { tail -20 $R/gpurun_out/tlc.log; exit 1; }
f=$(find $R/gpurun_out/tlc -name "*kernel_trace.csv" | head -1)
python $R/scripts/round_timeline.py $f --min-us 0 > $R/gpurun_out/committee_w1_waves${W}_full_timeline.txt
rm -rf $R/gpurun_out/tlc
wc -l $R/gpurun_out/committee_w1_waves${W}_full_timeline.txt
