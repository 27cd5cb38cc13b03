#!/bin/bash
# Kernel timelines of one committee round at world 1 (RCCL group of one) at 4 and 16 hardware queues.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for q in 0; do
timeout -k 10 180 python $R/bench.py --gpus 1 --force-dist --layout committee --waves 2 --hw-queues $q --steps 10 --warmup 3 > $R/gpurun_out/bench_committee_w1_q$q.log 2>&1 || { tail -30 $R/gpurun_out/bench_committee_w1_q$q.log; exit 1; }
echo "queues=$q $(tail -1 $R/gpurun_out/bench_committee_w1_q$q.log | cut -c100-230)"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl$q -o tl -- python $R/bench.py --gpus 1 --force-dist --layout committee --waves 2 --hw-queues $q --steps 3 --warmup 2 > $R/gpurun_out/tl$q.log 2>&1 || { tail -20 $R/gpurun_out/tl$q.log; exit 1; }
f=$(find $R/gpurun_out/tl$q -name "*kernel_trace.csv" | head -1)
python $R/scripts/round_timeline.py $f --min-us 15 > $R/gpurun_out/committee_w1_q${q}_timeline.txt
rm -rf $R/gpurun_out/tl$q
done
