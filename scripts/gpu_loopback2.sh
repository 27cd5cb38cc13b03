#!/bin/bash
# Loopback round with the probed compute stream: bench at waves 1/2/4/8 + timeline.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for w in 1 2 4 8; do
timeout -k 10 180 python bench.py --gpus 1 --force-dist --loopback --waves $w --dist-timeout 60 --steps 10 --warmup 3 > gpurun_out/r3_loopback_waves$w.log 2>&1 || { tail -30 gpurun_out/r3_loopback_waves$w.log; exit 1; }
tail -1 gpurun_out/r3_loopback_waves$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('waves', d['pipeline_waves'], 'ms', round(d['ms_per_step'],2), d['compute_stream_vs_rccl'])"
done
cd /tmp && export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tlc -o tl -- python $R/bench.py --gpus 1 --force-dist --loopback --layout committee --waves 4 --dist-timeout 60 --steps 3 --warmup 2 > $R/gpurun_out/tlc.log 2>&1 || { tail -20 $R/gpurun_out/tlc.log; exit 1; }
f=$(find $R/gpurun_out/tlc -name "*kernel_trace.csv" | head -1)
python $R/scripts/round_timeline.py $f --min-us 0 > $R/gpurun_out/r3_loopback_w1_waves4_timeline.txt
rm -rf $R/gpurun_out/tlc
grep -c rccl $R/gpurun_out/r3_loopback_w1_waves4_timeline.txt
