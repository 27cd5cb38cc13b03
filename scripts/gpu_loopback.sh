#!/bin/bash
# World-1 RCCL loopback: tests, the headline-size loopback round, its kernel timeline.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
echo "== loopback tests"; 
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -k "loopback" -x -v --timeout 200 --timeout-method thread > gpurun_out/loopback_tests.log 2>&1 || { tail -40 gpurun_out/loopback_tests.log; exit 1; }
tail -3 gpurun_out/loopback_tests.log
echo "== loopback headline size"
for w in 1 4; do
timeout -k 10 180 python bench.py --gpus 1 --force-dist --loopback --waves $w --dist-timeout 60 --steps 10 --warmup 3 > gpurun_out/r3_loopback_waves$w.log 2>&1 || { tail -30 gpurun_out/r3_loopback_waves$w.log; exit 1; }
tail -1 gpurun_out/r3_loopback_waves$w.log | cut -c1-330
done
echo "== unchunked ops (which message sizes RCCL's self send/recv carries correctly)"
for w in 4 2 1; do
timeout -k 10 180 python bench.py --gpus 1 --force-dist --loopback --waves $w --p2p-chunk-mb 16384 --dist-timeout 60 --steps 3 --warmup 1 > gpurun_out/r3_loopback_unchunked_waves$w.log 2>&1 && echo "waves $w unchunked: ok" || echo "waves $w unchunked: FAILED ($(grep -o 'device error word.*' gpurun_out/r3_loopback_unchunked_waves$w.log | head -1))"
done
echo "== loopback timeline"
cd /tmp && export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tlc -o tl -- python $R/bench.py --gpus 1 --force-dist --loopback --layout committee --waves 4 --dist-timeout 60 --steps 3 --warmup 2 > $R/gpurun_out/tlc.log 2>&1 || { tail -20 $R/gpurun_out/tlc.log; exit 1; }
f=$(find $R/gpurun_out/tlc -name "*kernel_trace.csv" | head -1)
python $R/scripts/round_timeline.py $f --min-us 0 > $R/gpurun_out/r3_loopback_w1_waves4_timeline.txt
rm -rf $R/gpurun_out/tlc
wc -l $R/gpurun_out/r3_loopback_w1_waves4_timeline.txt
