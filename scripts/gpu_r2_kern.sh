#!/bin/bash
# Kernel iteration loop: kernel tests, then the 1-GPU bench and a kernel timeline.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_share16.py -x -q --timeout 300 --timeout-method thread > gpurun_out/kern_tests.log 2>&1 || { tail -40 gpurun_out/kern_tests.log; exit 1; }
tail -2 gpurun_out/kern_tests.log
timeout -k 10 120 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_single.log 2>&1 || { tail -20 gpurun_out/bench_single.log; exit 1; }
echo "single $(tail -1 gpurun_out/bench_single.log | cut -c100-230)"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl -o tl -- python $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/tl.log 2>&1 || { tail -20 $R/gpurun_out/tl.log; exit 1; }
f=$(find $R/gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python $R/scripts/round_timeline.py $f --min-us 15 > $R/gpurun_out/single_timeline.txt
cat $R/gpurun_out/single_timeline.txt
rm -rf $R/gpurun_out/tl
