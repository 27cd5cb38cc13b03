set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_streaming.py -x -q > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_full.log 2>&1 && timeout -k 10 300 python bench.py --steps 20 --warmup 3 >> gpurun_out/bench_full.log 2>&1 && \
mkdir -p gpurun_out/prof && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_bench.log 2>&1
