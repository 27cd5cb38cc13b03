# Kernel numerics + MAC A/B + headline bench + rocprofv3 kernel stats, one GPU call.
#   gpurun --timeout 900 -- bash scripts/gpu_check.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/t.log 2>&1 && \
timeout -k 10 200 python -u scripts/debug/mac_bench.py > gpurun_out/mac_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --stages > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_bench.log 2>&1
